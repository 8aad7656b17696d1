/*
 * ec.c -- GF(2^255-19) and edwards25519 group arithmetic for the oracle,
 * plus Ed25519 (libsodium 1.0.18 rules) and ECVRF draft-03 (IOG fork).
 * TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * Representation: radix 2^51, 5 x uint64 limbs, unsigned __int128 products.
 * (The GPU kernels use radix 2^32 x 8 limbs; this is deliberately different.)
 * Scalar multiplication is plain MSB-first double-and-add on extended
 * coordinates; correctness of the group law is all that matters here, since
 * every verdict in the reference is a function of the resulting point
 * encodings, not of the evaluation strategy.
 *
 * Reference call sites: Ed25519 at Praos.hs:580 (OCert) and inside
 * KES.verifySignedKES (Praos.hs:582); VRF at Praos.hs:543.
 * Semantics restated from libsodium 1.0.18
 *   crypto_sign/ed25519/ref10/open.c `_crypto_sign_ed25519_verify_detached`
 *   crypto_core/ed25519/ref10/ed25519_ref10.c (frombytes, has_small_order,
 *   is_canonical, from_uniform)
 * and IOG libsodium `crypto_vrf/ietfdraft03/{verify,prove,convert}.c`
 * (versions pinned in SURVEY.md sec. 8c).
 */
#include <string.h>
#include "oracle.h"

typedef unsigned __int128 u128;
typedef struct { uint64_t v[5]; } fe;
static const uint64_t M51 = (1ULL << 51) - 1;

static void fe_0(fe *h) { memset(h, 0, sizeof *h); }
static void fe_1(fe *h) { fe_0(h); h->v[0] = 1; }
static void fe_small(fe *h, uint64_t x) { fe_0(h); h->v[0] = x; }

static void fe_carry(fe *h) {
  for (int k = 0; k < 2; k++) {
    uint64_t c;
    for (int i = 0; i < 4; i++) { c = h->v[i] >> 51; h->v[i] &= M51; h->v[i + 1] += c; }
    c = h->v[4] >> 51; h->v[4] &= M51; h->v[0] += 19 * c;
  }
}
static void fe_add(fe *h, const fe *f, const fe *g) {
  for (int i = 0; i < 5; i++) h->v[i] = f->v[i] + g->v[i];
  fe_carry(h);
}
static void fe_sub(fe *h, const fe *f, const fe *g) {
  /* add 4p to stay non-negative */
  static const uint64_t P4[5] = {0x1fffffffffffb4ULL, 0x1ffffffffffffcULL, 0x1ffffffffffffcULL,
                                 0x1ffffffffffffcULL, 0x1ffffffffffffcULL};
  for (int i = 0; i < 5; i++) h->v[i] = f->v[i] + P4[i] - g->v[i];
  fe_carry(h);
}
static void fe_neg(fe *h, const fe *f) { fe z; fe_0(&z); fe_sub(h, &z, f); }
static void fe_mul(fe *h, const fe *f, const fe *g) {
  const uint64_t *a = f->v, *b = g->v;
  u128 t[5];
  uint64_t b19[5];
  for (int i = 0; i < 5; i++) b19[i] = b[i] * 19;
  t[0] = (u128)a[0] * b[0] + (u128)a[1] * b19[4] + (u128)a[2] * b19[3] + (u128)a[3] * b19[2] + (u128)a[4] * b19[1];
  t[1] = (u128)a[0] * b[1] + (u128)a[1] * b[0] + (u128)a[2] * b19[4] + (u128)a[3] * b19[3] + (u128)a[4] * b19[2];
  t[2] = (u128)a[0] * b[2] + (u128)a[1] * b[1] + (u128)a[2] * b[0] + (u128)a[3] * b19[4] + (u128)a[4] * b19[3];
  t[3] = (u128)a[0] * b[3] + (u128)a[1] * b[2] + (u128)a[2] * b[1] + (u128)a[3] * b[0] + (u128)a[4] * b19[4];
  t[4] = (u128)a[0] * b[4] + (u128)a[1] * b[3] + (u128)a[2] * b[2] + (u128)a[3] * b[1] + (u128)a[4] * b[0];
  uint64_t r[5], c = 0;
  for (int i = 0; i < 5; i++) { t[i] += c; r[i] = (uint64_t)t[i] & M51; c = (uint64_t)(t[i] >> 51); }
  r[0] += c * 19;
  c = r[0] >> 51; r[0] &= M51; r[1] += c;
  memcpy(h->v, r, sizeof r);
}
static void fe_sq(fe *h, const fe *f) { fe_mul(h, f, f); }

/* canonical little-endian encoding */
static void fe_tobytes(uint8_t s[32], const fe *f) {
  fe h = *f;
  fe_carry(&h);
  /* now h < 2^255 + small; subtract p if >= p */
  uint64_t q = (h.v[0] + 19) >> 51;
  q = (h.v[1] + q) >> 51; q = (h.v[2] + q) >> 51; q = (h.v[3] + q) >> 51; q = (h.v[4] + q) >> 51;
  h.v[0] += 19 * q;
  uint64_t c;
  c = h.v[0] >> 51; h.v[0] &= M51; h.v[1] += c;
  c = h.v[1] >> 51; h.v[1] &= M51; h.v[2] += c;
  c = h.v[2] >> 51; h.v[2] &= M51; h.v[3] += c;
  c = h.v[3] >> 51; h.v[3] &= M51; h.v[4] += c;
  h.v[4] &= M51;
  uint8_t out[32] = {0};
  int bit = 0;
  for (int i = 0; i < 5; i++)
    for (int j = 0; j < 51; j++, bit++)
      if ((h.v[i] >> j) & 1) out[bit >> 3] |= (uint8_t)(1u << (bit & 7));
  memcpy(s, out, 32);
}
/* loads 255 bits (top bit ignored), value may be >= p (arithmetic is mod p) */
static void fe_frombytes(fe *h, const uint8_t s[32]) {
  fe_0(h);
  for (int bit = 0; bit < 255; bit++)
    if ((s[bit >> 3] >> (bit & 7)) & 1) h->v[bit / 51] |= 1ULL << (bit % 51);
}
static int fe_iszero(const fe *f) { uint8_t s[32]; fe_tobytes(s, f); uint8_t d = 0; for (int i = 0; i < 32; i++) d |= s[i]; return d == 0; }
static int fe_isnegative(const fe *f) { uint8_t s[32]; fe_tobytes(s, f); return s[0] & 1; }
static int fe_eq(const fe *a, const fe *b) { uint8_t x[32], y[32]; fe_tobytes(x, a); fe_tobytes(y, b); return memcmp(x, y, 32) == 0; }

/* f^e for e given as little-endian bytes (MSB-first square-and-multiply) */
static void fe_pow(fe *h, const fe *f, const uint8_t e[32]) {
  fe r; fe_1(&r);
  for (int bit = 255; bit >= 0; bit--) {
    fe_sq(&r, &r);
    if ((e[bit >> 3] >> (bit & 7)) & 1) fe_mul(&r, &r, f);
  }
  *h = r;
}
static uint8_t E_PM2[32], E_PM5D8[32], E_PM1D2[32], E_PM1D4[32];
static void fe_invert(fe *h, const fe *f) { fe_pow(h, f, E_PM2); }

typedef struct { fe X, Y, Z, T; } ge;
static fe FE_D, FE_D2, FE_SQRTM1, FE_A;
static ge GE_B;
static int inited = 0;

/* little-endian byte string of p - k, then shifted right */
static void sub_small_le(uint8_t out[32], uint32_t k) {
  /* p = 2^255 - 19 */
  uint8_t p[32];
  memset(p, 0xff, 32); p[31] = 0x7f; p[0] = 0xed;
  int borrow = 0;
  for (int i = 0; i < 32; i++) {
    int kb = i < 4 ? (int)((k >> (8 * i)) & 0xff) : 0;
    int v = p[i] - kb - borrow;
    borrow = v < 0; out[i] = (uint8_t)(v + (borrow ? 256 : 0));
  }
}
static void shr_le(uint8_t x[32], int n) {
  for (int k = 0; k < n; k++) {
    for (int i = 0; i < 32; i++) x[i] = (uint8_t)((x[i] >> 1) | ((i < 31 ? x[i + 1] & 1 : 0) << 7));
  }
}

static void ge_identity(ge *p) { fe_0(&p->X); fe_1(&p->Y); fe_1(&p->Z); fe_0(&p->T); }
/* unified addition, a = -1 twisted Edwards (add-2008-hwcd-3) */
static void ge_add(ge *r, const ge *p, const ge *q) {
  fe a, b, c, d, t1, t2, e, f, g, h;
  fe_sub(&t1, &p->Y, &p->X); fe_sub(&t2, &q->Y, &q->X); fe_mul(&a, &t1, &t2);
  fe_add(&t1, &p->Y, &p->X); fe_add(&t2, &q->Y, &q->X); fe_mul(&b, &t1, &t2);
  fe_mul(&c, &p->T, &q->T); fe_mul(&c, &c, &FE_D2);
  fe_mul(&d, &p->Z, &q->Z); fe_add(&d, &d, &d);
  fe_sub(&e, &b, &a); fe_sub(&f, &d, &c); fe_add(&g, &d, &c); fe_add(&h, &b, &a);
  fe_mul(&r->X, &e, &f); fe_mul(&r->Y, &g, &h); fe_mul(&r->T, &e, &h); fe_mul(&r->Z, &f, &g);
}
static void ge_dbl(ge *r, const ge *p) { ge_add(r, p, p); }
static void ge_neg(ge *r, const ge *p) { fe_neg(&r->X, &p->X); r->Y = p->Y; r->Z = p->Z; fe_neg(&r->T, &p->T); }

static void ge_tobytes(uint8_t s[32], const ge *p) {
  fe zi, x, y;
  fe_invert(&zi, &p->Z);
  fe_mul(&x, &p->X, &zi); fe_mul(&y, &p->Y, &zi);
  fe_tobytes(s, &y);
  s[31] ^= (uint8_t)(fe_isnegative(&x) << 7);
}

/* libsodium ge25519_frombytes: returns 0 ok / -1 not on curve.  y is taken
 * mod p from the low 255 bits (non-canonical y accepted); x = 0 with the sign
 * bit set is accepted and decodes to x = 0. */
static int ge_frombytes(ge *h, const uint8_t s[32]) {
  fe u, v, v3, vxx, chk, one;
  fe_1(&one);
  fe_frombytes(&h->Y, s);
  fe_1(&h->Z);
  fe_sq(&u, &h->Y);
  fe_mul(&v, &u, &FE_D);
  fe_sub(&u, &u, &one);            /* u = y^2 - 1 */
  fe_add(&v, &v, &one);            /* v = d y^2 + 1 */
  fe_sq(&v3, &v); fe_mul(&v3, &v3, &v);            /* v^3 */
  fe_sq(&h->X, &v3); fe_mul(&h->X, &h->X, &v); fe_mul(&h->X, &h->X, &u);  /* u v^7 */
  fe_pow(&h->X, &h->X, E_PM5D8);
  fe_mul(&h->X, &h->X, &v3); fe_mul(&h->X, &h->X, &u);   /* u v^3 (u v^7)^((p-5)/8) */
  fe_sq(&vxx, &h->X); fe_mul(&vxx, &vxx, &v);
  fe_sub(&chk, &vxx, &u);
  if (!fe_iszero(&chk)) {
    fe_add(&chk, &vxx, &u);
    if (!fe_iszero(&chk)) return -1;
    fe_mul(&h->X, &h->X, &FE_SQRTM1);
  }
  if (fe_isnegative(&h->X) != (s[31] >> 7)) fe_neg(&h->X, &h->X);
  fe_mul(&h->T, &h->X, &h->Y);
  return 0;
}

static void ge_scalarmult(ge *r, const uint8_t k[32], const ge *p) {
  ge acc; ge_identity(&acc);
  for (int bit = 255; bit >= 0; bit--) {
    ge_dbl(&acc, &acc);
    if ((k[bit >> 3] >> (bit & 7)) & 1) ge_add(&acc, &acc, p);
  }
  *r = acc;
}
static int ge_is_identity(const ge *p) { return fe_iszero(&p->X) && fe_eq(&p->Y, &p->Z); }

/* ---- scalars mod L (bit-serial reduction; simple and obviously right) ---- */
static const uint8_t L_LE[32] = {0xed, 0xd3, 0xf5, 0x5c, 0x1a, 0x63, 0x12, 0x58, 0xd6, 0x9c, 0xf7,
                                 0xa2, 0xde, 0xf9, 0xde, 0x14, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0x10};
/* r = x mod L, x little-endian of n bytes (n <= 64) */
static void sc_reduce_n(uint8_t r[32], const uint8_t *x, int n) {
  /* work in 64-bit words, 9 words (576 bits) */
  uint64_t acc[5] = {0}, Lw[5] = {0};
  for (int i = 0; i < 32; i++) Lw[i / 8] |= (uint64_t)L_LE[i] << (8 * (i % 8));
  for (int bit = 8 * n - 1; bit >= 0; bit--) {
    /* acc = 2*acc + bit */
    uint64_t carry = (x[bit >> 3] >> (bit & 7)) & 1;
    for (int i = 0; i < 5; i++) { uint64_t nc = acc[i] >> 63; acc[i] = (acc[i] << 1) | carry; carry = nc; }
    /* if acc >= L: acc -= L */
    int ge_ = 1;
    for (int i = 4; i >= 0; i--) { if (acc[i] != Lw[i]) { ge_ = acc[i] > Lw[i]; break; } }
    if (ge_) {
      uint64_t b = 0;
      for (int i = 0; i < 5; i++) { u128 d = (u128)acc[i] - Lw[i] - b; acc[i] = (uint64_t)d; b = (uint64_t)(d >> 64) & 1; }
    }
  }
  for (int i = 0; i < 32; i++) r[i] = (uint8_t)(acc[i / 8] >> (8 * (i % 8)));
}
static void sc_reduce64(uint8_t r[32], const uint8_t x[64]) { sc_reduce_n(r, x, 64); }
/* r = a*b + c mod L */
static void sc_muladd(uint8_t r[32], const uint8_t a[32], const uint8_t b[32], const uint8_t c[32]) {
  uint32_t t[17] = {0};
  uint64_t prod[16] = {0};
  for (int i = 0; i < 8; i++) {
    uint64_t ai = (uint64_t)a[4 * i] | ((uint64_t)a[4 * i + 1] << 8) | ((uint64_t)a[4 * i + 2] << 16) | ((uint64_t)a[4 * i + 3] << 24);
    uint64_t carry = 0;
    for (int j = 0; j < 8; j++) {
      uint64_t bj = (uint64_t)b[4 * j] | ((uint64_t)b[4 * j + 1] << 8) | ((uint64_t)b[4 * j + 2] << 16) | ((uint64_t)b[4 * j + 3] << 24);
      u128 s = (u128)ai * bj + prod[i + j] + carry;
      prod[i + j] = (uint64_t)s & 0xffffffffULL; carry = (uint64_t)(s >> 32);
    }
    prod[i + 8] += carry;
  }
  uint64_t carry = 0;
  for (int i = 0; i < 16; i++) {
    uint64_t ci = (i < 8) ? ((uint64_t)c[4 * i] | ((uint64_t)c[4 * i + 1] << 8) | ((uint64_t)c[4 * i + 2] << 16) | ((uint64_t)c[4 * i + 3] << 24)) : 0;
    uint64_t s = prod[i] + ci + carry;
    t[i] = (uint32_t)s; carry = s >> 32;
  }
  uint8_t x[68];
  for (int i = 0; i < 17; i++) for (int j = 0; j < 4; j++) if (4 * i + j < 68) x[4 * i + j] = (uint8_t)(t[i] >> (8 * j));
  sc_reduce_n(r, x, 64);
}
static int sc_is_canonical(const uint8_t s[32]) {
  for (int i = 31; i >= 0; i--) {
    if (s[i] < L_LE[i]) return 1;
    if (s[i] > L_LE[i]) return 0;
  }
  return 0; /* equal to L */
}

/* ---- init: constants derived, not transcribed ---- */
static void init(void) {
  if (inited) return;
  sub_small_le(E_PM2, 2);
  uint8_t t[32];
  sub_small_le(t, 5); shr_le(t, 3); memcpy(E_PM5D8, t, 32);
  sub_small_le(t, 1); shr_le(t, 1); memcpy(E_PM1D2, t, 32);
  sub_small_le(t, 1); shr_le(t, 2); memcpy(E_PM1D4, t, 32);
  fe n1, n2, inv;
  fe_small(&n1, 121665); fe_small(&n2, 121666);
  fe_invert(&inv, &n2); fe_mul(&FE_D, &n1, &inv); fe_neg(&FE_D, &FE_D);   /* d = -121665/121666 */
  fe_add(&FE_D2, &FE_D, &FE_D);
  fe two; fe_small(&two, 2); fe_pow(&FE_SQRTM1, &two, E_PM1D4);          /* 2^((p-1)/4) */
  fe_small(&FE_A, 486662);
  /* base point: y = 4/5, x even */
  fe four, five, y; fe_small(&four, 4); fe_small(&five, 5); fe_invert(&inv, &five); fe_mul(&y, &four, &inv);
  uint8_t enc[32]; fe_tobytes(enc, &y);
  inited = 1;
  ge_frombytes(&GE_B, enc);
}

/* ---- libsodium blacklist / canonicity (ed25519_ref10.c) ---- */
static int has_small_order(const uint8_t s[32]) {
  /* y in {0, 1, p-1, p, p+1, y8a, y8b} with the sign bit ignored */
  static const uint8_t y8a[32] = {0x26, 0xe8, 0x95, 0x8f, 0xc2, 0xb2, 0x27, 0xb0, 0x45, 0xc3, 0xf4, 0x89, 0xf2, 0xef, 0x98, 0xf0,
                                  0xd5, 0xdf, 0xac, 0x05, 0xd3, 0xc6, 0x33, 0x39, 0xb1, 0x38, 0x02, 0x88, 0x6d, 0x53, 0xfc, 0x05};
  static const uint8_t y8b[32] = {0xc7, 0x17, 0x6a, 0x70, 0x3d, 0x4d, 0xd8, 0x4f, 0xba, 0x3c, 0x0b, 0x76, 0x0d, 0x10, 0x67, 0x0f,
                                  0x2a, 0x20, 0x53, 0xfa, 0x2c, 0x39, 0xcc, 0xc6, 0x4e, 0xc7, 0xfd, 0x77, 0x92, 0xac, 0x03, 0x7a};
  uint8_t b[7][32];
  memset(b, 0, sizeof b);
  b[1][0] = 1;
  memcpy(b[2], y8a, 32); memcpy(b[3], y8b, 32);
  for (int k = 4; k < 7; k++) { memset(b[k], 0xff, 32); b[k][31] = 0x7f; }
  b[4][0] = 0xec; b[5][0] = 0xed; b[6][0] = 0xee;
  for (int k = 0; k < 7; k++) {
    if (memcmp(s, b[k], 31) == 0 && (s[31] & 0x7f) == b[k][31]) return 1;
  }
  return 0;
}
static int ge_is_canonical(const uint8_t s[32]) {
  /* y (255 bits) < p */
  if ((s[31] & 0x7f) != 0x7f) return 1;
  for (int i = 30; i > 0; i--) if (s[i] != 0xff) return 1;
  return s[0] < 0xed;
}

/* ---- Ed25519 ---- */
int orc_ed25519_verify(const uint8_t sig[64], const uint8_t *m, size_t n, const uint8_t pk[32]) {
  init();
  if (!sc_is_canonical(sig + 32) || has_small_order(sig)) return -1;
  if (!ge_is_canonical(pk) || has_small_order(pk)) return -1;
  ge A;
  if (ge_frombytes(&A, pk) != 0) return -1;
  /* h = SHA512(R || A || M) mod L */
  uint8_t hbuf[64], h[32];
  {
    uint8_t stackbuf[1024];
    uint8_t *buf = stackbuf;
    size_t tot = 64 + n;
    uint8_t *heap = NULL;
    if (tot > sizeof stackbuf) { extern void *malloc(size_t); heap = (uint8_t *)malloc(tot); buf = heap; }
    memcpy(buf, sig, 32); memcpy(buf + 32, pk, 32); memcpy(buf + 64, m, n);
    orc_sha512(hbuf, buf, tot);
    if (heap) { extern void free(void *); free(heap); }
  }
  sc_reduce64(h, hbuf);
  ge sB, hA, R;
  ge_scalarmult(&sB, sig + 32, &GE_B);
  ge_scalarmult(&hA, h, &A);
  ge_neg(&hA, &hA);
  ge_add(&R, &sB, &hA);
  uint8_t rcheck[32];
  ge_tobytes(rcheck, &R);
  return memcmp(rcheck, sig, 32) == 0 ? 0 : -1;
}

static void expand_seed(uint8_t az[64], const uint8_t seed[32]) {
  orc_sha512(az, seed, 32);
  az[0] &= 248; az[31] &= 127; az[31] |= 64;
}
void orc_ed25519_pk_from_seed(uint8_t pk[32], const uint8_t seed[32]) {
  init();
  uint8_t az[64]; ge A;
  expand_seed(az, seed);
  ge_scalarmult(&A, az, &GE_B);
  ge_tobytes(pk, &A);
}
void orc_ed25519_sign(uint8_t sig[64], const uint8_t *m, size_t n, const uint8_t seed[32]) {
  init();
  uint8_t az[64], pk[32], rh[64], r[32], hh[64], h[32];
  expand_seed(az, seed);
  ge A; ge_scalarmult(&A, az, &GE_B); ge_tobytes(pk, &A);
  extern void *malloc(size_t); extern void free(void *);
  uint8_t *buf = (uint8_t *)malloc(64 + n);
  memcpy(buf, az + 32, 32); memcpy(buf + 32, m, n);
  orc_sha512(rh, buf, 32 + n);
  sc_reduce64(r, rh);
  ge R; ge_scalarmult(&R, r, &GE_B); ge_tobytes(sig, &R);
  memcpy(buf, sig, 32); memcpy(buf + 32, pk, 32); memcpy(buf + 64, m, n);
  orc_sha512(hh, buf, 64 + n);
  free(buf);
  sc_reduce64(h, hh);
  sc_muladd(sig + 32, h, az, r);
}

/* ---- ECVRF-ED25519-SHA512-Elligator2, draft-03 ---- */
static void chi(fe *out, const fe *z) { fe_pow(out, z, E_PM1D2); }

/* libsodium ge25519_from_uniform (1.0.18); r has its sign bit already cleared
 * by the VRF caller, so x_sign is 0 */
static void from_uniform(uint8_t s[32], const uint8_t r[32]) {
  fe rr2, x, x2, x3, e, negx, one;
  uint8_t t[32];
  memcpy(t, r, 32);
  uint8_t x_sign = t[31] & 0x80;
  t[31] &= 0x7f;
  fe_1(&one);
  fe_frombytes(&rr2, t);
  fe_sq(&rr2, &rr2); fe_add(&rr2, &rr2, &rr2);   /* 2 r^2 */
  fe_add(&rr2, &rr2, &one);                       /* 1 + 2 r^2 */
  fe_invert(&rr2, &rr2);
  fe_mul(&x, &FE_A, &rr2); fe_neg(&x, &x);        /* x = -A / (1 + 2 r^2) */
  fe_sq(&x2, &x); fe_mul(&x3, &x, &x2);
  fe_add(&e, &x3, &x);
  fe_mul(&x2, &x2, &FE_A);
  fe_add(&e, &x2, &e);                            /* e = x^3 + A x^2 + x */
  chi(&e, &e);
  uint8_t eb[32]; fe_tobytes(eb, &e);
  int e_is_minus_1 = eb[1] & 1;
  if (e_is_minus_1) { fe_neg(&negx, &x); fe_sub(&x, &negx, &FE_A); }
  /* y_ed = (x - 1) / (x + 1) */
  fe xp1, xm1, inv, yed;
  fe_add(&xp1, &x, &one); fe_sub(&xm1, &x, &one);
  fe_invert(&inv, &xp1); fe_mul(&yed, &xm1, &inv);
  fe_tobytes(s, &yed);
  s[31] |= x_sign;
  ge p;
  ge_frombytes(&p, s);                            /* cannot fail (libsodium aborts) */
  ge_dbl(&p, &p); ge_dbl(&p, &p); ge_dbl(&p, &p); /* cofactor */
  ge_tobytes(s, &p);
}

static void hash_to_curve(uint8_t h[32], const ge *Y, const uint8_t *alpha, size_t alen) {
  extern void *malloc(size_t); extern void free(void *);
  uint8_t *buf = (uint8_t *)malloc(34 + alen), r[64];
  buf[0] = 0x04; buf[1] = 0x01;
  ge_tobytes(buf + 2, Y);
  memcpy(buf + 34, alpha, alen);
  orc_sha512(r, buf, 34 + alen);
  free(buf);
  r[31] &= 0x7f;
  from_uniform(h, r);
}
static void hash_points(uint8_t c[16], const ge *P1, const ge *P2, const ge *P3, const ge *P4) {
  uint8_t str[2 + 32 * 4], c1[64];
  str[0] = 0x04; str[1] = 0x02;
  ge_tobytes(str + 2, P1); ge_tobytes(str + 34, P2); ge_tobytes(str + 66, P3); ge_tobytes(str + 98, P4);
  orc_sha512(c1, str, sizeof str);
  memcpy(c, c1, 16);
}

int orc_vrf_proof_to_hash(uint8_t beta[64], const uint8_t proof[80]) {
  init();
  ge G;
  if (ge_frombytes(&G, proof) != 0) return -1;
  ge_dbl(&G, &G); ge_dbl(&G, &G); ge_dbl(&G, &G);
  uint8_t str[34];
  str[0] = 0x04; str[1] = 0x03;
  ge_tobytes(str + 2, &G);
  orc_sha512(beta, str, 34);
  return 0;
}

int orc_vrf_verify(uint8_t beta[64], const uint8_t pk[32], const uint8_t proof[80],
                   const uint8_t *alpha, size_t alphalen) {
  init();
  ge Y, G, H, U, V, t1, t2;
  if (has_small_order(pk) || ge_frombytes(&Y, pk) != 0) return -1;    /* vrf_validate_key */
  if (ge_frombytes(&G, proof) != 0) return -1;                         /* decode_proof */
  uint8_t c[32] = {0}, s64[64] = {0}, s[32], h[32], cp[16];
  memcpy(c, proof + 32, 16);
  memcpy(s64, proof + 48, 32);
  sc_reduce64(s, s64);
  hash_to_curve(h, &Y, alpha, alphalen);
  ge_frombytes(&H, h);
  ge_scalarmult(&t1, s, &GE_B); ge_scalarmult(&t2, c, &Y); ge_neg(&t2, &t2); ge_add(&U, &t1, &t2);
  ge_scalarmult(&t1, s, &H); ge_scalarmult(&t2, c, &G); ge_neg(&t2, &t2); ge_add(&V, &t1, &t2);
  hash_points(cp, &H, &G, &U, &V);
  if (memcmp(cp, c, 16) != 0) return -1;
  return orc_vrf_proof_to_hash(beta, proof);
}

void orc_vrf_pk_from_seed(uint8_t pk[32], const uint8_t seed[32]) { orc_ed25519_pk_from_seed(pk, seed); }

int orc_vrf_prove(uint8_t proof[80], const uint8_t seed[32], const uint8_t *alpha, size_t alphalen) {
  init();
  uint8_t az[64], pk[32], h[32], kbuf[64], k[32], c[32] = {0};
  expand_seed(az, seed);
  ge Y; ge_scalarmult(&Y, az, &GE_B); ge_tobytes(pk, &Y);
  if (ge_frombytes(&Y, pk) != 0) return -1;
  ge H, G, kB, kH;
  hash_to_curve(h, &Y, alpha, alphalen);
  ge_frombytes(&H, h);
  ge_scalarmult(&G, az, &H);
  uint8_t nb[64];
  memcpy(nb, az + 32, 32); memcpy(nb + 32, h, 32);
  orc_sha512(kbuf, nb, 64);
  sc_reduce64(k, kbuf);
  ge_scalarmult(&kB, k, &GE_B);
  ge_scalarmult(&kH, k, &H);
  hash_points(c, &H, &G, &kB, &kH);
  ge_tobytes(proof, &G);
  memcpy(proof + 32, c, 16);
  sc_muladd(proof + 48, c, az, k);
  return 0;
}

/* exported for tests: small-order / canonical predicates and point checks */
int orc_has_small_order(const uint8_t s[32]) { init(); return has_small_order(s); }
int orc_ge_decode_ok(const uint8_t s[32]) { init(); ge p; return ge_frombytes(&p, s) == 0; }
int orc_point_order_divides(const uint8_t s[32], int k) {
  init(); ge p, q; if (ge_frombytes(&p, s) != 0) return -1;
  uint8_t kk[32] = {0}; kk[0] = (uint8_t)k; ge_scalarmult(&q, kk, &p); return ge_is_identity(&q);
}

/* [s]B for a 32-byte LE scalar (no clamping); encoding out */
void orc_scalarmult_base(uint8_t out[32], const uint8_t s[32]) {
  init(); ge R; ge_scalarmult(&R, s, &GE_B); ge_tobytes(out, &R);
}
/* libsodium ge25519_frombytes then p3_tobytes; returns 1 if on curve */
int orc_ge_reencode(uint8_t out[32], const uint8_t in[32]) {
  init(); ge P; if (ge_frombytes(&P, in) != 0) { memset(out, 0, 32); return 0; }
  ge_tobytes(out, &P); return 1;
}
/* VRF draft-03 hash_to_curve(Y, alpha) encoding; returns 0 if pk undecodable */
int orc_vrf_hash_to_curve(uint8_t out[32], const uint8_t pk[32], const uint8_t *alpha, size_t alen) {
  init(); ge Y; if (ge_frombytes(&Y, pk) != 0) return 0;
  hash_to_curve(out, &Y, alpha, alen); return 1;
}
