/*
 * praos.c -- Sum6KES, the Fixed E34 leader check and the per-header Praos
 * check restatement.  TEST INFRASTRUCTURE ONLY (see oracle.h).
 */
#include <stdlib.h>
#include <string.h>
#include "oracle.h"

/* ------------------------------------------------------------------------
 * Sum6KES = SumKES Blake2b_256 (... (SingleKES Ed25519DSIGN)), depth 6.
 * cardano-crypto-class Cardano.Crypto.KES.Sum `verifyKES`:
 *   | hashPairOfVKeys (vk0, vk1) /= vk = Left "Reject"
 *   | t < _T      = verifyKES vk0 t     sigma
 *   | otherwise   = verifyKES vk1 (t-_T) sigma        (_T = 2^(d-1))
 * SingleKES ignores t (no assert in release builds) and is Ed25519 verify.
 * Raw signature: sigma_{d-1} || vk0 || vk1, so the leaf signature comes first
 * and the top level's pair last (verified by probe).
 * Caller: Praos.hs:582 (validateKESSignature), Shelley/Protocol/Praos.hs:85.
 * ------------------------------------------------------------------------ */
int orc_kes_verify(const uint8_t vk[32], uint32_t t, const uint8_t *m, size_t n,
                   const uint8_t sig[ORC_KES_SIG_BYTES]) {
  uint8_t cur[32], h[32];
  memcpy(cur, vk, 32);
  uint64_t tt = t;
  for (int d = ORC_KES_DEPTH; d >= 1; d--) {
    const uint8_t *pair = sig + 64 + 64 * (d - 1);
    orc_blake2b(h, 32, pair, 64);
    if (memcmp(h, cur, 32) != 0) return 1;               /* "Reject" */
    uint64_t T = 1ULL << (d - 1);
    if (tt < T) memcpy(cur, pair, 32);
    else { memcpy(cur, pair + 32, 32); tt -= T; }
  }
  return orc_ed25519_verify(sig, m, n, cur) == 0 ? 0 : 2;
}

/* expandSeed (Blake2b_256): r0 = H(0x01 || s), r1 = H(0x02 || s) */
static void expand(uint8_t r0[32], uint8_t r1[32], const uint8_t s[32]) {
  uint8_t b[33];
  memcpy(b + 1, s, 32);
  b[0] = 1; orc_blake2b(r0, 32, b, 33);
  b[0] = 2; orc_blake2b(r1, 32, b, 33);
}
static void kes_vk_rec(uint8_t vk[32], const uint8_t seed[32], int d) {
  if (d == 0) { orc_ed25519_pk_from_seed(vk, seed); return; }
  uint8_t r0[32], r1[32], pair[64];
  expand(r0, r1, seed);
  kes_vk_rec(pair, r0, d - 1);
  kes_vk_rec(pair + 32, r1, d - 1);
  orc_blake2b(vk, 32, pair, 64);
}
void orc_kes_vk_from_seed(uint8_t vk[32], const uint8_t seed[32]) { kes_vk_rec(vk, seed, ORC_KES_DEPTH); }

static void kes_sign_rec(uint8_t *sig, const uint8_t seed[32], int d, uint64_t t, const uint8_t *m, size_t n) {
  if (d == 0) { orc_ed25519_sign(sig, m, n, seed); return; }
  uint8_t r0[32], r1[32];
  expand(r0, r1, seed);
  uint8_t *pair = sig + 64 + 64 * (d - 1);
  kes_vk_rec(pair, r0, d - 1);
  kes_vk_rec(pair + 32, r1, d - 1);
  uint64_t T = 1ULL << (d - 1);
  if (t < T) kes_sign_rec(sig, r0, d - 1, t, m, n);
  else kes_sign_rec(sig, r1, d - 1, t - T, m, n);
}
int orc_kes_sign(uint8_t sig[ORC_KES_SIG_BYTES], const uint8_t seed[32], uint32_t t, const uint8_t *m, size_t n) {
  if (t >= (1u << ORC_KES_DEPTH)) return -1;
  kes_sign_rec(sig, seed, ORC_KES_DEPTH, t, m, n);
  return 0;
}

/* ------------------------------------------------------------------------
 * Leader check: cardano-protocol-tpraos `checkLeaderNatValue`, with
 * cardano-ledger-core `taylorExpCmp` and Data.Fixed E34 semantics:
 *   f == 1                     -> True
 *   recip_q = fromRational (2^256 / (2^256 - l))   -- raw floor(N/D)
 *   x       = -(fromRational sigma * c)            -- Fixed (*) floors
 *   taylorExpCmp 3 recip_q x: BELOW -> True; ABOVE / MaxReached -> False
 * Bignums are little-endian uint32 arrays; division is bit-serial.
 * Call site: Praos.hs:549 (validateVRFSignature), Praos.hs:505-526.
 * ------------------------------------------------------------------------ */
#define BW 32  /* 1024-bit capacity (TPraos: 2^512 * 10^34 products) */
typedef struct { uint32_t w[BW]; } bn;

static void bn_zero(bn *a) { memset(a, 0, sizeof *a); }
static int bn_cmp(const bn *a, const bn *b) {
  for (int i = BW - 1; i >= 0; i--) if (a->w[i] != b->w[i]) return a->w[i] < b->w[i] ? -1 : 1;
  return 0;
}
static void bn_add(bn *r, const bn *a, const bn *b) {
  uint64_t c = 0;
  for (int i = 0; i < BW; i++) { c += (uint64_t)a->w[i] + b->w[i]; r->w[i] = (uint32_t)c; c >>= 32; }
}
static void bn_sub(bn *r, const bn *a, const bn *b) { /* requires a >= b */
  int64_t br = 0;
  for (int i = 0; i < BW; i++) {
    int64_t d = (int64_t)a->w[i] - b->w[i] - br;
    br = d < 0; r->w[i] = (uint32_t)(d + (br ? (1LL << 32) : 0));
  }
}
static void bn_mul(bn *r, const bn *a, const bn *b) {
  uint32_t t[2 * BW] = {0};
  for (int i = 0; i < BW; i++) {
    uint64_t c = 0;
    for (int j = 0; j + i < 2 * BW && j < BW; j++) {
      c += (uint64_t)a->w[i] * b->w[j] + t[i + j];
      t[i + j] = (uint32_t)c; c >>= 32;
    }
  }
  memcpy(r->w, t, sizeof r->w);  /* callers keep products < 2^512 */
}
static void bn_mul_small(bn *r, const bn *a, uint32_t k) {
  uint64_t c = 0;
  for (int i = 0; i < BW; i++) { c += (uint64_t)a->w[i] * k; r->w[i] = (uint32_t)c; c >>= 32; }
}
static int bn_bitlen(const bn *a) {
  for (int i = BW - 1; i >= 0; i--) if (a->w[i]) { int b = 31; while (!((a->w[i] >> b) & 1)) b--; return 32 * i + b + 1; }
  return 0;
}
/* q = floor(a / d), rem optional; bit-serial */
static void bn_divmod(bn *q, bn *rem, const bn *a, const bn *d) {
  bn r, qq; bn_zero(&r); bn_zero(&qq);
  for (int bit = bn_bitlen(a) - 1; bit >= 0; bit--) {
    /* r = 2r + bit */
    uint32_t c = (a->w[bit >> 5] >> (bit & 31)) & 1;
    for (int i = 0; i < BW; i++) { uint32_t nc = r.w[i] >> 31; r.w[i] = (r.w[i] << 1) | c; c = nc; }
    if (bn_cmp(&r, d) >= 0) { bn_sub(&r, &r, d); qq.w[bit >> 5] |= 1u << (bit & 31); }
  }
  if (q) *q = qq;
  if (rem) *rem = r;
}
static void bn_from_le(bn *a, const uint8_t *b, int n) {
  bn_zero(a);
  for (int i = 0; i < n; i++) a->w[i / 4] |= (uint32_t)b[i] << (8 * (i % 4));
}
static void bn_from_be(bn *a, const uint8_t *b, int n) {
  bn_zero(a);
  for (int i = 0; i < n; i++) a->w[(n - 1 - i) / 4] |= (uint32_t)b[i] << (8 * ((n - 1 - i) % 4));
}
static void bn_pow10(bn *a, int e) { bn_zero(a); a->w[0] = 1; for (int i = 0; i < e; i++) bn_mul_small(a, a, 10); }
static int bn_is_zero(const bn *a) { for (int i = 0; i < BW; i++) if (a->w[i]) return 0; return 1; }

static int check_leader_n(const uint8_t *leader_be, int nbytes, const uint8_t sigma_fp[16],
                          const uint8_t c_raw[16], int f_is_one, int *iters) {
  if (iters) *iters = 0;
  if (f_is_one) return 1;
  bn R, l, D, N, q, sig, c, P, x, rem, two256;
  bn_pow10(&R, 34);
  bn_from_be(&l, leader_be, nbytes);
  bn_zero(&two256); two256.w[nbytes / 4] = 1;  /* certNatMax = 2^(8 * nbytes) */
  bn_sub(&D, &two256, &l);                     /* D = max - l  (>= 1) */
  bn_mul(&N, &two256, &R);                     /* N = max * R */
  bn_divmod(&q, NULL, &N, &D);                 /* recip_q raw */
  bn_from_le(&sig, sigma_fp, 16);
  /* c_raw is a signed 128-bit value, must be <= 0: |c| = -c */
  uint8_t neg[16];
  int carry = 1;
  for (int i = 0; i < 16; i++) { int v = (uint8_t)~c_raw[i] + carry; neg[i] = (uint8_t)v; carry = v >> 8; }
  if (!(c_raw[15] & 0x80)) { /* c >= 0: only c == 0 is meaningful -> x = 0 */
    for (int i = 0; i < 16; i++) if (c_raw[i]) return 0;
    memset(neg, 0, 16);
  }
  bn_from_le(&c, neg, 16);
  /* x = -floor(sigma * c / R) = ceil(sigma * |c| / R) */
  bn_mul(&P, &sig, &c);
  bn_divmod(&x, &rem, &P, &R);
  if (!bn_is_zero(&rem)) { bn one; bn_zero(&one); one.w[0] = 1; bn_add(&x, &x, &one); }
  /* taylorExpCmp 3 recip_q x: go 1000 0 x 1 1 */
  bn err = x, acc = R, t, errp, accp, e, hi, lo;
  for (int n = 0;; n++) {
    if (n == 1000) { if (iters) *iters = n; return 0; }  /* MaxReached */
    uint32_t k = (uint32_t)n + 2;                        /* divisor' */
    bn_mul(&t, &err, &x);
    bn_divmod(&t, NULL, &t, &R);                         /* err * x   (Fixed mul) */
    bn kk; bn_zero(&kk); kk.w[0] = k;
    bn_divmod(&errp, NULL, &t, &kk);                     /* / divisor' (Fixed div) */
    bn_add(&accp, &acc, &err);                           /* acc' = acc + err */
    bn_mul_small(&e, &errp, 3);                          /* |err' * 3| */
    bn_add(&hi, &accp, &e);
    if (bn_cmp(&q, &hi) >= 0) { if (iters) *iters = n + 1; return 0; }   /* ABOVE */
    if (bn_cmp(&accp, &e) > 0) {
      bn_sub(&lo, &accp, &e);
      if (bn_cmp(&q, &lo) < 0) { if (iters) *iters = n + 1; return 1; } /* BELOW */
    }
    err = errp; acc = accp;
  }
}

int orc_check_leader(const uint8_t leader_be[32], const uint8_t sigma_fp[16],
                     const uint8_t c_raw[16], int f_is_one, int *iters) {
  return check_leader_n(leader_be, 32, sigma_fp, c_raw, f_is_one, iters);
}
int orc_check_leader512(const uint8_t leader_be[64], const uint8_t sigma_fp[16],
                        const uint8_t c_raw[16], int f_is_one, int *iters) {
  return check_leader_n(leader_be, 64, sigma_fp, c_raw, f_is_one, iters);
}

/* ------------------------------------------------------------------------
 * Per-header checks, Praos.hs:441-606.  Every check is evaluated and
 * reported as a bit; the caller applies the reference's first-error order
 * (KES block :567-590, then VRF block :535-550).
 * ------------------------------------------------------------------------ */
static void be64(uint8_t *p, uint64_t v) { for (int i = 0; i < 8; i++) p[i] = (uint8_t)(v >> (56 - 8 * i)); }

void orc_praos_header(const orc_epoch *ep, const orc_header *h, orc_result *r) {
  memset(r, 0, sizeof *r);
  r->pool_idx = -1;
  /* validateKESSignature, Praos.hs:567-590 */
  uint64_t kp = h->slot / ep->slots_per_kes_period;
  uint64_t c0 = h->ocert_c0;
  if (!(c0 <= kp)) r->bits |= ORC_BIT_KES_BEFORE_START;
  if (!(kp < c0 + ep->max_kes_evo)) r->bits |= ORC_BIT_KES_AFTER_END;
  uint64_t t = kp >= c0 ? kp - c0 : 0;
  uint8_t msg[48];
  memcpy(msg, h->hot_vk, 32); be64(msg + 32, h->ocert_n); be64(msg + 40, c0);  /* ocertToSignable */
  if (orc_ed25519_verify(h->ocert_sig, msg, 48, h->cold_vk) != 0) r->bits |= ORC_BIT_OCERT_SIG;
  {
    /* KES with Word64 period semantics (t may exceed 2^6 when check 2 fails) */
    uint8_t cur[32], hh[32];
    memcpy(cur, h->hot_vk, 32);
    uint64_t tt = t;
    int bad = 0;
    for (int d = ORC_KES_DEPTH; d >= 1; d--) {
      const uint8_t *pair = h->kes_sig + 64 + 64 * (d - 1);
      orc_blake2b(hh, 32, pair, 64);
      if (memcmp(hh, cur, 32) != 0) { bad = 1; break; }
      uint64_t T = 1ULL << (d - 1);
      if (tt < T) memcpy(cur, pair, 32); else { memcpy(cur, pair + 32, 32); tt -= T; }
    }
    if (bad) r->bits |= ORC_BIT_KES_MERKLE;
    else if (orc_ed25519_verify(h->kes_sig, h->body, h->body_len, cur) != 0) r->bits |= ORC_BIT_KES_LEAF;
  }
  /* validateVRFSignature, Praos.hs:535-550 */
  orc_blake2b(r->issuer_hash, 28, h->cold_vk, 32);       /* hashKey: Blake2b-224 */
  int lo = 0, hi = (int)ep->npools - 1, idx = -1;
  while (lo <= hi) {
    int mid = (lo + hi) / 2;
    int c = memcmp(ep->pools[mid].hash28, r->issuer_hash, 28);
    if (c == 0) { idx = mid; break; }
    if (c < 0) lo = mid + 1; else hi = mid - 1;
  }
  r->pool_idx = idx;
  if (idx < 0) r->bits |= ORC_BIT_VRF_KEY_UNKNOWN;
  else {
    uint8_t vh[32];
    orc_blake2b(vh, 32, h->vrf_vk, 32);                   /* hashVerKeyVRF */
    if (memcmp(vh, ep->pools[idx].vrf_hash32, 32) != 0) r->bits |= ORC_BIT_VRF_KEY_WRONG;
  }
  uint8_t ain[40], alpha[32];
  be64(ain, h->slot);
  memcpy(ain + 8, ep->eta0, 32);
  orc_blake2b(alpha, 32, ain, ep->eta0_neutral ? 8 : 40);   /* mkInputVRF, Praos/VRF.hs:55-69 */
  uint8_t beta[64];
  if (orc_vrf_verify(beta, h->vrf_vk, h->vrf_proof, alpha, 32) != 0) r->bits |= ORC_BIT_VRF_PROOF;
  if (orc_vrf_proof_to_hash(r->beta, h->vrf_proof) != 0) memset(r->beta, 0, 64);
  if (memcmp(r->beta, h->vrf_out, 64) != 0) r->bits |= ORC_BIT_VRF_OUTPUT;
  uint8_t lb[65];
  lb[0] = 'L'; memcpy(lb + 1, h->vrf_out, 64);
  orc_blake2b(r->leader, 32, lb, 65);                     /* hashVRF SVRFLeader, Praos/VRF.hs:88-99 */
  lb[0] = 'N';
  uint8_t nv[32];
  orc_blake2b(nv, 32, lb, 65);
  orc_blake2b(r->nonce, 32, nv, 32);                      /* vrfNonceValue, Praos/VRF.hs:116-131 */
  if (idx >= 0 && !orc_check_leader(r->leader, ep->pools[idx].sigma_fp, ep->c_raw, ep->f_is_one, NULL))
    r->bits |= ORC_BIT_LEADER;
}

/* ------------------------------------------------------------------------
 * TPraos (cardano-protocol-tpraos), d = 0: praosVrfChecks (OVERLAY) then OCERT.
 * The OCERT predicates are the same as Praos.hs:567-590 (a2).
 * ------------------------------------------------------------------------ */
void orc_tpraos_seed(uint8_t out[32], uint64_t slot, const uint8_t eta0[32], int eta0_neutral, uint64_t k) {
  uint8_t in[40], h[32], kb[8], uc[32];
  be64(in, slot);
  memcpy(in + 8, eta0, 32);
  orc_blake2b(h, 32, in, eta0_neutral ? 8 : 40);           /* mkSeed: hash of BE64 slot || eta0 */
  be64(kb, k);
  orc_blake2b(uc, 32, kb, 8);                               /* mkNonceFromNumber k */
  for (int i = 0; i < 32; i++) out[i] = h[i] ^ uc[i];       /* Hash.xor */
}

void orc_tpraos_header(const orc_epoch *ep, const orc_tp_header *th, orc_tp_result *r) {
  const orc_header *h = &th->h;
  orc_result pr;
  memset(r, 0, sizeof *r);
  /* OCERT predicates and key lookups are shared with the Praos restatement */
  orc_praos_header(ep, h, &pr);
  r->bits = pr.bits & (ORC_BIT_KES_BEFORE_START | ORC_BIT_KES_AFTER_END | ORC_BIT_OCERT_SIG |
                       ORC_BIT_KES_MERKLE | ORC_BIT_KES_LEAF | ORC_BIT_VRF_KEY_UNKNOWN | ORC_BIT_VRF_KEY_WRONG);
  r->pool_idx = pr.pool_idx;
  uint8_t a_eta[32], a_l[32], beta[64];
  orc_tpraos_seed(a_eta, h->slot, ep->eta0, ep->eta0_neutral, 0);
  orc_tpraos_seed(a_l, h->slot, ep->eta0, ep->eta0_neutral, 1);
  if (orc_vrf_verify(beta, h->vrf_vk, h->vrf_proof, a_eta, 32) != 0) r->bits |= ORC_BIT_TP_VRF_NONCE;
  if (orc_vrf_proof_to_hash(r->beta_eta, h->vrf_proof) != 0) memset(r->beta_eta, 0, 64);
  if (memcmp(r->beta_eta, h->vrf_out, 64) != 0) r->bits |= ORC_BIT_TP_VRF_NONCE;
  if (orc_vrf_verify(beta, h->vrf_vk, th->leader_proof, a_l, 32) != 0) r->bits |= ORC_BIT_TP_VRF_LEADER;
  if (orc_vrf_proof_to_hash(r->beta_leader, th->leader_proof) != 0) memset(r->beta_leader, 0, 64);
  if (memcmp(r->beta_leader, th->leader_out, 64) != 0) r->bits |= ORC_BIT_TP_VRF_LEADER;
  orc_blake2b(r->nonce, 32, h->vrf_out, 64);                 /* mkNonceFromOutputVRF */
  if (r->pool_idx >= 0 &&
      !orc_check_leader512(th->leader_out, ep->pools[r->pool_idx].sigma_fp, ep->c_raw, ep->f_is_one, NULL))
    r->bits |= ORC_BIT_LEADER;
}
