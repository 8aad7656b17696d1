// praos_core.hpp -- per-lane verification procedures of the Praos header path.
//
//   ed25519_verify_core : libsodium 1.0.18 crypto_sign_ed25519_verify_detached
//                         (via cardano-crypto-class Ed25519DSIGN; Praos.hs:580, KES leaf)
//   kes_merkle          : cardano-crypto-class Sum6KES verifyKES tree walk (Praos.hs:582)
//   vrf_verify_core     : IOG crypto_vrf_ietfdraft03_verify + proof_to_hash (Praos.hs:543)
// plus the signing procedures used only by the synthetic-chain generator.
#pragma once
#include "hash.hpp"
#include "scalarmult.hpp"
#include "sc25519.hpp"

FE_INLINE uint32_t fsh16(uint32_t hi, uint32_t lo) { return __builtin_amdgcn_alignbit(hi, lo, 16); }

// SHA-512 of a message held in registers as LE u32 stream words S[0..NW),
// already padded with the 0x80 byte; NBYTES = message length (pre-padding).
template <int NW, int NBYTES>
FE_INLINE void sha512_regs(uint32_t out[16], const uint32_t S[NW]) {
  constexpr int NBLK = (NBYTES + 17 + 127) / 128;
  uint64_t H[8];
  sha512_init(H);
#pragma unroll
  for (int b = 0; b < NBLK; b++) {
    uint64_t W[16];
#pragma unroll
    for (int w = 0; w < 16; w++) {
      const int i0 = 32 * b + 2 * w, i1 = i0 + 1;
      const uint32_t lo = i0 < NW ? S[i0] : 0u;
      const uint32_t hi = i1 < NW ? S[i1] : 0u;
      W[w] = bswap64(((uint64_t)hi << 32) | lo);
    }
    if (b == NBLK - 1) W[15] = (uint64_t)NBYTES * 8u;
    sha512_block(H, W);
  }
  sha512_digest_words(out, H);
}

// stream = tag(2 bytes, LE u16) || parts (NP LE words) || 0x80
template <int NP>
FE_INLINE void stream2(uint32_t S[NP + 1], uint32_t tag16, const uint32_t P[NP]) {
  S[0] = (tag16 & 0xffffu) | (P[0] << 16);
#pragma unroll
  for (int i = 1; i < NP; i++) S[i] = fsh16(P[i], P[i - 1]);
  S[NP] = (P[NP - 1] >> 16) | (0x80u << 16);
}

// SHA-512 of (prefix[0..plen) || msg[0..len)); plen multiple of 8, <= 64.
// msg is 8-byte aligned and readable up to round_up(len, 8).
FE_INLINE void sha512_stream(uint32_t out[16], const uint32_t prefix[16], uint32_t plen,
                             const uint8_t* __restrict__ msg, uint32_t len) {
  uint64_t H[8];
  sha512_init(H);
  const uint32_t total = plen + len;
  const uint32_t nblocks = (total + 17u + 127u) >> 7;
  for (uint32_t blk = 0; blk < nblocks; blk++) {
    uint64_t W[16];
#pragma unroll
    for (int w = 0; w < 16; w++) {
      const uint32_t off = blk * 128u + 8u * w;
      uint64_t v;
      if (blk == 0 && (uint32_t)(8 * w) < plen) {
        v = be_word(prefix[2 * w], prefix[2 * w + 1]);
      } else {
        const uint32_t m = off - plen;
        uint64_t raw = 0;
        if (m < len) raw = *(const uint64_t*)(msg + m);
        const uint32_t valid = len > m ? (len - m) : 0u;
        if (valid < 8) {
          const uint64_t keep = valid == 0 ? 0ULL : (~0ULL >> (64 - 8 * valid));
          raw &= keep;
          if (len >= m && len < m + 8) raw |= 0x80ULL << (8 * (len - m));
        }
        v = bswap64(raw);
      }
      W[w] = v;
    }
    if (blk == nblocks - 1) W[15] = (uint64_t)total * 8u;
    sha512_block(H, W);
  }
  sha512_digest_words(out, H);
}

// ------------------------------------------------------------------ Ed25519
// hram: SHA-512(R || A || M) digest words.  Checks in libsodium order; all
// lanes do the full computation (rejections are folded in at the end).
// tab: the lane's 8-entry table of -A ({1..8}(-A), cached form).  Kernels pass a
// per-lane region of a global arena (kcommon.hpp lane_tab): each entry is 128
// contiguous bytes of the lane's own, so a digit-indexed select reads whole
// cache lines.  (A private array would live in swizzled scratch, where a
// lane-divergent index touches one dword per 128-byte line.)
FE_INLINE bool ed25519_verify_core(const uint32_t pk[8], const uint32_t R[8], const uint32_t S[8],
                                   const uint32_t hram[16], const ge_niels* __restrict__ btab,
                                   ge_cached* __restrict__ tab) {
  bool ok = sc_is_canonical(S) && !ge_has_small_order(R) && ge_is_canonical(pk) && !ge_has_small_order(pk);
  ge_p3 A;
  ok = ge_frombytes(A, pk, /*negate=*/true) && ok;
  uint32_t h[8], s[8];
  sc_reduce512(h, hram);
#pragma unroll
  for (int i = 0; i < 8; i++) s[i] = ok ? S[i] : 0u;      // keep the recoding in range (S < L)
  build_cached_table(tab, A);
  uint32_t hw[8], sw[8];
  sc_recode16(hw, h);
  sc_recode256(sw, s);
  ge_p1p1 x;
  STRAUS<64, 64, 0, 32, false>(x, tab, hw, nullptr, nullptr, btab, sw);   // [s]B - [h]A
  ge_p2 Rp;
  ge_p1p1_to_p2(Rp, x);
  uint32_t enc[8];
  ge_tobytes(enc, Rp.X, Rp.Y, Rp.Z);
  bool eq = true;
#pragma unroll
  for (int i = 0; i < 8; i++) eq &= enc[i] == R[i];
  return ok && eq;
}

// Same verification with the public key cached (k_keys.hip): kflag bit 0 =
// ge_is_canonical(pk) && !ge_has_small_order(pk) && decode ok; ktab = the key's
// multi-power tables (-A at 2^(16k)); btab = the global radix-2^16 comb of B.
// ed25519_cached_point: [s]B - [h]A in projective form, and the checks that need no
// encoding (S canonical, R not of small order, the key flag).
FE_INLINE bool ed25519_cached_point(ge_p2& Rp, const uint32_t R[8], const uint32_t S[8], const uint32_t hram[16],
                                    uint32_t kflag, const ge_cached* __restrict__ ktab,
                                    const ge_niels* __restrict__ btab) {
  bool ok = sc_is_canonical(S) && !ge_has_small_order(R) && (kflag & 1u) != 0;
  uint32_t h[8], s[8];
  sc_reduce512(h, hram);
#pragma unroll
  for (int i = 0; i < 8; i++) s[i] = ok ? S[i] : 0u;
  uint32_t hw[8], sw[8];
  sc_recode16(hw, h);
  sc_recode65536(sw, s);
  ge_p1p1 x;
  straus_comb<16, false>(x, ktab, hw, btab, sw);     // [s]B - [h]A: 4-window chain + comb (btab = global comb)
  ge_p1p1_to_p2(Rp, x);
  return ok;
}

FE_INLINE bool ed25519_verify_cached(const uint32_t R[8], const uint32_t S[8], const uint32_t hram[16],
                                     uint32_t kflag, const ge_cached* __restrict__ ktab,
                                     const ge_niels* __restrict__ btab) {
  ge_p2 Rp;
  const bool ok = ed25519_cached_point(Rp, R, S, hram, kflag, ktab, btab);
  uint32_t enc[8];
  ge_tobytes(enc, Rp.X, Rp.Y, Rp.Z);
  bool eq = true;
#pragma unroll
  for (int i = 0; i < 8; i++) eq &= enc[i] == R[i];
  return ok && eq;
}

// OCert signable: hot_vk(32) || BE64(n) || BE64(c0)  -> SHA-512(R||A||M), 112 bytes
FE_INLINE void ocert_hram(uint32_t out[16], const uint32_t R[8], const uint32_t A[8], const uint32_t hot[8],
                          uint64_t n, uint64_t c0) {
  uint64_t H[8];
  sha512_init(H);
  uint64_t W[16];
#pragma unroll
  for (int i = 0; i < 4; i++) {
    W[i] = be_word(R[2 * i], R[2 * i + 1]);
    W[4 + i] = be_word(A[2 * i], A[2 * i + 1]);
    W[8 + i] = be_word(hot[2 * i], hot[2 * i + 1]);
  }
  W[12] = n;                 // bytes are BE64(n): the big-endian word is n itself
  W[13] = c0;
  W[14] = 0x8000000000000000ULL;
  W[15] = 0;
  sha512_block(H, W);
#pragma unroll
  for (int i = 0; i < 15; i++) W[i] = 0;
  W[15] = 112u * 8u;
  sha512_block(H, W);
  sha512_digest_words(out, H);
}

// ------------------------------------------------------------------ Sum6KES
// Walks the tree top-down (Sum.verifyKES): at depth d the pair (vk0, vk1) is
// sig[64 + 64*(d-1) ..); Blake2b-256(vk0||vk1) must equal the current vk;
// t < 2^(d-1) selects vk0, else vk1 with t -= 2^(d-1).  Returns merkle_ok and
// the leaf Ed25519 vk.  t is a Word (64-bit) as in the reference.
FE_INLINE bool kes_merkle(uint32_t leaf_vk[8], const uint32_t vk[8], uint64_t t, const uint8_t* __restrict__ sig) {
  uint32_t cur[8];
#pragma unroll
  for (int i = 0; i < 8; i++) cur[i] = vk[i];
  bool ok = true;
#pragma unroll
  for (int d = 6; d >= 1; d--) {
    uint32_t pair[16];
    const uint4* p = (const uint4*)(sig + 64 + 64 * (d - 1));
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const uint4 v = p[q];
      pair[4 * q] = v.x; pair[4 * q + 1] = v.y; pair[4 * q + 2] = v.z; pair[4 * q + 3] = v.w;
    }
    uint32_t h[8];
    blake2b256_64(h, pair);
#pragma unroll
    for (int i = 0; i < 8; i++) ok &= h[i] == cur[i];
    const uint64_t T = 1ull << (d - 1);
    const bool right = t >= T;
    t = right ? t - T : t;
#pragma unroll
    for (int i = 0; i < 8; i++) cur[i] = right ? pair[8 + i] : pair[i];
  }
#pragma unroll
  for (int i = 0; i < 8; i++) leaf_vk[i] = cur[i];
  return ok;
}

// ------------------------------------------------------------------ VRF draft-03
__device__ __constant__ static const uint32_t FE_CURVE_A[8] = {486662u, 0, 0, 0, 0, 0, 0, 0};

// libsodium ge25519_from_uniform (the VRF caller has cleared r's sign bit),
// restated without its two field inversions: returns H = 8 * P projective
// (the encoding is deferred to the caller's batched inversion).
//   w = 1 + 2 r^2, Montgomery x1 = -A / w, x2 = -x1 - A; libsodium picks u = x1 when
//   chi(x1^3 + A x1^2 + x1) != -1, else x2, and y = (u - 1) / (u + 1) = N / D with
//     case 1: N1 = -(A + w),      D1 = w - A
//     case 2: N2 = A - A w - w,   D2 = A - A w + w.
//   P = ge25519_frombytes(y, sign 0): x = sqrt((N^2 - D^2) / (d N^2 + D^2)), x even.
// ONE exponentiation instead of two (chi, then the square root): with
// a1 = (N1^2 - D1^2) / (d N1^2 + D1^2) = -486664 x1^2 / g(x1), case 1 holds exactly
// when a1 is a square, and the case-2 ratio is a2 = a1 (w - 1) (g(x2) = 2 r^2 g(x1),
// x2 / x1 = w - 1).  The sqrt_ratio candidate s of a1 (s^2 (dN1^2 + D1^2) = a1-numerator
// times a 4th root of unity) then gives both roots: case 1 s or s sqrt(-1); case 2
// t = s 2^((p+3)/8) r or t sqrt(-1) (the same 4th-root argument, RFC 9380's Elligator 2
// sqrt trick).  libsodium's D = 0 corner (u + 1 = 0) is unreachable: w = A and
// w = A / (A - 1) need r^2 = (A - 1) / 2 resp. (A / (A - 1) - 1) / 2, both
// non-residues (tests/test_oracle.py::test_elligator_corner_unreachable).
__device__ __constant__ static const uint32_t FE_2_P38[8] = {   // 2^((p+3)/8) = 1 + sqrt(-1)
    0x4a0ea0b1u, 0xc4ee1b27u, 0xad2fe478u, 0x2f431806u, 0x3dfbd7a7u, 0x2b4d0099u, 0x4fc1df0bu, 0x2b832480u};

FE_INLINE void vrf_from_uniform(ge_p3& H, const uint32_t r[8]) {
  fe A, one, rf, w, t, Aw;
  fe_const(A, FE_CURVE_A);
  fe_set(one, 1);
  fe_frombytes32(rf, r);
  fe_sq(w, rf);
  fe_add(w, w, w);
  fe_add(w, w, one);                // w = 1 + 2 r^2 (never 0: -1/2 is a non-square)
  fe_mul(Aw, A, w);
  fe N1, D1, N2, D2;
  fe_add(N1, A, w);
  fe_neg(N1, N1);
  fe_sub(D1, w, A);
  fe_sub(t, A, Aw);
  fe_sub(N2, t, w);
  fe_add(D2, t, w);
  // case-1 ratio U / V and its sqrt_ratio candidate s = U V^3 (U V^7)^((p-5)/8)
  fe nn, dd, U, V, d, v3, s;
  fe_sq(nn, N1);
  fe_sq(dd, D1);
  fe_sub(U, nn, dd);
  fe_const(d, FE_D);
  fe_mul(V, nn, d);
  fe_add(V, V, dd);
  fe_sq(v3, V);
  fe_mul(v3, v3, V);                // V^3
  fe_sq(s, v3);
  fe_mul(s, s, V);
  fe_mul(s, s, U);                  // U V^7
  fe_pow22523(s, s);
  fe_mul(s, s, v3);
  fe_mul(s, s, U);
  fe sq1, chk, vss;
  fe_const(sq1, FE_SQRTM1);
  fe_sq(vss, s);
  fe_mul(vss, vss, V);
  fe_sub(chk, vss, U);
  const bool m1 = fe_iszero(chk);
  fe_add(chk, vss, U);
  const bool case1 = m1 || fe_iszero(chk);
  fe x1, x2, c;
  fe_mul(x1, s, sq1);
  fe_cmov(x1, s, m1);               // case 1: s or s sqrt(-1)
  fe_const(c, FE_2_P38);
  fe_mul(t, s, rf);
  fe_mul(t, t, c);                  // case 2 candidate
  fe U2, wm1;
  fe_sub(wm1, w, one);
  fe_mul(U2, U, wm1);
  fe_sq(vss, t);
  fe_mul(vss, vss, V);
  fe_sub(chk, vss, U2);
  const bool m2 = fe_iszero(chk);
  fe_mul(x2, t, sq1);
  fe_cmov(x2, t, m2);
  fe x = x2, N = N2, D = D2;
  fe_cmov(x, x1, case1);
  fe_cmov(N, N1, case1);
  fe_cmov(D, D1, case1);
  fe negx;
  fe_neg(negx, x);
  fe_cmov(x, negx, fe_isnegative(x));   // sign bit 0
  ge_p3 P;
  fe_mul(P.X, x, D);
  P.Y = N;
  P.Z = D;
  fe_mul(P.T, x, N);
  ge_p3 Q;
  ge_p3_dbl_to_p3(Q, P);
  ge_p3_dbl_to_p3(P, Q);
  ge_p3_dbl_to_p3(H, P);            // cofactor 8
}

// encoding of a point with Z == 1 (fresh from ge_frombytes)
FE_INLINE void ge_enc_affine(uint32_t s[8], const ge_p3& P) {
  fe_tobytes32(s, P.Y);
  s[7] |= (uint32_t)fe_isnegative(P.X) << 31;
}

// H from r = first 32 bytes of SHA-512(0x04 || 0x01 || Y || alpha), sign bit cleared
FE_INLINE void vrf_hash_to_curve(ge_p3& H, const uint32_t ys[8], const uint32_t alpha[8]) {
  uint32_t P[16], S[17], d[16];
#pragma unroll
  for (int i = 0; i < 8; i++) { P[i] = ys[i]; P[8 + i] = alpha[i]; }
  stream2<16>(S, 0x0104u, P);
  sha512_regs<17, 66>(d, S);
  uint32_t r[8];
#pragma unroll
  for (int i = 0; i < 8; i++) r[i] = d[i];
  r[7] &= 0x7fffffffu;
  vrf_from_uniform(H, r);
}

// beta = SHA-512(0x04 || 0x03 || enc(8 Gamma))
FE_INLINE void vrf_beta(uint32_t beta[16], const uint32_t g8[8]) {
  uint32_t S[9];
  stream2<8>(S, 0x0304u, g8);
  sha512_regs<9, 34>(beta, S);
}

// c' = SHA-512(0x04 || 0x02 || H || Gamma || U || V)[0..16)
FE_INLINE void vrf_hash_points(uint32_t c[4], const uint32_t h[8], const uint32_t g[8], const uint32_t u[8],
                               const uint32_t v[8]) {
  uint32_t P[32], S[33], d[16];
#pragma unroll
  for (int i = 0; i < 8; i++) { P[i] = h[i]; P[8 + i] = g[i]; P[16 + i] = u[i]; P[24 + i] = v[i]; }
  stream2<32>(S, 0x0204u, P);
  sha512_regs<33, 130>(d, S);
#pragma unroll
  for (int i = 0; i < 4; i++) c[i] = d[i];
}

// Returns proof validity; beta always computed from Gamma (gamma_ok tells if it decoded).
//   U = [s]B - [c]Y  : 33-window chain, s split over B and B' = 2^128 B (radix 256)
//   V = [s]H - [c]Gamma : 64-window chain, both bases per lane (radix 16)
// One batched inversion encodes H, U, V and 8 Gamma.
// CACHED: the VRF key comes from k_keys.hip (kinfo[0] bit 0 = key valid,
// kinfo[1..8] = canonical encoding of Y, ktab = tables of -Y at 2^(16k), k < 9)
// and U runs on a 4-window chain plus the fixed-base comb (btab = the global comb).
// vt: the lane's 16-entry table region (see ed25519_verify_core): {1..8}H, {1..8}(-Gamma)
// and, uncached, {1..8}(-Y) in its first half before H's table replaces it.
template <bool CACHED>
FE_INLINE bool vrf_verify_core(uint32_t beta[16], bool& gamma_ok, const uint32_t pk[8], const uint32_t gamma[8],
                               const uint32_t c4[4], const uint32_t s8[8], const uint32_t alpha[8],
                               const ge_niels* __restrict__ btab, ge_cached* __restrict__ vt,
                               const ge_cached* __restrict__ ktab = nullptr,
                               const uint32_t* __restrict__ kinfo = nullptr) {
  // vrf_validate_key: small order -> reject; ge25519_frombytes must succeed
  bool ok;
  ge_p3 Y, G;
  uint32_t ys[8];
  if constexpr (CACHED) {
    ok = (kinfo[0] & 1u) != 0;
#pragma unroll
    for (int i = 0; i < 8; i++) ys[i] = kinfo[1 + i];
  } else {
    ok = !ge_has_small_order(pk);
    ok = ge_frombytes(Y, pk, false) && ok;
    ge_enc_affine(ys, Y);
  }
  gamma_ok = ge_frombytes(G, gamma, false);
  // s reduced mod L (sc25519_reduce of s || 0^32)
  uint32_t sx[16], s[8], c[8];
#pragma unroll
  for (int i = 0; i < 16; i++) sx[i] = i < 8 ? s8[i] : 0u;
  sc_reduce512(s, sx);
#pragma unroll
  for (int i = 0; i < 8; i++) c[i] = i < 4 ? c4[i] : 0u;
  // H = hash_to_curve(canonical Y, alpha)
  ge_p3 H;
  vrf_hash_to_curve(H, ys, alpha);
  ge_p2 U, V;
  if constexpr (CACHED) {  // U = [s]B - [c]Y, cached -Y
    uint32_t cw[8], sw[8];
    sc_recode16(cw, c);
    sc_recode65536(sw, s);
    ge_p1p1 x;
    straus_comb<8, true>(x, ktab, cw, btab, sw);   // btab = the global comb
    ge_p1p1_to_p2(U, x);
  } else {  // U = [s]B - [c]Y
    ge_p3 nY = Y;
    fe_neg(nY.X, Y.X);
    fe_neg(nY.T, Y.T);
    ge_cached* ty = vt;
    build_cached_table(ty, nY);
    uint32_t cw[8], sw[8];
    sc_recode16(cw, c);
    sc_recode256(sw, s);
    ge_p1p1 x;
    STRAUS<33, 33, 0, 16, true>(x, ty, cw, nullptr, nullptr, btab, sw);
    ge_p1p1_to_p2(U, x);
  }
  {  // V = [s]H - [c]Gamma
    ge_p3 nG = G;
    fe_neg(nG.X, G.X);
    fe_neg(nG.T, G.T);
    ge_cached* th = vt;
    ge_cached* tg = vt + 8;
    build_cached_table(th, H);
    build_cached_table(tg, nG);
    uint32_t sw[8], cw[8];
    sc_recode16(sw, s);
    sc_recode16(cw, c);
    ge_p1p1 x;
    STRAUS<64, 64, 33, 0, false>(x, th, sw, tg, cw, nullptr, nullptr);
    ge_p1p1_to_p2(V, x);
  }
  // 8 Gamma
  ge_p3 G2, G4, G8;
  ge_p3_dbl_to_p3(G2, G);
  ge_p3_dbl_to_p3(G4, G2);
  ge_p3_dbl_to_p3(G8, G4);
  // batched inversion of U.Z, V.Z, G8.Z, H.Z
  fe z12, z123, z1234, inv, iu, iv, ig, ih;
  fe_mul(z12, U.Z, V.Z);
  fe_mul(z123, z12, G8.Z);
  fe_mul(z1234, z123, H.Z);
  fe_invert(inv, z1234);
  fe_mul(ih, inv, z123);            // 1/H.Z
  fe_mul(inv, inv, H.Z);            // 1/(U.Z V.Z G8.Z)
  fe_mul(ig, inv, z12);             // 1/G8.Z
  fe_mul(inv, inv, G8.Z);           // 1/(U.Z V.Z)
  fe_mul(iu, inv, V.Z);
  fe_mul(iv, inv, U.Z);
  uint32_t hs[8], us[8], vs[8], gs[8], g8s[8];
  ge_tobytes_zi(hs, H.X, H.Y, ih);
  ge_tobytes_zi(us, U.X, U.Y, iu);
  ge_tobytes_zi(vs, V.X, V.Y, iv);
  ge_tobytes_zi(g8s, G8.X, G8.Y, ig);
  ge_enc_affine(gs, G);
  uint32_t cp[4];
  vrf_hash_points(cp, hs, gs, us, vs);
  bool eq = true;
#pragma unroll
  for (int i = 0; i < 4; i++) eq &= cp[i] == c4[i];
  vrf_beta(beta, g8s);
  return ok && gamma_ok && eq;
}

// ------------------------------------------------------------------ VRF verify in stages
// The same verification as vrf_verify_core, split into independent pieces (k_vrf.hip):
// stage V (k_vrf_v) -- H = hash_to_curve, Gamma decode, 8 Gamma, V = [s]H - [c]Gamma --
// depends on the header alone; stage U (k_vrf_u) -- U = [s]B - [c]Y from the key's tables
// (k_keys.hip) or a per-lane chain -- depends on the key only; the two run concurrently
// (U of a cached key once its tables exist, U of an uncached key at once).  The join
// (k_vrf_join) -- one batched inversion, the challenge hash, beta -- reads both records.
// (vrf_fin_core = U + join in one lane, the two-stage form, kept for comparison.)
// Records in SoA planes of uint4 (plane p of item i at mid[p * stride + i], so a wave's
// access is one contiguous KB):
//   planes 0-5 V (X, Y, Z), 6-11 H, 12-17 8 Gamma, 18-19 enc(Gamma), 20 flags (x: Gamma
//   decoded; written by stage V), 21-26 U (X, Y, Z), 27 key flag (x: vrf_validate_key; stage U)
#define VRF_MID_PLANES 28
#define VRF_MID_V 0
#define VRF_MID_H 6
#define VRF_MID_G8 12
#define VRF_MID_GS 18
#define VRF_MID_FLAGS 20
#define VRF_MID_U 21
#define VRF_MID_KEY 27

FE_INLINE void mid_put(uint4* __restrict__ mid, size_t stride, size_t i, int plane, const uint32_t w[8]) {
  mid[(size_t)plane * stride + i] = make_uint4(w[0], w[1], w[2], w[3]);
  mid[(size_t)(plane + 1) * stride + i] = make_uint4(w[4], w[5], w[6], w[7]);
}
FE_INLINE void mid_get(uint32_t w[8], const uint4* __restrict__ mid, size_t stride, size_t i, int plane) {
  const uint4 a = mid[(size_t)plane * stride + i], b = mid[(size_t)(plane + 1) * stride + i];
  w[0] = a.x; w[1] = a.y; w[2] = a.z; w[3] = a.w; w[4] = b.x; w[5] = b.y; w[6] = b.z; w[7] = b.w;
}
FE_INLINE void mid_put_xyz(uint4* __restrict__ mid, size_t stride, size_t i, int plane, const fe& X, const fe& Y,
                           const fe& Z) {
  mid_put(mid, stride, i, plane, X.v);
  mid_put(mid, stride, i, plane + 2, Y.v);
  mid_put(mid, stride, i, plane + 4, Z.v);
}
FE_INLINE void mid_get_xyz(fe& X, fe& Y, fe& Z, const uint4* __restrict__ mid, size_t stride, size_t i, int plane) {
  mid_get(X.v, mid, stride, i, plane);
  mid_get(Y.v, mid, stride, i, plane + 2);
  mid_get(Z.v, mid, stride, i, plane + 4);
}

// The canonical encoding ge_enc_affine(ge_frombytes(pk)) that hash_to_curve reads, without
// the decode: y mod p with pk's sign bit.  Equal for every key that passes
// vrf_validate_key (x != 0 off the small-order points, so the sign bit is x's); for any
// other key the proof is rejected from the key flags whatever H is.
FE_INLINE void vrf_key_canonical(uint32_t ys[8], const uint32_t pk[8]) {
  fe y;
  fe_frombytes32(y, pk);
  fe_tobytes32(ys, y);
  ys[7] |= pk[7] & 0x80000000u;
}

// Stage V: writes H, 8 Gamma, enc(Gamma), the Gamma flag (before the chain, so none of
// them is live across it) and V.  vt: the lane's 16-entry table region ({1..8}H, {1..8}(-Gamma)).
FE_INLINE void vrf_v_core(uint4* __restrict__ mid, size_t stride, size_t i, const uint32_t pk[8],
                          const uint32_t gamma[8], const uint32_t c4[4], const uint32_t s8[8],
                          const uint32_t alpha[8], ge_cached* __restrict__ vt) {
  {
    uint32_t ys[8];
    vrf_key_canonical(ys, pk);
    ge_p3 H;
    vrf_hash_to_curve(H, ys, alpha);
    mid_put_xyz(mid, stride, i, VRF_MID_H, H.X, H.Y, H.Z);
    build_cached_table(vt, H);
  }
  {
    ge_p3 G;
    const bool gamma_ok = ge_frombytes(G, gamma, false);
    uint32_t gs[8];
    ge_enc_affine(gs, G);
    mid_put(mid, stride, i, VRF_MID_GS, gs);
    mid[(size_t)VRF_MID_FLAGS * stride + i] = make_uint4(gamma_ok ? 1u : 0u, 0u, 0u, 0u);
    ge_p3 G2, G4;
    ge_p3_dbl_to_p3(G2, G);
    ge_p3_dbl_to_p3(G4, G2);
    ge_p1p1 t;
    ge_p2 q;
    ge_p3_to_p2(q, G4);
    ge_p2_dbl(t, q);
    ge_p2 G8;
    ge_p1p1_to_p2(G8, t);
    mid_put_xyz(mid, stride, i, VRF_MID_G8, G8.X, G8.Y, G8.Z);
    fe_neg(G.X, G.X);
    fe_neg(G.T, G.T);
    build_cached_table(vt + 8, G);
  }
  uint32_t sx[16], s[8], c[8], sw[8], cw[8];
#pragma unroll
  for (int k = 0; k < 16; k++) sx[k] = k < 8 ? s8[k] : 0u;
  sc_reduce512(s, sx);
#pragma unroll
  for (int k = 0; k < 8; k++) c[k] = k < 4 ? c4[k] : 0u;
  sc_recode16(sw, s);
  sc_recode16(cw, c);
  ge_p1p1 x;
  STRAUS<64, 64, 33, 0, false>(x, vt, sw, vt + 8, cw, nullptr, nullptr);   // V = [s]H - [c]Gamma
  ge_p2 V;
  ge_p1p1_to_p2(V, x);
  mid_put_xyz(mid, stride, i, VRF_MID_V, V.X, V.Y, V.Z);
}

// Stage F: U, the batched inversion of U.Z V.Z (8 Gamma).Z H.Z, the challenge, beta.
// CACHED: kinfo / ktab of k_keys.hip and btab = the global radix-2^16 comb; otherwise Y is
// decoded per lane ({1..8}(-Y) in vt) and btab = the LDS tables {B, 2^128 B}.
template <bool CACHED>
FE_INLINE bool vrf_fin_core(uint32_t beta[16], bool& gamma_ok, const uint4* __restrict__ mid, size_t stride,
                            size_t i, const uint32_t pk[8], const uint32_t c4[4], const uint32_t s8[8],
                            const ge_niels* __restrict__ btab, ge_cached* __restrict__ vt,
                            const ge_cached* __restrict__ ktab, const uint32_t* __restrict__ kinfo) {
  bool ok;
  uint32_t sx[16], s[8], c[8], cw[8], sw[8];
#pragma unroll
  for (int k = 0; k < 16; k++) sx[k] = k < 8 ? s8[k] : 0u;
  sc_reduce512(s, sx);
#pragma unroll
  for (int k = 0; k < 8; k++) c[k] = k < 4 ? c4[k] : 0u;
  sc_recode16(cw, c);
  ge_p2 U;
  if constexpr (CACHED) {
    ok = (kinfo[0] & 1u) != 0;
    sc_recode65536(sw, s);
    ge_p1p1 x;
    straus_comb<8, true>(x, ktab, cw, btab, sw);
    ge_p1p1_to_p2(U, x);
  } else {
    ge_p3 Y;
    ok = !ge_has_small_order(pk);
    ok = ge_frombytes(Y, pk, false) && ok;
    fe_neg(Y.X, Y.X);
    fe_neg(Y.T, Y.T);
    build_cached_table(vt, Y);
    sc_recode256(sw, s);
    ge_p1p1 x;
    STRAUS<33, 33, 0, 16, true>(x, vt, cw, nullptr, nullptr, btab, sw);
    ge_p1p1_to_p2(U, x);
  }
  gamma_ok = (mid[(size_t)VRF_MID_FLAGS * stride + i].x & 1u) != 0;
  fe z12, z123, z1234, inv, zi;
  uint32_t hs[8], us[8], vs[8], gs[8], g8s[8];
  {
    ge_p2 V, G8;
    fe HZ;
    mid_get_xyz(V.X, V.Y, V.Z, mid, stride, i, VRF_MID_V);
    mid_get_xyz(G8.X, G8.Y, G8.Z, mid, stride, i, VRF_MID_G8);
    mid_get(HZ.v, mid, stride, i, VRF_MID_H + 4);
    fe_mul(z12, U.Z, V.Z);
    fe_mul(z123, z12, G8.Z);
    fe_mul(z1234, z123, HZ);
    fe_invert(inv, z1234);
    fe_mul(zi, inv, z123);            // 1/H.Z
    fe_mul(inv, inv, HZ);             // 1/(U.Z V.Z G8.Z)
    {
      fe HX, HY;
      mid_get(HX.v, mid, stride, i, VRF_MID_H);
      mid_get(HY.v, mid, stride, i, VRF_MID_H + 2);
      ge_tobytes_zi(hs, HX, HY, zi);
    }
    fe_mul(zi, inv, z12);             // 1/G8.Z
    ge_tobytes_zi(g8s, G8.X, G8.Y, zi);
    fe_mul(inv, inv, G8.Z);           // 1/(U.Z V.Z)
    fe_mul(zi, inv, V.Z);             // 1/U.Z
    ge_tobytes_zi(us, U.X, U.Y, zi);
    fe_mul(zi, inv, U.Z);             // 1/V.Z
    ge_tobytes_zi(vs, V.X, V.Y, zi);
  }
  mid_get(gs, mid, stride, i, VRF_MID_GS);
  uint32_t cp[4];
  vrf_hash_points(cp, hs, gs, us, vs);
  bool eq = true;
#pragma unroll
  for (int k = 0; k < 4; k++) eq &= cp[k] == c4[k];
  vrf_beta(beta, g8s);
  return ok && gamma_ok && eq;
}

// Stage U: U = [s]B - [c]Y into planes VRF_MID_U.., vrf_validate_key into VRF_MID_KEY.
// CACHED: kinfo / ktab of k_keys.hip and btab = the global radix-2^16 comb; otherwise Y is
// decoded per lane ({1..8}(-Y) in the lane's 8-entry table vt) and btab = LDS {B, 2^128 B}.
template <bool CACHED>
FE_INLINE void vrf_u_core(uint4* __restrict__ mid, size_t stride, size_t i, const uint32_t pk[8], const uint32_t c4[4],
                          const uint32_t s8[8], const ge_niels* __restrict__ btab, ge_cached* __restrict__ vt,
                          const ge_cached* __restrict__ ktab, const uint32_t* __restrict__ kinfo) {
  bool ok;
  uint32_t sx[16], s[8], c[8], cw[8], sw[8];
#pragma unroll
  for (int k = 0; k < 16; k++) sx[k] = k < 8 ? s8[k] : 0u;
  sc_reduce512(s, sx);
#pragma unroll
  for (int k = 0; k < 8; k++) c[k] = k < 4 ? c4[k] : 0u;
  sc_recode16(cw, c);
  ge_p1p1 x;
  if constexpr (CACHED) {
    ok = (kinfo[0] & 1u) != 0;
    sc_recode65536(sw, s);
    straus_comb<8, true>(x, ktab, cw, btab, sw);
  } else {
    ge_p3 Y;
    ok = !ge_has_small_order(pk);
    ok = ge_frombytes(Y, pk, false) && ok;
    fe_neg(Y.X, Y.X);
    fe_neg(Y.T, Y.T);
    build_cached_table(vt, Y);
    sc_recode256(sw, s);
    STRAUS<33, 33, 0, 16, true>(x, vt, cw, nullptr, nullptr, btab, sw);
  }
  ge_p2 U;
  ge_p1p1_to_p2(U, x);
  mid_put_xyz(mid, stride, i, VRF_MID_U, U.X, U.Y, U.Z);
  mid[(size_t)VRF_MID_KEY * stride + i] = make_uint4(ok ? 1u : 0u, 0u, 0u, 0u);
}

// Join: the batched inversion of U.Z V.Z (8 Gamma).Z H.Z, the four encodings, the
// challenge c' = SHA-512(0x04 || 0x02 || H || Gamma || U || V)[0..16) against c, beta.
FE_INLINE bool vrf_join_core(uint32_t beta[16], bool& gamma_ok, const uint4* __restrict__ mid, size_t stride, size_t i,
                             const uint32_t c4[4]) {
  const bool ok = (mid[(size_t)VRF_MID_KEY * stride + i].x & 1u) != 0;
  gamma_ok = (mid[(size_t)VRF_MID_FLAGS * stride + i].x & 1u) != 0;
  fe z12, z123, z1234, inv, zi;
  uint32_t hs[8], us[8], vs[8], gs[8], g8s[8];
  {
    fe UZ, VZ, G8Z, HZ;
    mid_get(UZ.v, mid, stride, i, VRF_MID_U + 4);
    mid_get(VZ.v, mid, stride, i, VRF_MID_V + 4);
    mid_get(G8Z.v, mid, stride, i, VRF_MID_G8 + 4);
    mid_get(HZ.v, mid, stride, i, VRF_MID_H + 4);
    fe_mul(z12, UZ, VZ);
    fe_mul(z123, z12, G8Z);
    fe_mul(z1234, z123, HZ);
    fe_invert_sel_inl(inv, z1234);   // inline: no caller-saved registers around a call
    fe_mul(zi, inv, z123);            // 1/H.Z
    fe_mul(inv, inv, HZ);             // 1/(U.Z V.Z G8.Z)
    fe X, Y;
    mid_get(X.v, mid, stride, i, VRF_MID_H);
    mid_get(Y.v, mid, stride, i, VRF_MID_H + 2);
    ge_tobytes_zi(hs, X, Y, zi);
    fe_mul(zi, inv, z12);             // 1/G8.Z
    mid_get(X.v, mid, stride, i, VRF_MID_G8);
    mid_get(Y.v, mid, stride, i, VRF_MID_G8 + 2);
    ge_tobytes_zi(g8s, X, Y, zi);
    fe_mul(inv, inv, G8Z);            // 1/(U.Z V.Z)
    fe_mul(zi, inv, VZ);              // 1/U.Z
    mid_get(X.v, mid, stride, i, VRF_MID_U);
    mid_get(Y.v, mid, stride, i, VRF_MID_U + 2);
    ge_tobytes_zi(us, X, Y, zi);
    fe_mul(zi, inv, UZ);              // 1/V.Z
    mid_get(X.v, mid, stride, i, VRF_MID_V);
    mid_get(Y.v, mid, stride, i, VRF_MID_V + 2);
    ge_tobytes_zi(vs, X, Y, zi);
  }
  mid_get(gs, mid, stride, i, VRF_MID_GS);
  uint32_t cp[4];
  vrf_hash_points(cp, hs, gs, us, vs);
  bool eq = true;
#pragma unroll
  for (int k = 0; k < 4; k++) eq &= cp[k] == c4[k];
  vrf_beta(beta, g8s);
  return ok && gamma_ok && eq;
}

// ------------------------------------------------------------------ signing (generator only)
// az = SHA-512(seed), clamped
FE_INLINE void ed25519_expand(uint32_t az[16], const uint32_t seed[8]) {
  uint32_t S[9];
#pragma unroll
  for (int i = 0; i < 8; i++) S[i] = seed[i];
  S[8] = 0x80u;
  sha512_regs<9, 32>(az, S);
  az[0] &= 0xfffffff8u;
  az[7] &= 0x7fffffffu;
  az[7] |= 0x40000000u;
}

// reduce a 256-bit scalar mod L ([a]P = [a mod L]P for P in the prime-order subgroup)
FE_INLINE void sc_reduce256(uint32_t r[8], const uint32_t a[8]) {
  uint32_t x[16];
#pragma unroll
  for (int i = 0; i < 16; i++) x[i] = i < 8 ? a[i] : 0u;
  sc_reduce512(r, x);
}

FE_INLINE void ed25519_pk_from_az(uint32_t pk[8], const uint32_t az[16], const ge_niels* __restrict__ btab) {
  uint32_t a[8];
  sc_reduce256(a, az);
  ge_p3 A;
  ge_scalarmult_base(A, a, btab);
  ge_tobytes(pk, A.X, A.Y, A.Z);
}

// RFC 8032 signature of msg (global memory, 8-aligned, len bytes)
FE_INLINE void ed25519_sign_core(uint32_t sig[16], const uint32_t az[16], const uint32_t pk[8],
                                 const uint8_t* __restrict__ msg, uint32_t len, const ge_niels* __restrict__ btab) {
  uint32_t pre[16], d[16], r[8], h[8], a[8];
#pragma unroll
  for (int i = 0; i < 16; i++) pre[i] = i < 8 ? az[8 + i] : 0u;
  sha512_stream(d, pre, 32, msg, len);
  sc_reduce512(r, d);
  ge_p3 R;
  ge_scalarmult_base(R, r, btab);
  uint32_t rs[8];
  ge_tobytes(rs, R.X, R.Y, R.Z);
#pragma unroll
  for (int i = 0; i < 8; i++) { pre[i] = rs[i]; pre[8 + i] = pk[i]; }
  sha512_stream(d, pre, 64, msg, len);
  sc_reduce512(h, d);
#pragma unroll
  for (int i = 0; i < 8; i++) a[i] = az[i];
  uint32_t S[8];
  sc_muladd(S, h, a, r);
#pragma unroll
  for (int i = 0; i < 8; i++) { sig[i] = rs[i]; sig[8 + i] = S[i]; }
}

// draft-03 prove (crypto_vrf_ietfdraft03_prove): proof = Gamma || c || s
FE_INLINE void vrf_prove_core(uint32_t proof[20], const uint32_t az[16], const uint32_t pk[8],
                              const uint32_t alpha[8], const ge_niels* __restrict__ btab) {
  ge_p3 Y;
  ge_frombytes(Y, pk, false);
  uint32_t ys[8], hs[8];
  ge_enc_affine(ys, Y);
  ge_p3 H;
  vrf_hash_to_curve(H, ys, alpha);
  ge_tobytes(hs, H.X, H.Y, H.Z);
  uint32_t x[8];
  sc_reduce256(x, az);
  ge_p3 G;
  ge_scalarmult_var(G, x, H);
  // k = SHA-512(az[32..64) || h_string) mod L
  uint32_t S[17], d[16], k[8];
#pragma unroll
  for (int i = 0; i < 8; i++) { S[i] = az[8 + i]; S[8 + i] = hs[i]; }
  S[16] = 0x80u;
  sha512_regs<17, 64>(d, S);
  sc_reduce512(k, d);
  ge_p3 kB, kH;
  ge_scalarmult_base(kB, k, btab);
  ge_scalarmult_var(kH, k, H);
  uint32_t gs[8], kbs[8], khs[8];
  ge_tobytes(gs, G.X, G.Y, G.Z);
  ge_tobytes(kbs, kB.X, kB.Y, kB.Z);
  ge_tobytes(khs, kH.X, kH.Y, kH.Z);
  uint32_t c4[4];
  vrf_hash_points(c4, hs, gs, kbs, khs);
  uint32_t c[8], s[8];
#pragma unroll
  for (int i = 0; i < 8; i++) c[i] = i < 4 ? c4[i] : 0u;
  sc_muladd(s, c, x, k);
#pragma unroll
  for (int i = 0; i < 8; i++) { proof[i] = gs[i]; proof[12 + i] = s[i]; }
#pragma unroll
  for (int i = 0; i < 4; i++) proof[8 + i] = c4[i];
}
