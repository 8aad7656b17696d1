// leader.hpp -- checkLeaderNatValue in bit-exact Fixed E34 arithmetic, per lane.
//
// Restates cardano-protocol-tpraos `checkLeaderNatValue` /
// cardano-ledger-core `taylorExpCmp` (called at Praos.hs:549):
//   recip_q = fromRational (2^256 / (2^256 - l))       -- raw floor(N / D)
//   x       = -(fromRational sigma * c)                 -- precomputed per pool
//   go n err acc divisor (from 0 x 1 1):
//     divisor' = divisor + 1;  err' = err * x / divisor';  acc' = acc + err
//     e = |err' * 3|
//     cmp >= acc' + e -> ABOVE (not leader); cmp < acc' - e -> BELOW (leader)
//     n == 1000 -> MaxReached (not leader)
// Fixed E34 raw ops: a*b = floor(ab / R), a / k = floor(a / k) (k integral),
// R = 10^34.  recip_q itself (a 370-bit quotient) is never formed:
// floor(N/D) >= T  <=>  N >= T*D  and  floor(N/D) < T  <=>  N < T*D.
#pragma once
#include "fe25519.hpp"

// R = 10^34 (4 words), mu = floor(2^256 / R) (5 words)
__device__ __constant__ static const uint32_t FX_R[4] = {0x00000000u, 0x378d8e64u, 0xbead87c0u, 0x0001ed09u};
__device__ __constant__ static const uint32_t FX_MU[5] = {0x113ebf96u, 0xf13bef0bu, 0x4ab4bd5au, 0x3c97da62u, 0x000084ecu};

// Barrett quotient floor(x / R) for x < 2^256 (8 words), mu = floor(2^256 / R)
FE_INLINE void fx_div_R(uint32_t q[8], const uint32_t x[8]) {
  const uint32_t* mu = FX_MU;
  // q1 = x >> 96 (5 words); q2 = q1 * mu (10 words); q3 = q2 >> 160 (5 words)
  uint32_t q2[10];
#pragma unroll
  for (int i = 0; i < 10; i++) q2[i] = 0;
#pragma unroll
  for (int i = 0; i < 5; i++) {
    uint64_t c = 0;
#pragma unroll
    for (int j = 0; j < 5; j++) {
      const uint64_t s = (uint64_t)x[3 + i] * mu[j] + q2[i + j] + c;
      q2[i + j] = (uint32_t)s;
      c = s >> 32;
    }
    q2[i + 5] = (uint32_t)c;
  }
  uint32_t q3[5];
#pragma unroll
  for (int i = 0; i < 5; i++) q3[i] = q2[5 + i];
  // r = x - q3 * R  (fits in 5 words since r < 3R)
  uint32_t p[5];
#pragma unroll
  for (int i = 0; i < 5; i++) p[i] = 0;
#pragma unroll
  for (int i = 0; i < 5; i++) {
    uint64_t c = 0;
#pragma unroll
    for (int j = 0; j < 4; j++) {
      if (i + j >= 5) continue;
      const uint64_t s = (uint64_t)q3[i] * FX_R[j] + p[i + j] + c;
      p[i + j] = (uint32_t)s;
      c = s >> 32;
    }
    if (i + 4 < 5) p[i + 4] += (uint32_t)c;
  }
  uint32_t r[5];
  uint32_t bw = 0;
#pragma unroll
  for (int i = 0; i < 5; i++) r[i] = subb(x[i], p[i], bw, &bw);
#pragma unroll
  for (int k = 0; k < 2; k++) {
    uint32_t u[5];
    uint32_t b2 = 0;
#pragma unroll
    for (int i = 0; i < 4; i++) u[i] = subb(r[i], FX_R[i], b2, &b2);
    u[4] = subb(r[4], 0, b2, &b2);
    const bool ge = b2 == 0;
#pragma unroll
    for (int i = 0; i < 5; i++) r[i] = ge ? u[i] : r[i];
    // q3 += ge
    uint32_t c = ge ? 1u : 0u;
#pragma unroll
    for (int i = 0; i < 5; i++) q3[i] = addc(q3[i], 0, c, &c);
  }
#pragma unroll
  for (int i = 0; i < 8; i++) q[i] = i < 5 ? q3[i] : 0;
}

// a (n words) * b (m words) -> r (n+m words)
template <int N, int M>
FE_INLINE void mp_mul(uint32_t r[N + M], const uint32_t a[N], const uint32_t b[M]) {
#pragma unroll
  for (int i = 0; i < N + M; i++) r[i] = 0;
#pragma unroll
  for (int i = 0; i < N; i++) {
    uint64_t c = 0;
#pragma unroll
    for (int j = 0; j < M; j++) {
      const uint64_t s = (uint64_t)a[i] * b[j] + r[i + j] + c;
      r[i + j] = (uint32_t)s;
      c = s >> 32;
    }
    r[i + M] = (uint32_t)c;
  }
}

// -1, 0, 1 compare of n-word numbers
template <int N>
FE_INLINE int mp_cmp(const uint32_t a[N], const uint32_t b[N]) {
  int r = 0;
#pragma unroll
  for (int i = 0; i < N; i++) {
    r = a[i] > b[i] ? 1 : (a[i] < b[i] ? -1 : r);
  }
  return r;
}

// floor(a / k), a: 8 words, 2 <= k < 2^16 (k = n + 2 <= 1001): 16-bit
// limbs so every step is a 32-bit by 32-bit division.
FE_INLINE void mp_div_small(uint32_t q[8], const uint32_t a[8], uint32_t k) {
  uint32_t rem = 0;
#pragma unroll
  for (int i = 7; i >= 0; i--) {
    const uint32_t hi = (rem << 16) | (a[i] >> 16);
    const uint32_t qh = hi / k;
    rem = hi - qh * k;
    const uint32_t lo = (rem << 16) | (a[i] & 0xffffu);
    const uint32_t ql = lo / k;
    rem = lo - ql * k;
    q[i] = (qh << 16) | ql;
  }
}

// Returns true = leader (BELOW).  l_le: leader value as LW LE words (natural,
// bound certNatMax = 2^(32 LW): LW = 8 for Praos (Blake2b-256 range extension,
// Praos/VRF.hs:103-112), LW = 16 for TPraos (raw 64-byte VRF output);
// x: Fixed raw x (4 words, >= 0).
template <int LW>
FE_INLINE bool leader_check_t(const uint32_t l_le[LW], const uint32_t x[4], int* iters_out) {
  constexpr int NW = LW + 5;          // N = 2^(32 LW) * R, plus one zero word
  constexpr int PW = 8 + LW + 1;      // (8-word value) * D
  // D = 2^(32 LW) - l  (LW + 1 words)
  uint32_t D[LW + 1];
  uint32_t bw = 0;
#pragma unroll
  for (int i = 0; i < LW; i++) D[i] = subb(0u, l_le[i], bw, &bw);
  D[LW] = 1u - bw;           // l == 0 -> D = 2^(32 LW)
  uint32_t N[NW];
#pragma unroll
  for (int i = 0; i < NW; i++) N[i] = 0;
#pragma unroll
  for (int i = 0; i < 4; i++) N[LW + i] = FX_R[i];
  uint32_t err[8], acc[8];
#pragma unroll
  for (int i = 0; i < 8; i++) { err[i] = i < 4 ? x[i] : 0; acc[i] = i < 4 ? FX_R[i] : 0; }
  // The iteration count is wave-uniform (every active lane is at the same n);
  // lanes that have decided stay masked off and the loop exits when all have,
  // so no value crosses a divergent loop exit.
  int res = -1, iters = 1000;
  for (int n = 0; n < 1000; n++) {
    if (res < 0) {
      const uint32_t k = (uint32_t)n + 2u;
      // t = floor(err * x / R);  err' = floor(t / k)
      uint32_t ex[12];
      mp_mul<8, 4>(ex, err, x);
      uint32_t t[8];
      fx_div_R(t, ex);      // err * x < 2^256 for every sane (sigma, f)
      uint32_t errp[8];
      mp_div_small(errp, t, k);
      // acc' = acc + err
      uint32_t accp[8];
      uint32_t c = 0;
#pragma unroll
      for (int i = 0; i < 8; i++) accp[i] = addc(acc[i], err[i], c, &c);
      // e = 3 * err'
      uint32_t e[8];
      uint64_t cc = 0;
#pragma unroll
      for (int i = 0; i < 8; i++) { cc += (uint64_t)errp[i] * 3u; e[i] = (uint32_t)cc; cc >>= 32; }
      // hi = acc' + e ; ABOVE iff N >= hi * D
      uint32_t hi[8];
      c = 0;
#pragma unroll
      for (int i = 0; i < 8; i++) hi[i] = addc(accp[i], e[i], c, &c);
      uint32_t hd[PW];
      mp_mul<8, LW + 1>(hd, hi, D);
      uint32_t big = 0;
#pragma unroll
      for (int i = NW; i < PW; i++) big |= hd[i];
      const bool above = big == 0 && mp_cmp<NW>(N, hd) >= 0;
      // lo = acc' - e (if non-negative); BELOW iff N < lo * D
      uint32_t lo[8];
      uint32_t b = 0;
#pragma unroll
      for (int i = 0; i < 8; i++) lo[i] = subb(accp[i], e[i], b, &b);
      uint32_t ld[PW];
      mp_mul<8, LW + 1>(ld, lo, D);
      uint32_t lbig = 0;
#pragma unroll
      for (int i = NW; i < PW; i++) lbig |= ld[i];
      const bool below = b == 0 && (lbig != 0 || mp_cmp<NW>(N, ld) < 0);
      if (above) { res = 0; iters = n + 1; }
      else if (below) { res = 1; iters = n + 1; }
#pragma unroll
      for (int i = 0; i < 8; i++) { err[i] = errp[i]; acc[i] = accp[i]; }
    }
    if (__all(res >= 0)) break;
  }
  const bool result = res == 1;                 // MaxReached -> not leader
  if (iters_out) *iters_out = iters;
  return result;
}

FE_INLINE bool leader_check(const uint32_t l_le[8], const uint32_t x[4], int* iters_out) {
  return leader_check_t<8>(l_le, x, iters_out);
}
