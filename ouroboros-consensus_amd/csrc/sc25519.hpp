// sc25519.hpp -- scalars modulo L = 2^252 + 27742317777372353535851937790883648493.
//
// Barrett reduction with 32-bit words (b = 2^32, k = 8, mu = floor(b^16 / L)).
// Used for h = SHA-512(R||A||M) mod L (Ed25519), s mod L (VRF proof s,
// reduced as libsodium's vrf_verify does) and the signer's S = r + h*a.
#pragma once
#include "fe25519.hpp"

__device__ __constant__ static const uint32_t SC_L[8] = {0x5cf5d3edu, 0x5812631au, 0xa2f79cd6u, 0x14def9deu,
                                                          0u, 0u, 0u, 0x10000000u};
__device__ __constant__ static const uint32_t SC_MU[9] = {0x0a2c131bu, 0xed9ce5a3u, 0x086329a7u, 0x2106215du, 0xffffffebu,
                                                           0xffffffffu, 0xffffffffu, 0xffffffffu, 0x0000000fu};

// r = x mod L, x = 16 LE words
FE_INLINE void sc_reduce512(uint32_t r[8], const uint32_t x[16]) {
  // q1 = x >> 224 (9 words); q2 = q1 * mu; q3 = q2 >> 288
  uint32_t q2[18];
#pragma unroll
  for (int i = 0; i < 18; i++) q2[i] = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    uint64_t c = 0;
#pragma unroll
    for (int j = 0; j < 9; j++) {
      const uint64_t s = (uint64_t)x[7 + i] * SC_MU[j] + q2[i + j] + c;
      q2[i + j] = (uint32_t)s;
      c = s >> 32;
    }
    q2[i + 9] = (uint32_t)c;
  }
  // r2 = (q3 * L) mod b^9
  uint32_t r2[9];
#pragma unroll
  for (int i = 0; i < 9; i++) r2[i] = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    uint64_t c = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) {
      if (i + j >= 9) continue;
      const uint64_t s = (uint64_t)q2[9 + i] * SC_L[j] + r2[i + j] + c;
      r2[i + j] = (uint32_t)s;
      c = s >> 32;
    }
    if (i + 8 < 9) r2[i + 8] = (uint32_t)c;
  }
  // t = x mod b^9 - r2 (mod b^9)
  uint32_t t[9];
  uint32_t bw = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) t[i] = subb(x[i], r2[i], bw, &bw);
  // at most two subtractions of L
#pragma unroll
  for (int k = 0; k < 2; k++) {
    uint32_t u[9];
    uint32_t b2 = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) u[i] = subb(t[i], SC_L[i], b2, &b2);
    u[8] = subb(t[8], 0, b2, &b2);
    const bool ge = b2 == 0;
#pragma unroll
    for (int i = 0; i < 9; i++) t[i] = ge ? u[i] : t[i];
  }
#pragma unroll
  for (int i = 0; i < 8; i++) r[i] = t[i];
}

// r = (a * b + c) mod L, all 8-word LE
FE_INLINE void sc_muladd(uint32_t r[8], const uint32_t a[8], const uint32_t b[8], const uint32_t c[8]) {
  uint32_t p[16];
#pragma unroll
  for (int i = 0; i < 16; i++) p[i] = i < 8 ? c[i] : 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint64_t cy = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) {
      const uint64_t s = (uint64_t)a[i] * b[j] + p[i + j] + cy;
      p[i + j] = (uint32_t)s;
      cy = s >> 32;
    }
    // propagate into the remaining words
#pragma unroll
    for (int k = i + 8; k < 16; k++) {
      const uint64_t s = (uint64_t)p[k] + cy;
      p[k] = (uint32_t)s;
      cy = s >> 32;
    }
  }
  sc_reduce512(r, p);
}

// S < L (libsodium sc25519_is_canonical)
FE_INLINE bool sc_is_canonical(const uint32_t s[8]) {
  uint32_t b = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) subb(s[i], SC_L[i], b, &b);
  return b != 0;
}
