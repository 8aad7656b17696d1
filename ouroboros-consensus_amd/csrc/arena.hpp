// arena.hpp -- byte-arena loads and multi-block Blake2b-256 shared by the
// stored-bytes kernels (k_decode.hip headers, k_block.hip block bodies).
// ld64u: 8 bytes at any offset as two aligned 8-byte loads + a funnel shift;
// callers pad the arena by 16 bytes so the second load never leaves it.
#pragma once
#include "kcommon.hpp"

__device__ __forceinline__ uint64_t ld64a(const uint8_t* __restrict__ p, uint64_t a) {
  return *(const uint64_t*)(p + a);
}
// 8 bytes at an arbitrary offset (little-endian)
__device__ __forceinline__ uint64_t ld64u(const uint8_t* __restrict__ p, uint64_t pos) {
  const uint64_t a = pos & ~7ull;
  const uint32_t sh = (uint32_t)(pos & 7u) * 8u;
  const uint64_t lo = ld64a(p, a);
  if (sh == 0) return lo;
  const uint64_t hi = ld64a(p, a + 8);
  return (lo >> sh) | (hi << (64u - sh));
}

// Blake2b compression (RFC 7693 F) for the multi-block header hash
__device__ __forceinline__ void b2b_compress(uint64_t h[8], const uint64_t m[16], uint64_t t, bool last) {
  constexpr uint8_t S[12][16] = {
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15}, {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3},
    {11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4}, {7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8},
    {9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13}, {2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9},
    {12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11}, {13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10},
    {6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5}, {10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0},
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15}, {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3}};
  uint64_t v[16];
#pragma unroll
  for (int i = 0; i < 8; i++) { v[i] = h[i]; v[i + 8] = B2B_IV[i]; }
  v[12] ^= t;
  if (last) v[14] = ~v[14];
#pragma unroll
  for (int r = 0; r < 12; r++) {
    B2B_G(0, 4, 8, 12, m[S[r][0]], m[S[r][1]]);
    B2B_G(1, 5, 9, 13, m[S[r][2]], m[S[r][3]]);
    B2B_G(2, 6, 10, 14, m[S[r][4]], m[S[r][5]]);
    B2B_G(3, 7, 11, 15, m[S[r][6]], m[S[r][7]]);
    B2B_G(0, 5, 10, 15, m[S[r][8]], m[S[r][9]]);
    B2B_G(1, 6, 11, 12, m[S[r][10]], m[S[r][11]]);
    B2B_G(2, 7, 8, 13, m[S[r][12]], m[S[r][13]]);
    B2B_G(3, 4, 9, 14, m[S[r][14]], m[S[r][15]]);
  }
#pragma unroll
  for (int i = 0; i < 8; i++) h[i] ^= v[i] ^ v[i + 8];
}

// one 128-byte message block of p[pos, pos + len) starting at byte `base` (zero padded)
__device__ __forceinline__ void b2b_load_block(uint64_t m[16], const uint8_t* __restrict__ p, uint64_t pos,
                                               uint64_t len, uint64_t base) {
#pragma unroll
  for (int k = 0; k < 16; k++) {
    const uint64_t o = base + 8 * k;
    uint64_t w = o < len ? ld64u(p, pos + o) : 0;
    if (o < len && len - o < 8) w &= (1ull << (8 * (len - o))) - 1;
    m[k] = w;
  }
}

// Blake2b-256 of p[pos, pos + len).  Register double buffering: block b + 1 is
// loaded before block b is compressed, so its (uncoalesced, per-lane) loads are
// in flight during ~2k VALU instructions -- latency hidden even at one wave per
// SIMD, which is what a batch of long block segments gives.
__device__ __forceinline__ void b2b256_range(uint32_t out[8], const uint8_t* __restrict__ p, uint64_t pos,
                                             uint64_t len) {
  uint64_t h[8];
#pragma unroll
  for (int i = 0; i < 8; i++) h[i] = B2B_IV[i];
  h[0] ^= 0x01010000ULL ^ 32u;
  const uint64_t nblk = len == 0 ? 1 : (len + 127) / 128;
  uint64_t nxt[16];
  b2b_load_block(nxt, p, pos, len, 0);
  for (uint64_t b = 0; b < nblk; b++) {
    uint64_t m[16];
#pragma unroll
    for (int k = 0; k < 16; k++) m[k] = nxt[k];
    const uint64_t base = 128 * b;
    if (b + 1 < nblk) b2b_load_block(nxt, p, pos, len, base + 128);
    const bool last = b + 1 == nblk;
    b2b_compress(h, m, last ? len : base + 128, last);
  }
#pragma unroll
  for (int i = 0; i < 4; i++) { out[2 * i] = (uint32_t)h[i]; out[2 * i + 1] = (uint32_t)(h[i] >> 32); }
}
