// host_util.hpp -- host-side helpers of libpraos_hip (C++; no device code).
//   * BLAKE2b-224 for issuer hashes of headers whose pool is not in the
//     distribution (praos_apply_batch needs hashKey for the counter map,
//     Praos.hs:595-606);
//   * x = -(fromRational sigma * c) in Fixed E34 (checkLeaderNatValue's x,
//     precomputed once per pool and epoch).
#pragma once
#include <cstdint>
#include <cstring>

namespace praos_host {

inline uint64_t ror64(uint64_t x, int n) { return (x >> n) | (x << (64 - n)); }

inline void blake2b(uint8_t* out, size_t outlen, const uint8_t* m, size_t n) {
  static const uint64_t IV[8] = {0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL, 0x3c6ef372fe94f82bULL,
                                 0xa54ff53a5f1d36f1ULL, 0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL,
                                 0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL};
  static const uint8_t S[12][16] = {
      {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15}, {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3},
      {11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4}, {7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8},
      {9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13}, {2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9},
      {12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11}, {13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10},
      {6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5}, {10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0},
      {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15}, {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3}};
  uint64_t h[8];
  for (int i = 0; i < 8; i++) h[i] = IV[i];
  h[0] ^= 0x01010000ULL ^ (uint64_t)outlen;
  size_t off = 0;
  auto compress = [&](const uint8_t* blk, uint64_t t, bool last) {
    uint64_t mm[16], v[16];
    for (int i = 0; i < 16; i++) { uint64_t w; std::memcpy(&w, blk + 8 * i, 8); mm[i] = w; }
    for (int i = 0; i < 8; i++) { v[i] = h[i]; v[i + 8] = IV[i]; }
    v[12] ^= t;
    if (last) v[14] = ~v[14];
    auto G = [&](int a, int b, int c, int d, uint64_t x, uint64_t y) {
      v[a] = v[a] + v[b] + x; v[d] = ror64(v[d] ^ v[a], 32);
      v[c] = v[c] + v[d]; v[b] = ror64(v[b] ^ v[c], 24);
      v[a] = v[a] + v[b] + y; v[d] = ror64(v[d] ^ v[a], 16);
      v[c] = v[c] + v[d]; v[b] = ror64(v[b] ^ v[c], 63);
    };
    for (int r = 0; r < 12; r++) {
      const uint8_t* s = S[r];
      G(0, 4, 8, 12, mm[s[0]], mm[s[1]]); G(1, 5, 9, 13, mm[s[2]], mm[s[3]]);
      G(2, 6, 10, 14, mm[s[4]], mm[s[5]]); G(3, 7, 11, 15, mm[s[6]], mm[s[7]]);
      G(0, 5, 10, 15, mm[s[8]], mm[s[9]]); G(1, 6, 11, 12, mm[s[10]], mm[s[11]]);
      G(2, 7, 8, 13, mm[s[12]], mm[s[13]]); G(3, 4, 9, 14, mm[s[14]], mm[s[15]]);
    }
    for (int i = 0; i < 8; i++) h[i] ^= v[i] ^ v[i + 8];
  };
  while (n - off > 128) { off += 128; compress(m + off - 128, off, false); }
  uint8_t blk[128] = {0};
  std::memcpy(blk, m + off, n - off);
  compress(blk, n, true);
  for (size_t i = 0; i < outlen; i++) out[i] = (uint8_t)(h[i / 8] >> (8 * (i % 8)));
}

// ---- 256-bit unsigned helpers (4 x u64 LE) ----
struct u256 { uint64_t w[4]; };

inline u256 mul128(const uint8_t a_le[16], const uint8_t b_le[16]) {
  uint64_t a[2], b[2];
  std::memcpy(a, a_le, 16);
  std::memcpy(b, b_le, 16);
  u256 r{};
  for (int i = 0; i < 2; i++) {
    unsigned __int128 c = 0;
    for (int j = 0; j < 2; j++) {
      c += (unsigned __int128)a[i] * b[j] + r.w[i + j];
      r.w[i + j] = (uint64_t)c;
      c >>= 64;
    }
    r.w[i + 2] += (uint64_t)c;
  }
  return r;
}

// ceil(x / d) for 128-bit d, bit-serial (per pool, once per epoch)
inline void ceil_div_256_128(uint8_t q_le[16], const u256& x, unsigned __int128 d, bool* overflow) {
  unsigned __int128 rem = 0;
  u256 q{};
  for (int bit = 255; bit >= 0; bit--) {
    const bool top = (rem >> 127) != 0;
    rem = (rem << 1) | ((x.w[bit / 64] >> (bit % 64)) & 1);
    if (top || rem >= d) { rem -= d; q.w[bit / 64] |= 1ull << (bit % 64); }
  }
  if (rem != 0) {  // +1
    for (int i = 0; i < 4; i++) { if (++q.w[i] != 0) break; }
  }
  *overflow = (q.w[2] | q.w[3]) != 0;
  std::memcpy(q_le, q.w, 16);
}

// x_raw = -floor(sigma_fp * c_raw / R) = ceil(sigma_fp * |c| / R) for c_raw <= 0.
// Rejected above X_MAX = 16 R: the device Taylor loop (leader.hpp) keeps err * x in
// 256 bits, and err_n <= R e^X, so err * x <= R^2 X e^X < 2^226 * 2^28 for X <= 16
// (sigma |ln(1-f)| <= 16 covers every f <= 1 - e^-16).
inline bool leader_x_raw(uint8_t x_le[16], const uint8_t sigma_fp[16], const uint8_t c_raw[16]) {
  unsigned __int128 c;
  std::memcpy(&c, c_raw, 16);
  const bool neg = (c >> 127) != 0;
  if (!neg) {  // c >= 0: only c == 0 is meaningful (x = 0)
    std::memset(x_le, 0, 16);
    return c == 0;
  }
  unsigned __int128 mag = ~c + 1;
  uint8_t mag_le[16];
  std::memcpy(mag_le, &mag, 16);
  u256 p = mul128(sigma_fp, mag_le);
  unsigned __int128 R = (unsigned __int128)1;
  for (int i = 0; i < 34; i++) R *= 10;
  bool of = false;
  ceil_div_256_128(x_le, p, R, &of);
  if (of) return false;
  unsigned __int128 x;
  std::memcpy(&x, x_le, 16);
  return x <= 16 * R;
}

}  // namespace praos_host
