// host_util.hpp -- host-side helpers of libpraos_hip (C++; no device code).
//   * BLAKE2b-224 for issuer hashes of headers whose pool is not in the
//     distribution (praos_apply_batch needs hashKey for the counter map,
//     Praos.hs:595-606);
//   * x = -(fromRational sigma * c) in Fixed E34 (checkLeaderNatValue's x,
//     precomputed once per pool and epoch).
#pragma once
#include <cstdint>
#include <cstring>

#include "praos_hip.h"

namespace praos_host {

inline uint64_t ror64(uint64_t x, int n) { return (x >> n) | (x << (64 - n)); }

// BLAKE2b (RFC 7693), unkeyed.  The 16 working words live in locals and the 12
// rounds are unrolled with compile-time message schedules, so the compiler keeps the
// whole compression in registers (~3x faster than an indexed v[16] array; the
// sequential evolving-nonce chain of the fold is one compression per header).
#define PH_G(a, b, c, d, x, y)               \
  a = a + b + (x); d = ror64(d ^ a, 32);     \
  c = c + d;       b = ror64(b ^ c, 24);     \
  a = a + b + (y); d = ror64(d ^ a, 16);     \
  c = c + d;       b = ror64(b ^ c, 63);
#define PH_ROUND(s0, s1, s2, s3, s4, s5, s6, s7, s8, s9, s10, s11, s12, s13, s14, s15) \
  PH_G(v0, v4, v8, v12, M[s0], M[s1]) PH_G(v1, v5, v9, v13, M[s2], M[s3])          \
  PH_G(v2, v6, v10, v14, M[s4], M[s5]) PH_G(v3, v7, v11, v15, M[s6], M[s7])        \
  PH_G(v0, v5, v10, v15, M[s8], M[s9]) PH_G(v1, v6, v11, v12, M[s10], M[s11])      \
  PH_G(v2, v7, v8, v13, M[s12], M[s13]) PH_G(v3, v4, v9, v14, M[s14], M[s15])

// compression over message words M (inlined into its callers: where M's words are known
// constants -- the zero half of a 64-byte message -- the compiler drops their additions)
__attribute__((always_inline)) inline void blake2b_compress_words(uint64_t h[8], const uint64_t M[16], uint64_t t,
                                                                  bool last) {
  static constexpr uint64_t IV[8] = {0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL, 0x3c6ef372fe94f82bULL,
                                     0xa54ff53a5f1d36f1ULL, 0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL,
                                     0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL};
  uint64_t v0 = h[0], v1 = h[1], v2 = h[2], v3 = h[3], v4 = h[4], v5 = h[5], v6 = h[6], v7 = h[7];
  uint64_t v8 = IV[0], v9 = IV[1], v10 = IV[2], v11 = IV[3], v12 = IV[4] ^ t, v13 = IV[5];
  uint64_t v14 = last ? ~IV[6] : IV[6], v15 = IV[7];
  PH_ROUND(0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15)
  PH_ROUND(14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3)
  PH_ROUND(11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4)
  PH_ROUND(7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8)
  PH_ROUND(9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13)
  PH_ROUND(2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9)
  PH_ROUND(12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11)
  PH_ROUND(13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10)
  PH_ROUND(6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5)
  PH_ROUND(10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0)
  PH_ROUND(0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15)
  PH_ROUND(14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3)
  h[0] ^= v0 ^ v8; h[1] ^= v1 ^ v9; h[2] ^= v2 ^ v10; h[3] ^= v3 ^ v11;
  h[4] ^= v4 ^ v12; h[5] ^= v5 ^ v13; h[6] ^= v6 ^ v14; h[7] ^= v7 ^ v15;
}

inline void blake2b_compress(uint64_t h[8], const uint8_t blk[128], uint64_t t, bool last) {
  uint64_t M[16];
  std::memcpy(M, blk, 128);                          // little-endian host
  blake2b_compress_words(h, M, t, last);
}
#undef PH_ROUND
#undef PH_G

inline void blake2b(uint8_t* out, size_t outlen, const uint8_t* m, size_t n) {
  uint64_t h[8] = {0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL, 0x3c6ef372fe94f82bULL, 0xa54ff53a5f1d36f1ULL,
                   0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL, 0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL};
  h[0] ^= 0x01010000ULL ^ (uint64_t)outlen;
  size_t off = 0;
  while (n - off > 128) { off += 128; blake2b_compress(h, m + off - 128, off, false); }
  uint8_t blk[128] = {0};
  std::memcpy(blk, m + off, n - off);
  blake2b_compress(h, blk, n, true);
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

// a ⭒ b (Nonce semigroup): Neutral is the identity, else Blake2b-256(a || b).
inline praos_nonce nonce_combine(const praos_nonce& a, const praos_nonce& b) {
  if (a.neutral) return b;
  if (b.neutral) return a;
  // Blake2b-256 of the 64-byte a || b: one compression whose second message half is the
  // constant zero padding (the fold's and the replay's nonce chains are one of these per header)
  uint64_t M[16] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  std::memcpy(M, a.hash, 32);
  std::memcpy(M + 4, b.hash, 32);
  uint64_t h[8] = {0x6a09e667f3bcc908ULL ^ 0x01010020ULL, 0xbb67ae8584caa73bULL, 0x3c6ef372fe94f82bULL,
                   0xa54ff53a5f1d36f1ULL, 0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL, 0x1f83d9abfb41bd6bULL,
                   0x5be0cd19137e2179ULL};
  blake2b_compress_words(h, M, 64, true);
  praos_nonce r;
  std::memcpy(r.hash, h, 32);                        // little-endian host
  r.neutral = 0;
  return r;
}

inline bool nonce_eq(const praos_nonce& a, const praos_nonce& b) {
  if (a.neutral || b.neutral) return a.neutral && b.neutral;
  return std::memcmp(a.hash, b.hash, 32) == 0;
}

}  // namespace praos_host
