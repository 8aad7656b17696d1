// hash.hpp -- per-lane SHA-512 (FIPS 180-4) and single-block BLAKE2b (RFC 7693).
//
// SHA-512 is the hash inside Ed25519 and the VRF draft-03 suite; BLAKE2b-256 /
// -224 are cardano-crypto-class `Blake2b_256` / `Blake2b_224` (KES vk pairs,
// mkInputVRF Praos/VRF.hs:55-69, hashVRF :88-99, hashKey Praos.hs:552).  Every
// BLAKE2b input on the Praos path fits one 128-byte block, so only that form
// exists here.  64-bit words live in VGPR pairs; rotates lower to v_alignbit.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define H_INLINE __device__ __forceinline__

// 64-bit rotate right by a constant as two v_alignbit_b32 (funnel shifts of the
// 32-bit halves) instead of two 64-bit shifts + two ORs; n = 32 is a half swap.
H_INLINE uint64_t ror64(uint64_t x, int n) {
  const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  if (n == 32) return ((uint64_t)lo << 32) | hi;
  if (n < 32)
    return ((uint64_t)__builtin_amdgcn_alignbit(lo, hi, n) << 32) | __builtin_amdgcn_alignbit(hi, lo, n);
  const int m = n - 32;
  return ((uint64_t)__builtin_amdgcn_alignbit(hi, lo, m) << 32) | __builtin_amdgcn_alignbit(lo, hi, m);
}
H_INLINE uint64_t bswap64(uint64_t x) { return __builtin_bswap64(x); }

__device__ __constant__ static const uint64_t SHA512_K[80] = {
  0x428a2f98d728ae22ULL, 0x7137449123ef65cdULL, 0xb5c0fbcfec4d3b2fULL, 0xe9b5dba58189dbbcULL,
  0x3956c25bf348b538ULL, 0x59f111f1b605d019ULL, 0x923f82a4af194f9bULL, 0xab1c5ed5da6d8118ULL,
  0xd807aa98a3030242ULL, 0x12835b0145706fbeULL, 0x243185be4ee4b28cULL, 0x550c7dc3d5ffb4e2ULL,
  0x72be5d74f27b896fULL, 0x80deb1fe3b1696b1ULL, 0x9bdc06a725c71235ULL, 0xc19bf174cf692694ULL,
  0xe49b69c19ef14ad2ULL, 0xefbe4786384f25e3ULL, 0x0fc19dc68b8cd5b5ULL, 0x240ca1cc77ac9c65ULL,
  0x2de92c6f592b0275ULL, 0x4a7484aa6ea6e483ULL, 0x5cb0a9dcbd41fbd4ULL, 0x76f988da831153b5ULL,
  0x983e5152ee66dfabULL, 0xa831c66d2db43210ULL, 0xb00327c898fb213fULL, 0xbf597fc7beef0ee4ULL,
  0xc6e00bf33da88fc2ULL, 0xd5a79147930aa725ULL, 0x06ca6351e003826fULL, 0x142929670a0e6e70ULL,
  0x27b70a8546d22ffcULL, 0x2e1b21385c26c926ULL, 0x4d2c6dfc5ac42aedULL, 0x53380d139d95b3dfULL,
  0x650a73548baf63deULL, 0x766a0abb3c77b2a8ULL, 0x81c2c92e47edaee6ULL, 0x92722c851482353bULL,
  0xa2bfe8a14cf10364ULL, 0xa81a664bbc423001ULL, 0xc24b8b70d0f89791ULL, 0xc76c51a30654be30ULL,
  0xd192e819d6ef5218ULL, 0xd69906245565a910ULL, 0xf40e35855771202aULL, 0x106aa07032bbd1b8ULL,
  0x19a4c116b8d2d0c8ULL, 0x1e376c085141ab53ULL, 0x2748774cdf8eeb99ULL, 0x34b0bcb5e19b48a8ULL,
  0x391c0cb3c5c95a63ULL, 0x4ed8aa4ae3418acbULL, 0x5b9cca4f7763e373ULL, 0x682e6ff3d6b2b8a3ULL,
  0x748f82ee5defb2fcULL, 0x78a5636f43172f60ULL, 0x84c87814a1f0ab72ULL, 0x8cc702081a6439ecULL,
  0x90befffa23631e28ULL, 0xa4506cebde82bde9ULL, 0xbef9a3f7b2c67915ULL, 0xc67178f2e372532bULL,
  0xca273eceea26619cULL, 0xd186b8c721c0c207ULL, 0xeada7dd6cde0eb1eULL, 0xf57d4f7fee6ed178ULL,
  0x06f067aa72176fbaULL, 0x0a637dc5a2c898a6ULL, 0x113f9804bef90daeULL, 0x1b710b35131c471bULL,
  0x28db77f523047d84ULL, 0x32caab7b40c72493ULL, 0x3c9ebe0a15c9bebcULL, 0x431d67c49c100d4cULL,
  0x4cc5d4becb3e42b6ULL, 0x597f299cfc657e2aULL, 0x5fcb6fab3ad6faecULL, 0x6c44198c4a475817ULL};

H_INLINE void sha512_init(uint64_t H[8]) {
  H[0] = 0x6a09e667f3bcc908ULL; H[1] = 0xbb67ae8584caa73bULL; H[2] = 0x3c6ef372fe94f82bULL;
  H[3] = 0xa54ff53a5f1d36f1ULL; H[4] = 0x510e527fade682d1ULL; H[5] = 0x9b05688c2b3e6c1fULL;
  H[6] = 0x1f83d9abfb41bd6bULL; H[7] = 0x5be0cd19137e2179ULL;
}

// One SHA-512 round on the working variables v[] named for round j (a = v[-j mod 8], ..., h =
// v[7 - j mod 8]): no register rotation, the next round reads the same array renamed.
#define SHA512_ROUND(j, kw)                                                                       \
  do {                                                                                           \
    uint64_t& a_ = v[(8 - ((j) & 7)) & 7];                                                       \
    uint64_t& b_ = v[(9 - ((j) & 7)) & 7];                                                       \
    uint64_t& c_ = v[(10 - ((j) & 7)) & 7];                                                      \
    uint64_t& d_ = v[(11 - ((j) & 7)) & 7];                                                      \
    uint64_t& e_ = v[(12 - ((j) & 7)) & 7];                                                      \
    uint64_t& f_ = v[(13 - ((j) & 7)) & 7];                                                      \
    uint64_t& g_ = v[(14 - ((j) & 7)) & 7];                                                      \
    uint64_t& h_ = v[(15 - ((j) & 7)) & 7];                                                      \
    const uint64_t t1_ = h_ + (ror64(e_, 14) ^ ror64(e_, 18) ^ ror64(e_, 41)) + ((e_ & f_) ^ (~e_ & g_)) + (kw); \
    const uint64_t t2_ = (ror64(a_, 28) ^ ror64(a_, 34) ^ ror64(a_, 39)) + ((a_ & b_) ^ (c_ & (a_ ^ b_))); \
    d_ += t1_;                                                                                   \
    h_ = t1_ + t2_;                                                                              \
  } while (0)

// W: 16 big-endian message words (already byte-swapped); consumed in place.  Rounds in
// blocks of 16 with constant W indices and renamed working variables (an 80-round unroll
// request is not honoured at this size: the rolled loop then indexed W through
// s_set_gpr_idx and rotated a..h with eight 64-bit moves per round); the first block
// unrolled, the message schedule's four blocks one runtime loop.
H_INLINE void sha512_block(uint64_t H[8], uint64_t W[16]) {
  uint64_t v[8];
#pragma unroll
  for (int i = 0; i < 8; i++) v[i] = H[i];
#pragma unroll
  for (int j = 0; j < 16; j++) SHA512_ROUND(j, SHA512_K[j] + W[j]);
#pragma clang loop unroll(disable)
  for (int r = 16; r < 80; r += 16) {
#pragma unroll
    for (int j = 0; j < 16; j++) {
      const uint64_t w15 = W[(j + 1) & 15], w2 = W[(j + 14) & 15];
      const uint64_t s0 = ror64(w15, 1) ^ ror64(w15, 8) ^ (w15 >> 7);
      const uint64_t s1 = ror64(w2, 19) ^ ror64(w2, 61) ^ (w2 >> 6);
      W[j] += s0 + W[(j + 9) & 15] + s1;
      SHA512_ROUND(j, SHA512_K[r + j] + W[j]);
    }
  }
#pragma unroll
  for (int i = 0; i < 8; i++) H[i] += v[i];
}

// digest as 16 little-endian u32 words (byte order of the 64-byte output)
H_INLINE void sha512_digest_words(uint32_t out[16], const uint64_t H[8]) {
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint64_t le = bswap64(H[i]);
    out[2 * i] = (uint32_t)le;
    out[2 * i + 1] = (uint32_t)(le >> 32);
  }
}

// load big-endian message word from 8 little-endian bytes given as two u32
H_INLINE uint64_t be_word(uint32_t lo, uint32_t hi) { return bswap64(((uint64_t)hi << 32) | lo); }

// SHA-512 of (prefix[0..64) || msg[0..len)), msg 8-byte aligned in global
// memory and readable up to round_up(len, 8).  Returns digest words.
// Lanes may have different lengths (the loop runs to the wave's maximum).
H_INLINE void sha512_prefix64_msg(uint32_t out[16], const uint32_t prefix[16],
                                  const uint8_t* __restrict__ msg, uint32_t len) {
  uint64_t H[8];
  sha512_init(H);
  const uint32_t total = 64u + len;
  const uint32_t nblocks = (total + 17u + 127u) >> 7;
  for (uint32_t blk = 0; blk < nblocks; blk++) {
    uint64_t W[16];
#pragma unroll
    for (int w = 0; w < 16; w++) {
      const uint32_t off = blk * 128u + 8u * w;            // stream offset
      uint64_t v;
      if (blk == 0 && w < 8) {
        v = be_word(prefix[2 * w], prefix[2 * w + 1]);
      } else {
        const uint32_t m = off - 64u;                      // message offset
        uint64_t raw = 0;
        if (m < len) raw = *(const uint64_t*)(msg + m);
        // bytes >= len are zero; byte at len is 0x80
        const uint32_t valid = len > m ? (len - m) : 0u;   // bytes of message in this word
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

// ---------------------------------------------------------------- BLAKE2b
__device__ __constant__ static const uint64_t B2B_IV[8] = {
  0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL, 0x3c6ef372fe94f82bULL, 0xa54ff53a5f1d36f1ULL,
  0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL, 0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL};

#define B2B_G(a, b, c, d, x, y)                    \
  do {                                             \
    v[a] = v[a] + v[b] + (x); v[d] = ror64(v[d] ^ v[a], 32); \
    v[c] = v[c] + v[d];       v[b] = ror64(v[b] ^ v[c], 24); \
    v[a] = v[a] + v[b] + (y); v[d] = ror64(v[d] ^ v[a], 16); \
    v[c] = v[c] + v[d];       v[b] = ror64(v[b] ^ v[c], 63); \
  } while (0)

// One-block BLAKE2b (unkeyed): m = 16 little-endian words (zero padded),
// len <= 128 message bytes, outlen in {28, 32}.  Output: h[0..3] words.
H_INLINE void blake2b_1block(uint64_t h[4], const uint64_t m[16], uint32_t len, uint32_t outlen) {
  constexpr uint8_t S[12][16] = {
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15}, {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3},
    {11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4}, {7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8},
    {9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13}, {2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9},
    {12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11}, {13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10},
    {6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5}, {10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0},
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15}, {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3}};
  uint64_t v[16];
  uint64_t h0[8];
#pragma unroll
  for (int i = 0; i < 8; i++) h0[i] = B2B_IV[i];
  h0[0] ^= 0x01010000ULL ^ (uint64_t)outlen;
#pragma unroll
  for (int i = 0; i < 8; i++) { v[i] = h0[i]; v[i + 8] = B2B_IV[i]; }
  v[12] ^= (uint64_t)len;
  v[14] = ~v[14];
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
  for (int i = 0; i < 4; i++) h[i] = h0[i] ^ v[i] ^ v[i + 8];
}

// BLAKE2b-256 of 64 bytes given as 16 LE u32 words -> 8 LE u32 words
H_INLINE void blake2b256_64(uint32_t out[8], const uint32_t in[16]) {
  uint64_t m[16];
#pragma unroll
  for (int i = 0; i < 8; i++) m[i] = ((uint64_t)in[2 * i + 1] << 32) | in[2 * i];
#pragma unroll
  for (int i = 8; i < 16; i++) m[i] = 0;
  uint64_t h[4];
  blake2b_1block(h, m, 64, 32);
#pragma unroll
  for (int i = 0; i < 4; i++) { out[2 * i] = (uint32_t)h[i]; out[2 * i + 1] = (uint32_t)(h[i] >> 32); }
}
// BLAKE2b-{224,256} of 32 bytes (8 LE words)
H_INLINE void blake2b_32(uint32_t out[8], const uint32_t in[8], uint32_t outlen) {
  uint64_t m[16];
#pragma unroll
  for (int i = 0; i < 4; i++) m[i] = ((uint64_t)in[2 * i + 1] << 32) | in[2 * i];
#pragma unroll
  for (int i = 4; i < 16; i++) m[i] = 0;
  uint64_t h[4];
  blake2b_1block(h, m, 32, outlen);
#pragma unroll
  for (int i = 0; i < 4; i++) { out[2 * i] = (uint32_t)h[i]; out[2 * i + 1] = (uint32_t)(h[i] >> 32); }
}
// BLAKE2b-256 of (tag byte || 64 bytes)  -- hashVRF "L"/"N" range extension
H_INLINE void blake2b256_tag64(uint32_t out[8], uint32_t tag, const uint32_t in[16]) {
  uint64_t m[16];
  uint64_t prev = tag & 0xffu;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint64_t w = ((uint64_t)in[2 * i + 1] << 32) | in[2 * i];
    m[i] = prev | (w << 8);
    prev = w >> 56;
  }
  m[8] = prev;
#pragma unroll
  for (int i = 9; i < 16; i++) m[i] = 0;
  uint64_t h[4];
  blake2b_1block(h, m, 65, 32);
#pragma unroll
  for (int i = 0; i < 4; i++) { out[2 * i] = (uint32_t)h[i]; out[2 * i + 1] = (uint32_t)(h[i] >> 32); }
}
// mkInputVRF: BLAKE2b-256(BE64(slot) || eta0) (eta0 omitted when neutral)
H_INLINE void mk_input_vrf(uint32_t out[8], uint64_t slot, const uint32_t eta0[8], bool neutral) {
  uint64_t m[16];
  m[0] = bswap64(slot);
#pragma unroll
  for (int i = 0; i < 4; i++) m[1 + i] = neutral ? 0 : (((uint64_t)eta0[2 * i + 1] << 32) | eta0[2 * i]);
#pragma unroll
  for (int i = 5; i < 16; i++) m[i] = 0;
  uint64_t h[4];
  blake2b_1block(h, m, neutral ? 8u : 40u, 32);
#pragma unroll
  for (int i = 0; i < 4; i++) { out[2 * i] = (uint32_t)h[i]; out[2 * i + 1] = (uint32_t)(h[i] >> 32); }
}

// TPraos mkSeed (cardano-protocol-tpraos BHeader.mkSeed): Blake2b256(BE64(slot) || eta0)
// XOR ucNonce, ucNonce = mkNonceFromNumber k = Blake2b256(BE64(k)), k = 0 (seedEta), 1 (seedL).
H_INLINE void tpraos_seed(uint32_t out[8], uint64_t slot, const uint32_t eta0[8], bool neutral, uint64_t k) {
  uint32_t h[8], uc[8];
  mk_input_vrf(h, slot, eta0, neutral);
  uint64_t m[16];
  m[0] = bswap64(k);
#pragma unroll
  for (int i = 1; i < 16; i++) m[i] = 0;
  uint64_t hh[4];
  blake2b_1block(hh, m, 8, 32);
#pragma unroll
  for (int i = 0; i < 4; i++) { uc[2 * i] = (uint32_t)hh[i]; uc[2 * i + 1] = (uint32_t)(hh[i] >> 32); }
#pragma unroll
  for (int i = 0; i < 8; i++) out[i] = h[i] ^ uc[i];
}
// mkNonceFromOutputVRF: Blake2b256 of the 64-byte VRF output (16 LE words)
H_INLINE void blake2b256_of64(uint32_t out[8], const uint32_t in[16]) { blake2b256_64(out, in); }
