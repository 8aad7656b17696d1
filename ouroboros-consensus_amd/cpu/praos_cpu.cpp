// praos_cpu.cpp -- libpraos_cpu.so: the CPU twin of libpraos_hip.
//
// A multi-threaded C++ implementation of the header-crypto part of the
// include/praos_hip.h ABI (praos_open / praos_set_epoch / praos_verify_headers and
// the single-primitive batches), written for x86-64 host cores: GF(2^255-19) in
// radix 2^51 with 64x64->128 products, Straus double-scalar multiplication with
// sliding signed windows (width 5 for per-signature bases, width 8 over a static
// table of odd multiples of B), Elligator2 without inversions, and the Fixed E34
// leader test by cross-multiplication.  Semantics are those of the reference's
// crypto as restated in SURVEY.md Appendix C (libsodium 1.0.18 Ed25519 rules, IOG
// ECVRF draft-03, Sum6KES, checkLeaderNatValue) -- the same restatement the GPU
// kernels follow; tests/test_cpu_twin.py gates it against the oracle bit for bit.
//
// It is the timed CPU baseline of bench.py (the Haskell reference cannot run in
// this pipeline) and a library a caller can choose EXPLICITLY; libpraos_hip never
// falls back to it.  Entry points not listed here (device-resident batches,
// decode, block integrity, generator) exist only in libpraos_hip.
#include "praos_hip.h"

#include <algorithm>
#include <array>
#include <atomic>
#include <cstdio>
#include <cstring>
#include <map>
#include <string>
#include <thread>
#include <vector>

#include <sched.h>

namespace {

typedef unsigned __int128 u128;

// ============================================================ hashes
const uint64_t K512[80] = {
    0x428a2f98d728ae22ULL, 0x7137449123ef65cdULL, 0xb5c0fbcfec4d3b2fULL, 0xe9b5dba58189dbbcULL, 0x3956c25bf348b538ULL,
    0x59f111f1b605d019ULL, 0x923f82a4af194f9bULL, 0xab1c5ed5da6d8118ULL, 0xd807aa98a3030242ULL, 0x12835b0145706fbeULL,
    0x243185be4ee4b28cULL, 0x550c7dc3d5ffb4e2ULL, 0x72be5d74f27b896fULL, 0x80deb1fe3b1696b1ULL, 0x9bdc06a725c71235ULL,
    0xc19bf174cf692694ULL, 0xe49b69c19ef14ad2ULL, 0xefbe4786384f25e3ULL, 0x0fc19dc68b8cd5b5ULL, 0x240ca1cc77ac9c65ULL,
    0x2de92c6f592b0275ULL, 0x4a7484aa6ea6e483ULL, 0x5cb0a9dcbd41fbd4ULL, 0x76f988da831153b5ULL, 0x983e5152ee66dfabULL,
    0xa831c66d2db43210ULL, 0xb00327c898fb213fULL, 0xbf597fc7beef0ee4ULL, 0xc6e00bf33da88fc2ULL, 0xd5a79147930aa725ULL,
    0x06ca6351e003826fULL, 0x142929670a0e6e70ULL, 0x27b70a8546d22ffcULL, 0x2e1b21385c26c926ULL, 0x4d2c6dfc5ac42aedULL,
    0x53380d139d95b3dfULL, 0x650a73548baf63deULL, 0x766a0abb3c77b2a8ULL, 0x81c2c92e47edaee6ULL, 0x92722c851482353bULL,
    0xa2bfe8a14cf10364ULL, 0xa81a664bbc423001ULL, 0xc24b8b70d0f89791ULL, 0xc76c51a30654be30ULL, 0xd192e819d6ef5218ULL,
    0xd69906245565a910ULL, 0xf40e35855771202aULL, 0x106aa07032bbd1b8ULL, 0x19a4c116b8d2d0c8ULL, 0x1e376c085141ab53ULL,
    0x2748774cdf8eeb99ULL, 0x34b0bcb5e19b48a8ULL, 0x391c0cb3c5c95a63ULL, 0x4ed8aa4ae3418acbULL, 0x5b9cca4f7763e373ULL,
    0x682e6ff3d6b2b8a3ULL, 0x748f82ee5defb2fcULL, 0x78a5636f43172f60ULL, 0x84c87814a1f0ab72ULL, 0x8cc702081a6439ecULL,
    0x90befffa23631e28ULL, 0xa4506cebde82bde9ULL, 0xbef9a3f7b2c67915ULL, 0xc67178f2e372532bULL, 0xca273eceea26619cULL,
    0xd186b8c721c0c207ULL, 0xeada7dd6cde0eb1eULL, 0xf57d4f7fee6ed178ULL, 0x06f067aa72176fbaULL, 0x0a637dc5a2c898a6ULL,
    0x113f9804bef90daeULL, 0x1b710b35131c471bULL, 0x28db77f523047d84ULL, 0x32caab7b40c72493ULL, 0x3c9ebe0a15c9bebcULL,
    0x431d67c49c100d4cULL, 0x4cc5d4becb3e42b6ULL, 0x597f299cfc657e2aULL, 0x5fcb6fab3ad6faecULL, 0x6c44198c4a475817ULL};

inline uint64_t ror(uint64_t x, int n) { return (x >> n) | (x << (64 - n)); }
inline uint64_t ld_be64(const uint8_t* p) {
  uint64_t v;
  std::memcpy(&v, p, 8);
  return __builtin_bswap64(v);
}
inline uint64_t ld_le64(const uint8_t* p) {
  uint64_t v;
  std::memcpy(&v, p, 8);
  return v;
}

void sha512_block(uint64_t H[8], const uint8_t* blk) {
  uint64_t W[80];
  for (int i = 0; i < 16; i++) W[i] = ld_be64(blk + 8 * i);
  for (int i = 16; i < 80; i++) {
    const uint64_t s0 = ror(W[i - 15], 1) ^ ror(W[i - 15], 8) ^ (W[i - 15] >> 7);
    const uint64_t s1 = ror(W[i - 2], 19) ^ ror(W[i - 2], 61) ^ (W[i - 2] >> 6);
    W[i] = W[i - 16] + s0 + W[i - 7] + s1;
  }
  uint64_t a = H[0], b = H[1], c = H[2], d = H[3], e = H[4], f = H[5], g = H[6], h = H[7];
  for (int i = 0; i < 80; i++) {
    const uint64_t t1 = h + (ror(e, 14) ^ ror(e, 18) ^ ror(e, 41)) + ((e & f) ^ (~e & g)) + K512[i] + W[i];
    const uint64_t t2 = (ror(a, 28) ^ ror(a, 34) ^ ror(a, 39)) + ((a & b) ^ (a & c) ^ (b & c));
    h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
  }
  H[0] += a; H[1] += b; H[2] += c; H[3] += d; H[4] += e; H[5] += f; H[6] += g; H[7] += h;
}

// SHA-512 of the concatenation of up to 4 parts
void sha512(uint8_t out[64], const uint8_t* p0, size_t n0, const uint8_t* p1 = nullptr, size_t n1 = 0,
            const uint8_t* p2 = nullptr, size_t n2 = 0, const uint8_t* p3 = nullptr, size_t n3 = 0) {
  uint64_t H[8] = {0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL, 0x3c6ef372fe94f82bULL, 0xa54ff53a5f1d36f1ULL,
                   0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL, 0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL};
  uint8_t buf[128];
  size_t fill = 0, total = 0;
  const uint8_t* ps[4] = {p0, p1, p2, p3};
  const size_t ns[4] = {n0, n1, n2, n3};
  for (int k = 0; k < 4; k++) {
    const uint8_t* p = ps[k];
    size_t n = ns[k];
    total += n;
    while (n) {
      if (fill == 0 && n >= 128) { sha512_block(H, p); p += 128; n -= 128; continue; }
      const size_t t = std::min(n, 128 - fill);
      std::memcpy(buf + fill, p, t);
      fill += t; p += t; n -= t;
      if (fill == 128) { sha512_block(H, buf); fill = 0; }
    }
  }
  buf[fill++] = 0x80;
  if (fill > 112) { std::memset(buf + fill, 0, 128 - fill); sha512_block(H, buf); fill = 0; }
  std::memset(buf + fill, 0, 128 - fill);
  const uint64_t bits = (uint64_t)total * 8;
  for (int i = 0; i < 8; i++) buf[127 - i] = (uint8_t)(bits >> (8 * i));
  sha512_block(H, buf);
  for (int i = 0; i < 8; i++) {
    const uint64_t v = __builtin_bswap64(H[i]);
    std::memcpy(out + 8 * i, &v, 8);
  }
}

const uint64_t B2B_IV[8] = {0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL, 0x3c6ef372fe94f82bULL,
                            0xa54ff53a5f1d36f1ULL, 0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL,
                            0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL};
const uint8_t B2B_SIGMA[12][16] = {
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15}, {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3},
    {11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4}, {7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8},
    {9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13}, {2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9},
    {12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11}, {13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10},
    {6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5}, {10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0},
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15}, {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3}};

void b2b_compress(uint64_t h[8], const uint8_t* blk, uint64_t t, bool last) {
  uint64_t m[16], v[16];
  for (int i = 0; i < 16; i++) m[i] = ld_le64(blk + 8 * i);
  for (int i = 0; i < 8; i++) { v[i] = h[i]; v[i + 8] = B2B_IV[i]; }
  v[12] ^= t;
  if (last) v[14] = ~v[14];
#define G(a, b, c, d, x, y)                        \
  v[a] = v[a] + v[b] + (x); v[d] = ror(v[d] ^ v[a], 32); \
  v[c] = v[c] + v[d]; v[b] = ror(v[b] ^ v[c], 24);       \
  v[a] = v[a] + v[b] + (y); v[d] = ror(v[d] ^ v[a], 16); \
  v[c] = v[c] + v[d]; v[b] = ror(v[b] ^ v[c], 63);
  for (int r = 0; r < 12; r++) {
    const uint8_t* s = B2B_SIGMA[r];
    G(0, 4, 8, 12, m[s[0]], m[s[1]]) G(1, 5, 9, 13, m[s[2]], m[s[3]])
    G(2, 6, 10, 14, m[s[4]], m[s[5]]) G(3, 7, 11, 15, m[s[6]], m[s[7]])
    G(0, 5, 10, 15, m[s[8]], m[s[9]]) G(1, 6, 11, 12, m[s[10]], m[s[11]])
    G(2, 7, 8, 13, m[s[12]], m[s[13]]) G(3, 4, 9, 14, m[s[14]], m[s[15]])
  }
#undef G
  for (int i = 0; i < 8; i++) h[i] ^= v[i] ^ v[i + 8];
}

// BLAKE2b (unkeyed) of the concatenation of two parts, outlen <= 64
void blake2b(uint8_t* out, size_t outlen, const uint8_t* p0, size_t n0, const uint8_t* p1 = nullptr, size_t n1 = 0) {
  uint64_t h[8];
  for (int i = 0; i < 8; i++) h[i] = B2B_IV[i];
  h[0] ^= 0x01010000ULL ^ (uint64_t)outlen;
  uint8_t buf[128];
  size_t fill = 0;
  uint64_t t = 0;
  const size_t total = n0 + n1;
  const uint8_t* ps[2] = {p0, p1};
  const size_t ns[2] = {n0, n1};
  for (int k = 0; k < 2; k++) {
    const uint8_t* p = ps[k];
    size_t n = ns[k];
    while (n) {
      if (fill == 128) { t += 128; b2b_compress(h, buf, t, false); fill = 0; }
      const size_t c = std::min(n, 128 - fill);
      std::memcpy(buf + fill, p, c);
      fill += c; p += c; n -= c;
    }
  }
  std::memset(buf + fill, 0, 128 - fill);
  b2b_compress(h, buf, total, true);
  uint8_t full[64];
  for (int i = 0; i < 8; i++) std::memcpy(full + 8 * i, &h[i], 8);
  std::memcpy(out, full, outlen);
}

// ============================================================ GF(2^255 - 19), radix 2^51
struct fe { uint64_t v[5]; };
constexpr uint64_t M51 = (1ULL << 51) - 1;

inline void fe_0(fe& h) { std::memset(&h, 0, sizeof h); }
inline void fe_1(fe& h) { fe_0(h); h.v[0] = 1; }
inline void fe_carry(fe& h) {
  uint64_t c;
  c = h.v[0] >> 51; h.v[0] &= M51; h.v[1] += c;
  c = h.v[1] >> 51; h.v[1] &= M51; h.v[2] += c;
  c = h.v[2] >> 51; h.v[2] &= M51; h.v[3] += c;
  c = h.v[3] >> 51; h.v[3] &= M51; h.v[4] += c;
  c = h.v[4] >> 51; h.v[4] &= M51; h.v[0] += 19 * c;
}
// inputs with limbs < 2^53 give limbs < 2^52 after the carry
inline void fe_add(fe& h, const fe& f, const fe& g) {
  for (int i = 0; i < 5; i++) h.v[i] = f.v[i] + g.v[i];
  fe_carry(h);
}
inline void fe_sub(fe& h, const fe& f, const fe& g) {   // + 4p keeps every limb positive
  h.v[0] = f.v[0] + 0x1fffffffffffb4ULL - g.v[0];
  for (int i = 1; i < 5; i++) h.v[i] = f.v[i] + 0x1ffffffffffffcULL - g.v[i];
  fe_carry(h);
}
inline void fe_neg(fe& h, const fe& f) { fe z; fe_0(z); fe_sub(h, z, f); }
inline void fe_mul(fe& h, const fe& f, const fe& g) {
  const uint64_t *a = f.v, *b = g.v;
  const uint64_t b1 = b[1] * 19, b2 = b[2] * 19, b3 = b[3] * 19, b4 = b[4] * 19;
  u128 t0 = (u128)a[0] * b[0] + (u128)a[1] * b4 + (u128)a[2] * b3 + (u128)a[3] * b2 + (u128)a[4] * b1;
  u128 t1 = (u128)a[0] * b[1] + (u128)a[1] * b[0] + (u128)a[2] * b4 + (u128)a[3] * b3 + (u128)a[4] * b2;
  u128 t2 = (u128)a[0] * b[2] + (u128)a[1] * b[1] + (u128)a[2] * b[0] + (u128)a[3] * b4 + (u128)a[4] * b3;
  u128 t3 = (u128)a[0] * b[3] + (u128)a[1] * b[2] + (u128)a[2] * b[1] + (u128)a[3] * b[0] + (u128)a[4] * b4;
  u128 t4 = (u128)a[0] * b[4] + (u128)a[1] * b[3] + (u128)a[2] * b[2] + (u128)a[3] * b[1] + (u128)a[4] * b[0];
  t1 += (uint64_t)(t0 >> 51); uint64_t r0 = (uint64_t)t0 & M51;
  t2 += (uint64_t)(t1 >> 51); uint64_t r1 = (uint64_t)t1 & M51;
  t3 += (uint64_t)(t2 >> 51); uint64_t r2 = (uint64_t)t2 & M51;
  t4 += (uint64_t)(t3 >> 51); uint64_t r3 = (uint64_t)t3 & M51;
  const uint64_t c = (uint64_t)(t4 >> 51); uint64_t r4 = (uint64_t)t4 & M51;
  r0 += c * 19;
  r1 += r0 >> 51; r0 &= M51;
  h.v[0] = r0; h.v[1] = r1; h.v[2] = r2; h.v[3] = r3; h.v[4] = r4;
}
inline void fe_sq(fe& h, const fe& f) {
  const uint64_t* a = f.v;
  const uint64_t d0 = a[0] * 2, d1 = a[1] * 2, d2 = a[2] * 2 * 19, d4 = a[4] * 19, d419 = d4 * 2;
  const uint64_t a3_19 = a[3] * 19;
  u128 t0 = (u128)a[0] * a[0] + (u128)d419 * a[1] + (u128)d2 * a[3];
  u128 t1 = (u128)d0 * a[1] + (u128)d419 * a[2] + (u128)a3_19 * a[3];
  u128 t2 = (u128)d0 * a[2] + (u128)a[1] * a[1] + (u128)d419 * a[3];
  u128 t3 = (u128)d0 * a[3] + (u128)d1 * a[2] + (u128)d4 * a[4];
  u128 t4 = (u128)d0 * a[4] + (u128)d1 * a[3] + (u128)a[2] * a[2];
  t1 += (uint64_t)(t0 >> 51); uint64_t r0 = (uint64_t)t0 & M51;
  t2 += (uint64_t)(t1 >> 51); uint64_t r1 = (uint64_t)t1 & M51;
  t3 += (uint64_t)(t2 >> 51); uint64_t r2 = (uint64_t)t2 & M51;
  t4 += (uint64_t)(t3 >> 51); uint64_t r3 = (uint64_t)t3 & M51;
  const uint64_t c = (uint64_t)(t4 >> 51); uint64_t r4 = (uint64_t)t4 & M51;
  r0 += c * 19;
  r1 += r0 >> 51; r0 &= M51;
  h.v[0] = r0; h.v[1] = r1; h.v[2] = r2; h.v[3] = r3; h.v[4] = r4;
}
inline void fe_sqn(fe& h, const fe& f, int n) { fe_sq(h, f); for (int i = 1; i < n; i++) fe_sq(h, h); }
inline void fe_mul_small(fe& h, const fe& f, uint64_t k) {
  u128 c = 0;
  for (int i = 0; i < 5; i++) { c += (u128)f.v[i] * k; h.v[i] = (uint64_t)c & M51; c >>= 51; }
  h.v[0] += (uint64_t)c * 19;
  fe_carry(h);
}

void fe_tobytes(uint8_t s[32], const fe& f) {
  fe h = f;
  fe_carry(h);
  fe_carry(h);
  uint64_t q = (h.v[0] + 19) >> 51;
  q = (h.v[1] + q) >> 51; q = (h.v[2] + q) >> 51; q = (h.v[3] + q) >> 51; q = (h.v[4] + q) >> 51;
  h.v[0] += 19 * q;
  uint64_t c;
  c = h.v[0] >> 51; h.v[0] &= M51; h.v[1] += c;
  c = h.v[1] >> 51; h.v[1] &= M51; h.v[2] += c;
  c = h.v[2] >> 51; h.v[2] &= M51; h.v[3] += c;
  c = h.v[3] >> 51; h.v[3] &= M51; h.v[4] += c;
  h.v[4] &= M51;
  const uint64_t w0 = h.v[0] | (h.v[1] << 51), w1 = (h.v[1] >> 13) | (h.v[2] << 38),
                 w2 = (h.v[2] >> 26) | (h.v[3] << 25), w3 = (h.v[3] >> 39) | (h.v[4] << 12);
  std::memcpy(s, &w0, 8); std::memcpy(s + 8, &w1, 8); std::memcpy(s + 16, &w2, 8); std::memcpy(s + 24, &w3, 8);
}
// low 255 bits; values >= p are fine (arithmetic is mod p)
void fe_frombytes(fe& h, const uint8_t s[32]) {
  const uint64_t w0 = ld_le64(s), w1 = ld_le64(s + 8), w2 = ld_le64(s + 16), w3 = ld_le64(s + 24);
  h.v[0] = w0 & M51;
  h.v[1] = ((w0 >> 51) | (w1 << 13)) & M51;
  h.v[2] = ((w1 >> 38) | (w2 << 26)) & M51;
  h.v[3] = ((w2 >> 25) | (w3 << 39)) & M51;
  h.v[4] = (w3 >> 12) & M51;
}
bool fe_iszero(const fe& f) { uint8_t s[32]; fe_tobytes(s, f); uint8_t d = 0; for (int i = 0; i < 32; i++) d |= s[i]; return d == 0; }
bool fe_isnegative(const fe& f) { uint8_t s[32]; fe_tobytes(s, f); return s[0] & 1; }

void fe_pow2_250_1(fe& t0, fe& z11, const fe& z) {
  fe t1, t2, t3;
  fe_sq(t0, z);
  fe_sqn(t1, t0, 2);
  fe_mul(t1, z, t1);
  fe_mul(z11, t0, t1);
  fe_sq(t0, z11);
  fe_mul(t0, t1, t0);
  fe_sqn(t1, t0, 5); fe_mul(t0, t1, t0);
  fe_sqn(t1, t0, 10); fe_mul(t1, t1, t0);
  fe_sqn(t2, t1, 20); fe_mul(t1, t2, t1);
  fe_sqn(t1, t1, 10); fe_mul(t0, t1, t0);
  fe_sqn(t1, t0, 50); fe_mul(t1, t1, t0);
  fe_sqn(t3, t1, 100); fe_mul(t1, t3, t1);
  fe_sqn(t1, t1, 50); fe_mul(t0, t1, t0);
}
void fe_invert(fe& r, const fe& z) { fe t0, z11; fe_pow2_250_1(t0, z11, z); fe_sqn(t0, t0, 5); fe_mul(r, t0, z11); }
void fe_pow22523(fe& r, const fe& z) { fe t0, z11; fe_pow2_250_1(t0, z11, z); fe_sqn(t0, t0, 2); fe_mul(r, t0, z); }
void fe_chi(fe& r, const fe& z) {                // z^((p-1)/2)
  fe t0, z11, t1;
  fe_pow2_250_1(t0, z11, z);
  fe_sqn(t0, t0, 4);
  fe_sq(t1, z); fe_mul(t1, t1, z); fe_sq(t1, t1);
  fe_mul(r, t0, t1);
}

fe FE_D, FE_D2, FE_SQRTM1, FE_A;

// ============================================================ edwards25519
struct ge_p2 { fe X, Y, Z; };
struct ge_p3 { fe X, Y, Z, T; };
struct ge_p1p1 { fe X, Y, Z, T; };
struct ge_cached { fe YpX, YmX, Z, T2d; };
struct ge_niels { fe ypx, ymx, xy2d; };

inline void p1p1_to_p2(ge_p2& r, const ge_p1p1& p) { fe_mul(r.X, p.X, p.T); fe_mul(r.Y, p.Y, p.Z); fe_mul(r.Z, p.Z, p.T); }
inline void p1p1_to_p3(ge_p3& r, const ge_p1p1& p) {
  fe_mul(r.X, p.X, p.T); fe_mul(r.Y, p.Y, p.Z); fe_mul(r.Z, p.Z, p.T); fe_mul(r.T, p.X, p.Y);
}
inline void p3_to_cached(ge_cached& c, const ge_p3& p) {
  fe_add(c.YpX, p.Y, p.X); fe_sub(c.YmX, p.Y, p.X); c.Z = p.Z; fe_mul(c.T2d, p.T, FE_D2);
}
inline void p2_dbl(ge_p1p1& r, const ge_p2& p) {
  fe t0;
  fe_sq(r.X, p.X); fe_sq(r.Z, p.Y); fe_sq(r.T, p.Z); fe_add(r.T, r.T, r.T);
  fe_add(r.Y, p.X, p.Y); fe_sq(t0, r.Y);
  fe_add(r.Y, r.Z, r.X); fe_sub(r.Z, r.Z, r.X); fe_sub(r.X, t0, r.Y); fe_sub(r.T, r.T, r.Z);
}
inline void p3_dbl(ge_p1p1& r, const ge_p3& p) { ge_p2 q{p.X, p.Y, p.Z}; p2_dbl(r, q); }
inline void ge_add(ge_p1p1& r, const ge_p3& p, const ge_cached& q) {
  fe t0;
  fe_add(r.X, p.Y, p.X); fe_sub(r.Y, p.Y, p.X);
  fe_mul(r.Z, r.X, q.YpX); fe_mul(r.Y, r.Y, q.YmX); fe_mul(r.T, q.T2d, p.T); fe_mul(r.X, p.Z, q.Z);
  fe_add(t0, r.X, r.X);
  fe_sub(r.X, r.Z, r.Y); fe_add(r.Y, r.Z, r.Y); fe_add(r.Z, t0, r.T); fe_sub(r.T, t0, r.T);
}
inline void ge_sub(ge_p1p1& r, const ge_p3& p, const ge_cached& q) {
  fe t0;
  fe_add(r.X, p.Y, p.X); fe_sub(r.Y, p.Y, p.X);
  fe_mul(r.Z, r.X, q.YmX); fe_mul(r.Y, r.Y, q.YpX); fe_mul(r.T, q.T2d, p.T); fe_mul(r.X, p.Z, q.Z);
  fe_add(t0, r.X, r.X);
  fe_sub(r.X, r.Z, r.Y); fe_add(r.Y, r.Z, r.Y); fe_sub(r.Z, t0, r.T); fe_add(r.T, t0, r.T);
}
inline void ge_madd(ge_p1p1& r, const ge_p3& p, const ge_niels& q) {
  fe t0;
  fe_add(r.X, p.Y, p.X); fe_sub(r.Y, p.Y, p.X);
  fe_mul(r.Z, r.X, q.ypx); fe_mul(r.Y, r.Y, q.ymx); fe_mul(r.T, q.xy2d, p.T);
  fe_add(t0, p.Z, p.Z);
  fe_sub(r.X, r.Z, r.Y); fe_add(r.Y, r.Z, r.Y); fe_add(r.Z, t0, r.T); fe_sub(r.T, t0, r.T);
}
inline void ge_msub(ge_p1p1& r, const ge_p3& p, const ge_niels& q) {
  fe t0;
  fe_add(r.X, p.Y, p.X); fe_sub(r.Y, p.Y, p.X);
  fe_mul(r.Z, r.X, q.ymx); fe_mul(r.Y, r.Y, q.ypx); fe_mul(r.T, q.xy2d, p.T);
  fe_add(t0, p.Z, p.Z);
  fe_sub(r.X, r.Z, r.Y); fe_add(r.Y, r.Z, r.Y); fe_sub(r.Z, t0, r.T); fe_add(r.T, t0, r.T);
}
inline void p3_dbl_to_p3(ge_p3& r, const ge_p3& p) { ge_p1p1 t; p3_dbl(t, p); p1p1_to_p3(r, t); }

void ge_tobytes(uint8_t s[32], const fe& X, const fe& Y, const fe& Z) {
  fe zi, x, y;
  fe_invert(zi, Z);
  fe_mul(x, X, zi);
  fe_mul(y, Y, zi);
  fe_tobytes(s, y);
  s[31] ^= (uint8_t)(fe_isnegative(x) << 7);
}

// libsodium ge25519_frombytes' square root: x = u v^3 (u v^7)^((p-5)/8), times
// sqrt(-1) when v x^2 != u; false when neither v x^2 == u nor == -u
bool fe_sqrt_ratio(fe& x, const fe& u, const fe& v) {
  fe v3, vxx, chk;
  fe_sq(v3, v); fe_mul(v3, v3, v);
  fe_sq(x, v3); fe_mul(x, x, v); fe_mul(x, x, u);
  fe_pow22523(x, x);
  fe_mul(x, x, v3); fe_mul(x, x, u);
  fe_sq(vxx, x); fe_mul(vxx, vxx, v);
  fe_sub(chk, vxx, u);
  if (fe_iszero(chk)) return true;
  fe_add(chk, vxx, u);
  if (!fe_iszero(chk)) return false;
  fe_mul(x, x, FE_SQRTM1);
  return true;
}

// libsodium 1.0.18 ge25519_frombytes (y from the low 255 bits mod p; the sign bit
// picks x; x = 0 with the sign bit set decodes to x = 0)
bool ge_frombytes(ge_p3& h, const uint8_t s[32]) {
  fe u, v, one;
  fe_1(one);
  fe_frombytes(h.Y, s);
  fe_1(h.Z);
  fe_sq(u, h.Y);
  fe_mul(v, u, FE_D);
  fe_sub(u, u, one);
  fe_add(v, v, one);
  if (!fe_sqrt_ratio(h.X, u, v)) return false;
  if (fe_isnegative(h.X) != ((s[31] >> 7) != 0)) fe_neg(h.X, h.X);
  fe_mul(h.T, h.X, h.Y);
  return true;
}

bool has_small_order(const uint8_t s[32]) {     // libsodium blacklist, sign bit ignored
  static const uint8_t y8a[32] = {0x26, 0xe8, 0x95, 0x8f, 0xc2, 0xb2, 0x27, 0xb0, 0x45, 0xc3, 0xf4,
                                  0x89, 0xf2, 0xef, 0x98, 0xf0, 0xd5, 0xdf, 0xac, 0x05, 0xd3, 0xc6,
                                  0x33, 0x39, 0xb1, 0x38, 0x02, 0x88, 0x6d, 0x53, 0xfc, 0x05};
  static const uint8_t y8b[32] = {0xc7, 0x17, 0x6a, 0x70, 0x3d, 0x4d, 0xd8, 0x4f, 0xba, 0x3c, 0x0b,
                                  0x76, 0x0d, 0x10, 0x67, 0x0f, 0x2a, 0x20, 0x53, 0xfa, 0x2c, 0x39,
                                  0xcc, 0xc6, 0x4e, 0xc7, 0xfd, 0x77, 0x92, 0xac, 0x03, 0x7a};
  uint8_t t[32];
  std::memcpy(t, s, 32);
  t[31] &= 0x7f;
  if (!std::memcmp(t, y8a, 32) || !std::memcmp(t, y8b, 32)) return true;
  bool mid0 = true, mid1 = true;
  for (int i = 1; i < 31; i++) { mid0 &= t[i] == 0; mid1 &= t[i] == 0xff; }
  if (mid0 && t[31] == 0 && (t[0] == 0 || t[0] == 1)) return true;
  if (mid1 && t[31] == 0x7f && (t[0] == 0xec || t[0] == 0xed || t[0] == 0xee)) return true;
  return false;
}
bool ge_is_canonical(const uint8_t s[32]) {
  if ((s[31] & 0x7f) != 0x7f) return true;
  for (int i = 30; i > 0; i--) if (s[i] != 0xff) return true;
  return s[0] < 0xed;
}

// ============================================================ scalars mod L
// little-endian 64-bit limbs; Barrett with mu = floor(2^512 / L)
const uint64_t LW[4] = {0x5812631a5cf5d3edULL, 0x14def9dea2f79cd6ULL, 0, 0x1000000000000000ULL};
uint64_t MU[5];

void mp_mul(uint64_t* r, const uint64_t* a, int na, const uint64_t* b, int nb) {
  std::memset(r, 0, 8 * (na + nb));
  for (int i = 0; i < na; i++) {
    u128 c = 0;
    for (int j = 0; j < nb; j++) { c += (u128)a[i] * b[j] + r[i + j]; r[i + j] = (uint64_t)c; c >>= 64; }
    r[i + nb] = (uint64_t)c;
  }
}
int mp_cmp(const uint64_t* a, const uint64_t* b, int n) {
  for (int i = n - 1; i >= 0; i--) if (a[i] != b[i]) return a[i] < b[i] ? -1 : 1;
  return 0;
}
uint64_t mp_sub(uint64_t* r, const uint64_t* a, const uint64_t* b, int n) {   // returns borrow
  uint64_t br = 0;
  for (int i = 0; i < n; i++) {
    const u128 d = (u128)a[i] - b[i] - br;
    r[i] = (uint64_t)d;
    br = (uint64_t)(d >> 64) & 1;
  }
  return br;
}
uint64_t mp_add(uint64_t* r, const uint64_t* a, const uint64_t* b, int n) {   // returns carry
  u128 c = 0;
  for (int i = 0; i < n; i++) { c += (u128)a[i] + b[i]; r[i] = (uint64_t)c; c >>= 64; }
  return (uint64_t)c;
}

// r = x mod L for a 64-byte little-endian x
void sc_reduce64(uint8_t r[32], const uint8_t x[64]) {
  uint64_t X[8], q[13], qL[9], rr[9];
  for (int i = 0; i < 8; i++) X[i] = ld_le64(x + 8 * i);
  mp_mul(q, X, 8, MU, 5);                 // x * mu, the quotient estimate is q >> 512
  const uint64_t* qh = q + 8;             // 5 limbs
  mp_mul(qL, qh, 5, LW, 4);               // 9 limbs
  uint64_t Xe[9];
  std::memcpy(Xe, X, 64);
  Xe[8] = 0;
  mp_sub(rr, Xe, qL, 9);                  // r = x - q L, 0 <= r < 3L
  uint64_t L9[9] = {LW[0], LW[1], LW[2], LW[3], 0, 0, 0, 0, 0};
  while (mp_cmp(rr, L9, 9) >= 0) mp_sub(rr, rr, L9, 9);
  for (int i = 0; i < 4; i++) std::memcpy(r + 8 * i, &rr[i], 8);
}
void sc_reduce32(uint8_t r[32], const uint8_t x[32]) {
  uint8_t w[64] = {0};
  std::memcpy(w, x, 32);
  sc_reduce64(r, w);
}
bool sc_is_canonical(const uint8_t s[32]) {
  uint64_t S[4];
  for (int i = 0; i < 4; i++) S[i] = ld_le64(s + 8 * i);
  return mp_cmp(S, LW, 4) < 0;
}

// ============================================================ scalar multiplication
// signed sliding-window recoding (odd digits |d| < 2^(w-1)), libsodium `slide` generalised
void slide(int8_t r[256], const uint8_t a[32], int w) {
  for (int i = 0; i < 256; i++) r[i] = 1 & (a[i >> 3] >> (i & 7));
  const int maxd = (1 << (w - 1)) - 1;
  for (int i = 0; i < 256; i++) {
    if (!r[i]) continue;
    for (int b = 1; b <= w + 1 && i + b < 256; b++) {
      if (!r[i + b]) continue;
      if (r[i] + (r[i + b] << b) <= maxd) {
        r[i] += r[i + b] << b;
        r[i + b] = 0;
      } else if (r[i] - (r[i + b] << b) >= -maxd) {
        r[i] -= r[i + b] << b;
        for (int k = i + b; k < 256; k++) {
          if (!r[k]) { r[k] = 1; break; }
          r[k] = 0;
        }
      } else {
        break;
      }
    }
  }
}

constexpr int WB = 8;                       // fixed-base window (odd multiples up to 127 B)
ge_niels BTAB[1 << (WB - 2)];               // {1, 3, 5, ..., 127} B, affine niels
ge_p3 GE_B;

void odd_multiples(ge_cached* t, int cnt, const ge_p3& P) {   // t[k] = (2k+1) P
  ge_p1p1 x;
  ge_p3 P2, acc = P;
  p3_dbl(x, P);
  p1p1_to_p3(P2, x);
  ge_cached c2;
  p3_to_cached(c2, P2);
  p3_to_cached(t[0], P);
  for (int k = 1; k < cnt; k++) {
    ge_add(x, acc, c2);
    p1p1_to_p3(acc, x);
    p3_to_cached(t[k], acc);
  }
}

// out = sum of [a_i] P_i with sliding windows; P_i given as odd-multiple tables
// (cached, width 5) plus optionally [b] B over the static table (width 8)
struct Term { const int8_t* d; const ge_cached* tab; };
void straus(ge_p3& out, const Term* terms, int nt, const int8_t* bd) {
  int top = 255;
  auto any = [&](int i) {
    for (int k = 0; k < nt; k++) if (terms[k].d[i]) return true;
    return bd && bd[i];
  };
  while (top >= 0 && !any(top)) top--;
  ge_p2 r;
  fe_0(r.X); fe_1(r.Y); fe_1(r.Z);
  ge_p1p1 t;
  ge_p3 u;
  for (int i = top; i >= 0; i--) {
    p2_dbl(t, r);
    bool conv = false;
    for (int k = 0; k < nt; k++) {
      const int d = terms[k].d[i];
      if (!d) continue;
      p1p1_to_p3(u, t);
      if (d > 0) ge_add(t, u, terms[k].tab[d / 2]);
      else ge_sub(t, u, terms[k].tab[(-d) / 2]);
      conv = true;
    }
    if (bd && bd[i]) {
      p1p1_to_p3(u, t);
      if (bd[i] > 0) ge_madd(t, u, BTAB[bd[i] / 2]);
      else ge_msub(t, u, BTAB[(-bd[i]) / 2]);
      conv = true;
    }
    (void)conv;
    p1p1_to_p2(r, t);
  }
  if (top < 0) { fe_0(out.X); fe_1(out.Y); fe_1(out.Z); fe_0(out.T); return; }
  p1p1_to_p3(out, t);
}

struct Init {
  Init() {
    fe n1, n2, inv;
    fe_0(n1); n1.v[0] = 121665;
    fe_0(n2); n2.v[0] = 121666;
    fe_invert(inv, n2);
    fe_mul(FE_D, n1, inv);
    fe_neg(FE_D, FE_D);
    fe_add(FE_D2, FE_D, FE_D);
    // sqrt(-1) = 2^((p-1)/4): (p-1)/4 = 2^253 - 5
    fe two, t0, z11, t1;
    fe_0(two); two.v[0] = 2;
    fe_pow2_250_1(t0, z11, two);            // 2^250 - 1
    fe_sqn(t0, t0, 3);                      // 2^253 - 8
    fe_sq(t1, two); fe_mul(t1, t1, two);    // 2^3 = exponent 3
    fe_mul(FE_SQRTM1, t0, t1);              // 2^253 - 5
    fe_0(FE_A); FE_A.v[0] = 486662;
    // B: y = 4/5, x even
    fe four, five, y;
    fe_0(four); four.v[0] = 4;
    fe_0(five); five.v[0] = 5;
    fe_invert(inv, five);
    fe_mul(y, four, inv);
    uint8_t enc[32];
    fe_tobytes(enc, y);
    ge_frombytes(GE_B, enc);
    ge_cached tc[1 << (WB - 2)];
    odd_multiples(tc, 1 << (WB - 2), GE_B);
    for (int k = 0; k < (1 << (WB - 2)); k++) {     // to affine niels
      fe zi, x, yy;
      fe_sub(yy, tc[k].YpX, tc[k].YmX);             // 2X
      fe_add(x, tc[k].YpX, tc[k].YmX);              // 2Y
      fe_invert(zi, tc[k].Z);
      fe_mul(yy, yy, zi); fe_mul(x, x, zi);         // 2x, 2y
      fe half;
      fe_0(half); half.v[0] = 2;
      fe_invert(half, half);
      fe_mul(yy, yy, half); fe_mul(x, x, half);     // x, y
      fe_add(BTAB[k].ypx, x, yy);
      fe_sub(BTAB[k].ymx, x, yy);
      fe xy;
      fe_mul(xy, x, yy);
      fe_mul(BTAB[k].xy2d, xy, FE_D2);
    }
    // mu = floor(2^512 / L), bit-serial once
    uint64_t rem[5] = {0, 0, 0, 0, 0}, q[5] = {0, 0, 0, 0, 0};
    const uint64_t L5[5] = {LW[0], LW[1], LW[2], LW[3], 0};
    for (int bit = 512; bit >= 0; bit--) {
      uint64_t c = bit == 512 ? 1 : 0;
      for (int i = 0; i < 5; i++) { const uint64_t nc = rem[i] >> 63; rem[i] = (rem[i] << 1) | c; c = nc; }
      if (mp_cmp(rem, L5, 5) >= 0) {
        mp_sub(rem, rem, L5, 5);
        if (bit < 320) q[bit / 64] |= 1ULL << (bit % 64);
      }
    }
    std::memcpy(MU, q, sizeof MU);
  }
} g_init;

// ============================================================ Ed25519 (libsodium 1.0.18 verify_detached)
bool ed25519_verify(const uint8_t sig[64], const uint8_t* m, size_t n, const uint8_t pk[32]) {
  if (!sc_is_canonical(sig + 32) || has_small_order(sig)) return false;
  if (!ge_is_canonical(pk) || has_small_order(pk)) return false;
  ge_p3 A;
  if (!ge_frombytes(A, pk)) return false;
  uint8_t hh[64], h[32];
  sha512(hh, sig, 32, pk, 32, m, n);
  sc_reduce64(h, hh);
  // R' = [S]B - [h]A
  ge_cached ta[8];
  odd_multiples(ta, 8, A);
  int8_t hd[256], sd[256];
  slide(hd, h, 5);
  for (int i = 0; i < 256; i++) hd[i] = (int8_t)-hd[i];
  slide(sd, sig + 32, WB);
  Term t{hd, ta};
  ge_p3 R;
  straus(R, &t, 1, sd);
  uint8_t enc[32];
  ge_tobytes(enc, R.X, R.Y, R.Z);
  return std::memcmp(enc, sig, 32) == 0;
}

// ============================================================ Sum6KES
// 0 ok, 1 Merkle "Reject", 2 leaf Ed25519 failure; t is a Word (Praos.hs:582)
int kes_verify(const uint8_t vk[32], uint64_t t, const uint8_t* m, size_t n, const uint8_t* sig) {
  uint8_t cur[32], h[32];
  std::memcpy(cur, vk, 32);
  for (int d = 6; d >= 1; d--) {
    const uint8_t* pair = sig + 64 + 64 * (d - 1);
    blake2b(h, 32, pair, 64);
    if (std::memcmp(h, cur, 32) != 0) return 1;
    const uint64_t T = 1ULL << (d - 1);
    if (t < T) std::memcpy(cur, pair, 32);
    else { std::memcpy(cur, pair + 32, 32); t -= T; }
  }
  return ed25519_verify(sig, m, n, cur) ? 0 : 2;
}

// ============================================================ ECVRF-ED25519-SHA512-Elligator2, draft-03
// libsodium ge25519_from_uniform (sign bit already cleared), then x 8: H projective
void vrf_from_uniform(ge_p3& H, const uint8_t r[32]) {
  fe one, w, t, q, e, A2, Aw;
  fe_1(one);
  fe_frombytes(w, r);
  fe_sq(w, w); fe_add(w, w, w); fe_add(w, w, one);          // w = 1 + 2 r^2
  fe_sq(A2, FE_A);
  fe_mul(Aw, FE_A, w);
  fe_mul(t, A2, w); fe_sub(q, A2, t); fe_sq(t, w); fe_add(q, q, t);   // Q = A^2 - A^2 w + w^2
  fe_mul(q, q, Aw); fe_neg(e, q);                           // e ~ -A w Q (same character as x^3 + A x^2 + x)
  fe_chi(e, e);
  uint8_t eb[32];
  fe_tobytes(eb, e);
  const bool e_is_minus_1 = eb[1] & 1;
  fe N, D;
  if (!e_is_minus_1) { fe_add(N, FE_A, w); fe_neg(N, N); fe_sub(D, w, FE_A); }
  else { fe_sub(t, FE_A, Aw); fe_sub(N, t, w); fe_add(D, t, w); }
  if (fe_iszero(D)) { fe_0(N); fe_1(D); }
  fe nn, dd, u, v, x;
  fe_sq(nn, N); fe_sq(dd, D);
  fe_sub(u, nn, dd);
  fe_mul(v, nn, FE_D); fe_add(v, v, dd);
  fe_sqrt_ratio(x, u, v);
  if (fe_isnegative(x)) fe_neg(x, x);
  ge_p3 P;
  fe_mul(P.X, x, D); P.Y = N; P.Z = D; fe_mul(P.T, x, N);
  ge_p3 Q;
  p3_dbl_to_p3(Q, P); p3_dbl_to_p3(P, Q); p3_dbl_to_p3(H, P);
}

void enc_affine(uint8_t s[32], const ge_p3& P) {     // Z == 1
  fe_tobytes(s, P.Y);
  s[31] |= (uint8_t)(fe_isnegative(P.X) << 7);
}

// Returns proof validity; beta = proof_to_hash (zeros when Gamma does not decode)
bool vrf_verify(uint8_t beta[64], const uint8_t pk[32], const uint8_t proof[80], const uint8_t alpha[32]) {
  std::memset(beta, 0, 64);
  ge_p3 G;
  const bool gamma_ok = ge_frombytes(G, proof);
  if (gamma_ok) {
    ge_p3 G2, G4, G8;
    p3_dbl_to_p3(G2, G); p3_dbl_to_p3(G4, G2); p3_dbl_to_p3(G8, G4);
    uint8_t str[34];
    str[0] = 0x04; str[1] = 0x03;
    ge_tobytes(str + 2, G8.X, G8.Y, G8.Z);
    sha512(beta, str, 34);
  }
  ge_p3 Y;
  if (has_small_order(pk) || !ge_frombytes(Y, pk) || !gamma_ok) return false;
  uint8_t ys[32], r[64], c[32] = {0}, s[32];
  enc_affine(ys, Y);
  const uint8_t pre[2] = {0x04, 0x01};
  sha512(r, pre, 2, ys, 32, alpha, 32);
  r[31] &= 0x7f;
  ge_p3 H;
  vrf_from_uniform(H, r);
  std::memcpy(c, proof + 32, 16);
  sc_reduce32(s, proof + 48);
  // U = [s]B - [c]Y ;  V = [s]H - [c]Gamma
  ge_cached ty[8], th[8], tg[8];
  odd_multiples(ty, 8, Y);
  odd_multiples(th, 8, H);
  odd_multiples(tg, 8, G);
  int8_t cd[256], sd5[256], sd8[256];
  slide(cd, c, 5);
  for (int i = 0; i < 256; i++) cd[i] = (int8_t)-cd[i];
  slide(sd5, s, 5);
  slide(sd8, s, WB);
  ge_p3 U, V;
  Term tu{cd, ty};
  straus(U, &tu, 1, sd8);
  Term tv[2] = {{sd5, th}, {cd, tg}};
  straus(V, tv, 2, nullptr);
  uint8_t str[2 + 4 * 32], hs[32], cp[64];
  str[0] = 0x04; str[1] = 0x02;
  ge_tobytes(hs, H.X, H.Y, H.Z);
  std::memcpy(str + 2, hs, 32);
  enc_affine(str + 34, G);                 // canonical re-encoding of the decoded Gamma
  ge_tobytes(str + 66, U.X, U.Y, U.Z);
  ge_tobytes(str + 98, V.X, V.Y, V.Z);
  sha512(cp, str, sizeof str);
  return std::memcmp(cp, c, 16) == 0;
}

// ============================================================ leader check (Fixed E34)
// Natural numbers as little-endian u64 limbs, fixed capacity.
constexpr int NL = 16;
struct nat { uint64_t w[NL]; };
inline void nat_zero(nat& a) { std::memset(&a, 0, sizeof a); }
void nat_mul(nat& r, const nat& a, const nat& b) {
  uint64_t t[2 * NL];
  mp_mul(t, a.w, NL, b.w, NL);
  std::memcpy(r.w, t, sizeof r.w);        // callers keep products < 2^(64 NL)
}
uint64_t nat_divsmall(nat& q, const nat& a, uint64_t d) {
  u128 rem = 0;
  for (int i = NL - 1; i >= 0; i--) {
    rem = (rem << 64) | a.w[i];
    q.w[i] = (uint64_t)(rem / d);
    rem %= d;
  }
  return (uint64_t)rem;
}
const uint64_t TEN17 = 100000000000000000ULL;
void nat_div_R(nat& q, const nat& a) { nat t; nat_divsmall(t, a, TEN17); nat_divsmall(q, t, TEN17); }
nat nat_R() { nat r; nat_zero(r); r.w[0] = TEN17; nat t; nat_zero(t); t.w[0] = TEN17; nat_mul(r, r, t); return r; }

// checkLeaderNatValue (Praos.hs:549): bound 2^(8 nbytes); x = Fixed raw (>= 0)
bool leader_check(const uint8_t* l_be, int nbytes, const uint8_t x_le[16]) {
  const nat R = nat_R();
  nat l, D, N, x;
  nat_zero(l); nat_zero(D); nat_zero(N); nat_zero(x);
  for (int i = 0; i < nbytes; i++) l.w[(nbytes - 1 - i) / 8] |= (uint64_t)l_be[i] << (8 * ((nbytes - 1 - i) % 8));
  nat maxv;
  nat_zero(maxv);
  maxv.w[nbytes / 8] = 1;
  mp_sub(D.w, maxv.w, l.w, NL);                       // D = certNatMax - l
  for (int i = 0; i < 2; i++) N.w[nbytes / 8 + i] = R.w[i];   // N = certNatMax * R
  std::memcpy(x.w, x_le, 16);
  nat err = x, acc = R;
  for (int n = 0; n < 1000; n++) {
    nat t, errp, accp, e, hi, lo, hd;
    nat_mul(t, err, x);
    nat_div_R(t, t);
    nat_divsmall(errp, t, (uint64_t)n + 2);
    mp_add(accp.w, acc.w, err.w, NL);
    nat_zero(e);
    e.w[0] = 3;
    nat_mul(e, errp, e);
    mp_add(hi.w, accp.w, e.w, NL);
    nat_mul(hd, hi, D);
    if (mp_cmp(N.w, hd.w, NL) >= 0) return false;    // recip_q >= acc' + e: ABOVE
    if (mp_cmp(accp.w, e.w, NL) > 0) {
      mp_sub(lo.w, accp.w, e.w, NL);
      nat ld;
      nat_mul(ld, lo, D);
      if (mp_cmp(N.w, ld.w, NL) < 0) return true;    // recip_q < acc' - e: BELOW
    }
    err = errp;
    acc = accp;
  }
  return false;                                        // MaxReached
}

// x = -floor(sigma * c / R) (= ceil(sigma |c| / R) for c <= 0); false when out of range
bool leader_x_raw(uint8_t x_le[16], const uint8_t sigma_fp[16], const uint8_t c_raw[16]) {
  u128 c, s;
  std::memcpy(&c, c_raw, 16);
  std::memcpy(&s, sigma_fp, 16);
  if (!(c >> 127)) { std::memset(x_le, 0, 16); return c == 0; }
  const u128 mag = ~c + 1;
  nat a, b, p, q, R = nat_R();
  nat_zero(a); nat_zero(b);
  std::memcpy(a.w, &s, 16);
  std::memcpy(b.w, &mag, 16);
  nat_mul(p, a, b);
  nat_div_R(q, p);
  nat back;
  nat_mul(back, q, R);
  if (mp_cmp(back.w, p.w, NL) != 0) {
    nat one;
    nat_zero(one);
    one.w[0] = 1;
    mp_add(q.w, q.w, one.w, NL);
  }
  for (int i = 2; i < NL; i++) if (q.w[i]) return false;
  u128 xv;
  std::memcpy(&xv, q.w, 16);
  u128 r16 = ((u128)TEN17 * TEN17) * 16;
  if (xv > r16) return false;
  std::memcpy(x_le, &xv, 16);
  return true;
}

void be64(uint8_t* p, uint64_t v) { for (int i = 0; i < 8; i++) p[i] = (uint8_t)(v >> (56 - 8 * i)); }

// ============================================================ threads
int usable_cores() {
  cpu_set_t set;
  if (sched_getaffinity(0, sizeof set, &set) == 0) return std::max(1, CPU_COUNT(&set));
  return std::max(1u, std::thread::hardware_concurrency());
}

template <typename F>
void parallel_for(size_t n, int nthreads, F&& f) {
  if (n == 0) return;
  nthreads = std::max(1, std::min<int>(nthreads, (int)((n + 31) / 32)));
  std::atomic<size_t> next{0};
  auto work = [&]() {
    for (;;) {
      const size_t i0 = next.fetch_add(32);
      if (i0 >= n) break;
      const size_t i1 = std::min(n, i0 + 32);
      for (size_t i = i0; i < i1; i++) f(i);
    }
  };
  std::vector<std::thread> th;
  for (int k = 1; k < nthreads; k++) th.emplace_back(work);
  work();
  for (auto& t : th) t.join();
}

}  // namespace

struct praos_ctx {
  int threads = 0;                        // 0: every usable core
  std::string err;
  bool have_epoch = false;
  praos_params params{};
  uint8_t eta0[32] = {0};
  int eta0_neutral = 1;
  std::vector<praos_pool> pools;          // sorted by hash
  std::vector<int32_t> order;             // sorted index -> caller index
  std::vector<std::array<uint8_t, 16>> x; // per sorted pool
  int nthreads() const { return threads > 0 ? threads : usable_cores(); }
};

extern "C" {

int praos_abi_version(void) { return PRAOS_ABI_VERSION; }
const char* praos_last_error(praos_ctx* c) { return c ? c->err.c_str() : "no context"; }
praos_ctx* praos_open(int device) { (void)device; return new praos_ctx(); }
void praos_close(praos_ctx* c) { delete c; }

/* PRAOS_OPT_THREADS (CPU twin only): worker threads, 0 = every usable core */
int praos_set_option(praos_ctx* c, int opt, int value) {
  if (!c) return PRAOS_E_ARG;
  if (opt == 4) { c->threads = value < 0 ? 0 : value; return PRAOS_OK; }
  return PRAOS_OK;                        // GPU options are accepted and ignored
}

int praos_set_epoch(praos_ctx* c, const uint8_t eta0[32], const praos_pool* pools, uint32_t npools,
                    const praos_params* params) {
  if (!c || !params || (npools && !pools) || params->slots_per_kes_period == 0) return PRAOS_E_ARG;
  std::vector<int32_t> order(npools);
  for (uint32_t i = 0; i < npools; i++) order[i] = (int32_t)i;
  std::sort(order.begin(), order.end(),
            [&](int32_t a, int32_t b) { return std::memcmp(pools[a].hash28, pools[b].hash28, 28) < 0; });
  std::vector<praos_pool> sorted(npools);
  std::vector<std::array<uint8_t, 16>> xs(npools);
  c->have_epoch = false;
  for (uint32_t s = 0; s < npools; s++) {
    sorted[s] = pools[order[s]];
    if (!leader_x_raw(xs[s].data(), sorted[s].sigma_fp, params->c_raw)) {
      c->err = "sigma * activeSlotLog out of range";
      return PRAOS_E_ARG;
    }
  }
  c->pools.swap(sorted);
  c->order.swap(order);
  c->x.swap(xs);
  c->params = *params;
  c->eta0_neutral = eta0 == nullptr;
  std::memset(c->eta0, 0, 32);
  if (eta0) std::memcpy(c->eta0, eta0, 32);
  c->have_epoch = true;
  return PRAOS_OK;
}

int praos_verify_headers(praos_ctx* c, const praos_headers* h, praos_out* out) {
  if (!c || !h || !out || !out->bits) return PRAOS_E_ARG;
  if (!c->have_epoch) return PRAOS_E_STATE;
  const praos_params P = c->params;
  parallel_for(h->n, c->nthreads(), [&](size_t i) {
    uint16_t b = 0;
    const uint64_t slot = h->slot[i], c0 = h->ocert_c0[i];
    // validateKESSignature (Praos.hs:567-590)
    const uint64_t kp = slot / P.slots_per_kes_period;
    if (!(c0 <= kp)) b |= PRAOS_BIT_KES_BEFORE_START;
    if (!(kp < c0 + P.max_kes_evo)) b |= PRAOS_BIT_KES_AFTER_END;
    uint8_t msg[48];
    std::memcpy(msg, h->hot_vk + 32 * i, 32);
    be64(msg + 32, h->ocert_n[i]);
    be64(msg + 40, c0);
    if (!ed25519_verify(h->ocert_sig + 64 * i, msg, 48, h->cold_vk + 32 * i)) b |= PRAOS_BIT_OCERT_SIG;
    const uint64_t off = h->body_off[i], len = h->body_len[i];
    if (off > h->body_bytes_len || len > h->body_bytes_len - off) {
      b |= PRAOS_BIT_INPUT;
    } else {
      const int k = kes_verify(h->hot_vk + 32 * i, kp >= c0 ? kp - c0 : 0, h->body_bytes + off, len,
                               h->kes_sig + 448 * i);
      if (k == 1) b |= PRAOS_BIT_KES_MERKLE;
      if (k == 2) b |= PRAOS_BIT_KES_LEAF;
    }
    // validateVRFSignature (Praos.hs:528-556)
    uint8_t hk[28];
    blake2b(hk, 28, h->cold_vk + 32 * i, 32);
    int lo = 0, hi = (int)c->pools.size() - 1, idx = -1;
    while (lo <= hi) {
      const int mid = (lo + hi) / 2;
      const int r = std::memcmp(c->pools[mid].hash28, hk, 28);
      if (r == 0) { idx = mid; break; }
      if (r < 0) lo = mid + 1; else hi = mid - 1;
    }
    if (idx < 0) {
      b |= PRAOS_BIT_VRF_KEY_UNKNOWN;
    } else {
      uint8_t vh[32];
      blake2b(vh, 32, h->vrf_vk + 32 * i, 32);
      if (std::memcmp(vh, c->pools[idx].vrf_hash32, 32) != 0) b |= PRAOS_BIT_VRF_KEY_WRONG;
    }
    uint8_t sb[8], alpha[32], beta[64];
    be64(sb, slot);
    blake2b(alpha, 32, sb, 8, c->eta0, c->eta0_neutral ? 0 : 32);     // mkInputVRF
    const uint8_t* vout = h->vrf_out + 64 * i;
    if (!vrf_verify(beta, h->vrf_vk + 32 * i, h->vrf_proof + 80 * i, alpha)) b |= PRAOS_BIT_VRF_PROOF;
    if (P.vrf_check_output && std::memcmp(beta, vout, 64) != 0) b |= PRAOS_BIT_VRF_OUTPUT;
    const uint8_t tagL = 'L', tagN = 'N';
    uint8_t lv[32], nv[32], nn[32];
    blake2b(lv, 32, &tagL, 1, vout, 64);                               // vrfLeaderValue
    blake2b(nv, 32, &tagN, 1, vout, 64);
    blake2b(nn, 32, nv, 32);                                           // vrfNonceValue
    if (idx >= 0 && !P.f_is_one && !leader_check(lv, 32, c->x[idx].data())) b |= PRAOS_BIT_LEADER;
    out->bits[i] = b;
    if (out->pool_idx) out->pool_idx[i] = idx < 0 ? -1 : c->order[idx];
    if (out->beta) std::memcpy(out->beta + 64 * i, beta, 64);
    if (out->leader) std::memcpy(out->leader + 32 * i, lv, 32);
    if (out->nonce) std::memcpy(out->nonce + 32 * i, nn, 32);
  });
  return PRAOS_OK;
}

// TPraos (Shelley..Alonzo, d = 0): SL.updateChainDepState's header crypto (TPraos.hs:378-387,
// cardano-protocol-tpraos OCERT + OVERLAY praosVrfChecks).  The OCERT predicates are the
// Praos ones; the two VRF certificates are checked against mkSeed seedEta / seedL
// (Blake2b-256(BE64 slot || eta0) xor Blake2b-256(BE64 k), k = 0 / 1), the leader test takes
// the 64-byte leader certificate output against the 2^512 bound, and the nonce is
// mkNonceFromOutputVRF (Blake2b-256 of the eta output).  No overlay schedule here (d = 0).
int praos_verify_tpraos_headers(praos_ctx* c, const praos_tpraos_headers* th, praos_tpraos_out* out) {
  if (!c || !th || !out || !out->bits || (th->h.n && (!th->leader_out || !th->leader_proof))) return PRAOS_E_ARG;
  if (!c->have_epoch) return PRAOS_E_STATE;
  const praos_headers* h = &th->h;
  const praos_params P = c->params;
  parallel_for(h->n, c->nthreads(), [&](size_t i) {
    uint16_t b = 0;
    const uint64_t slot = h->slot[i], c0 = h->ocert_c0[i];
    const uint64_t kp = slot / P.slots_per_kes_period;
    if (!(c0 <= kp)) b |= PRAOS_BIT_KES_BEFORE_START;
    if (!(kp < c0 + P.max_kes_evo)) b |= PRAOS_BIT_KES_AFTER_END;
    uint8_t msg[48];
    std::memcpy(msg, h->hot_vk + 32 * i, 32);
    be64(msg + 32, h->ocert_n[i]);
    be64(msg + 40, c0);
    if (!ed25519_verify(h->ocert_sig + 64 * i, msg, 48, h->cold_vk + 32 * i)) b |= PRAOS_BIT_OCERT_SIG;
    const uint64_t off = h->body_off[i], len = h->body_len[i];
    if (off > h->body_bytes_len || len > h->body_bytes_len - off) {
      b |= PRAOS_BIT_INPUT;
    } else {
      const int k = kes_verify(h->hot_vk + 32 * i, kp >= c0 ? kp - c0 : 0, h->body_bytes + off, len,
                               h->kes_sig + 448 * i);
      if (k == 1) b |= PRAOS_BIT_KES_MERKLE;
      if (k == 2) b |= PRAOS_BIT_KES_LEAF;
    }
    // praosVrfChecks: the issuer's pool, its registered VRF key
    uint8_t hk[28];
    blake2b(hk, 28, h->cold_vk + 32 * i, 32);
    int lo = 0, hi = (int)c->pools.size() - 1, idx = -1;
    while (lo <= hi) {
      const int mid = (lo + hi) / 2;
      const int r = std::memcmp(c->pools[mid].hash28, hk, 28);
      if (r == 0) { idx = mid; break; }
      if (r < 0) lo = mid + 1; else hi = mid - 1;
    }
    if (idx < 0) {
      b |= PRAOS_BIT_VRF_KEY_UNKNOWN;
    } else {
      uint8_t vh[32];
      blake2b(vh, 32, h->vrf_vk + 32 * i, 32);
      if (std::memcmp(vh, c->pools[idx].vrf_hash32, 32) != 0) b |= PRAOS_BIT_VRF_KEY_WRONG;
    }
    // the two certificates: mkSeed seedEta (k = 0), seedL (k = 1)
    uint8_t sb[8], hs[32];
    be64(sb, slot);
    blake2b(hs, 32, sb, 8, c->eta0, c->eta0_neutral ? 0 : 32);
    const uint8_t* certs_out[2] = {h->vrf_out + 64 * i, th->leader_out + 64 * i};
    const uint8_t* certs_proof[2] = {h->vrf_proof + 80 * i, th->leader_proof + 80 * i};
    uint8_t* betas[2] = {out->beta_eta ? out->beta_eta + 64 * i : nullptr,
                         out->beta_leader ? out->beta_leader + 64 * i : nullptr};
    for (int k = 0; k < 2; k++) {
      uint8_t kb[8], uc[32], alpha[32], beta[64];
      be64(kb, (uint64_t)k);
      blake2b(uc, 32, kb, 8);                                         // mkNonceFromNumber k
      for (int j = 0; j < 32; j++) alpha[j] = hs[j] ^ uc[j];          // Hash.xor
      const bool ok = vrf_verify(beta, h->vrf_vk + 32 * i, certs_proof[k], alpha);
      if (!ok || (P.vrf_check_output && std::memcmp(beta, certs_out[k], 64) != 0))
        b |= k == 0 ? PRAOS_BIT_TP_VRF_NONCE : PRAOS_BIT_TP_VRF_LEADER;
      if (betas[k]) std::memcpy(betas[k], beta, 64);
    }
    if (idx >= 0 && !P.f_is_one && !leader_check(certs_out[1], 64, c->x[idx].data())) b |= PRAOS_BIT_LEADER;
    out->bits[i] = b;
    if (out->pool_idx) out->pool_idx[i] = idx < 0 ? -1 : c->order[idx];
    if (out->nonce) blake2b(out->nonce + 32 * i, 32, certs_out[0], 64);   // mkNonceFromOutputVRF
  });
  return PRAOS_OK;
}

int praos_verify_ocert(praos_ctx* c, size_t n, const uint8_t* cold_vk, const uint8_t* hot_vk, const uint64_t* ocert_n,
                       const uint64_t* ocert_c0, const uint8_t* sig, uint8_t* ok) {
  if (!c || (n && (!cold_vk || !hot_vk || !ocert_n || !ocert_c0 || !sig || !ok))) return PRAOS_E_ARG;
  parallel_for(n, c->nthreads(), [&](size_t i) {
    uint8_t msg[48];
    std::memcpy(msg, hot_vk + 32 * i, 32);
    be64(msg + 32, ocert_n[i]);
    be64(msg + 40, ocert_c0[i]);
    ok[i] = ed25519_verify(sig + 64 * i, msg, 48, cold_vk + 32 * i) ? 1 : 0;
  });
  return PRAOS_OK;
}

int praos_verify_kes(praos_ctx* c, size_t n, const uint8_t* vk, const uint32_t* period, const uint8_t* sig,
                     const uint64_t* msg_off, const uint32_t* msg_len, const uint8_t* msg_bytes, size_t msg_bytes_len,
                     uint8_t* result) {
  if (!c || (n && (!vk || !period || !sig || !msg_off || !msg_len || !result))) return PRAOS_E_ARG;
  parallel_for(n, c->nthreads(), [&](size_t i) {
    if (msg_off[i] > msg_bytes_len || msg_len[i] > msg_bytes_len - msg_off[i]) { result[i] = 1; return; }
    result[i] = (uint8_t)kes_verify(vk + 32 * i, period[i], msg_bytes + msg_off[i], msg_len[i], sig + 448 * i);
  });
  return PRAOS_OK;
}

int praos_verify_vrf(praos_ctx* c, size_t n, const uint8_t* vk, const uint8_t* proof, const uint8_t* alpha,
                     uint8_t* ok, uint8_t* beta) {
  if (!c || (n && (!vk || !proof || !alpha || !ok))) return PRAOS_E_ARG;
  parallel_for(n, c->nthreads(), [&](size_t i) {
    uint8_t b[64];
    ok[i] = vrf_verify(b, vk + 32 * i, proof + 80 * i, alpha + 32 * i) ? 1 : 0;
    if (beta) std::memcpy(beta + 64 * i, b, 64);
  });
  return PRAOS_OK;
}

int praos_check_leader(praos_ctx* c, size_t n, const uint8_t* leader, const uint8_t* sigma_fp,
                       const praos_params* params, uint8_t* is_leader) {
  if (!c || !params || (n && (!leader || !sigma_fp || !is_leader))) return PRAOS_E_ARG;
  std::vector<std::array<uint8_t, 16>> xs(n);
  for (size_t i = 0; i < n; i++)
    if (!leader_x_raw(xs[i].data(), sigma_fp + 16 * i, params->c_raw)) { c->err = "x out of range"; return PRAOS_E_ARG; }
  parallel_for(n, c->nthreads(), [&](size_t i) {
    is_leader[i] = params->f_is_one ? 1 : (leader_check(leader + 32 * i, 32, xs[i].data()) ? 1 : 0);
  });
  return PRAOS_OK;
}

}  // extern "C"
