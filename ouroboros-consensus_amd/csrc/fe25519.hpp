// fe25519.hpp -- GF(2^255-19) arithmetic for gfx950, one field element per lane.
//
// Representation: 8 x 32-bit limbs, radix 2^32, value in [0, 2^256) ("weakly
// reduced": congruent mod p, canonicalised only for encoding / comparison).
//
// Why radix 2^32 (measured on MI355X, tools/microbench/intrate.hip at 3 waves per SIMD):
// v_mad_u64_u32 (32x32+64 -> 64 with carry-out) issues at ~5.0 SIMD cycles per wave64
// instruction, a carry add at ~4.6 and other VOP3 ops at ~4.4, so a full 32-bit MAC costs
// barely more than an add.  The 8x8 schoolbook product is 64 MACs, each paired with one
// v_addc_co_u32 that counts the column carry; reduction folds the high 256 bits with
// 2^256 = 38 (mod p).  This beats radix 2^25.5 (100 MACs + 64-bit carry chains) and 9 x 29-bit
// limbs (81 carry-free MACs, but a 64-bit shift and mask per column: 771 / 661 vs 744 / 574
// cycles per multiply / squaring, tools/microbench/fe29.hip), and uses 8 VGPRs per element.
// The shipped products are the generated columns of fe_cols.hpp (PRAOS_MACG, below).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define FE_INLINE __device__ __forceinline__

struct fe { uint32_t v[8]; };

// acc(64) += a*b with the carry-out counted into top.  gfx950 needs two wait
// states between a VALU write of VCC and a VALU read of it as carry-in (the
// compiler inserts the same `s_nop 1` in its own carry chains).  FE_MAC / FE_MAC2 are the
// PRAOS_MACG=0 forms; FE_MAC3 / FE_MAC4 (the ILP-4 builds) are padding-free already.
#define FE_MAC(acc, top, a, b)                                                     \
  asm("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\ts_nop 1\n\tv_addc_co_u32 %1, vcc, 0, %1, vcc" \
      : "+v"(acc), "+v"(top) : "v"(a), "v"(b) : "vcc")
// first MAC of a column: top := carry-out (no zero-initialised top register to copy in)
#define FE_MAC0(acc, top, a, b)                                                    \
  asm("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\ts_nop 1\n\tv_cndmask_b32_e64 %1, 0, 1, vcc" \
      : "+v"(acc), "=v"(top) : "v"(a), "v"(b) : "vcc")

FE_INLINE uint32_t addc(uint32_t a, uint32_t b, uint32_t cin, uint32_t* cout) {
  return __builtin_addc(a, b, cin, cout);
}
FE_INLINE uint32_t subb(uint32_t a, uint32_t b, uint32_t bin, uint32_t* bout) {
  return __builtin_subc(a, b, bin, bout);
}

FE_INLINE void fe_set(fe& r, uint32_t x) {
  r.v[0] = x;
#pragma unroll
  for (int i = 1; i < 8; i++) r.v[i] = 0;
}
FE_INLINE void fe_const(fe& r, const uint32_t c[8]) {
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = c[i];
}

// PRAOS_RED_BRANCH=1: the second fold's carry propagation in a rarely taken branch (below)
#ifndef PRAOS_RED_BRANCH
#define PRAOS_RED_BRANCH 1
#endif

// r = t[0..15] mod p, t = 512-bit product
FE_INLINE void fe_reduce512(fe& r, const uint32_t t[16]) {
  uint64_t s[8];
#pragma unroll
  for (int i = 0; i < 8; i++) s[i] = (uint64_t)t[8 + i] * 38u + t[i];
  uint32_t c = 0;
  r.v[0] = (uint32_t)s[0];
#pragma unroll
  for (int i = 1; i < 8; i++) r.v[i] = addc((uint32_t)s[i], (uint32_t)(s[i - 1] >> 32), c, &c);
  uint32_t k = (uint32_t)(s[7] >> 32) + c;           // < 40
#if PRAOS_RED_BRANCH
  // 38 k < 1520 carries out of limb 0 only when limb 0 >= 2^32 - 1520 (probability < 2^-21
  // per product): the seven-limb carry propagation runs in a branch the wave almost never
  // takes, instead of as a serial VCC chain in every product.
  r.v[0] = addc(r.v[0], k * 38u, 0, &c);
  if (__builtin_expect(c != 0, 0)) {
#pragma unroll
    for (int i = 1; i < 8; i++) r.v[i] = addc(r.v[i], 0, c, &c);
    r.v[0] += 38u * c;                               // cannot carry: value wrapped to < 2^11
  }
#else
  uint64_t s0 = (uint64_t)k * 38u + r.v[0];
  r.v[0] = (uint32_t)s0;
  c = (uint32_t)(s0 >> 32);
#pragma unroll
  for (int i = 1; i < 8; i++) r.v[i] = addc(r.v[i], 0, c, &c);
  r.v[0] += 38u * c;                                 // cannot carry: value wrapped to < 2^11
#endif
}

// PRAOS_MACG=1: the products come from fe_cols.hpp (tools/gen_fe_cols.py), each column one asm
// block with its MACs software-pipelined so no carry read needs s_nop padding; 0 keeps the
// FE_MAC / FE_MAC2 forms below (the A/B reference).
#ifndef PRAOS_MACG
#define PRAOS_MACG 1
#endif
#include "fe_cols.hpp"

// 2 t[0 .. 16) + the diagonal squares a_i^2, reduced: the square from its cross products
FE_INLINE void fe_sq_finish(fe& r, uint32_t (&t)[16], const fe& a) {
#pragma unroll
  for (int i = 15; i > 0; i--) t[i] = (t[i] << 1) | (t[i - 1] >> 31);
  t[0] = 0;
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint64_t d = (uint64_t)a.v[i] * a.v[i];
    t[2 * i] = addc(t[2 * i], (uint32_t)d, c, &c);
    t[2 * i + 1] = addc(t[2 * i + 1], (uint32_t)(d >> 32), c, &c);
  }
  fe_reduce512(r, t);
}

FE_INLINE void fe_mul(fe& r, const fe& a, const fe& b) {
  uint32_t t[16];
#if PRAOS_MACG
  fe_prod_g(t, a, b);
#else
  uint64_t acc = (uint64_t)a.v[0] * b.v[0];
  t[0] = (uint32_t)acc;
  acc >>= 32;
#pragma unroll
  for (int k = 1; k < 15; k++) {
    uint32_t top;
    const int i0 = k < 8 ? 0 : k - 7;                // first i of column k (j = k - i <= 7)
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const int j = k - i;
      if (j < 0 || j > 7) continue;
      if (i == i0) FE_MAC0(acc, top, a.v[i], b.v[j]);
      else FE_MAC(acc, top, a.v[i], b.v[j]);
    }
    t[k] = (uint32_t)acc;
    acc = (acc >> 32) | ((uint64_t)top << 32);
  }
  t[15] = (uint32_t)acc;
#endif
  fe_reduce512(r, t);
}

FE_INLINE void fe_sq(fe& r, const fe& a) {
  uint32_t t[16];
#if PRAOS_MACG
  fe_cross_g(t, a);
#else
  // cross products a_i a_j, i < j
  uint64_t acc = 0;
  t[0] = 0;
#pragma unroll
  for (int k = 1; k < 15; k++) {
    uint32_t top = 0;                                // stays 0 in column 14 (no i < j there)
    const int i0 = k < 8 ? 0 : k - 7;
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const int j = k - i;
      if (j <= i || j > 7) continue;
      if (i == i0) FE_MAC0(acc, top, a.v[i], a.v[j]);
      else FE_MAC(acc, top, a.v[i], a.v[j]);
    }
    t[k] = (uint32_t)acc;
    acc = (acc >> 32) | ((uint64_t)top << 32);
  }
  t[15] = (uint32_t)acc;
#endif
  fe_sq_finish(r, t, a);                             // cross sum < 2^511: doubling loses no bit
}

// ---- two independent products interleaved MAC by MAC (ILP for the group formulas,
// whose multiplications come in independent groups of 2-4).  Each product keeps its
// carry in its own SGPR pair; the other product's mad + an s_nop 0 give the two wait
// states between a carry write and its read.  tools/microbench/femul2.hip: at 3 waves
// per SIMD (the verify kernels' occupancy) 835 -> 788 SIMD cycles per multiply.
#ifndef PRAOS_ILP2
#define PRAOS_ILP2 1
#endif
// The first product's carry goes through VCC (its carry add encodes as VOP2, issued in
// fewer cycles than the VOP3 form an SGPR-pair carry needs), the second's through an
// SGPR pair; PRAOS_MAC2_VCC=0 keeps both in SGPR pairs (the A/B reference).
#ifndef PRAOS_MAC2_VCC
#define PRAOS_MAC2_VCC 1
#endif
#if PRAOS_MAC2_VCC
#define FE_MAC2(acc1, top1, a1, b1, acc2, top2, a2, b2)                                    \
  do {                                                                                   \
    uint64_t c2_;                                                                        \
    asm("v_mad_u64_u32 %0, vcc, %5, %6, %0\n\tv_mad_u64_u32 %1, %4, %7, %8, %1\n\ts_nop 0\n\t" \
        "v_addc_co_u32 %2, vcc, 0, %2, vcc\n\tv_addc_co_u32 %3, %4, 0, %3, %4"             \
        : "+v"(acc1), "+v"(acc2), "+v"(top1), "+v"(top2), "=&s"(c2_)                     \
        : "v"(a1), "v"(b1), "v"(a2), "v"(b2) : "vcc");                                   \
  } while (0)
#define FE_MAC2_0(acc1, top1, a1, b1, acc2, top2, a2, b2)                                  \
  do {                                                                                   \
    uint64_t c2_;                                                                        \
    asm("v_mad_u64_u32 %0, vcc, %5, %6, %0\n\tv_mad_u64_u32 %1, %4, %7, %8, %1\n\ts_nop 0\n\t" \
        "v_addc_co_u32 %2, vcc, 0, %9, vcc\n\tv_cndmask_b32_e64 %3, 0, 1, %4"              \
        : "+v"(acc1), "+v"(acc2), "=v"(top1), "=v"(top2), "=&s"(c2_)                     \
        : "v"(a1), "v"(b1), "v"(a2), "v"(b2), "v"(0u) : "vcc");                          \
  } while (0)
#else
#define FE_MAC2(acc1, top1, a1, b1, acc2, top2, a2, b2)                                    \
  do {                                                                                   \
    uint64_t c1_, c2_;                                                                   \
    asm("v_mad_u64_u32 %0, %4, %6, %7, %0\n\tv_mad_u64_u32 %1, %5, %8, %9, %1\n\ts_nop 0\n\t" \
        "v_addc_co_u32 %2, %4, 0, %2, %4\n\tv_addc_co_u32 %3, %5, 0, %3, %5"              \
        : "+v"(acc1), "+v"(acc2), "+v"(top1), "+v"(top2), "=&s"(c1_), "=&s"(c2_)         \
        : "v"(a1), "v"(b1), "v"(a2), "v"(b2));                                           \
  } while (0)
#define FE_MAC2_0(acc1, top1, a1, b1, acc2, top2, a2, b2)                                  \
  do {                                                                                   \
    uint64_t c1_, c2_;                                                                   \
    asm("v_mad_u64_u32 %0, %4, %6, %7, %0\n\tv_mad_u64_u32 %1, %5, %8, %9, %1\n\ts_nop 0\n\t" \
        "v_cndmask_b32_e64 %2, 0, 1, %4\n\tv_cndmask_b32_e64 %3, 0, 1, %5"                \
        : "+v"(acc1), "+v"(acc2), "=v"(top1), "=v"(top2), "=&s"(c1_), "=&s"(c2_)         \
        : "v"(a1), "v"(b1), "v"(a2), "v"(b2));                                           \
  } while (0)

#endif

// r1 = a1 b1, r2 = a2 b2 (outputs may alias any input: written after both products)
FE_INLINE void fe_mul2(fe& r1, const fe& a1, const fe& b1, fe& r2, const fe& a2, const fe& b2) {
#if PRAOS_ILP2 && PRAOS_MACG
  uint32_t t1[16], t2[16];
  fe_prod2_g(t1, t2, a1, b1, a2, b2);
  fe_reduce512(r1, t1);
  fe_reduce512(r2, t2);
#elif PRAOS_ILP2
  uint32_t t1[16], t2[16];
  uint64_t acc1 = (uint64_t)a1.v[0] * b1.v[0], acc2 = (uint64_t)a2.v[0] * b2.v[0];
  t1[0] = (uint32_t)acc1;
  t2[0] = (uint32_t)acc2;
  acc1 >>= 32;
  acc2 >>= 32;
#pragma unroll
  for (int k = 1; k < 15; k++) {
    uint32_t top1, top2;
    const int i0 = k < 8 ? 0 : k - 7;
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const int j = k - i;
      if (j < 0 || j > 7) continue;
      if (i == i0) FE_MAC2_0(acc1, top1, a1.v[i], b1.v[j], acc2, top2, a2.v[i], b2.v[j]);
      else FE_MAC2(acc1, top1, a1.v[i], b1.v[j], acc2, top2, a2.v[i], b2.v[j]);
    }
    t1[k] = (uint32_t)acc1;
    t2[k] = (uint32_t)acc2;
    acc1 = (acc1 >> 32) | ((uint64_t)top1 << 32);
    acc2 = (acc2 >> 32) | ((uint64_t)top2 << 32);
  }
  t1[15] = (uint32_t)acc1;
  t2[15] = (uint32_t)acc2;
  fe_reduce512(r1, t1);
  fe_reduce512(r2, t2);
#else
  fe x, y;
  fe_mul(x, a1, b1);
  fe_mul(y, a2, b2);
  r1 = x;
  r2 = y;
#endif
}

// r1 = a1^2, r2 = a2^2 (outputs may alias inputs)
FE_INLINE void fe_sq2(fe& r1, const fe& a1, fe& r2, const fe& a2) {
#if PRAOS_ILP2 && PRAOS_MACG
  uint32_t t1[16], t2[16];
  fe_cross2_g(t1, t2, a1, a2);
  fe_sq_finish(r1, t1, a1);
  fe_sq_finish(r2, t2, a2);
#elif PRAOS_ILP2
  uint32_t t1[16], t2[16];
  uint64_t acc1 = 0, acc2 = 0;
  t1[0] = 0;
  t2[0] = 0;
#pragma unroll
  for (int k = 1; k < 15; k++) {
    uint32_t top1 = 0, top2 = 0;
    const int i0 = k < 8 ? 0 : k - 7;
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const int j = k - i;
      if (j <= i || j > 7) continue;
      if (i == i0) FE_MAC2_0(acc1, top1, a1.v[i], a1.v[j], acc2, top2, a2.v[i], a2.v[j]);
      else FE_MAC2(acc1, top1, a1.v[i], a1.v[j], acc2, top2, a2.v[i], a2.v[j]);
    }
    t1[k] = (uint32_t)acc1;
    t2[k] = (uint32_t)acc2;
    acc1 = (acc1 >> 32) | ((uint64_t)top1 << 32);
    acc2 = (acc2 >> 32) | ((uint64_t)top2 << 32);
  }
  t1[15] = (uint32_t)acc1;
  t2[15] = (uint32_t)acc2;
#pragma unroll
  for (int i = 15; i > 0; i--) {
    t1[i] = (t1[i] << 1) | (t1[i - 1] >> 31);
    t2[i] = (t2[i] << 1) | (t2[i - 1] >> 31);
  }
  t1[0] = 0;
  t2[0] = 0;
  uint32_t c1 = 0, c2 = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint64_t d1 = (uint64_t)a1.v[i] * a1.v[i], d2 = (uint64_t)a2.v[i] * a2.v[i];
    t1[2 * i] = addc(t1[2 * i], (uint32_t)d1, c1, &c1);
    t1[2 * i + 1] = addc(t1[2 * i + 1], (uint32_t)(d1 >> 32), c1, &c1);
    t2[2 * i] = addc(t2[2 * i], (uint32_t)d2, c2, &c2);
    t2[2 * i + 1] = addc(t2[2 * i + 1], (uint32_t)(d2 >> 32), c2, &c2);
  }
  fe_reduce512(r1, t1);
  fe_reduce512(r2, t2);
#else
  fe x, y;
  fe_sq(x, a1);
  fe_sq(y, a2);
  r1 = x;
  r2 = y;
#endif
}

// ---- three / four independent products interleaved MAC by MAC (modules built with
// PRAOS_ILP4: the group formulas' products come in independent groups of 3 and 4 --
// p1p1 -> p2 / p3 conversions, the four squarings of a doubling, the additions).  Product 1
// carries through VCC (VOP2 carry add), the others through SGPR pairs; each carry is read
// >= 2 instructions after its write, so no wait-state padding is needed.
// tools/microbench/femul4.hip: one wave per SIMD 1137 -> 971 SIMD cycles per multiply
// against the two-way interleave (the latency-bound small batches), 803 -> 777 at 3 waves.
#define FE_MAC3(A, T, X, Y)                                                                   \
  do {                                                                                       \
    uint64_t c1_, c2_;                                                                       \
    asm("v_mad_u64_u32 %0, vcc, %8, %9, %0\n\tv_mad_u64_u32 %1, %6, %10, %11, %1\n\t"          \
        "v_mad_u64_u32 %2, %7, %12, %13, %2\n\t"                                             \
        "v_addc_co_u32 %3, vcc, 0, %3, vcc\n\tv_addc_co_u32 %4, %6, 0, %4, %6\n\t"             \
        "v_addc_co_u32 %5, %7, 0, %5, %7"                                                    \
        : "+v"(A[0]), "+v"(A[1]), "+v"(A[2]), "+v"(T[0]), "+v"(T[1]), "+v"(T[2]), "=&s"(c1_),  \
          "=&s"(c2_)                                                                         \
        : "v"(X[0]), "v"(Y[0]), "v"(X[1]), "v"(Y[1]), "v"(X[2]), "v"(Y[2])                   \
        : "vcc");                                                                            \
  } while (0)
#define FE_MAC3_0(A, T, X, Y)                                                                 \
  do {                                                                                       \
    uint64_t c1_, c2_;                                                                       \
    asm("v_mad_u64_u32 %0, vcc, %8, %9, %0\n\tv_mad_u64_u32 %1, %6, %10, %11, %1\n\t"          \
        "v_mad_u64_u32 %2, %7, %12, %13, %2\n\t"                                             \
        "v_cndmask_b32_e64 %3, 0, 1, vcc\n\tv_cndmask_b32_e64 %4, 0, 1, %6\n\t"                \
        "v_cndmask_b32_e64 %5, 0, 1, %7"                                                     \
        : "+v"(A[0]), "+v"(A[1]), "+v"(A[2]), "=v"(T[0]), "=v"(T[1]), "=v"(T[2]), "=&s"(c1_),  \
          "=&s"(c2_)                                                                         \
        : "v"(X[0]), "v"(Y[0]), "v"(X[1]), "v"(Y[1]), "v"(X[2]), "v"(Y[2])                   \
        : "vcc");                                                                            \
  } while (0)
#define FE_MAC4(A, T, X, Y)                                                                   \
  do {                                                                                       \
    uint64_t c1_, c2_, c3_;                                                                  \
    asm("v_mad_u64_u32 %0, vcc, %11, %12, %0\n\tv_mad_u64_u32 %1, %8, %13, %14, %1\n\t"        \
        "v_mad_u64_u32 %2, %9, %15, %16, %2\n\tv_mad_u64_u32 %3, %10, %17, %18, %3\n\t"        \
        "v_addc_co_u32 %4, vcc, 0, %4, vcc\n\tv_addc_co_u32 %5, %8, 0, %5, %8\n\t"             \
        "v_addc_co_u32 %6, %9, 0, %6, %9\n\tv_addc_co_u32 %7, %10, 0, %7, %10"                 \
        : "+v"(A[0]), "+v"(A[1]), "+v"(A[2]), "+v"(A[3]), "+v"(T[0]), "+v"(T[1]), "+v"(T[2]),  \
          "+v"(T[3]), "=&s"(c1_), "=&s"(c2_), "=&s"(c3_)                                     \
        : "v"(X[0]), "v"(Y[0]), "v"(X[1]), "v"(Y[1]), "v"(X[2]), "v"(Y[2]), "v"(X[3]), "v"(Y[3]) \
        : "vcc");                                                                            \
  } while (0)
#define FE_MAC4_0(A, T, X, Y)                                                                 \
  do {                                                                                       \
    uint64_t c1_, c2_, c3_;                                                                  \
    asm("v_mad_u64_u32 %0, vcc, %11, %12, %0\n\tv_mad_u64_u32 %1, %8, %13, %14, %1\n\t"        \
        "v_mad_u64_u32 %2, %9, %15, %16, %2\n\tv_mad_u64_u32 %3, %10, %17, %18, %3\n\t"        \
        "v_cndmask_b32_e64 %4, 0, 1, vcc\n\tv_cndmask_b32_e64 %5, 0, 1, %8\n\t"                \
        "v_cndmask_b32_e64 %6, 0, 1, %9\n\tv_cndmask_b32_e64 %7, 0, 1, %10"                    \
        : "+v"(A[0]), "+v"(A[1]), "+v"(A[2]), "+v"(A[3]), "=v"(T[0]), "=v"(T[1]), "=v"(T[2]),  \
          "=v"(T[3]), "=&s"(c1_), "=&s"(c2_), "=&s"(c3_)                                     \
        : "v"(X[0]), "v"(Y[0]), "v"(X[1]), "v"(Y[1]), "v"(X[2]), "v"(Y[2]), "v"(X[3]), "v"(Y[3]) \
        : "vcc");                                                                            \
  } while (0)

// t[m][0 .. 16) = a[m] * b[m] for m < M (M = 3 or 4), product scanning, MACs interleaved
template <int M>
FE_INLINE void fe_prodN(uint32_t (&t)[M][16], const fe* const (&a)[M], const fe* const (&b)[M]) {
  static_assert(M == 3 || M == 4, "three or four products");
  uint64_t acc[M];
#pragma unroll
  for (int m = 0; m < M; m++) {
    acc[m] = (uint64_t)a[m]->v[0] * b[m]->v[0];
    t[m][0] = (uint32_t)acc[m];
    acc[m] >>= 32;
  }
#pragma unroll
  for (int k = 1; k < 15; k++) {
    uint32_t top[M];
    const int i0 = k < 8 ? 0 : k - 7;
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const int j = k - i;
      if (j < 0 || j > 7) continue;
      uint32_t x[M], y[M];
#pragma unroll
      for (int m = 0; m < M; m++) { x[m] = a[m]->v[i]; y[m] = b[m]->v[j]; }
      if constexpr (M == 4) {
        if (i == i0) FE_MAC4_0(acc, top, x, y);
        else FE_MAC4(acc, top, x, y);
      } else {
        if (i == i0) FE_MAC3_0(acc, top, x, y);
        else FE_MAC3(acc, top, x, y);
      }
    }
#pragma unroll
    for (int m = 0; m < M; m++) {
      t[m][k] = (uint32_t)acc[m];
      acc[m] = (acc[m] >> 32) | ((uint64_t)top[m] << 32);
    }
  }
#pragma unroll
  for (int m = 0; m < M; m++) t[m][15] = (uint32_t)acc[m];
}

// r_m = a_m b_m (outputs may alias any input: written after every product)
FE_INLINE void fe_mul3(fe& r1, const fe& a1, const fe& b1, fe& r2, const fe& a2, const fe& b2, fe& r3, const fe& a3,
                       const fe& b3) {
  uint32_t t[3][16];
  const fe* const a[3] = {&a1, &a2, &a3};
  const fe* const b[3] = {&b1, &b2, &b3};
  fe_prodN<3>(t, a, b);
  fe_reduce512(r1, t[0]);
  fe_reduce512(r2, t[1]);
  fe_reduce512(r3, t[2]);
}
FE_INLINE void fe_mul4(fe& r1, const fe& a1, const fe& b1, fe& r2, const fe& a2, const fe& b2, fe& r3, const fe& a3,
                       const fe& b3, fe& r4, const fe& a4, const fe& b4) {
  uint32_t t[4][16];
  const fe* const a[4] = {&a1, &a2, &a3, &a4};
  const fe* const b[4] = {&b1, &b2, &b3, &b4};
  fe_prodN<4>(t, a, b);
  fe_reduce512(r1, t[0]);
  fe_reduce512(r2, t[1]);
  fe_reduce512(r3, t[2]);
  fe_reduce512(r4, t[3]);
}
// r_m = a_m^2, m < 4: cross products interleaved, then doubled, diagonal added
FE_INLINE void fe_sq4(fe& r1, const fe& a1, fe& r2, const fe& a2, fe& r3, const fe& a3, fe& r4, const fe& a4) {
  const fe* const a[4] = {&a1, &a2, &a3, &a4};
  uint32_t t[4][16];
  uint64_t acc[4] = {0, 0, 0, 0};
#pragma unroll
  for (int m = 0; m < 4; m++) t[m][0] = 0;
#pragma unroll
  for (int k = 1; k < 15; k++) {
    uint32_t top[4] = {0, 0, 0, 0};                  // stays 0 in column 14 (no i < j there)
    const int i0 = k < 8 ? 0 : k - 7;
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const int j = k - i;
      if (j <= i || j > 7) continue;
      uint32_t x[4], y[4];
#pragma unroll
      for (int m = 0; m < 4; m++) { x[m] = a[m]->v[i]; y[m] = a[m]->v[j]; }
      if (i == i0) FE_MAC4_0(acc, top, x, y);
      else FE_MAC4(acc, top, x, y);
    }
#pragma unroll
    for (int m = 0; m < 4; m++) {
      t[m][k] = (uint32_t)acc[m];
      acc[m] = (acc[m] >> 32) | ((uint64_t)top[m] << 32);
    }
  }
#pragma unroll
  for (int m = 0; m < 4; m++) {
    t[m][15] = (uint32_t)acc[m];
#pragma unroll
    for (int i = 15; i > 0; i--) t[m][i] = (t[m][i] << 1) | (t[m][i - 1] >> 31);
    t[m][0] = 0;
    uint32_t c = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const uint64_t d = (uint64_t)a[m]->v[i] * a[m]->v[i];
      t[m][2 * i] = addc(t[m][2 * i], (uint32_t)d, c, &c);
      t[m][2 * i + 1] = addc(t[m][2 * i + 1], (uint32_t)(d >> 32), c, &c);
    }
  }
  fe_reduce512(r1, t[0]);
  fe_reduce512(r2, t[1]);
  fe_reduce512(r3, t[2]);
  fe_reduce512(r4, t[3]);
}

// The fold of the 2^256 carry (borrow) adds (subtracts) 38 at limb 0; that carries (borrows)
// further only when limb 0 >= 2^32 - 38 (< 38): with PRAOS_RED_BRANCH the propagation runs in a
// branch the wave almost never takes, as in fe_reduce512.
FE_INLINE void fe_add(fe& r, const fe& a, const fe& b) {
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = addc(a.v[i], b.v[i], c, &c);
  uint32_t c2 = 0;
  r.v[0] = addc(r.v[0], 38u * c, 0, &c2);
#if PRAOS_RED_BRANCH
  if (__builtin_expect(c2 != 0, 0)) {
#pragma unroll
    for (int i = 1; i < 8; i++) r.v[i] = addc(r.v[i], 0, c2, &c2);
    r.v[0] += 38u * c2;
  }
#else
#pragma unroll
  for (int i = 1; i < 8; i++) r.v[i] = addc(r.v[i], 0, c2, &c2);
  r.v[0] += 38u * c2;
#endif
}

FE_INLINE void fe_sub(fe& r, const fe& a, const fe& b) {
  uint32_t bw = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = subb(a.v[i], b.v[i], bw, &bw);
  uint32_t b2 = 0;
  r.v[0] = subb(r.v[0], 38u * bw, 0, &b2);
#if PRAOS_RED_BRANCH
  if (__builtin_expect(b2 != 0, 0)) {
#pragma unroll
    for (int i = 1; i < 8; i++) r.v[i] = subb(r.v[i], 0, b2, &b2);
    r.v[0] -= 38u * b2;
  }
#else
#pragma unroll
  for (int i = 1; i < 8; i++) r.v[i] = subb(r.v[i], 0, b2, &b2);
  r.v[0] -= 38u * b2;
#endif
}

FE_INLINE void fe_neg(fe& r, const fe& a) {
  fe z;
  fe_set(z, 0);
  fe_sub(r, z, a);
}

FE_INLINE void fe_cmov(fe& r, const fe& a, bool c) {
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = c ? a.v[i] : r.v[i];
}

// canonical representative in [0, p)
FE_INLINE void fe_canon(fe& r, const fe& a) {
  // fold bit 255
  uint32_t top = a.v[7] >> 31;
  uint32_t c = 0;
  r.v[0] = addc(a.v[0], 19u * top, 0, &c);
#pragma unroll
  for (int i = 1; i < 7; i++) r.v[i] = addc(a.v[i], 0, c, &c);
  r.v[7] = (a.v[7] & 0x7fffffffu) + c;               // now < 2^255 + 19
  // subtract p if r >= p  <=>  r + 19 >= 2^255
  uint32_t u[8];
  c = 0;
  u[0] = addc(r.v[0], 19u, 0, &c);
#pragma unroll
  for (int i = 1; i < 8; i++) u[i] = addc(r.v[i], 0, c, &c);
  const bool ge = (u[7] >> 31) != 0;
  u[7] &= 0x7fffffffu;
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = ge ? u[i] : r.v[i];
}

FE_INLINE void fe_tobytes32(uint32_t w[8], const fe& a) {   // little-endian words
  fe c;
  fe_canon(c, a);
#pragma unroll
  for (int i = 0; i < 8; i++) w[i] = c.v[i];
}

FE_INLINE bool fe_iszero(const fe& a) {
  fe c;
  fe_canon(c, a);
  uint32_t o = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) o |= c.v[i];
  return o == 0;
}
FE_INLINE bool fe_isnegative(const fe& a) {
  fe c;
  fe_canon(c, a);
  return c.v[0] & 1;
}
// 255-bit load: top bit cleared, value may be >= p (arithmetic is mod p)
FE_INLINE void fe_frombytes32(fe& r, const uint32_t w[8]) {
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = w[i];
  r.v[7] &= 0x7fffffffu;
}

FE_INLINE void fe_sqn(fe& r, const fe& a, int n) {
  fe_sq(r, a);
#pragma clang loop unroll(disable)
  for (int i = 1; i < n; i++) fe_sq(r, r);
}

// z^(2^250 - 1) and helpers, shared by invert / pow22523 (standard chain)
FE_INLINE void fe_pow2_250_1(fe& t0, fe& z11, const fe& z) {
  fe t1, t2, t3;
  fe_sq(t0, z);                 // 2
  fe_sqn(t1, t0, 2);            // 8
  fe_mul(t1, z, t1);            // 9
  fe_mul(z11, t0, t1);          // 11
  fe_sq(t0, z11);               // 22
  fe_mul(t0, t1, t0);           // 2^5 - 1
  fe_sqn(t1, t0, 5);
  fe_mul(t0, t1, t0);           // 2^10 - 1
  fe_sqn(t1, t0, 10);
  fe_mul(t1, t1, t0);           // 2^20 - 1
  fe_sqn(t2, t1, 20);
  fe_mul(t1, t2, t1);           // 2^40 - 1
  fe_sqn(t1, t1, 10);
  fe_mul(t0, t1, t0);           // 2^50 - 1
  fe_sqn(t1, t0, 50);
  fe_mul(t1, t1, t0);           // 2^100 - 1
  fe_sqn(t3, t1, 100);
  fe_mul(t1, t3, t1);           // 2^200 - 1
  fe_sqn(t1, t1, 50);
  fe_mul(t0, t1, t0);           // 2^250 - 1
}

FE_INLINE void fe_invert_inl(fe& r, const fe& z) {      // z^(p-2)
  fe t0, z11;
  fe_pow2_250_1(t0, z11, z);
  fe_sqn(t0, t0, 5);            // 2^255 - 2^5
  fe_mul(r, t0, z11);           // 2^255 - 21
}

FE_INLINE void fe_pow22523_inl(fe& r, const fe& z) {    // z^((p-5)/8) = z^(2^252 - 3)
  fe t0, z11;
  fe_pow2_250_1(t0, z11, z);
  fe_sqn(t0, t0, 2);            // 2^252 - 4
  fe_mul(r, t0, z);             // 2^252 - 3
}

// Legendre symbol z^((p-1)/2) = z^(2^254 - 10)
FE_INLINE void fe_chi_inl(fe& r, const fe& z) {
  fe t0, z11;
  fe_pow2_250_1(t0, z11, z);    // 2^250 - 1
  fe_sqn(t0, t0, 4);            // 2^254 - 16
  fe t1;
  fe_sq(t1, z);                 // 2
  fe_mul(t1, t1, z);            // 3
  fe_sq(t1, t1);                // 6
  fe_mul(r, t0, t1);            // 2^254 - 10
}

// Exponentiation chains (~255 squarings each) are emitted once per kernel
// module and called by value: the call overhead is < 1% of the chain, and
// inlining every call site multiplied compile time and code size.
__device__ __noinline__ fe fe_invert_v(fe z) { fe r; fe_invert_inl(r, z); return r; }
__device__ __noinline__ fe fe_pow22523_v(fe z) { fe r; fe_pow22523_inl(r, z); return r; }
__device__ __noinline__ fe fe_chi_v(fe z) { fe r; fe_chi_inl(r, z); return r; }

// PRAOS_INV_GCD=1: the inversions by the binary GCD of fe_inv_gcd.hpp (Pornin's algorithm,
// ~2.5x fewer SIMD cycles than the Fermat chain); 0 keeps z^(p-2) (the A/B reference).  The
// result is the same field element; a GCD that did not end (never observed) takes Fermat's.
#ifndef PRAOS_INV_GCD
#define PRAOS_INV_GCD 1
#endif
#include "fe_inv_gcd.hpp"
__device__ __constant__ static const uint32_t FE_GCD_CTAB[18][8] = FEG_CTAB;   // 2^(-30 k) mod p
FE_INLINE void fe_invert_gcd_inl(fe& r, const fe& z) {
  fe y, v, c;
  fe_canon(y, z);
  int k;
  const bool ok = feg_core(v.v, y.v, &k);
  fe_const(c, FE_GCD_CTAB[k]);                       // k is wave-uniform: scalar loads
  fe_mul(r, v, c);
  if (__builtin_expect(!ok, 0)) r = fe_invert_v(z);
}
__device__ __noinline__ fe fe_invert_gcd_v(fe z) { fe r; fe_invert_gcd_inl(r, z); return r; }
FE_INLINE void fe_invert_sel_inl(fe& r, const fe& z) {   // the inline form PRAOS_INV_GCD selects
#if PRAOS_INV_GCD
  fe_invert_gcd_inl(r, z);
#else
  fe_invert_inl(r, z);
#endif
}

#if FE_POW_INLINE   // a module whose kernels keep values live across the chain (no call spills)
#if PRAOS_INV_GCD
FE_INLINE void fe_invert(fe& r, const fe& z) { fe_invert_gcd_inl(r, z); }
#else
FE_INLINE void fe_invert(fe& r, const fe& z) { fe_invert_inl(r, z); }
#endif
FE_INLINE void fe_pow22523(fe& r, const fe& z) { fe_pow22523_inl(r, z); }
#else
#if PRAOS_INV_GCD
FE_INLINE void fe_invert(fe& r, const fe& z) { r = fe_invert_gcd_v(z); }
#else
FE_INLINE void fe_invert(fe& r, const fe& z) { r = fe_invert_v(z); }
#endif
FE_INLINE void fe_pow22523(fe& r, const fe& z) { r = fe_pow22523_v(z); }
#endif
FE_INLINE void fe_chi(fe& r, const fe& z) { r = fe_chi_v(z); }

__device__ __constant__ static const uint32_t FE_D[8] = {0x135978a3u, 0x75eb4dcau, 0x4141d8abu, 0x00700a4du,
                                                          0x7779e898u, 0x8cc74079u, 0x2b6ffe73u, 0x52036ceeu};
__device__ __constant__ static const uint32_t FE_D2[8] = {0x26b2f159u, 0xebd69b94u, 0x8283b156u, 0x00e0149au,
                                                           0xeef3d130u, 0x198e80f2u, 0x56dffce7u, 0x2406d9dcu};
__device__ __constant__ static const uint32_t FE_SQRTM1[8] = {0x4a0ea0b0u, 0xc4ee1b27u, 0xad2fe478u, 0x2f431806u,
                                                               0x3dfbd7a7u, 0x2b4d0099u, 0x4fc1df0bu, 0x2b832480u};
