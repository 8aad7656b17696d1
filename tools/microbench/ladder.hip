// Prices the field representation on the group operations stage V is made of ("adds
// included"), not on products alone (fe29.hip): one Straus window of k_vrf_v's ladder --
// 4 doublings (dbl-2008-hwcd: 4 squarings + 3 products + the additions / subtractions, the
// last one to extended coordinates) and 2 cached additions (add-2008-hwcd-3: 4 products +
// 4 additions + 3 subtractions, each followed by its conversion) -- repeated ITERS times per
// lane, in two representations of GF(2^255-19):
//
//   lib   the library's 8 x 32-bit limbs (fe25519.hpp / ge25519.hpp as compiled into k_vrf_v:
//         generated MAC columns, carried additions with the rare-branch fold); PRAOS_ILP4=1
//         builds the ILP-4 formulas of the small-batch module instead
//   f29   9 x 29-bit limbs: every column sum of a product fits 64 bits (81 carry-free mads, one
//         carry pass); additions lazy (limb-wise, no carry), subtractions limb-wise with a 2p
//         bias, and a carry pass before a product whenever an input could exceed the
//         product's 2^30.4 limb bound
//
// Reports SIMD cycles per window at exactly 1..4 waves per SIMD and checks that both
// representations end on the same point (encoded).  Not used by the library.
// Build: hipcc --offload-arch=gfx950 -O3 -I../../ouroboros-consensus_amd/csrc [-DPRAOS_ILP4=1] -o ladder ladder.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include "ge25519.hpp"

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); return 1; } } while (0)

constexpr int ITERS = 64;

// ------------------------------------------------------------------ 9 x 29
constexpr uint32_t M29 = (1u << 29) - 1;
struct f29 { uint32_t v[9]; };

FE_INLINE void f29_from(f29& r, const fe& a) {
  fe c;
  fe_canon(c, a);
#pragma unroll
  for (int k = 0; k < 9; k++) {
    const int bit = 29 * k, w = bit >> 5, s = bit & 31;
    uint64_t x = c.v[w];
    if (w + 1 < 8) x |= (uint64_t)c.v[w + 1] << 32;
    r.v[k] = (uint32_t)(x >> s) & M29;
  }
}
// x * 2^bit as an 8 x 32 element (x < 2^32; the part at or above 2^256 folded with 38)
FE_INLINE void fe_term(fe& r, uint32_t x, int bit) {
  fe_set(r, 0);
  if (bit + 32 > 256) {                    // split x at 2^(256 - bit)
    const int keep = 256 - bit;
    const uint32_t hi = x >> keep;
    x &= (1u << keep) - 1u;
    r.v[0] = hi * 38u;                     // hi < 2^8: no overflow
  }
  const int w = bit >> 5, sft = bit & 31;
  r.v[w] += x << sft;
  if (sft && w + 1 < 8) r.v[w + 1] += x >> (32 - sft);
}
// any lazy value (limbs < 2^32) -> 8 x 32, mod p
FE_INLINE void f29_to(fe& r, const f29& a) {
  fe_set(r, 0);
#pragma unroll
  for (int k = 0; k < 9; k++) {
    fe t;
    fe_term(t, a.v[k], 29 * k);
    fe_add(r, r, t);
  }
}

FE_INLINE void f29_carry(f29& r, const uint64_t (&T)[9]) {
  uint64_t c = 0;
#pragma unroll
  for (int k = 0; k < 9; k++) {
    const uint64_t u = T[k] + c;
    r.v[k] = (uint32_t)u & M29;
    c = u >> 29;
  }
  // fold everything at or above 2^255 (limb 8's bits 23.. and the carry at 2^261) with 19, so a
  // reduced value's limb 8 stays below 2^23 and the subtraction's 2p bias covers it
  const uint64_t top = ((uint64_t)(r.v[8] >> 23)) + (c << 6);
  r.v[8] &= (1u << 23) - 1u;
  const uint64_t u0 = (uint64_t)r.v[0] + top * 19u;
  r.v[0] = (uint32_t)u0 & M29;
  r.v[1] += (uint32_t)(u0 >> 29);
}
FE_INLINE void f29_weak(f29& a) {                      // a carry pass: limbs back under 2^29 (+ small)
  uint64_t T[9];
#pragma unroll
  for (int k = 0; k < 9; k++) T[k] = a.v[k];
  f29_carry(a, T);
}
FE_INLINE void f29_mul(f29& r, const f29& a, const f29& b) {
  uint32_t t[18];
  uint64_t S = 0;
#pragma unroll
  for (int k = 0; k < 17; k++) {
#pragma unroll
    for (int i = 0; i < 9; i++) {
      const int j = k - i;
      if (j < 0 || j > 8) continue;
      S += (uint64_t)a.v[i] * b.v[j];
    }
    t[k] = (uint32_t)S & M29;
    S >>= 29;
  }
  t[17] = (uint32_t)S;
  uint64_t T[9];
#pragma unroll
  for (int k = 0; k < 9; k++) T[k] = (uint64_t)t[k + 9] * 1216u + t[k];
  f29_carry(r, T);
}
FE_INLINE void f29_sq(f29& r, const f29& a) {
  uint32_t a2[9];
#pragma unroll
  for (int i = 0; i < 9; i++) a2[i] = a.v[i] << 1;
  uint32_t t[18];
  uint64_t S = 0;
#pragma unroll
  for (int k = 0; k < 17; k++) {
#pragma unroll
    for (int i = 0; i < 9; i++) {
      const int j = k - i;
      if (j <= i || j > 8) continue;
      S += (uint64_t)a2[i] * a.v[j];
    }
    if ((k & 1) == 0 && k / 2 < 9) S += (uint64_t)a.v[k / 2] * a.v[k / 2];
    t[k] = (uint32_t)S & M29;
    S >>= 29;
  }
  t[17] = (uint32_t)S;
  uint64_t T[9];
#pragma unroll
  for (int k = 0; k < 9; k++) T[k] = (uint64_t)t[k + 9] * 1216u + t[k];
  f29_carry(r, T);
}
FE_INLINE void f29_add(f29& r, const f29& a, const f29& b) {
#pragma unroll
  for (int k = 0; k < 9; k++) r.v[k] = a.v[k] + b.v[k];
}
// a - b + 2p (b's limbs below 2^30 - 38)
FE_INLINE void f29_sub(f29& r, const f29& a, const f29& b) {
  r.v[0] = a.v[0] + ((1u << 30) - 38u) - b.v[0];
#pragma unroll
  for (int k = 1; k < 8; k++) r.v[k] = a.v[k] + ((1u << 30) - 2u) - b.v[k];
  r.v[8] = a.v[8] + ((1u << 24) - 2u) - b.v[8];
}

struct g29_p2 { f29 X, Y, Z; };
struct g29_p3 { f29 X, Y, Z, T; };
struct g29_p1p1 { f29 X, Y, Z, T; };
struct g29_cached { f29 YpX, YmX, Z, T2d; };

// the p1p1 coordinates below are sums / differences of reduced products: a carry pass each before
// they feed a product (their limbs reach 2^30.6, the products take 2^30.4)
FE_INLINE void g29_p1p1_to_p2(g29_p2& r, g29_p1p1 p) {
  f29_weak(p.X); f29_weak(p.Y); f29_weak(p.Z); f29_weak(p.T);
  f29_mul(r.X, p.X, p.T); f29_mul(r.Y, p.Y, p.Z); f29_mul(r.Z, p.Z, p.T);
}
FE_INLINE void g29_p1p1_to_p3(g29_p3& r, g29_p1p1 p) {
  f29_weak(p.X); f29_weak(p.Y); f29_weak(p.Z); f29_weak(p.T);
  f29_mul(r.X, p.X, p.T); f29_mul(r.Y, p.Y, p.Z); f29_mul(r.Z, p.Z, p.T); f29_mul(r.T, p.X, p.Y);
}
FE_INLINE void g29_dbl(g29_p1p1& r, const g29_p2& p) {
  f29 t0, s;
  f29_add(s, p.X, p.Y);                    // < 2^30: a product input as it is
  f29_sq(r.X, p.X); f29_sq(r.Z, p.Y); f29_sq(r.T, p.Z); f29_sq(t0, s);
  f29_add(r.T, r.T, r.T);
  f29_add(r.Y, r.Z, r.X);
  f29_sub(r.Z, r.Z, r.X);
  f29_sub(r.X, t0, r.Y);
  f29_weak(r.Z);                           // (r.Z is subtracted below: keep its limbs under the bias)
  f29_sub(r.T, r.T, r.Z);
}
FE_INLINE void g29_add(g29_p1p1& r, const g29_p3& p, const g29_cached& q) {
  f29 t0, a, b;
  f29_add(a, p.Y, p.X);
  f29_sub(b, p.Y, p.X);
  f29_weak(b);
  f29_mul(r.Z, a, q.YpX); f29_mul(r.Y, b, q.YmX); f29_mul(r.T, q.T2d, p.T); f29_mul(r.X, p.Z, q.Z);
  f29_add(t0, r.X, r.X);
  f29_sub(r.X, r.Z, r.Y);
  f29_add(r.Y, r.Z, r.Y);
  f29_add(r.Z, t0, r.T);
  f29_sub(r.T, t0, r.T);
}

// ------------------------------------------------------------------ kernels
// The starting point and the two cached addends are derived from the lane id; the loop is the
// window; the result is the affine encoding's hash (8 x 32 path for all three).
FE_INLINE void start_points(ge_p2& P, ge_cached& Q1, ge_cached& Q2, uint32_t t) {
  // P = [t+2]B-ish: any valid points serve; build them with the library (8 x 32)
  ge_p3 A, B3;
  ge_p3_identity(A);
  fe_set(A.X, 0);
  // a fixed valid point: the base point's coordinates
  const uint32_t bx[8] = {0x8f25d51au, 0xc9562d60u, 0x9525a7b2u, 0x692cc760u, 0xfdd6dc5cu, 0xc0a4e231u,
                          0xcd6e53feu, 0x216936d3u};
  const uint32_t by[8] = {0x66666658u, 0x66666666u, 0x66666666u, 0x66666666u, 0x66666666u, 0x66666666u,
                          0x66666666u, 0x66666666u};
  fe_const(A.X, bx);
  fe_const(A.Y, by);
  fe_set(A.Z, 1);
  fe_mul(A.T, A.X, A.Y);
  // scramble per lane: a few doublings and additions
  ge_cached cA;
  ge_p3_to_cached(cA, A);
  B3 = A;
  for (uint32_t k = 0; k < (t & 7) + 1; k++) ge_p3_dbl_to_p3(B3, B3);
  ge_p1p1 x;
  ge_add(x, B3, cA);
  ge_p1p1_to_p3(B3, x);
  ge_p3_to_p2(P, B3);
  ge_p3 C = B3;
  ge_p3_dbl_to_p3(C, C);
  ge_p3_to_cached(Q1, C);
  ge_p3_dbl_to_p3(C, C);
  ge_p3_to_cached(Q2, C);
}

FE_INLINE uint32_t hash_point(const fe& X, const fe& Y, const fe& Z) {
  uint32_t s[8];
  ge_tobytes(s, X, Y, Z);
  uint32_t h = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) h = h * 0x9e3779b1u + s[i];
  return h;
}

__global__ void __launch_bounds__(256) k_lib(uint32_t* out) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  ge_p2 P;
  ge_cached Q1, Q2;
  start_points(P, Q1, Q2, t);
  for (int it = 0; it < ITERS; it++) {
    ge_p1p1 x;
    ge_p3 P3;
#pragma unroll 1
    for (int d = 0; d < 3; d++) { ge_p2_dbl(x, P); ge_p1p1_to_p2(P, x); }
    ge_p2_dbl(x, P);
    ge_p1p1_to_p3(P3, x);
    ge_add(x, P3, Q1);
    ge_p1p1_to_p3(P3, x);
    ge_add(x, P3, Q2);
    ge_p1p1_to_p2(P, x);
  }
  out[t] = hash_point(P.X, P.Y, P.Z);
}

__global__ void __launch_bounds__(256) k_f29(uint32_t* out) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  ge_p2 P0;
  ge_cached Q1l, Q2l;
  start_points(P0, Q1l, Q2l, t);
  g29_p2 P;
  g29_cached Q1, Q2;
  f29_from(P.X, P0.X); f29_from(P.Y, P0.Y); f29_from(P.Z, P0.Z);
  f29_from(Q1.YpX, Q1l.YpX); f29_from(Q1.YmX, Q1l.YmX); f29_from(Q1.Z, Q1l.Z); f29_from(Q1.T2d, Q1l.T2d);
  f29_from(Q2.YpX, Q2l.YpX); f29_from(Q2.YmX, Q2l.YmX); f29_from(Q2.Z, Q2l.Z); f29_from(Q2.T2d, Q2l.T2d);
  for (int it = 0; it < ITERS; it++) {
    g29_p1p1 x;
    g29_p3 P3;
#pragma unroll 1
    for (int d = 0; d < 3; d++) { g29_dbl(x, P); g29_p1p1_to_p2(P, x); }
    g29_dbl(x, P);
    g29_p1p1_to_p3(P3, x);
    g29_add(x, P3, Q1);
    g29_p1p1_to_p3(P3, x);
    g29_add(x, P3, Q2);
    g29_p1p1_to_p2(P, x);
  }
  fe X, Y, Z;
  f29_to(X, P.X); f29_to(Y, P.Y); f29_to(Z, P.Z);
  out[t] = hash_point(X, Y, Z);
}

template <int V>
static int run(uint32_t* d, int blocks, float* ms) {
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  for (int rep = 0; rep < 2; rep++) {
    if (rep) CHK(hipEventRecord(e0));
    if (V == 0) hipLaunchKernelGGL(k_lib, dim3(blocks), dim3(256), 0, 0, d);
    else hipLaunchKernelGGL(k_f29, dim3(blocks), dim3(256), 0, 0, d);
    if (rep) CHK(hipEventRecord(e1));
    CHK(hipDeviceSynchronize());
  }
  CHK(hipEventElapsedTime(ms, e0, e1));
  return 0;
}

int main() {
  hipDeviceProp_t p;
  CHK(hipGetDeviceProperties(&p, 0));
  const int ncu = p.multiProcessorCount;
  const char* names[2] = {"lib 8x32", "f29 9x29"};
  uint32_t* d;
  CHK(hipMalloc(&d, (size_t)ncu * 4 * 256 * 4));
  const size_t maxl = (size_t)ncu * 4 * 256;
  uint32_t* h[2];
  for (int v = 0; v < 2; v++) h[v] = new uint32_t[maxl];
  int bad = 0;
  printf("PRAOS_ILP4=%d  one Straus window = 4 doublings + 2 cached additions (+ conversions), %d windows per lane\n",
         PRAOS_ILP4, ITERS);
  for (int W = 1; W <= 4; W++) {
    const int blocks = ncu * W;                 // 256-thread blocks: 4 waves per block, one per SIMD
    const size_t lanes = (size_t)blocks * 256;
    for (int v = 0; v < 2; v++) {
      float ms;
      const int rc = v == 0 ? run<0>(d, blocks, &ms) : run<1>(d, blocks, &ms);
      if (rc) return rc;
      CHK(hipMemcpy(h[v], d, lanes * 4, hipMemcpyDeviceToHost));
      size_t diff = 0;
      if (v > 0)
        for (size_t i = 0; i < lanes; i++) diff += h[v][i] != h[0][i];
      bad += diff != 0;
      printf("W=%d %-12s %8.3f ms  %8.0f SIMD cycles per wave-window (2.4 GHz)  %s\n", W, names[v], ms,
             ms * 1e-3 * 2.4e9 * ncu * 4 / ((double)lanes / 64 * ITERS), v ? (diff ? "MISMATCH" : "== lib") : "");
    }
  }
  return bad ? 2 : 0;
}
