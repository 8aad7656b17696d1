// Point-doubling chains, one lane per point vs a 4-lane group per point, on gfx950.
//
// Question (DESIGN.md section 8, strong scaling): stage V of a 54k-header shard is
// latency-bound (one wave per SIMD, each lane a ~250-doubling chain).  Splitting a
// point's doubling over a quad of lanes -- X^2, Y^2, Z^2, (X+Y)^2 on lanes 0..3, then
// X3 = E F, Y3 = G H, Z3 = F G on lanes 0..2, the operands exchanged with DPP quad
// permutes -- does ~1.7x the instructions but fills 4x the waves.  Which is faster for
// 252 doublings at 54k and at 432k points?
//   single : the kernels' ge_p2_dbl + ge_p1p1_to_p2 (ILP-2 squarings / products)
//   quad   : the 4-lane form; every lane of the quad ends with the full (X3, Y3, Z3)
//   pair   : a 2-lane form (two squarings and up to two products per lane, ILP-2)
// Both must give the same point.
// Build: hipcc --offload-arch=gfx950 -O3 -I../../ouroboros-consensus_amd/csrc -o dbl4lane dbl4lane.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstring>

#include "ge25519.hpp"

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); return 1; } } while (0)

constexpr int DBLS = 252;

__device__ __forceinline__ void start_point(ge_p2& P, uint32_t t) {
  // any projective (X : Y : Z) works for a doubling-chain timing and equality check
#pragma unroll
  for (int i = 0; i < 8; i++) {
    P.X.v[i] = 0x9e3779b9u * (t + 3 * i + 1);
    P.Y.v[i] = 0x85ebca6bu ^ (t * 7 + i);
    P.Z.v[i] = i == 0 ? 1u + (t & 0xff) : 0u;
  }
  P.X.v[7] &= 0x7fffffffu;
  P.Y.v[7] &= 0x7fffffffu;
}

__global__ void __launch_bounds__(256) k_single(uint32_t* out, size_t n) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  ge_p2 P;
  start_point(P, (uint32_t)t);
  ge_p1p1 x;
#pragma clang loop unroll(disable)
  for (int k = 0; k < DBLS; k++) {
    ge_p2_dbl(x, P);
    ge_p1p1_to_p2(P, x);
  }
#pragma unroll
  for (int i = 0; i < 8; i++) {
    out[24 * t + i] = P.X.v[i];
    out[24 * t + 8 + i] = P.Y.v[i];
    out[24 * t + 16 + i] = P.Z.v[i];
  }
}

// all lanes of the quad read lane k's value
template <int K>
__device__ __forceinline__ uint32_t quad_bcast(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, K | (K << 2) | (K << 4) | (K << 6), 0xf, 0xf, false);
}
template <int K>
__device__ __forceinline__ void fe_bcast(fe& r, const fe& a) {
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = quad_bcast<K>(a.v[i]);
}
__device__ __forceinline__ void fe_sel(fe& r, bool c, const fe& a, const fe& b) {
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = c ? a.v[i] : b.v[i];
}

__global__ void __launch_bounds__(256) k_quad(uint32_t* out, size_t n) {
  const size_t g = (size_t)blockIdx.x * blockDim.x + threadIdx.x;   // lane; point = g / 4
  const size_t t = g >> 2;
  const int q = (int)(threadIdx.x & 3);
  // 4 n lanes = whole quads; lanes past them run on dummy points and write nothing
  ge_p2 P;
  start_point(P, (uint32_t)t);
  fe in, s, A, B, C, T0, rX, rY, rZ, rT, a, b, p;
#pragma clang loop unroll(disable)
  for (int k = 0; k < DBLS; k++) {
    fe_add(T0, P.X, P.Y);
    fe_sel(in, q == 0, P.X, P.Y);
    fe_sel(in, q < 2, in, P.Z);
    fe_sel(in, q < 3, in, T0);
    fe_sq(s, in);                                     // X^2 | Y^2 | Z^2 | (X+Y)^2
    fe_bcast<0>(A, s);
    fe_bcast<1>(B, s);
    fe_bcast<2>(C, s);
    fe_bcast<3>(T0, s);
    fe_add(rY, B, A);                                 // as ge_p2_dbl: p1p1 (rX, rY, rZ, rT)
    fe_sub(rZ, B, A);
    fe_sub(rX, T0, rY);
    fe_add(rT, C, C);
    fe_sub(rT, rT, rZ);
    fe_sel(a, q == 1, rY, rX);                        // X3 = rX rT | Y3 = rY rZ | Z3 = rZ rT
    fe_sel(a, q == 2, rZ, a);
    fe_sel(b, q == 1, rZ, rT);
    fe_mul(p, a, b);
    fe_bcast<0>(P.X, p);
    fe_bcast<1>(P.Y, p);
    fe_bcast<2>(P.Z, p);
  }
  if (g < 4 * n && q == 0) {
#pragma unroll
    for (int i = 0; i < 8; i++) {
      out[24 * t + i] = P.X.v[i];
      out[24 * t + 8 + i] = P.Y.v[i];
      out[24 * t + 16 + i] = P.Z.v[i];
    }
  }
}


// lanes 2j, 2j+1 read lane K of their pair (DPP quad_perm inside the quad: pairs (0,1), (2,3))
template <int K>
__device__ __forceinline__ uint32_t pair_bcast(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, K | (K << 2) | ((2 + K) << 4) | ((2 + K) << 6), 0xf, 0xf, false);
}
template <int K>
__device__ __forceinline__ void fe_pbcast(fe& r, const fe& a) {
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = pair_bcast<K>(a.v[i]);
}

// 2-lane form: lane 0 of the pair squares X, Y and forms X3, Y3; lane 1 squares Z, X+Y and
// forms Z3 (its second product slot idle)
__global__ void __launch_bounds__(256) k_pair(uint32_t* out, size_t n) {
  const size_t g = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t t = g >> 1;
  const int q = (int)(threadIdx.x & 1);
  ge_p2 P;
  start_point(P, (uint32_t)t);
  fe i1, i2, s1, s2, A, B, C, T0, rX, rY, rZ, rT, a1, b1, a2, b2, p1, p2;
#pragma clang loop unroll(disable)
  for (int k = 0; k < DBLS; k++) {
    fe_add(T0, P.X, P.Y);
    fe_sel(i1, q == 0, P.X, P.Z);
    fe_sel(i2, q == 0, P.Y, T0);
    fe_sq2(s1, i1, s2, i2);                            // lane 0: X^2, Y^2 | lane 1: Z^2, (X+Y)^2
    fe_pbcast<0>(A, s1);
    fe_pbcast<0>(B, s2);
    fe_pbcast<1>(C, s1);
    fe_pbcast<1>(T0, s2);
    fe_add(rY, B, A);
    fe_sub(rZ, B, A);
    fe_sub(rX, T0, rY);
    fe_add(rT, C, C);
    fe_sub(rT, rT, rZ);
    fe_sel(a1, q == 0, rX, rZ);                        // lane 0: X3 = rX rT, Y3 = rY rZ | lane 1: Z3 = rZ rT
    fe_sel(a2, q == 0, rY, rZ);
    fe_sel(b2, q == 0, rZ, rT);
    fe_mul2(p1, a1, rT, p2, a2, b2);
    fe_pbcast<0>(P.X, p1);
    fe_pbcast<0>(P.Y, p2);
    fe_pbcast<1>(P.Z, p1);
  }
  if (g < 2 * n && q == 0) {
#pragma unroll
    for (int i = 0; i < 8; i++) {
      out[24 * t + i] = P.X.v[i];
      out[24 * t + 8 + i] = P.Y.v[i];
      out[24 * t + 16 + i] = P.Z.v[i];
    }
  }
}

static void canon(uint32_t w[8]) {
  for (int rep = 0; rep < 3; rep++) {
    uint64_t top = w[7] >> 31;
    w[7] &= 0x7fffffff;
    uint64_t c = top * 19;
    for (int i = 0; i < 8; i++) { c += w[i]; w[i] = (uint32_t)c; c >>= 32; }
  }
  uint32_t u[8]; uint64_t c = 19;
  for (int i = 0; i < 8; i++) { c += w[i]; u[i] = (uint32_t)c; c >>= 32; }
  if (u[7] >> 31) { u[7] &= 0x7fffffff; memcpy(w, u, 32); }
}

int main() {
  const size_t sizes[3] = {54000, 108000, 432000};
  const size_t maxn = 432000;
  uint32_t* d; CHK(hipMalloc(&d, maxn * 96));
  uint32_t* a = new uint32_t[maxn * 24];
  uint32_t* b = new uint32_t[maxn * 24];
  hipEvent_t e0, e1; CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
  int bad_total = 0;
  for (size_t n : sizes) {
    float ms[3];
    uint32_t* c = new uint32_t[n * 24];
    for (int v = 0; v < 3; v++) {
      const size_t lanes = v == 1 ? 4 * n : v == 2 ? 2 * n : n;
      const unsigned blocks = (unsigned)((lanes + 255) / 256);
      for (int rep = 0; rep < 2; rep++) {
        CHK(hipEventRecord(e0));
        if (v == 1) hipLaunchKernelGGL(k_quad, dim3(blocks), dim3(256), 0, 0, d, n);
        else if (v == 2) hipLaunchKernelGGL(k_pair, dim3(blocks), dim3(256), 0, 0, d, n);
        else hipLaunchKernelGGL(k_single, dim3(blocks), dim3(256), 0, 0, d, n);
        CHK(hipEventRecord(e1));
        CHK(hipEventSynchronize(e1));
        CHK(hipEventElapsedTime(&ms[v], e0, e1));
      }
      CHK(hipMemcpy(v == 1 ? b : v == 2 ? c : a, d, n * 96, hipMemcpyDeviceToHost));
    }
    // compare projective points: X_a Z_b == X_b Z_a etc. is needless here -- the same formulas
    // in the same order give the same representatives up to the final reduction
    size_t bad = 0;
    for (size_t i = 0; i < n * 3; i++) {
      canon(a + 8 * i); canon(b + 8 * i); canon(c + 8 * i);
      bad += memcmp(a + 8 * i, b + 8 * i, 32) != 0 || memcmp(a + 8 * i, c + 8 * i, 32) != 0;
    }
    delete[] c;
    bad_total += bad != 0;
    printf("%7zu points x %d doublings: one lane %7.3f ms (%5zu waves)   2-lane pair %7.3f ms (%5zu waves, %.2f)"
           "   4-lane quad %7.3f ms (%5zu waves, %.2f)  %s\n",
           n, DBLS, ms[0], (n + 63) / 64, ms[2], (2 * n + 63) / 64, ms[2] / ms[0], ms[1], (4 * n + 63) / 64,
           ms[1] / ms[0], bad ? "MISMATCH" : "equal");
  }
  CHK(hipFree(d));
  return bad_total ? 2 : 0;
}
