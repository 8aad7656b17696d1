// Field-multiply ILP microbenchmark, 4 interleaved products (gfx950).
//
// Question (small batches, round 3): a 54k-header shard is < 1 wave per SIMD, so every
// verify chain runs latency-bound.  How much faster is one wave when four independent
// products (a group formula's multiplications come in independent groups of 3-4) are
// interleaved MAC by MAC, each with its carry in its own SGPR pair, than with the two-way
// interleave (fe_mul2) the kernels use?
//   ilp1 : one chain (fe_mul), ilp2 : two interleaved (fe_mul2), ilp4 : four interleaved
// Run at 1, 2, 3 waves per SIMD.  Build: hipcc --offload-arch=gfx950 -O3 -o femul4 femul4.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstring>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); return 1; } } while (0)
#define DI __device__ __forceinline__

constexpr int ITERS = 512;

struct f32 { uint32_t v[8]; };
DI uint32_t addc(uint32_t a, uint32_t b, uint32_t cin, uint32_t* cout) { return __builtin_addc(a, b, cin, cout); }
DI void red512(f32& r, const uint32_t t[16]) {
  uint64_t s[8];
#pragma unroll
  for (int i = 0; i < 8; i++) s[i] = (uint64_t)t[8 + i] * 38u + t[i];
  uint32_t c = 0;
  r.v[0] = (uint32_t)s[0];
#pragma unroll
  for (int i = 1; i < 8; i++) r.v[i] = addc((uint32_t)s[i], (uint32_t)(s[i - 1] >> 32), c, &c);
  uint32_t k = (uint32_t)(s[7] >> 32) + c;
  uint64_t s0 = (uint64_t)k * 38u + r.v[0];
  r.v[0] = (uint32_t)s0;
  c = (uint32_t)(s0 >> 32);
#pragma unroll
  for (int i = 1; i < 8; i++) r.v[i] = addc(r.v[i], 0, c, &c);
  r.v[0] += 38u * c;
}
#define MAC1(acc, top, a, b) \
  asm("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\ts_nop 1\n\tv_addc_co_u32 %1, vcc, 0, %1, vcc" \
      : "+v"(acc), "+v"(top) : "v"(a), "v"(b) : "vcc")
#define MAC2(acc1, top1, a1, b1, acc2, top2, a2, b2)                                           \
  do {                                                                                        \
    uint64_t c1_, c2_;                                                                        \
    asm("v_mad_u64_u32 %0, %4, %6, %7, %0\n\tv_mad_u64_u32 %1, %5, %8, %9, %1\n\ts_nop 0\n\t"   \
        "v_addc_co_u32 %2, %4, 0, %2, %4\n\tv_addc_co_u32 %3, %5, 0, %3, %5"                   \
        : "+v"(acc1), "+v"(acc2), "+v"(top1), "+v"(top2), "=&s"(c1_), "=&s"(c2_)              \
        : "v"(a1), "v"(b1), "v"(a2), "v"(b2));                                                \
  } while (0)
// four mads, then the four carry adds: every carry is read >= 3 instructions after its write
#define MAC4(A, T, a, b, k)                                                                     \
  do {                                                                                        \
    uint64_t c0_, c1_, c2_, c3_;                                                              \
    asm("v_mad_u64_u32 %0, %8, %12, %13, %0\n\tv_mad_u64_u32 %1, %9, %14, %15, %1\n\t"          \
        "v_mad_u64_u32 %2, %10, %16, %17, %2\n\tv_mad_u64_u32 %3, %11, %18, %19, %3\n\t"        \
        "v_addc_co_u32 %4, %8, 0, %4, %8\n\tv_addc_co_u32 %5, %9, 0, %5, %9\n\t"                \
        "v_addc_co_u32 %6, %10, 0, %6, %10\n\tv_addc_co_u32 %7, %11, 0, %7, %11"               \
        : "+v"(A[0]), "+v"(A[1]), "+v"(A[2]), "+v"(A[3]), "+v"(T[0]), "+v"(T[1]), "+v"(T[2]), \
          "+v"(T[3]), "=&s"(c0_), "=&s"(c1_), "=&s"(c2_), "=&s"(c3_)                          \
        : "v"(a[0]), "v"(b[0]), "v"(a[1]), "v"(b[1]), "v"(a[2]), "v"(b[2]), "v"(a[3]), "v"(b[3])); \
  } while (0)

DI void mul1(f32& r, const f32& a, const f32& b) {
  uint32_t t[16];
  uint64_t acc = (uint64_t)a.v[0] * b.v[0];
  t[0] = (uint32_t)acc;
  acc >>= 32;
#pragma unroll
  for (int k = 1; k < 15; k++) {
    uint32_t top = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const int j = k - i;
      if (j < 0 || j > 7) continue;
      MAC1(acc, top, a.v[i], b.v[j]);
    }
    t[k] = (uint32_t)acc;
    acc = (acc >> 32) | ((uint64_t)top << 32);
  }
  t[15] = (uint32_t)acc;
  red512(r, t);
}

template <int N>
DI void mulN(f32* r, const f32* a, const f32* b) {
  uint32_t t[N][16];
  uint64_t acc[N];
#pragma unroll
  for (int q = 0; q < N; q++) {
    acc[q] = (uint64_t)a[q].v[0] * b[q].v[0];
    t[q][0] = (uint32_t)acc[q];
    acc[q] >>= 32;
  }
#pragma unroll
  for (int k = 1; k < 15; k++) {
    uint32_t top[N];
#pragma unroll
    for (int q = 0; q < N; q++) top[q] = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const int j = k - i;
      if (j < 0 || j > 7) continue;
      if constexpr (N == 2) {
        MAC2(acc[0], top[0], a[0].v[i], b[0].v[j], acc[1], top[1], a[1].v[i], b[1].v[j]);
      } else {
        const uint32_t av[4] = {a[0].v[i], a[1].v[i], a[2].v[i], a[3].v[i]};
        const uint32_t bv[4] = {b[0].v[j], b[1].v[j], b[2].v[j], b[3].v[j]};
        MAC4(acc, top, av, bv, 0);
      }
    }
#pragma unroll
    for (int q = 0; q < N; q++) {
      t[q][k] = (uint32_t)acc[q];
      acc[q] = (acc[q] >> 32) | ((uint64_t)top[q] << 32);
    }
  }
#pragma unroll
  for (int q = 0; q < N; q++) {
    t[q][15] = (uint32_t)acc[q];
    red512(r[q], t[q]);
  }
}

// V: 0 ilp1 (4 chains, one after the other), 1 ilp2 (2 x 2), 2 ilp4
template <int V>
__global__ void __launch_bounds__(256) kern(uint32_t* out, uint32_t seed) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  f32 x[4], y;
#pragma unroll
  for (int q = 0; q < 4; q++)
#pragma unroll
    for (int i = 0; i < 8; i++) x[q].v[i] = seed * (t + (3 + 2 * q) * i + q + 1);
#pragma unroll
  for (int i = 0; i < 8; i++) y.v[i] = seed ^ (t * 7 + i);
#pragma unroll
  for (int q = 0; q < 4; q++) x[q].v[7] &= 0x7fffffff;
  y.v[7] &= 0x7fffffff;
  const f32 yy[4] = {y, y, y, y};
  for (int it = 0; it < ITERS; it++) {
    if constexpr (V == 0) {
#pragma unroll
      for (int q = 0; q < 4; q++) mul1(x[q], x[q], y);
    } else if constexpr (V == 1) {
      mulN<2>(x, x, yy);
      mulN<2>(x + 2, x + 2, yy);
    } else {
      mulN<4>(x, x, yy);
    }
  }
#pragma unroll
  for (int q = 0; q < 4; q++)
#pragma unroll
    for (int i = 0; i < 8; i++) out[32 * t + 8 * q + i] = x[q].v[i];
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

template <int V>
static int run(uint32_t* dout, int blocks, double* ms) {
  hipEvent_t e0, e1; CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
  hipLaunchKernelGGL(kern<V>, dim3(blocks), dim3(256), 0, 0, dout, 0x9e3779b9u);
  CHK(hipDeviceSynchronize());
  CHK(hipEventRecord(e0));
  hipLaunchKernelGGL(kern<V>, dim3(blocks), dim3(256), 0, 0, dout, 0x9e3779b9u);
  CHK(hipEventRecord(e1));
  CHK(hipEventSynchronize(e1));
  float t; CHK(hipEventElapsedTime(&t, e0, e1)); *ms = t;
  return 0;
}

int main() {
  hipDeviceProp_t p; CHK(hipGetDeviceProperties(&p, 0));
  const int ncu = p.multiProcessorCount;
  const char* names[3] = {"ilp1: one chain at a time", "ilp2: two interleaved", "ilp4: four interleaved"};
  const size_t maxlanes = (size_t)ncu * 3 * 256;
  uint32_t* d; CHK(hipMalloc(&d, maxlanes * 128));
  uint32_t* ref = new uint32_t[maxlanes * 32];
  uint32_t* got = new uint32_t[maxlanes * 32];
  int bad_total = 0;
  for (int W = 1; W <= 3; W++) {
    const int blocks = ncu * W;
    const size_t lanes = (size_t)blocks * 256;
    for (int v = 0; v < 3; v++) {
      double ms;
      int rc = v == 0 ? run<0>(d, blocks, &ms) : v == 1 ? run<1>(d, blocks, &ms) : run<2>(d, blocks, &ms);
      if (rc) return rc;
      CHK(hipMemcpy(got, d, lanes * 128, hipMemcpyDeviceToHost));
      for (size_t i = 0; i < lanes * 4; i++) canon(got + 8 * i);
      size_t bad = 0;
      if (v == 0) memcpy(ref, got, lanes * 128);
      else for (size_t i = 0; i < lanes * 32; i++) bad += got[i] != ref[i];
      bad_total += bad != 0;
      const double muls = (double)lanes * ITERS * 4;
      printf("W=%d waves/SIMD  %-28s %8.3f ms  %7.2f G mul/s  %6.1f SIMD cycles per wave-mul (2.4 GHz)  %s\n", W,
             names[v], ms, muls / ms / 1e6, ms * 1e-3 * 2.4e9 * ncu * 4 / (muls / 64),
             v ? (bad ? "MISMATCH vs ilp1" : "== ilp1") : "");
    }
  }
  CHK(hipFree(d));
  return bad_total ? 2 : 0;
}
