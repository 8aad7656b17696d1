// Field-multiply latency / ILP microbenchmark for gfx950.
//
// Question: is the per-lane GF(2^255-19) multiply (fe25519.hpp: one serial
// chain of 64 x {v_mad_u64_u32, s_nop 1, v_addc_co_u32}) issue-bound or
// latency-bound at the occupancy the verify kernels run at (3 waves/SIMD)?
//   single : x = x*y, the kernel's fe_mul, one chain per lane
//   seq2   : two chains per lane, fe_mul twice (the asm blocks serialise on VCC)
//   ilp2   : two chains interleaved MAC by MAC, carries in two SGPR pairs,
//            s_nop 0 between the two mads and the two addcs
//   ilp2n  : the same without the s_nop (hazard probe: results must still agree)
// Each is run at 1, 2, 3, 4 waves per SIMD (blocks of 4 waves, ncu * W blocks).
// Build: hipcc --offload-arch=gfx950 -O3 -o femul2 femul2.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstring>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); return 1; } } while (0)
#define DI __device__ __forceinline__

constexpr int ITERS = 1024;

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
#define MAC_ASM(acc, top, a, b) \
  asm("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\ts_nop 1\n\tv_addc_co_u32 %1, vcc, 0, %1, vcc" \
      : "+v"(acc), "+v"(top) : "v"(a), "v"(b) : "vcc")
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
      MAC_ASM(acc, top, a.v[i], b.v[j]);
    }
    t[k] = (uint32_t)acc;
    acc = (acc >> 32) | ((uint64_t)top << 32);
  }
  t[15] = (uint32_t)acc;
  red512(r, t);
}

// two MACs of independent products, carries in compiler-chosen SGPR pairs
#define MAC2_NOP(acc1, top1, a1, b1, acc2, top2, a2, b2)                                         \
  do {                                                                                          \
    uint64_t c1_, c2_;                                                                          \
    asm("v_mad_u64_u32 %0, %4, %6, %7, %0\n\t"                                                  \
        "v_mad_u64_u32 %1, %5, %8, %9, %1\n\t"                                                  \
        "s_nop 0\n\t"                                                                           \
        "v_addc_co_u32 %2, %4, 0, %2, %4\n\t"                                                   \
        "v_addc_co_u32 %3, %5, 0, %3, %5"                                                       \
        : "+v"(acc1), "+v"(acc2), "+v"(top1), "+v"(top2), "=&s"(c1_), "=&s"(c2_)                \
        : "v"(a1), "v"(b1), "v"(a2), "v"(b2));                                                  \
  } while (0)
#define MAC2_RAW(acc1, top1, a1, b1, acc2, top2, a2, b2)                                         \
  do {                                                                                          \
    uint64_t c1_, c2_;                                                                          \
    asm("v_mad_u64_u32 %0, %4, %6, %7, %0\n\t"                                                  \
        "v_mad_u64_u32 %1, %5, %8, %9, %1\n\t"                                                  \
        "v_addc_co_u32 %2, %4, 0, %2, %4\n\t"                                                   \
        "v_addc_co_u32 %3, %5, 0, %3, %5"                                                       \
        : "+v"(acc1), "+v"(acc2), "+v"(top1), "+v"(top2), "=&s"(c1_), "=&s"(c2_)                \
        : "v"(a1), "v"(b1), "v"(a2), "v"(b2));                                                  \
  } while (0)

template <bool NOP>
DI void mul2(f32& r1, const f32& a1, const f32& b1, f32& r2, const f32& a2, const f32& b2) {
  uint32_t t1[16], t2[16];
  uint64_t acc1 = (uint64_t)a1.v[0] * b1.v[0], acc2 = (uint64_t)a2.v[0] * b2.v[0];
  t1[0] = (uint32_t)acc1; t2[0] = (uint32_t)acc2;
  acc1 >>= 32; acc2 >>= 32;
#pragma unroll
  for (int k = 1; k < 15; k++) {
    uint32_t top1 = 0, top2 = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const int j = k - i;
      if (j < 0 || j > 7) continue;
      if constexpr (NOP) MAC2_NOP(acc1, top1, a1.v[i], b1.v[j], acc2, top2, a2.v[i], b2.v[j]);
      else MAC2_RAW(acc1, top1, a1.v[i], b1.v[j], acc2, top2, a2.v[i], b2.v[j]);
    }
    t1[k] = (uint32_t)acc1; t2[k] = (uint32_t)acc2;
    acc1 = (acc1 >> 32) | ((uint64_t)top1 << 32);
    acc2 = (acc2 >> 32) | ((uint64_t)top2 << 32);
  }
  t1[15] = (uint32_t)acc1; t2[15] = (uint32_t)acc2;
  red512(r1, t1);
  red512(r2, t2);
}

// V: 0 single (1 chain), 1 seq2, 2 ilp2, 3 ilp2n
template <int V>
__global__ void __launch_bounds__(256) kern(uint32_t* out, uint32_t seed) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  f32 x, z, y;
#pragma unroll
  for (int i = 0; i < 8; i++) { x.v[i] = seed * (t + 3 * i + 1); z.v[i] = seed * (t + 5 * i + 2); y.v[i] = seed ^ (t * 7 + i); }
  x.v[7] &= 0x7fffffff; z.v[7] &= 0x7fffffff; y.v[7] &= 0x7fffffff;
  for (int it = 0; it < ITERS; it++) {
    if constexpr (V == 0) {
      mul1(x, x, y);
    } else if constexpr (V == 1) {
      mul1(x, x, y);
      mul1(z, z, y);
    } else {
      mul2<V == 2>(x, x, y, z, z, y);
    }
  }
#pragma unroll
  for (int i = 0; i < 8; i++) { out[16 * t + i] = x.v[i]; out[16 * t + 8 + i] = V == 0 ? 0u : z.v[i]; }
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
  const char* names[4] = {"single chain (fe_mul)", "two chains, sequential fe_mul", "two chains interleaved + s_nop 0",
                          "two chains interleaved, no s_nop"};
  const int maxblocks = ncu * 4;
  const size_t maxlanes = (size_t)maxblocks * 256;
  uint32_t* d; CHK(hipMalloc(&d, maxlanes * 64));
  uint32_t* ref = new uint32_t[maxlanes * 16];
  uint32_t* got = new uint32_t[maxlanes * 16];
  int bad_total = 0;
  for (int W = 1; W <= 4; W++) {
    const int blocks = ncu * W;
    const size_t lanes = (size_t)blocks * 256;
    for (int v = 0; v < 4; v++) {
      double ms;
      int rc = v == 0 ? run<0>(d, blocks, &ms) : v == 1 ? run<1>(d, blocks, &ms) : v == 2 ? run<2>(d, blocks, &ms)
                                                                                          : run<3>(d, blocks, &ms);
      if (rc) return rc;
      CHK(hipMemcpy(got, d, lanes * 64, hipMemcpyDeviceToHost));
      for (size_t i = 0; i < lanes * 2; i++) canon(got + 8 * i);
      size_t bad = 0;
      if (v == 1) memcpy(ref, got, lanes * 64);
      if (v >= 2) for (size_t i = 0; i < lanes * 16; i++) bad += got[i] != ref[i];
      if (v == 0) for (size_t i = 0; i < lanes; i++) bad += memcmp(got + 16 * i, got + 16 * i, 32) != 0;
      bad_total += bad != 0;
      const double muls = (double)lanes * ITERS * (v == 0 ? 1 : 2);
      printf("W=%d waves/SIMD  %-36s %8.3f ms  %7.2f G mul/s  %6.1f SIMD cycles per wave-mul (2.4 GHz)  %s\n", W,
             names[v], ms, muls / ms / 1e6, ms * 1e-3 * 2.4e9 * ncu * 4 / (muls / 64),
             v >= 2 ? (bad ? "MISMATCH vs seq2" : "== seq2") : "");
    }
  }
  CHK(hipFree(d));
  return bad_total ? 2 : 0;
}
