// fe25519.hpp product forms A/B: build with -DPRAOS_MACG=0 (FE_MAC / FE_MAC2, s_nop padded) and
// -DPRAOS_MACG=1 (fe_cols.hpp, software-pipelined columns), run both, compare the checksums.
//   mul  : x = x*y            (fe_mul, one product)
//   sq   : x = x^2            (fe_sq)
//   mul2 : x = x*y, z = z*y   (fe_mul2, two products interleaved)
//   sq2  : x = x^2, z = z^2   (fe_sq2)
//   addsub: two fe_add + two fe_sub, dependent (per "product" read: per add / sub)
// at 1..4 waves per SIMD (blocks of 4 waves, CUs x W blocks).
// Build: hipcc --offload-arch=gfx950 -O3 -I../../ouroboros-consensus_amd/csrc -DPRAOS_MACG=1 -o femul6_g femul6.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include "fe25519.hpp"

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); return 1; } } while (0)

constexpr int ITERS = 1024;

template <int V>
__global__ void __launch_bounds__(256) kern(uint32_t* out, uint32_t seed) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  fe x, z, y;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    x.v[i] = seed * (t + 3 * i + 1);
    z.v[i] = seed * (t + 5 * i + 2);
    y.v[i] = seed ^ (t * 7 + i);
  }
  for (int it = 0; it < ITERS; it++) {
    if constexpr (V == 0) fe_mul(x, x, y);
    else if constexpr (V == 1) fe_sq(x, x);
    else if constexpr (V == 2) fe_mul2(x, x, y, z, z, y);
    else if constexpr (V == 3) fe_sq2(x, x, z, z);
    else {
      fe_add(x, x, y);
      fe_sub(z, z, x);
      fe_add(y, y, z);
      fe_sub(x, x, z);
    }
  }
  uint32_t h = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) h = h * 0x9e3779b1u + x.v[i] + 7u * z.v[i];
  out[t] = h;
}

template <int V>
static int run(uint32_t* d, int blocks, float* ms) {
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  hipLaunchKernelGGL(kern<V>, dim3(blocks), dim3(256), 0, 0, d, 0x9e3779b9u);
  CHK(hipDeviceSynchronize());
  CHK(hipEventRecord(e0));
  hipLaunchKernelGGL(kern<V>, dim3(blocks), dim3(256), 0, 0, d, 0x9e3779b9u);
  CHK(hipEventRecord(e1));
  CHK(hipEventSynchronize(e1));
  CHK(hipEventElapsedTime(ms, e0, e1));
  return 0;
}

int main() {
  hipDeviceProp_t p;
  CHK(hipGetDeviceProperties(&p, 0));
  const int ncu = p.multiProcessorCount;
  const char* names[5] = {"fe_mul", "fe_sq", "fe_mul2", "fe_sq2", "addsub"};
  uint32_t* d;
  CHK(hipMalloc(&d, (size_t)ncu * 4 * 256 * 4));
  uint32_t* h = new uint32_t[(size_t)ncu * 4 * 256];
  printf("PRAOS_MACG=%d\n", PRAOS_MACG);
  for (int W = 1; W <= 4; W++) {
    const int blocks = ncu * W;
    const size_t lanes = (size_t)blocks * 256;
    for (int v = 0; v < 5; v++) {
      float ms;
      int rc = v == 0   ? run<0>(d, blocks, &ms)
               : v == 1 ? run<1>(d, blocks, &ms)
               : v == 2 ? run<2>(d, blocks, &ms)
               : v == 3 ? run<3>(d, blocks, &ms)
                        : run<4>(d, blocks, &ms);
      if (rc) return rc;
      CHK(hipMemcpy(h, d, lanes * 4, hipMemcpyDeviceToHost));
      uint64_t sum = 0;
      for (size_t i = 0; i < lanes; i++) sum = sum * 1000003u + h[i];
      const double products = (double)lanes * ITERS * (v == 4 ? 4 : v >= 2 ? 2 : 1);
      printf("W=%d %-8s %8.3f ms  %7.1f SIMD cycles per wave-product (2.4 GHz)  checksum %016llx\n", W, names[v], ms,
             ms * 1e-3 * 2.4e9 * ncu * 4 / (products / 64), (unsigned long long)sum);
    }
  }
  CHK(hipFree(d));
  return 0;
}
