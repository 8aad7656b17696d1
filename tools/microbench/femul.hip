// GF(2^255-19) multiply microbenchmark for gfx950: which limb layout and MAC
// form the per-lane field arithmetic should use.
//   r32asm : radix 2^32, 8 limbs, product scanning, MAC = v_mad_u64_u32 + s_nop + v_addc (fe25519.hpp)
//   r32c   : radix 2^32, the same schedule with the carries left to the compiler (__builtin_addc)
//   r26    : radix 2^25.5, 10 limbs, 100 v_mad_u64_u32 into 10 independent 64-bit column sums
//            (no carry flags), one carry pass
//   r32col : radix 2^32, one asm block per column (fe_col.hpp): the MACs' carries in
//            separate SGPR pairs, counted after the column, no s_nop per MAC
// Each lane runs a dependent chain of multiplies (like a scalar-multiplication
// chain); results are compared across variants mod p.
// Build: hipcc --offload-arch=gfx950 -O3 -o femul femul.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include "fe_col.hpp"
#include <cstdio>
#include <cstring>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); return 1; } } while (0)
#define DI __device__ __forceinline__

constexpr int ITERS = 2048;

// ---------------------------------------------------------------- radix 2^32
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
template <bool ASM>
DI void mul32(f32& r, const f32& a, const f32& b) {
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
      if constexpr (ASM) {
        MAC_ASM(acc, top, a.v[i], b.v[j]);
      } else {
        const uint64_t p = (uint64_t)a.v[i] * b.v[j];
        uint32_t c1, c2;
        const uint32_t lo = addc((uint32_t)acc, (uint32_t)p, 0, &c1);
        const uint32_t hi = addc((uint32_t)(acc >> 32), (uint32_t)(p >> 32), c1, &c2);
        acc = ((uint64_t)hi << 32) | lo;
        top += c2;
      }
    }
    t[k] = (uint32_t)acc;
    acc = (acc >> 32) | ((uint64_t)top << 32);
  }
  t[15] = (uint32_t)acc;
  red512(r, t);
}

template <int M>
DI void col_dispatch(uint64_t& acc, uint32_t& top, const uint32_t* x, const uint32_t* y) { FeCol<M>::mac(acc, top, x, y); }

DI void mul32col(f32& r, const f32& a, const f32& b) {
  uint32_t t[16];
  uint64_t acc = (uint64_t)a.v[0] * b.v[0];
  t[0] = (uint32_t)acc;
  acc >>= 32;
#pragma unroll
  for (int k = 1; k < 15; k++) {
    uint32_t top = 0, x[8], y[8];
    int m = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const int j = k - i;
      if (j < 0 || j > 7) continue;
      x[m] = a.v[i];
      y[m] = b.v[j];
      m++;
    }
    switch (m) {
      case 1: col_dispatch<1>(acc, top, x, y); break;
      case 2: col_dispatch<2>(acc, top, x, y); break;
      case 3: col_dispatch<3>(acc, top, x, y); break;
      case 4: col_dispatch<4>(acc, top, x, y); break;
      case 5: col_dispatch<5>(acc, top, x, y); break;
      case 6: col_dispatch<6>(acc, top, x, y); break;
      case 7: col_dispatch<7>(acc, top, x, y); break;
      default: col_dispatch<8>(acc, top, x, y); break;
    }
    t[k] = (uint32_t)acc;
    acc = (acc >> 32) | ((uint64_t)top << 32);
  }
  t[15] = (uint32_t)acc;
  red512(r, t);
}

// ---------------------------------------------------------------- radix 2^25.5
// limbs: even i 26 bits, odd i 25 bits; value = sum f_i 2^ceil(25.5 i)
struct f26 { uint32_t v[10]; };
DI void carry26(f26& r, uint64_t h[10]) {
  uint64_t c;
  c = h[0] >> 26; h[1] += c; h[0] &= 0x3ffffff;
  c = h[4] >> 26; h[5] += c; h[4] &= 0x3ffffff;
  c = h[1] >> 25; h[2] += c; h[1] &= 0x1ffffff;
  c = h[5] >> 25; h[6] += c; h[5] &= 0x1ffffff;
  c = h[2] >> 26; h[3] += c; h[2] &= 0x3ffffff;
  c = h[6] >> 26; h[7] += c; h[6] &= 0x3ffffff;
  c = h[3] >> 25; h[4] += c; h[3] &= 0x1ffffff;
  c = h[7] >> 25; h[8] += c; h[7] &= 0x1ffffff;
  c = h[4] >> 26; h[5] += c; h[4] &= 0x3ffffff;
  c = h[8] >> 26; h[9] += c; h[8] &= 0x3ffffff;
  c = h[9] >> 25; h[0] += c * 19; h[9] &= 0x1ffffff;
  c = h[0] >> 26; h[1] += c; h[0] &= 0x3ffffff;
#pragma unroll
  for (int i = 0; i < 10; i++) r.v[i] = (uint32_t)h[i];
}
DI void mul26(f26& r, const f26& f, const f26& g) {
  uint32_t g19[10], f2[10];
#pragma unroll
  for (int i = 0; i < 10; i++) { g19[i] = 19u * g.v[i]; f2[i] = (i & 1) ? 2u * f.v[i] : f.v[i]; }
  uint64_t h[10];
#pragma unroll
  for (int k = 0; k < 10; k++) {
    uint64_t s = 0;
#pragma unroll
    for (int i = 0; i < 10; i++) {
      const int j = k - i;
      // odd i and odd j: the product sits one bit above limb k's position
      if (j >= 0) s += (uint64_t)((i & 1) && (j & 1) ? f2[i] : f.v[i]) * g.v[j];
      else s += (uint64_t)((i & 1) && ((j + 10) & 1) ? f2[i] : f.v[i]) * g19[j + 10];
    }
    h[k] = s;
  }
  carry26(r, h);
}

// ---------------------------------------------------------------- kernels
template <int V>
__global__ void __launch_bounds__(256) kern(uint32_t* out, uint32_t seed) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if constexpr (V < 2 || V == 3) {
    f32 x, y;
#pragma unroll
    for (int i = 0; i < 8; i++) { x.v[i] = seed * (t + 3 * i + 1); y.v[i] = seed ^ (t * 7 + i); }
    x.v[7] &= 0x7fffffff; y.v[7] &= 0x7fffffff;
    for (int it = 0; it < ITERS; it++) {
      if constexpr (V == 3) mul32col(x, x, y);
      else mul32<V == 0>(x, x, y);
    }
#pragma unroll
    for (int i = 0; i < 8; i++) out[10 * t + i] = x.v[i];
  } else {
    f26 x, y;
    // same field values as the 2^32 variant: split the 255-bit numbers
    uint32_t xw[8], yw[8];
#pragma unroll
    for (int i = 0; i < 8; i++) { xw[i] = seed * (t + 3 * i + 1); yw[i] = seed ^ (t * 7 + i); }
    xw[7] &= 0x7fffffff; yw[7] &= 0x7fffffff;
    const int pos[10] = {0, 26, 51, 77, 102, 128, 153, 179, 204, 230};
#pragma unroll
    for (int l = 0; l < 10; l++) {
      const int w = (l & 1) ? 25 : 26;
      uint64_t vx = 0, vy = 0;
      const int b = pos[l], wi = b / 32, sh = b % 32;
      vx = xw[wi] >> sh; vy = yw[wi] >> sh;
      if (wi + 1 < 8 && sh + w > 32) { vx |= (uint64_t)xw[wi + 1] << (32 - sh); vy |= (uint64_t)yw[wi + 1] << (32 - sh); }
      x.v[l] = (uint32_t)(vx & ((1u << w) - 1)); y.v[l] = (uint32_t)(vy & ((1u << w) - 1));
    }
    for (int it = 0; it < ITERS; it++) mul26(x, x, y);
#pragma unroll
    for (int l = 0; l < 10; l++) out[10 * t + l] = x.v[l];
  }
}

static void canon(uint32_t w[8]) {   // reduce a < 2^256 value mod p (host)
  for (int rep = 0; rep < 3; rep++) {
    uint64_t top = w[7] >> 31;
    w[7] &= 0x7fffffff;
    uint64_t c = top * 19;
    for (int i = 0; i < 8; i++) { c += w[i]; w[i] = (uint32_t)c; c >>= 32; }
  }
  // subtract p if >= p
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
  const int blocks = ncu * 16;              // 16 waves / CU = 4 per SIMD
  const size_t lanes = (size_t)blocks * 256;
  uint32_t* d; CHK(hipMalloc(&d, lanes * 40));
  uint32_t* h[4];
  const char* names[4] = {"radix 2^32, asm MAC (v_mad_u64_u32 + s_nop + v_addc)", "radix 2^32, compiler carries",
                          "radix 2^25.5, 100 MACs into 10 column sums",
                          "radix 2^32, column asm blocks (carries in SGPR pairs)"};
  double ms[4];
  for (int v = 0; v < 4; v++) {
    h[v] = new uint32_t[lanes * 8];
    int rc = v == 0 ? run<0>(d, blocks, &ms[v]) : v == 1 ? run<1>(d, blocks, &ms[v]) :
             v == 2 ? run<2>(d, blocks, &ms[v]) : run<3>(d, blocks, &ms[v]);
    if (rc) return rc;
    uint32_t* raw = new uint32_t[lanes * 10];
    CHK(hipMemcpy(raw, d, lanes * 40, hipMemcpyDeviceToHost));
    for (size_t i = 0; i < lanes; i++) {
      uint32_t* w = h[v] + 8 * i;
      if (v != 2) { memcpy(w, raw + 10 * i, 32); }
      else {   // sum limb_l * 2^pos_l into 9 words with carries
        static const int pos[10] = {0, 26, 51, 77, 102, 128, 153, 179, 204, 230};
        uint64_t acc[9] = {0};
        for (int l = 0; l < 10; l++) {
          const unsigned __int128 val = (unsigned __int128)raw[10 * i + l] << (pos[l] % 32);
          int wi = pos[l] / 32;
          unsigned __int128 c = val;
          for (int k = wi; k < 9 && c; k++) { c += acc[k]; acc[k] = (uint32_t)c; c >>= 32; }
        }
        uint64_t c = acc[8] * 38;        // 2^256 = 38 mod p
        for (int k = 0; k < 8; k++) { c += acc[k]; w[k] = (uint32_t)c; c >>= 32; }
        c *= 38;
        for (int k = 0; k < 8 && c; k++) { c += w[k]; w[k] = (uint32_t)c; c >>= 32; }
      }
      canon(w);
    }
    delete[] raw;
    const double muls = (double)lanes * ITERS;
    printf("%-58s %8.3f ms  %7.2f G mul/s  %6.1f SIMD cycles per wave-mul (at 2.4 GHz, %d CUs)\n", names[v], ms[v],
           muls / ms[v] / 1e6, ms[v] * 1e-3 * 2.4e9 * ncu * 4 / (muls / 64), ncu);
  }
  size_t bad = 0;
  for (size_t i = 0; i < lanes * 8; i++) bad += (h[0][i] != h[1][i]) + (h[0][i] != h[2][i]) + (h[0][i] != h[3][i]);
  printf("results equal mod p across variants: %s (%zu word mismatches)\n", bad ? "NO" : "yes", bad);
  return bad ? 2 : 0;
}
