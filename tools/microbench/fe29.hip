// Prototype: GF(2^255-19) products in 9 limbs of 29 bits (every column sum fits 64 bits, so a
// MAC is one v_mad_u64_u32 with no carry add) against fe25519.hpp's 8 x 32-bit products.
// Reports SIMD cycles per product at 1..4 waves per SIMD and checks the results equal
// (converted back to 8 x 32 and canonicalised).  Not used by the library.
// Build: hipcc --offload-arch=gfx950 -O3 -I../../ouroboros-consensus_amd/csrc -o fe29 fe29.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include "fe25519.hpp"

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); return 1; } } while (0)

constexpr int ITERS = 1024;
constexpr uint32_t M29 = (1u << 29) - 1;

struct f29 { uint32_t v[9]; };

FE_INLINE void to29(f29& r, const fe& a) {       // a < 2^256 -> 9 x 29 (value < 2^261)
#pragma unroll
  for (int k = 0; k < 9; k++) {
    const int bit = 29 * k, w = bit >> 5, s = bit & 31;
    uint64_t x = a.v[w];
    if (w + 1 < 8) x |= (uint64_t)a.v[w + 1] << 32;
    r.v[k] = (uint32_t)(x >> s) & M29;
  }
}
FE_INLINE void from29(fe& r, const f29& a) {     // limbs < 2^29 assumed after a carry pass
  // value may be up to 2^261: fold bits >= 255 (times 19) while packing
  uint32_t w[9] = {0};
  uint64_t acc = 0;
  int nb = 0, o = 0;
#pragma unroll
  for (int k = 0; k < 9; k++) {
    acc |= (uint64_t)a.v[k] << nb;
    nb += 29;
    while (nb >= 32) { w[o++] = (uint32_t)acc; acc >>= 32; nb -= 32; }
  }
  w[o] = (uint32_t)acc;                            // o == 8: bits 256..260
  fe t;
#pragma unroll
  for (int i = 0; i < 8; i++) t.v[i] = w[i];
  // + w[8] * 2^256 = w[8] * 38
  uint32_t c = 0;
  t.v[0] = addc(t.v[0], w[8] * 38u, 0, &c);
#pragma unroll
  for (int i = 1; i < 8; i++) t.v[i] = addc(t.v[i], 0, c, &c);
  t.v[0] += 38u * c;
  r = t;
}

// carry pass + fold of T_k (k < 9) with T_k < 2^41: limbs < 2^29 except limb 0 < 2^29 + 2^23
FE_INLINE void carry29(f29& r, const uint64_t (&T)[9]) {
  uint64_t c = 0;
#pragma unroll
  for (int k = 0; k < 9; k++) {
    const uint64_t u = T[k] + c;
    r.v[k] = (uint32_t)u & M29;
    c = u >> 29;
  }
  // c at 2^261 = 2^6 * 2^255 = 64 * 19 = 1216
  const uint64_t u0 = (uint64_t)r.v[0] + c * 1216u;
  r.v[0] = (uint32_t)u0 & M29;
  r.v[1] += (uint32_t)(u0 >> 29);
}

FE_INLINE void fe29_mul(f29& r, const f29& a, const f29& b) {
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
  carry29(r, T);
}

FE_INLINE void fe29_sq(f29& r, const f29& a) {
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
  carry29(r, T);
}

template <int V>
__global__ void __launch_bounds__(256) kern(uint32_t* out, uint32_t seed) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  fe x, y;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    x.v[i] = seed * (t + 3 * i + 1);
    y.v[i] = seed ^ (t * 7 + i);
  }
  if constexpr (V == 0) {
    for (int it = 0; it < ITERS; it++) fe_mul(x, x, y);
  } else if constexpr (V == 1) {
    for (int it = 0; it < ITERS; it++) fe_sq(x, x);
  } else {
    f29 a, b;
    to29(a, x);
    to29(b, y);
    for (int it = 0; it < ITERS; it++) {
      if constexpr (V == 2) fe29_mul(a, a, b);
      else fe29_sq(a, a);
    }
    from29(x, a);
  }
  fe c;
  fe_canon(c, x);
  uint32_t h = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) h = h * 0x9e3779b1u + c.v[i];
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
  const char* names[4] = {"fe_mul 8x32", "fe_sq 8x32", "fe29_mul", "fe29_sq"};
  uint32_t* d;
  CHK(hipMalloc(&d, (size_t)ncu * 4 * 256 * 4));
  const size_t maxl = (size_t)ncu * 4 * 256;
  uint32_t* h[4];
  for (int v = 0; v < 4; v++) h[v] = new uint32_t[maxl];
  int bad = 0;
  for (int W = 1; W <= 4; W++) {
    const int blocks = ncu * W;
    const size_t lanes = (size_t)blocks * 256;
    for (int v = 0; v < 4; v++) {
      float ms;
      int rc = v == 0 ? run<0>(d, blocks, &ms) : v == 1 ? run<1>(d, blocks, &ms) : v == 2 ? run<2>(d, blocks, &ms)
                                                                                          : run<3>(d, blocks, &ms);
      if (rc) return rc;
      CHK(hipMemcpy(h[v], d, lanes * 4, hipMemcpyDeviceToHost));
      size_t diff = 0;
      if (v >= 2)
        for (size_t i = 0; i < lanes; i++) diff += h[v][i] != h[v - 2][i];
      bad += diff != 0;
      printf("W=%d %-12s %8.3f ms  %7.1f SIMD cycles per wave-product (2.4 GHz)  %s\n", W, names[v], ms,
             ms * 1e-3 * 2.4e9 * ncu * 4 / ((double)lanes * ITERS / 64), v >= 2 ? (diff ? "MISMATCH" : "== 8x32") : "");
    }
  }
  return bad ? 2 : 0;
}
