// GF(2^255-19) multiply microbenchmark, round 4: the two product forms the round-3 review
// asked to A/B against the shipped radix-2^32 schoolbook (fe25519.hpp fe_mul).
//   school : radix 2^32, 8 limbs, 64 MACs (v_mad_u64_u32 + s_nop + v_addc per MAC), the shipped form
//   karat  : radix 2^32, one level of subtractive Karatsuba on 4-limb halves: three 4x4 products
//            (48 MACs) + |a0 - a1|, |b0 - b1| with their signs, z1 = z0 + z2 -/+ |.||.|, added at 2^128
//   r29    : 9 x 29-bit limbs (261 bits, weakly reduced), 81 v_mad_u64_u32 into 17 carry-free 64-bit
//            column sums (< 9 * 2^58), one carry pass, the columns >= 9 folded with 2^261 = 1216 (mod p),
//            a second short carry pass
// Every lane runs a dependent chain of ITERS multiplies (x := x * y), like a scalar
// multiplication; the results are converted to canonical bytes on the host and compared.
// Occupancy: --waves W per SIMD (W * 4 blocks of 256 lanes per CU).
// Build: hipcc --offload-arch=gfx950 -O3 -o femul5 femul5.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); return 1; } } while (0)
#define DI __device__ __forceinline__

constexpr int ITERS = 2048;

struct f32 { uint32_t v[8]; };
DI uint32_t addc(uint32_t a, uint32_t b, uint32_t cin, uint32_t* cout) { return __builtin_addc(a, b, cin, cout); }
DI uint32_t subb(uint32_t a, uint32_t b, uint32_t bin, uint32_t* bout) { return __builtin_subc(a, b, bin, bout); }

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

#define MAC(acc, top, a, b) \
  asm("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\ts_nop 1\n\tv_addc_co_u32 %1, vcc, 0, %1, vcc" \
      : "+v"(acc), "+v"(top) : "v"(a), "v"(b) : "vcc")
#define MAC0(acc, top, a, b) \
  asm("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\ts_nop 1\n\tv_cndmask_b32_e64 %1, 0, 1, vcc" \
      : "+v"(acc), "=v"(top) : "v"(a), "v"(b) : "vcc")

// t[0 .. 2N) = a[0 .. N) * b[0 .. N), product scanning
template <int N>
DI void prod(uint32_t* t, const uint32_t* a, const uint32_t* b) {
  uint64_t acc = (uint64_t)a[0] * b[0];
  t[0] = (uint32_t)acc;
  acc >>= 32;
#pragma unroll
  for (int k = 1; k < 2 * N - 1; k++) {
    uint32_t top;
    const int i0 = k < N ? 0 : k - (N - 1);
#pragma unroll
    for (int i = 0; i < N; i++) {
      const int j = k - i;
      if (j < 0 || j > N - 1) continue;
      if (i == i0) MAC0(acc, top, a[i], b[j]);
      else MAC(acc, top, a[i], b[j]);
    }
    t[k] = (uint32_t)acc;
    acc = (acc >> 32) | ((uint64_t)top << 32);
  }
  t[2 * N - 1] = (uint32_t)acc;
}

DI void mul_school(f32& r, const f32& a, const f32& b) {
  uint32_t t[16];
  prod<8>(t, a.v, b.v);
  red512(r, t);
}

// |x - y| of 4-limb halves; returns 1 when x < y
DI uint32_t absdiff4(uint32_t d[4], const uint32_t* x, const uint32_t* y) {
  uint32_t bw = 0;
#pragma unroll
  for (int i = 0; i < 4; i++) d[i] = subb(x[i], y[i], bw, &bw);
  const uint32_t m = 0u - bw;                    // all ones when negative: two's complement negate
  uint32_t c = bw;
#pragma unroll
  for (int i = 0; i < 4; i++) d[i] = addc(d[i] ^ m, 0, c, &c);
  return bw;
}

DI void mul_karat(f32& r, const f32& a, const f32& b) {
  uint32_t z0[8], z2[8], z1[8], da[4], db[4];
  prod<4>(z0, a.v, b.v);
  prod<4>(z2, a.v + 4, b.v + 4);
  const uint32_t sa = absdiff4(da, a.v, a.v + 4), sb = absdiff4(db, b.v, b.v + 4);
  prod<4>(z1, da, db);
  // mid = z0 + z2 - (a0 - a1)(b0 - b1) = z0 + z2 - s * |da||db|, s = +1 when the signs agree
  uint32_t m[9], c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) m[i] = addc(z0[i], z2[i], c, &c);
  m[8] = c;
  const uint32_t neg = sa ^ sb;                  // signs differ: add |da||db|, else subtract it
  const uint32_t mk = neg - 1u;                  // all ones when subtracting
  c = mk & 1u;                                   // subtract = add the complement + 1
#pragma unroll
  for (int i = 0; i < 8; i++) m[i] = addc(m[i], z1[i] ^ mk, c, &c);
  m[8] = addc(m[8], mk, c, &c);                  // (the 9-limb result is non-negative, < 2^257)
  uint32_t t[16];
#pragma unroll
  for (int i = 0; i < 4; i++) t[i] = z0[i];
  c = 0;
#pragma unroll
  for (int i = 4; i < 8; i++) t[i] = addc(z0[i], m[i - 4], c, &c);
#pragma unroll
  for (int i = 8; i < 12; i++) t[i] = addc(z2[i - 8], m[i - 4], c, &c);
  t[12] = addc(z2[4], m[8], c, &c);
#pragma unroll
  for (int i = 13; i < 16; i++) t[i] = addc(z2[i - 8], 0, c, &c);
  red512(r, t);
}

// ---------------------------------------------------------------- 9 x 29-bit limbs
struct f29 { uint32_t v[9]; };
constexpr uint32_t M29 = (1u << 29) - 1;
DI void mul_r29(f29& r, const f29& a, const f29& b) {
  uint64_t t[17];
#pragma unroll
  for (int k = 0; k < 17; k++) {
    uint64_t s = 0;
#pragma unroll
    for (int i = 0; i < 9; i++) {
      const int j = k - i;
      if (j >= 0 && j < 9) s += (uint64_t)a.v[i] * b.v[j];       // v_mad_u64_u32, no carry flag
    }
    t[k] = s;
  }
  // carry pass over the 17 columns: l_k < 2^29, the carry out of column 16 is l_17
  uint32_t l[18];
  uint64_t c = 0;
#pragma unroll
  for (int k = 0; k < 17; k++) {
    const uint64_t s = t[k] + c;
    l[k] = (uint32_t)s & M29;
    c = s >> 29;
  }
  l[17] = (uint32_t)c;                           // < 2^35 does not occur: values < 2^261 keep it < 2^32
  // fold 2^(29 (k + 9)) = 2^(29 k) * 1216 (mod p), second carry pass
  uint64_t d[9];
#pragma unroll
  for (int k = 0; k < 9; k++) d[k] = (uint64_t)l[k + 9] * 1216u + l[k];
  c = 0;
#pragma unroll
  for (int k = 0; k < 9; k++) {
    const uint64_t s = d[k] + c;
    r.v[k] = (uint32_t)s & M29;
    c = s >> 29;
  }
  // carry out of 2^261: < 2^12, times 1216 into limb 0 (a further carry is < 2^29 + 2^23: kept)
  const uint64_t s0 = (uint64_t)r.v[0] + c * 1216u;
  r.v[0] = (uint32_t)s0 & M29;
  r.v[1] += (uint32_t)(s0 >> 29);
}

template <int V>
__global__ void __launch_bounds__(256) kern(uint32_t* out, uint32_t seed) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t xw[8], yw[8];
#pragma unroll
  for (int i = 0; i < 8; i++) { xw[i] = seed * (t + 3 * i + 1); yw[i] = seed ^ (t * 7 + i); }
  xw[7] &= 0x7fffffff; yw[7] &= 0x7fffffff;
  if constexpr (V < 2) {
    f32 x, y;
#pragma unroll
    for (int i = 0; i < 8; i++) { x.v[i] = xw[i]; y.v[i] = yw[i]; }
    for (int it = 0; it < ITERS; it++) {
      if constexpr (V == 0) mul_school(x, x, y);
      else mul_karat(x, x, y);
    }
#pragma unroll
    for (int i = 0; i < 8; i++) out[9 * t + i] = x.v[i];
    out[9 * t + 8] = 0;
  } else {
    f29 x, y;
#pragma unroll
    for (int l = 0; l < 9; l++) {                // split the 255-bit values into 29-bit limbs
      const int b = 29 * l, wi = b / 32, sh = b % 32;
      uint64_t vx = xw[wi] >> sh, vy = yw[wi] >> sh;
      if (wi + 1 < 8) { vx |= (uint64_t)xw[wi + 1] << (32 - sh); vy |= (uint64_t)yw[wi + 1] << (32 - sh); }
      x.v[l] = (uint32_t)vx & M29;
      y.v[l] = (uint32_t)vy & M29;
    }
    for (int it = 0; it < ITERS; it++) mul_r29(x, x, y);
#pragma unroll
    for (int l = 0; l < 9; l++) out[9 * t + l] = x.v[l];
  }
}

// host: value mod p as 8 canonical words
static void canon_words(const uint32_t* raw, int v, uint32_t w[8]) {
  unsigned __int128 acc[10] = {0};
  uint64_t words[10] = {0};
  if (v < 2) {
    for (int i = 0; i < 8; i++) words[i] = raw[i];
  } else {
    for (int l = 0; l < 9; l++) {
      const int b = 29 * l;
      const unsigned __int128 val = (unsigned __int128)raw[l] << (b % 32);
      acc[b / 32] += (uint64_t)val & 0xffffffffu;
      acc[b / 32 + 1] += (uint64_t)(val >> 32);
    }
    unsigned __int128 c = 0;
    for (int k = 0; k < 10; k++) { c += acc[k]; words[k] = (uint32_t)c; c >>= 32; }
  }
  // fold bits >= 255 repeatedly: 2^255 = 19
  for (int rep = 0; rep < 4; rep++) {
    uint64_t top = (words[7] >> 31) | (words[8] << 1) | (words[9] << 33);
    words[7] &= 0x7fffffff; words[8] = words[9] = 0;
    unsigned __int128 c = (unsigned __int128)top * 19;
    for (int i = 0; i < 10; i++) { c += words[i]; words[i] = (uint32_t)c; c >>= 32; }
  }
  uint32_t u[8]; uint64_t c = 19;
  for (int i = 0; i < 8; i++) { c += words[i]; u[i] = (uint32_t)c; c >>= 32; }
  for (int i = 0; i < 8; i++) w[i] = (uint32_t)words[i];
  if (u[7] >> 31) { u[7] &= 0x7fffffff; memcpy(w, u, 32); }
}

template <int V>
static int run(uint32_t* dout, int blocks, double* ms) {
  hipEvent_t e0, e1; CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
  hipLaunchKernelGGL(kern<V>, dim3(blocks), dim3(256), 0, 0, dout, 0x9e3779b9u);
  CHK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int rep = 0; rep < 3; rep++) {
    CHK(hipEventRecord(e0));
    hipLaunchKernelGGL(kern<V>, dim3(blocks), dim3(256), 0, 0, dout, 0x9e3779b9u);
    CHK(hipEventRecord(e1));
    CHK(hipEventSynchronize(e1));
    float t; CHK(hipEventElapsedTime(&t, e0, e1));
    if (t < best) best = t;
  }
  *ms = best;
  return 0;
}

int main(int argc, char** argv) {
  hipDeviceProp_t p; CHK(hipGetDeviceProperties(&p, 0));
  const int ncu = p.multiProcessorCount;
  int waves = 3;
  for (int i = 1; i + 1 < argc; i++) if (!strcmp(argv[i], "--waves")) waves = atoi(argv[i + 1]);
  const int blocks = ncu * 4 * waves;            // 4 SIMDs per CU, one 256-lane block = 4 waves
  const size_t lanes = (size_t)blocks * 256;
  uint32_t* d; CHK(hipMalloc(&d, lanes * 36));
  const char* names[3] = {"radix 2^32 schoolbook, 64 MACs (shipped fe_mul)",
                          "radix 2^32 one-level Karatsuba, 48 MACs + fix-ups",
                          "9 x 29-bit limbs, 81 carry-free MADs + 2 carry passes"};
  uint32_t* h[3];
  double ms[3];
  uint32_t* raw = new uint32_t[lanes * 9];
  for (int v = 0; v < 3; v++) {
    int rc = v == 0 ? run<0>(d, blocks, &ms[v]) : v == 1 ? run<1>(d, blocks, &ms[v]) : run<2>(d, blocks, &ms[v]);
    if (rc) return rc;
    CHK(hipMemcpy(raw, d, lanes * 36, hipMemcpyDeviceToHost));
    h[v] = new uint32_t[lanes * 8];
    for (size_t i = 0; i < lanes; i++) canon_words(raw + 9 * i, v, h[v] + 8 * i);
    const double muls = (double)lanes * ITERS;
    printf("%-56s %8.3f ms  %7.2f G mul/s  %6.1f SIMD cycles per wave-mul (%d waves/SIMD, 2.4 GHz, %d CUs)\n",
           names[v], ms[v], muls / ms[v] / 1e6, ms[v] * 1e-3 * 2.4e9 * ncu * 4 / (muls / 64), waves, ncu);
  }
  size_t bad = 0;
  for (size_t i = 0; i < lanes * 8; i++) bad += (h[0][i] != h[1][i]) + (h[0][i] != h[2][i]);
  printf("results equal mod p across variants: %s (%zu word mismatches)\n", bad ? "NO" : "yes", bad);
  printf("speed vs schoolbook: karatsuba %.3fx, 9x29 %.3fx\n", ms[0] / ms[1], ms[0] / ms[2]);
  return bad ? 2 : 0;
}
