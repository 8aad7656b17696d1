// Integer-VALU issue-rate microbenchmark for gfx950 (MI355X).
//
// Purpose: pick the GF(2^255-19) limb representation from MEASURED rates of
// the candidate multiply instructions (v_mad_u64_u32, v_mul_lo/hi_u32,
// 24-bit forms) against plain 32-bit adds.  Each thread runs 8 independent
// dependency chains of one instruction so issue rate, not latency, is timed.
//
// Build: hipcc --offload-arch=gfx950 -O3 -o intrate intrate.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); return 1; } } while (0)

constexpr int ITERS = 4096;

enum Op { ADD_U32, MAD_U64_U32, MUL_LO_U32, MUL_HI_U32, MAD_U32_U24, MUL_HI_U32_U24,
          ADD_CO_U32, ADDC_CO_U32, FMA_F64, ADD3_U32, LSHL_ADD, ALIGNBIT, MAD_U64_U32_DEP, NOPS };
static const char* names[] = {"v_add_u32", "v_mad_u64_u32", "v_mul_lo_u32", "v_mul_hi_u32",
  "v_mad_u32_u24", "v_mul_hi_u32_u24", "v_add_co_u32", "v_add_co+v_addc_co (pair)", "v_fma_f64",
  "v_add3_u32", "v_lshl_add_u32", "v_alignbit_b32", "v_mad_u64_u32 (1 chain, latency)"};

template <int OP>
__global__ void __launch_bounds__(256) kern(uint32_t* out, uint32_t seed) {
  uint32_t a = seed ^ threadIdx.x, b = seed * 7 + blockIdx.x;
  uint32_t x[8]; uint64_t y[8]; double d[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) { x[k] = a + k; y[k] = (uint64_t)(b + k) << 3; d[k] = (double)(a + k); }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if constexpr (OP == ADD_U32) asm volatile("v_add_u32 %0, %1, %0" : "+v"(x[k]) : "v"(a));
      if constexpr (OP == MAD_U64_U32) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(y[k]) : "v"(a), "v"(b) : "vcc");
      if constexpr (OP == MUL_LO_U32) asm volatile("v_mul_lo_u32 %0, %1, %0" : "+v"(x[k]) : "v"(a));
      if constexpr (OP == MUL_HI_U32) asm volatile("v_mul_hi_u32 %0, %1, %0" : "+v"(x[k]) : "v"(a));
      if constexpr (OP == MAD_U32_U24) asm volatile("v_mad_u32_u24 %0, %1, %2, %0" : "+v"(x[k]) : "v"(a), "v"(b));
      if constexpr (OP == MUL_HI_U32_U24) asm volatile("v_mul_hi_u32_u24 %0, %1, %0" : "+v"(x[k]) : "v"(a));
      if constexpr (OP == ADD_CO_U32) asm volatile("v_add_co_u32 %0, vcc, %1, %0" : "+v"(x[k]) : "v"(a) : "vcc");
      if constexpr (OP == ADDC_CO_U32) asm volatile("v_add_co_u32 %0, vcc, %1, %0\n\tv_addc_co_u32 %0, vcc, %1, %0, vcc" : "+v"(x[k]) : "v"(a) : "vcc");
      if constexpr (OP == FMA_F64) asm volatile("v_fma_f64 %0, %1, %2, %0" : "+v"(d[k]) : "v"(d[(k + 1) & 7]), "v"(d[(k + 2) & 7]));
      if constexpr (OP == ADD3_U32) asm volatile("v_add3_u32 %0, %1, %2, %0" : "+v"(x[k]) : "v"(a), "v"(b));
      if constexpr (OP == LSHL_ADD) asm volatile("v_lshl_add_u32 %0, %1, 3, %0" : "+v"(x[k]) : "v"(a));
      if constexpr (OP == ALIGNBIT) asm volatile("v_alignbit_b32 %0, %1, %0, 7" : "+v"(x[k]) : "v"(a));
      if constexpr (OP == MAD_U64_U32_DEP) { if (k == 0) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(y[0]) : "v"(a), "v"(b) : "vcc"); }
    }
  }
  uint32_t acc = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) acc += x[k] + (uint32_t)y[k] + (uint32_t)(y[k] >> 32) + (uint32_t)d[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <int OP>
static int run(uint32_t* dout, int blocks, double clk_ghz, int ncu) {
  hipEvent_t e0, e1; CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
  hipLaunchKernelGGL(kern<OP>, dim3(blocks), dim3(256), 0, 0, dout, 1u);  // warm
  CHK(hipDeviceSynchronize());
  CHK(hipEventRecord(e0));
  for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(kern<OP>, dim3(blocks), dim3(256), 0, 0, dout, 1u + r);
  CHK(hipEventRecord(e1)); CHK(hipEventSynchronize(e1));
  float ms; CHK(hipEventElapsedTime(&ms, e0, e1));
  double per = (OP == MAD_U64_U32_DEP) ? 1.0 : 8.0;
  double instr = 3.0 * blocks * 256.0 * ITERS * per;   // lane-instructions
  double rate = instr / (ms * 1e-3);                    // lane-instr/s
  double per_cu_clk = rate / (ncu * clk_ghz * 1e9);
  printf("%-34s %8.3f ms  %10.2f T lane-instr/s  %7.2f lane-instr/clk/CU  (%.2f cyc per wave64-instr per SIMD)\n",
         names[OP], ms / 3, rate / 1e12, per_cu_clk, 4.0 * 64.0 / per_cu_clk);
  return 0;
}

int main() {
  hipDeviceProp_t p; CHK(hipGetDeviceProperties(&p, 0));
  int ncu = p.multiProcessorCount; double clk = p.clockRate / 1e6;
  printf("device %s  CUs=%d  clock=%.3f GHz\n", p.gcnArchName, ncu, clk);
  uint32_t* d; int blocks = ncu * 8; CHK(hipMalloc(&d, blocks * 256 * 4));
  run<ADD_U32>(d, blocks, clk, ncu); run<MAD_U64_U32>(d, blocks, clk, ncu); run<MUL_LO_U32>(d, blocks, clk, ncu);
  run<MUL_HI_U32>(d, blocks, clk, ncu); run<MAD_U32_U24>(d, blocks, clk, ncu); run<MUL_HI_U32_U24>(d, blocks, clk, ncu);
  run<ADD_CO_U32>(d, blocks, clk, ncu); run<ADDC_CO_U32>(d, blocks, clk, ncu); run<FMA_F64>(d, blocks, clk, ncu);
  run<ADD3_U32>(d, blocks, clk, ncu); run<LSHL_ADD>(d, blocks, clk, ncu); run<ALIGNBIT>(d, blocks, clk, ncu);
  run<MAD_U64_U32_DEP>(d, blocks, clk, ncu);
  CHK(hipFree(d));
  return 0;
}
