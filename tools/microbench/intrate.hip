// Integer-VALU issue-cost table for gfx950 (MI355X), by waves per SIMD.
//
// Round 5 rewrite of the round-1 probe (profiles/r01_intrate_microbench.txt), which ran 8
// waves per SIMD off the wall clock and could not separate issue cost from latency.  Here:
//   * W = 1, 2, 3, 4 waves per SIMD: blocks of 256 lanes (one wave per SIMD of a CU), W x CUs
//     blocks; every wave records its SIMD (HW_ID, XCC_ID) and its shader-clock start / end,
//     and the host groups waves by SIMD, so a SIMD's cost is measured on the waves that
//     actually shared it (cycles from the first start to the last end / instructions issued
//     there) and SIMDs holding another count than W are reported, not mixed in;
//   * C = 8 independent chains per wave (16 for the multiplies: one wave alone then shows
//     its issue cost, not the latency of one chain);
//   * the carry-writing forms both through VCC (one register shared by every chain, as
//     FE_MAC in csrc/fe25519.hpp) and through an SGPR pair per chain (as FE_MAC2's second
//     product), and the MAC sequences the field multiply is made of.
// The figure that matters is "SIMD cycles per wave64 instruction": 2 = the guide's VALU peak
// (32 lanes / clk per SIMD), which the 78.6 T int32 ops/s roofline peak assumes.
//
// Build: hipcc --offload-arch=gfx950 -O3 -o intrate intrate.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <map>
#include <vector>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); exit(1); } } while (0)

constexpr int ITERS = 512;     // x REP x C instructions per wave
constexpr int REP = 4;

enum Op {
  ADD_U32, ADD3_U32, LSHL_ADD, CNDMASK, MAD_VCC, MAD_SGPR, MAD_SGPR_DISTINCT, MUL_LO, MUL_HI, MAD_U24, MUL_U24,
  MUL_HI_U24, ADD_CO_VCC, ADD_CO_SGPR, ADDC_SGPR, ADDC_VCC_SERIAL, FMA_F64, MAC_FE, MAC2_FE, MAC_SGPR_NONOP, NOPS
};
struct OpInfo { const char* name; int chains; int valu_per_op; const char* note; };
static const OpInfo ops[NOPS] = {
  {"v_add_u32", 8, 1, "VOP2"},
  {"v_add3_u32", 8, 1, "VOP3, 3 sources"},
  {"v_lshl_add_u32", 8, 1, "VOP3"},
  {"v_cndmask_b32_e64", 8, 1, "VOP3, SGPR-pair mask (the MAC0 carry read)"},
  {"v_mad_u64_u32 (carry -> vcc)", 16, 1, "every chain writes VCC (FE_MAC)"},
  {"v_mad_u64_u32 (carry -> own sgpr)", 16, 1, "SGPR pair per chain"},
  {"v_mad_u64_u32 (distinct a,b)", 16, 1, "per-chain multiplicands, SGPR carry (a field product's MACs)"},
  {"v_mul_lo_u32", 16, 1, ""},
  {"v_mul_hi_u32", 16, 1, ""},
  {"v_mad_u32_u24", 16, 1, "VOP3"},
  {"v_mul_u32_u24", 16, 1, "VOP2"},
  {"v_mul_hi_u32_u24", 16, 1, "VOP2"},
  {"v_add_co_u32 (carry -> vcc)", 8, 1, "VOP2, every chain writes VCC"},
  {"v_add_co_u32 (carry -> own sgpr)", 8, 1, "VOP3b"},
  {"v_addc_co_u32 (own sgpr carry)", 8, 1, "VOP3b, carry in/out an SGPR pair per chain"},
  {"v_addc_co_u32 (one vcc chain)", 1, 1, "serial through VCC + s_nop 1: carry-chain latency"},
  {"v_fma_f64", 8, 1, "for scale"},
  {"MAC = mad(vcc) + s_nop 1 + addc(vcc)", 8, 2, "FE_MAC as shipped, per MAC"},
  {"MAC2 = 2 mad + s_nop 0 + 2 addc", 4, 4, "FE_MAC2 as shipped (vcc + sgpr), per pair"},
  {"MAC, sgpr carries, no nop", 8, 2, "mad(own sgpr) + addc(own sgpr), 8 MACs interleaved"},
};

constexpr int chains_of(int op) {
  return (op >= MAD_VCC && op <= MUL_HI_U24) ? 16 : (op == ADDC_VCC_SERIAL ? 1 : (op == MAC2_FE ? 4 : 8));
}

template <int OP>
__global__ void __launch_bounds__(256) kern(uint32_t* out, unsigned long long* rec, uint32_t seed) {
  const uint32_t a = seed ^ threadIdx.x, b = seed * 7u + blockIdx.x;
  constexpr int C = chains_of(OP);
  uint32_t x[16], top[16], av[16], bv[16];
  uint64_t y[16], cs[16];
  double d[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    x[k] = a + k; top[k] = b ^ k; av[k] = a * (k + 3); bv[k] = b * (k + 5);
    y[k] = (uint64_t)(b + k) << 3; cs[k] = 0; d[k] = (double)(a + k);
  }
  const uint64_t mask = (uint64_t)b * 0x9E3779B97F4A7C15ull;
  __syncthreads();
  const unsigned long long t0 = clock64(), r0 = wall_clock64();
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int r = 0; r < REP; ++r) {
#pragma unroll
      for (int k = 0; k < C; ++k) {
        if constexpr (OP == ADD_U32) asm volatile("v_add_u32 %0, %1, %0" : "+v"(x[k]) : "v"(a));
        if constexpr (OP == ADD3_U32) asm volatile("v_add3_u32 %0, %1, %2, %0" : "+v"(x[k]) : "v"(a), "v"(b));
        if constexpr (OP == LSHL_ADD) asm volatile("v_lshl_add_u32 %0, %1, 3, %0" : "+v"(x[k]) : "v"(a));
        if constexpr (OP == CNDMASK) asm volatile("v_cndmask_b32_e64 %0, %1, %0, %2" : "+v"(x[k]) : "v"(a), "s"(mask));
        if constexpr (OP == MAD_VCC)
          asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(y[k]) : "v"(a), "v"(b) : "vcc");
        if constexpr (OP == MAD_SGPR)
          asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(y[k]), "+s"(cs[k]) : "v"(a), "v"(b));
        if constexpr (OP == MAD_SGPR_DISTINCT)
          asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(y[k]), "+s"(cs[k]) : "v"(av[k]), "v"(bv[(k + 3) & 15]));
        if constexpr (OP == MUL_LO) asm volatile("v_mul_lo_u32 %0, %1, %0" : "+v"(x[k]) : "v"(a));
        if constexpr (OP == MUL_HI) asm volatile("v_mul_hi_u32 %0, %1, %0" : "+v"(x[k]) : "v"(a));
        if constexpr (OP == MAD_U24) asm volatile("v_mad_u32_u24 %0, %1, %2, %0" : "+v"(x[k]) : "v"(a), "v"(b));
        if constexpr (OP == MUL_U24) asm volatile("v_mul_u32_u24 %0, %1, %0" : "+v"(x[k]) : "v"(a));
        if constexpr (OP == MUL_HI_U24) asm volatile("v_mul_hi_u32_u24 %0, %1, %0" : "+v"(x[k]) : "v"(a));
        if constexpr (OP == ADD_CO_VCC) asm volatile("v_add_co_u32 %0, vcc, %1, %0" : "+v"(x[k]) : "v"(a) : "vcc");
        if constexpr (OP == ADD_CO_SGPR)
          asm volatile("v_add_co_u32 %0, %1, %2, %0" : "+v"(x[k]), "+s"(cs[k]) : "v"(a));
        if constexpr (OP == ADDC_SGPR)
          asm volatile("v_addc_co_u32 %0, %1, %2, %0, %1" : "+v"(x[k]), "+s"(cs[k]) : "v"(a));
        if constexpr (OP == ADDC_VCC_SERIAL)
          asm volatile("v_addc_co_u32 %0, vcc, %1, %0, vcc\n\ts_nop 1" : "+v"(x[0]) : "v"(a) : "vcc");
        if constexpr (OP == FMA_F64) asm volatile("v_fma_f64 %0, %1, %2, %0" : "+v"(d[k]) : "v"(d[(k + 1) & 15]), "v"(d[(k + 2) & 15]));
        if constexpr (OP == MAC_FE)
          asm volatile("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\ts_nop 1\n\tv_addc_co_u32 %1, vcc, 0, %1, vcc"
                       : "+v"(y[k]), "+v"(top[k]) : "v"(av[k]), "v"(bv[(k + 3) & 15]) : "vcc");
        if constexpr (OP == MAC2_FE) {
          uint64_t c2;
          asm volatile("v_mad_u64_u32 %0, vcc, %5, %6, %0\n\tv_mad_u64_u32 %1, %4, %7, %8, %1\n\ts_nop 0\n\t"
                       "v_addc_co_u32 %2, vcc, 0, %2, vcc\n\tv_addc_co_u32 %3, %4, 0, %3, %4"
                       : "+v"(y[2 * k]), "+v"(y[2 * k + 1]), "+v"(top[2 * k]), "+v"(top[2 * k + 1]), "=&s"(c2)
                       : "v"(av[k]), "v"(bv[k]), "v"(av[k + 4]), "v"(bv[k + 4]) : "vcc");
        }
        if constexpr (OP == MAC_SGPR_NONOP)   // mad k writes cs[k]; addc k reads it 7 VALU later
          asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(y[k]), "=s"(cs[k]) : "v"(av[k]), "v"(bv[(k + 3) & 15]));
      }
      if constexpr (OP == MAC_SGPR_NONOP) {
#pragma unroll
        for (int k = 0; k < C; ++k)
          asm volatile("v_addc_co_u32 %0, %1, 0, %0, %1" : "+v"(top[k]), "+s"(cs[k]));
      }
    }
  }
  const unsigned long long t1 = clock64(), r1 = wall_clock64();
  uint32_t acc = 0;
#pragma unroll
  for (int k = 0; k < 16; ++k) acc += x[k] + top[k] + (uint32_t)y[k] + (uint32_t)(y[k] >> 32) + (uint32_t)cs[k] + (uint32_t)d[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
  if ((threadIdx.x & 63) == 0) {
    const uint32_t hw = __builtin_amdgcn_s_getreg(GETREG_IMMED(31, 0, 4));      // HW_ID
    const uint32_t xcc = __builtin_amdgcn_s_getreg(GETREG_IMMED(3, 0, 20));     // XCC_ID
    const size_t w = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    rec[4 * w + 0] = t0;
    rec[4 * w + 1] = t1;
    rec[4 * w + 2] = ((unsigned long long)xcc << 32) | (hw & 0x7F30u);         // SIMD, CU, SH, SE
    rec[4 * w + 3] = r1 - r0;
  }
}

struct Row { double cpi_med, cpi_min, cpi_max, ghz; int simds, simds_other; };

template <int OP>
static Row run(int ncu, int W, uint32_t* dout, unsigned long long* drec) {
  const int blocks = ncu * W;
  hipLaunchKernelGGL(kern<OP>, dim3(blocks), dim3(256), 0, 0, dout, drec, 1u);     // warm
  CHK(hipDeviceSynchronize());
  hipLaunchKernelGGL(kern<OP>, dim3(blocks), dim3(256), 0, 0, dout, drec, 2u);
  CHK(hipDeviceSynchronize());
  std::vector<unsigned long long> rec(4 * (size_t)blocks * 4);
  CHK(hipMemcpy(rec.data(), drec, rec.size() * 8, hipMemcpyDeviceToHost));
  constexpr int C = chains_of(OP);
  const double per_wave = (double)ITERS * REP * C * ops[OP].valu_per_op;     // VALU instructions per wave
  struct S { unsigned long long t0 = ~0ull, t1 = 0; int waves = 0; double ghz = 0; };
  std::map<unsigned long long, S> simd;
  for (size_t w = 0; w < rec.size() / 4; ++w) {
    S& s = simd[rec[4 * w + 2]];
    s.t0 = std::min(s.t0, rec[4 * w + 0]);
    s.t1 = std::max(s.t1, rec[4 * w + 1]);
    s.waves++;
    s.ghz = (double)(rec[4 * w + 1] - rec[4 * w + 0]) / (rec[4 * w + 3] * 10.0);   // wall clock: 100 MHz
  }
  std::vector<double> cpi;
  double ghz = 0;
  int other = 0;
  for (auto& [k, s] : simd) {
    if (s.waves != W) { other++; continue; }
    cpi.push_back((double)(s.t1 - s.t0) / (per_wave * W));
    ghz += s.ghz;
  }
  std::sort(cpi.begin(), cpi.end());
  Row r{};
  r.simds = (int)cpi.size();
  r.simds_other = other;
  if (!cpi.empty()) {
    r.cpi_med = cpi[cpi.size() / 2];
    r.cpi_min = cpi.front();
    r.cpi_max = cpi.back();
    r.ghz = ghz / cpi.size();
  }
  return r;
}

template <int OP>
static void table_row(int ncu, uint32_t* dout, unsigned long long* drec) {
  Row r[4];
  for (int W = 1; W <= 4; ++W) r[W - 1] = run<OP>(ncu, W, dout, drec);
  printf("%-38s C=%-2d", ops[OP].name, chains_of(OP));
  for (int W = 0; W < 4; ++W) printf(" | %6.2f", r[W].cpi_med);
  printf(" | ");
  for (int W = 0; W < 4; ++W) printf("%d/%d ", r[W].simds, r[W].simds_other);
  printf("| %.2f GHz | %s\n", r[2].ghz, ops[OP].note);
  fflush(stdout);
}

int main() {
  hipDeviceProp_t p;
  CHK(hipGetDeviceProperties(&p, 0));
  const int ncu = p.multiProcessorCount;
  printf("device %s  CUs=%d  clockRate=%.3f GHz\n", p.gcnArchName, ncu, p.clockRate / 1e6);
  printf("SIMD cycles per wave64 VALU instruction (median over SIMDs holding exactly W waves; s_nop not counted)\n");
  printf("%-38s %-4s | %6s | %6s | %6s | %6s | SIMDs used/other per W | clock | note\n", "op", "", "W=1", "W=2", "W=3",
         "W=4");
  uint32_t* dout;
  unsigned long long* drec;
  CHK(hipMalloc(&dout, (size_t)ncu * 4 * 256 * 4));
  CHK(hipMalloc(&drec, (size_t)ncu * 4 * 4 * 4 * 8));
  table_row<ADD_U32>(ncu, dout, drec);
  table_row<ADD3_U32>(ncu, dout, drec);
  table_row<LSHL_ADD>(ncu, dout, drec);
  table_row<CNDMASK>(ncu, dout, drec);
  table_row<MAD_VCC>(ncu, dout, drec);
  table_row<MAD_SGPR>(ncu, dout, drec);
  table_row<MAD_SGPR_DISTINCT>(ncu, dout, drec);
  table_row<MUL_LO>(ncu, dout, drec);
  table_row<MUL_HI>(ncu, dout, drec);
  table_row<MAD_U24>(ncu, dout, drec);
  table_row<MUL_U24>(ncu, dout, drec);
  table_row<MUL_HI_U24>(ncu, dout, drec);
  table_row<ADD_CO_VCC>(ncu, dout, drec);
  table_row<ADD_CO_SGPR>(ncu, dout, drec);
  table_row<ADDC_SGPR>(ncu, dout, drec);
  table_row<ADDC_VCC_SERIAL>(ncu, dout, drec);
  table_row<FMA_F64>(ncu, dout, drec);
  table_row<MAC_FE>(ncu, dout, drec);
  table_row<MAC2_FE>(ncu, dout, drec);
  table_row<MAC_SGPR_NONOP>(ncu, dout, drec);
  CHK(hipFree(dout));
  CHK(hipFree(drec));
  return 0;
}
