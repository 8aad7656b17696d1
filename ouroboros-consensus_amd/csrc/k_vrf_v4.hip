// k_vrf_v4.hip -- stage V of the staged VRF verify (k_vrf_stage.hip k_vrf_v: alpha, H =
// hash_to_curve, Gamma, 8 Gamma, V = [s]H - [c]Gamma, the stage record) built with the ILP-4
// group formulas (PRAOS_ILP4, ge25519.hpp: the 3-4 independent products of every doubling /
// addition / conversion interleaved MAC by MAC) at 2 waves per SIMD.  For batches whose V
// waves do not fill the SIMDs (a 54k-header shard is 844 waves for 1,024 SIMDs) each chain
// runs latency-bound, and the wider interleave shortens it (tools/microbench/femul4.hip: one
// wave per SIMD, 1137 -> 971 SIMD cycles per multiply).  Identical operations and output.
#define PRAOS_ILP4 1
#include "k_vrf.hpp"

__global__ void __launch_bounds__(NT, 2) k_vrf_v4(size_t n, size_t i0, size_t i1, VrfIn a, uint4* __restrict__ mid) {
  const size_t i = i0 + (size_t)blockIdx.x * blockDim.x + threadIdx.x;   // headers [i0, i1), record stride n
  if (i >= i1) return;
  if (a.wave_prio) __builtin_amdgcn_s_setprio(3);
  uint32_t pk[8], pr[20], alpha[8];
  load_words(pk, a.vrf_vk + 32 * i, 8);
  load_words(pr, a.vrf_proof + 80 * i, 20);
  header_alpha(alpha, a, i);
  vrf_v_core(mid, n, i, pk, pr, pr + 8, pr + 12, alpha, lane_tab(a.tabs, i, LT_VRF));
}

// The same kernel holding its SIMD alone: touching a255 makes every wave allocate its 202
// VGPRs plus the 256 accumulation registers (460 of the SIMD's 512), so no other wave of
// the step's kernels (all above 52 VGPRs) is placed beside it.  A 54k-header step's 844 V
// waves then take 211 CUs whole and the short first-level chains (uncached verifies, key
// precomputes) run on the remaining CUs instead of sharing SIMDs with V.
__global__ void __launch_bounds__(NT, 1) k_vrf_v4x(size_t n, size_t i0, size_t i1, VrfIn a, uint4* __restrict__ mid) {
  asm volatile("v_accvgpr_write_b32 a255, 0" ::: "a255");
  const size_t i = i0 + (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= i1) return;
  if (a.wave_prio) __builtin_amdgcn_s_setprio(3);
  uint32_t pk[8], pr[20], alpha[8];
  load_words(pk, a.vrf_vk + 32 * i, 8);
  load_words(pr, a.vrf_proof + 80 * i, 20);
  header_alpha(alpha, a, i);
  vrf_v_core(mid, n, i, pk, pr, pr + 8, pr + 12, alpha, lane_tab(a.tabs, i, LT_VRF));
}

// Stage U of a cached key (k_vrf_stage.hip k_vrf_u) from the same ILP-4 build: small batches
__global__ void __launch_bounds__(NT, 2) k_vrf_u4(size_t stride, const uint32_t* __restrict__ list,
                                                  const uint32_t* __restrict__ count,
                                                  const int32_t* __restrict__ item_entry,
                                                  const ge_cached* __restrict__ ktab,
                                                  const uint32_t* __restrict__ kinfo,
                                                  const ge_niels* __restrict__ comb,
                                                  const uint8_t* __restrict__ vrf_proof, uint4* __restrict__ mid,
                                                  int prio) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (size_t)*count) return;
  wave_setprio(prio);
  const size_t i = list[t];
  const size_t e = (size_t)item_entry[i];
  uint32_t pr[20];
  load_words(pr, vrf_proof + 80 * i, 20);
  vrf_u_core<true>(mid, stride, i, nullptr, pr + 8, pr + 12, comb, nullptr, ktab + e * KT_STRIDE, kinfo + 9 * e);
}

void launch_vrf_u4(hipStream_t stream, size_t n, const uint32_t* list, const uint32_t* count, const int32_t* item_entry,
                   const ge_cached* ktab, const uint32_t* kinfo, const ge_niels* comb, const uint8_t* vrf_proof,
                   void* mid, int prio) {
  hipLaunchKernelGGL(k_vrf_u4, dim3((unsigned)((n + NT - 1) / NT)), dim3(NT), 0, stream, n, list, count, item_entry,
                     ktab, kinfo, comb, vrf_proof, (uint4*)mid, prio);
}

void launch_vrf_v4(hipStream_t stream, size_t n, size_t i0, size_t i1, const uint8_t* vrf_vk,
                   const uint8_t* vrf_proof, const uint64_t* slot, const uint32_t* eta0, int eta0_neutral,
                   const uint8_t* eta_idx, ge_cached* tabs, void* mid, int wave_prio, int tp_seed, int excl) {
  VrfIn a = vrf_in(nullptr, vrf_vk, nullptr, vrf_proof, slot, eta0, eta0_neutral, eta_idx, nullptr, nullptr,
                   nullptr, 0, 0, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, tabs);
  a.wave_prio = wave_prio;
  a.tp_seed = tp_seed;
  i1 = i1 < n ? i1 : n;
  if (i1 <= i0) return;
  const dim3 grid((unsigned)((i1 - i0 + NT - 1) / NT));
  if (excl)
    hipLaunchKernelGGL(k_vrf_v4x, grid, dim3(NT), 0, stream, n, i0, i1, a, (uint4*)mid);
  else
    hipLaunchKernelGGL(k_vrf_v4, grid, dim3(NT), 0, stream, n, i0, i1, a, (uint4*)mid);
}
