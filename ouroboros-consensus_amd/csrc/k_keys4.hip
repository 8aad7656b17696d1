// k_keys4.hip -- the key-cache precompute (k_keys.hip k_key_precompute: decode, checks, the
// 15 x 16-doubling chain to the chunk bases) built with the ILP-4 group formulas
// (PRAOS_ILP4, as k_vrf_v4.hip).  In a small batch the precompute is a few dozen waves of
// one long chain each on the cached verifies' critical path; the wider interleave shortens
// the chain.  Identical operations and output.
#define PRAOS_ILP4 1
#include "k_keys.hpp"

__global__ void __launch_bounds__(64) k_key_precompute4(int kind, const uint32_t* __restrict__ counters,
                                                         uint32_t max_entries, const uint32_t* __restrict__ entry_rep,
                                                         const uint8_t* __restrict__ keys, ge_cached* __restrict__ ktab,
                                                         uint32_t* __restrict__ kinfo, int wave_prio,
                                                         const uint32_t* __restrict__ base) {
  if (wave_prio) __builtin_amdgcn_s_setprio(3);
  const uint32_t ne = min(counters[0], max_entries);
  for (uint32_t e = (base ? *base : 0u) + blockIdx.x * blockDim.x + threadIdx.x; e < ne; e += gridDim.x * blockDim.x)
    key_precompute_entry(kind, e, entry_rep, keys, ktab, kinfo);
}

void launch_key_precompute4(int kind, hipStream_t stream, const uint32_t* counters, uint32_t max_entries,
                            const uint32_t* entry_rep, const uint8_t* keys, ge_cached* ktab, uint32_t* kinfo,
                            int wave_prio, const uint32_t* base, uint32_t span) {
  hipLaunchKernelGGL(k_key_precompute4, dim3((span + 63) / 64), dim3(64), 0, stream, kind, counters, max_entries,
                     entry_rep, keys, ktab, kinfo, wave_prio, base);
}
