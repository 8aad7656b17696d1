#pragma once
// kcommon.hpp -- shared pieces of the gfx950 kernel modules of libpraos_hip
// (one header / signature per lane).
//
// Data layout in HBM (struct of arrays, one record per header per field,
// records 8/16-byte aligned so each lane issues dwordx4 loads):
//   slot u64[n] | cold_vk [n][32] | vrf_vk [n][32] | vrf_out [n][64] | vrf_proof [n][80]
//   hot_vk [n][32] | ocert_n u64[n] | ocert_c0 u64[n] | ocert_sig [n][64]
//   kes_sig [n][448] | body_off u64[n] | body_len u32[n] | body arena (8-aligned, +8 pad)
// Outputs: bits u16[n] (OR-accumulated by the kernels), pool_idx i32[n],
//   beta [n][64], leader [n][32] (big-endian natural), nonce [n][32].
// Epoch tables: pool hash28 (7 words, sorted), vrf hash (8 words), x_raw (4 words).
#include "praos_core.hpp"
#include "leader.hpp"
#include "praos_hip.h"
#include "launch.hpp"

#define NT 256                      // threads per block (4 waves)
// minimum waves per SIMD requested from the register allocator
#ifndef LB_ED
#define LB_ED 3
#endif
#ifndef LB_VRF
#define LB_VRF 3
#endif

// Per-lane point tables in global memory (praos_api.hip allocates them per batch):
// item i owns `entries` cached points, 128 contiguous bytes each, at arena + i *
// entries -- 8 for an Ed25519 verify (KES leaf, OCert), 16 for a VRF verify.
#define LT_ED 8
#define LT_VRF 16
__device__ __forceinline__ ge_cached* lane_tab(ge_cached* __restrict__ arena, size_t i, int entries) {
  return arena + i * (size_t)entries;
}

__device__ __forceinline__ void load_words(uint32_t* w, const uint8_t* p, int nwords) {
  const uint4* q = (const uint4*)p;
  for (int i = 0; i < nwords / 4; i++) {
    const uint4 v = q[i];
    w[4 * i] = v.x; w[4 * i + 1] = v.y; w[4 * i + 2] = v.z; w[4 * i + 3] = v.w;
  }
}
__device__ __forceinline__ void store_words(uint8_t* p, const uint32_t* w, int nwords) {
  uint4* q = (uint4*)p;
  for (int i = 0; i < nwords / 4; i++) q[i] = make_uint4(w[4 * i], w[4 * i + 1], w[4 * i + 2], w[4 * i + 3]);
}

// Fixed-base comb in global memory (k_init_btab): BCOMB_T tables of BTAB_N niels,
// table j = {1..128} 256^j B.  The cached-key chains read it in place (L2-resident);
// the per-lane-base chains stage the ones they use into LDS, compacted in increasing
// t: MASK bit t = comb table 8t = {1..128} 2^(64 t) B, i.e. 0b0001 = {B} (Ed25519
// verify), 0b0101 = {B, 2^128 B} (VRF U, signing).
template <int MASK>
__device__ __forceinline__ const ge_niels* stage_btab(const ge_niels* __restrict__ g, ge_niels* s) {
  constexpr int W4 = BTAB_WORDS / 4;                  // uint4 per table
  int slot = 0;
#pragma unroll
  for (int t = 0; t < 4; t++) {
    if (MASK & (1 << t)) {
      const uint4* src = (const uint4*)g + 8 * t * W4;
      uint4* dst = (uint4*)s + slot * W4;
      for (int i = threadIdx.x; i < W4; i += blockDim.x) dst[i] = src[i];
      slot++;
    }
  }
  __syncthreads();
  return s;
}

// s_setprio takes an immediate: wave priority 2 or 3 from a runtime value (0 and others: unchanged)
__device__ __forceinline__ void wave_setprio(int p) {
  if (p == 3) __builtin_amdgcn_s_setprio(3);
  else if (p == 2) __builtin_amdgcn_s_setprio(2);
}
