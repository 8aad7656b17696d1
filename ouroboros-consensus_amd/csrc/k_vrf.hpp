#pragma once
// k_vrf.hpp -- pieces shared by the VRF kernel modules (k_vrf.hip: the one-kernel verify and
// TPraos; k_vrf_stage.hip: the staged header pipeline)
#include "kcommon.hpp"

// Header mode: issuer hash -> pool (binary search), VRF key hash, alpha =
// mkInputVRF(slot, eta0), proof verify, beta, output check, leader/nonce values.
// Plain mode (ok_out != null): alpha given per item; ok_out, beta only.
struct VrfIn {
  const uint8_t* __restrict__ cold_vk;
  const uint8_t* __restrict__ vrf_vk;
  const uint8_t* __restrict__ vrf_out;
  const uint8_t* __restrict__ vrf_proof;
  const uint64_t* __restrict__ slot;
  const uint32_t* __restrict__ eta0;     // eta_idx == null: the epoch nonce (8 words)
  int eta0_neutral;
  const uint8_t* __restrict__ eta_idx;   // several epochs per batch: header i uses entry eta_idx[i]
                                         // of eta0 = table of 9-word entries (nonce, neutral flag)
  const uint32_t* __restrict__ pool_hash;
  const uint32_t* __restrict__ pool_vrf;
  const int32_t* __restrict__ pool_map;
  uint32_t npools;
  int check_output;
  const uint8_t* __restrict__ alpha_in;
  uint16_t* __restrict__ bits;
  int32_t* __restrict__ pool_idx;
  int32_t* __restrict__ pool_sorted_idx;
  uint8_t* __restrict__ beta_out;
  uint8_t* __restrict__ leader_out;
  uint8_t* __restrict__ nonce_out;
  uint8_t* __restrict__ ok_out;
  ge_cached* __restrict__ tabs;          // per-lane tables (LT_VRF entries per item)
  int wave_prio;                         // stage V / join waves at s_setprio 3 (small batches)
  int tp_seed;                           // stage V alpha: 0 Praos mkInputVRF; 1 + k TPraos mkSeed
                                         // with ucNonce k (0 seedEta, 1 seedL)
  int pre;                               // join: the pool part ran ahead (k_vrf_pool wrote bits[i])
};

// issuer pool: hashKey (Blake2b-224 of the cold vk, Praos.hs:552) -> sorted index or -1
__device__ __forceinline__ int32_t pool_search(const uint32_t hk[8], const uint32_t* __restrict__ pool_hash,
                                               uint32_t npools) {
  int lo = 0, hi = (int)npools - 1;
  while (lo <= hi) {
    const int mid = (lo + hi) >> 1;
    const uint32_t* ph = pool_hash + 7 * mid;
    int c = 0;
    for (int k = 0; k < 7 && c == 0; k++) {
      const uint32_t x = __builtin_bswap32(ph[k]), q = __builtin_bswap32(hk[k]);   // byte order
      c = x < q ? -1 : (x > q ? 1 : 0);
    }
    if (c == 0) return mid;
    if (c < 0) lo = mid + 1; else hi = mid - 1;
  }
  return -1;
}

// alpha = mkInputVRF(slot, eta) of header i (Praos/VRF.hs:55-69), or for a TPraos
// certificate mkSeed(ucNonce, slot, eta) (TPraos.hs:378-387 -> BHeader.mkSeed)
__device__ __forceinline__ void header_alpha(uint32_t alpha[8], const VrfIn& a, size_t i) {
  uint32_t e0[8];
  const uint32_t* ep = a.eta_idx ? a.eta0 + 9 * (uint32_t)a.eta_idx[i] : a.eta0;
#pragma unroll
  for (int k = 0; k < 8; k++) e0[k] = ep[k];
  const bool neutral = a.eta_idx ? ep[8] != 0 : a.eta0_neutral != 0;
  if (a.tp_seed) tpraos_seed(alpha, a.slot[i], e0, neutral, (uint64_t)(a.tp_seed - 1));
  else mk_input_vrf(alpha, a.slot[i], e0, neutral);
}

static inline VrfIn vrf_in(const uint8_t* cold_vk, const uint8_t* vrf_vk, const uint8_t* vrf_out, const uint8_t* vrf_proof,
                    const uint64_t* slot, const uint32_t* eta0, int eta0_neutral, const uint8_t* eta_idx,
                    const uint32_t* pool_hash, const uint32_t* pool_vrf, const int32_t* pool_map, uint32_t npools,
                    int check_output, uint16_t* bits, int32_t* pool_idx, int32_t* pool_sorted_idx, uint8_t* beta_out,
                    uint8_t* leader_out, uint8_t* nonce_out, ge_cached* tabs) {
  return VrfIn{cold_vk, vrf_vk, vrf_out, vrf_proof, slot, eta0, eta0_neutral, eta_idx, pool_hash, pool_vrf, pool_map,
               npools, check_output, nullptr, bits, pool_idx, pool_sorted_idx, beta_out, leader_out, nonce_out, nullptr,
               tabs};
}
