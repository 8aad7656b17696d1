// k_vrf.hip -- ECVRF draft-03 verify + pool lookup + range extension kernel.
#include "k_vrf.hpp"

// ------------------------------------------------------------------ VRF
// Items: i in [0, n) or list[0 .. *count) (key-cache partition, k_keys.hip):
// k_vrf takes the misses, k_vrf_ck the hits (cached VRF key, short U chain).
template <bool CACHED>
__device__ __forceinline__ void vrf_item(const VrfIn& a, size_t i, const ge_niels* __restrict__ btab,
                                         const ge_cached* __restrict__ ktab, const uint32_t* __restrict__ kinfo) {
  uint32_t pk[8], pr[20], alpha[8];
  load_words(pk, a.vrf_vk + 32 * i, 8);
  load_words(pr, a.vrf_proof + 80 * i, 20);
  uint16_t b = 0;
  int32_t sidx = -1;
  if (a.alpha_in) {
    load_words(alpha, a.alpha_in + 32 * i, 8);
  } else {
    uint32_t e0[8];
    const uint32_t* ep = a.eta_idx ? a.eta0 + 9 * (uint32_t)a.eta_idx[i] : a.eta0;
#pragma unroll
    for (int k = 0; k < 8; k++) e0[k] = ep[k];
    const bool neutral = a.eta_idx ? ep[8] != 0 : a.eta0_neutral != 0;
    mk_input_vrf(alpha, a.slot[i], e0, neutral);                  // Praos/VRF.hs:55-69
    uint32_t cv[8], hk[8];
    load_words(cv, a.cold_vk + 32 * i, 8);
    blake2b_32(hk, cv, 28);
    sidx = pool_search(hk, a.pool_hash, a.npools);
    if (sidx < 0) {
      b |= PRAOS_BIT_VRF_KEY_UNKNOWN;                              // Praos.hs:537
    } else {
      uint32_t vh[8];
      blake2b_32(vh, pk, 32);                                      // hashVerKeyVRF
      bool same = true;
#pragma unroll
      for (int k = 0; k < 8; k++) same &= vh[k] == a.pool_vrf[8 * sidx + k];
      if (!same) b |= PRAOS_BIT_VRF_KEY_WRONG;                     // Praos.hs:539-541
    }
  }
  uint32_t beta[16];
  bool gamma_ok;
  const bool proof_ok =
      vrf_verify_core<CACHED>(beta, gamma_ok, pk, pr, pr + 8, pr + 12, alpha, btab, lane_tab(a.tabs, i, LT_VRF),
                              ktab, kinfo);
  if (!gamma_ok) {
#pragma unroll
    for (int k = 0; k < 16; k++) beta[k] = 0;
  }
  if (a.ok_out) {
    a.ok_out[i] = proof_ok ? 1 : 0;
    if (a.beta_out) store_words(a.beta_out + 64 * i, beta, 16);
    return;
  }
  uint32_t out[16];
  load_words(out, a.vrf_out + 64 * i, 16);
  bool out_eq = true;
#pragma unroll
  for (int k = 0; k < 16; k++) out_eq &= out[k] == beta[k];
  if (!proof_ok) b |= PRAOS_BIT_VRF_PROOF;                         // Praos.hs:543-547
  if (!out_eq && a.check_output) b |= PRAOS_BIT_VRF_OUTPUT;
  // range extension of the CERTIFIED output (Praos/VRF.hs:88-131)
  uint32_t lv[8], nv[8], nn[8];
  blake2b256_tag64(lv, 'L', out);
  blake2b256_tag64(nv, 'N', out);
  blake2b_32(nn, nv, 32);
  if (a.leader_out) store_words(a.leader_out + 32 * i, lv, 8);
  if (a.nonce_out) store_words(a.nonce_out + 32 * i, nn, 8);
  if (a.beta_out) store_words(a.beta_out + 64 * i, beta, 16);
  a.pool_idx[i] = sidx < 0 ? -1 : a.pool_map[sidx];
  a.pool_sorted_idx[i] = sidx;
  a.bits[i] = b;
}

__global__ void __launch_bounds__(NT, LB_VRF) k_vrf(size_t n, const uint32_t* __restrict__ list,
                                                    const uint32_t* __restrict__ count,
                                                    const ge_niels* __restrict__ gbtab, VrfIn a) {
  const size_t items = list ? (size_t)*count : n;
  if ((size_t)blockIdx.x * NT >= items) return;
  __shared__ ge_niels sbtab[2 * BTAB_N];
  const ge_niels* btab = stage_btab<5>(gbtab, sbtab);
  const size_t t = (size_t)blockIdx.x * NT + threadIdx.x;
  if (t >= items) return;
  vrf_item<false>(a, list ? list[t] : t, btab, nullptr, nullptr);
}

__global__ void __launch_bounds__(NT, LB_VRF) k_vrf_ck(const uint32_t* __restrict__ list,
                                                       const uint32_t* __restrict__ count,
                                                       const int32_t* __restrict__ item_entry,
                                                       const ge_cached* __restrict__ ktab,
                                                       const uint32_t* __restrict__ kinfo,
                                                       const ge_niels* __restrict__ gbtab, VrfIn a) {
  const size_t items = *count;
  if ((size_t)blockIdx.x * NT >= items) return;
  const ge_niels* btab = gbtab;                                 // the radix-2^16 comb, read in place
  const size_t t = (size_t)blockIdx.x * NT + threadIdx.x;
  if (t >= items) return;
  const size_t i = list[t];
  const size_t e = (size_t)item_entry[i];
  vrf_item<true>(a, i, btab, ktab + e * KT_STRIDE, kinfo + 9 * e);
}


// ------------------------------------------------------------------ TPraos VRF
// cardano-protocol-tpraos OVERLAY.praosVrfChecks: pool lookup, VRF key hash,
// verifyCertified for the eta cert with mkSeed seedEta and for the leader cert
// with mkSeed seedL (VRFKeyBadNonce / VRFKeyBadLeaderValue); the leader value is
// the certified leader output itself (checked by k_leader with a 2^512 bound).
// Overlay schedule (ovl_class != null, host-classified, praos_set_overlay): class -2
// = NotActiveSlotOVERLAY (no VRF check); class k >= 0 = the k-th genesis key's slot:
// pbftVrfChecks against its delegate (gen: delegate hash 7 words + pad | VRF hash 8)
// -- cold-key hash and VRF-key hash compared, both certificates verified, no pool
// and no leader test (pool_sorted = -1 makes k_leader skip the header).
__global__ void __launch_bounds__(NT, LB_VRF) k_vrf_tp(
    size_t n, const ge_niels* __restrict__ gbtab, const uint8_t* __restrict__ cold_vk,
    const uint8_t* __restrict__ vrf_vk, const uint8_t* __restrict__ eta_out, const uint8_t* __restrict__ eta_proof,
    const uint8_t* __restrict__ l_out, const uint8_t* __restrict__ l_proof, const uint64_t* __restrict__ slot,
    const uint32_t* __restrict__ eta0, int eta0_neutral, const uint32_t* __restrict__ pool_hash,
    const uint32_t* __restrict__ pool_vrf, const int32_t* __restrict__ pool_map, uint32_t npools, int check_output,
    uint16_t* __restrict__ bits, int32_t* __restrict__ pool_idx, int32_t* __restrict__ pool_sorted_idx,
    uint8_t* __restrict__ beta_eta, uint8_t* __restrict__ beta_l, uint8_t* __restrict__ nonce_out,
    ge_cached* __restrict__ tabs, const int32_t* __restrict__ ovl_class, const uint32_t* __restrict__ gen,
    const uint8_t* __restrict__ eta_idx) {
  if ((size_t)blockIdx.x * NT >= n) return;
  __shared__ ge_niels sbtab[2 * BTAB_N];
  const ge_niels* btab = stage_btab<5>(gbtab, sbtab);
  const size_t i = (size_t)blockIdx.x * NT + threadIdx.x;
  if (i >= n) return;
  uint32_t pk[8], e0[8];
  load_words(pk, vrf_vk + 32 * i, 8);
  // eta_idx: several epochs per batch, eta0 = table of 9-word entries (nonce, neutral flag)
  const uint32_t* ep = eta_idx ? eta0 + 9 * (uint32_t)eta_idx[i] : eta0;
  const bool neutral = eta_idx ? ep[8] != 0 : eta0_neutral != 0;
#pragma unroll
  for (int k = 0; k < 8; k++) e0[k] = ep[k];
  uint16_t b = 0;
  uint32_t cv[8], hk[8];
  load_words(cv, cold_vk + 32 * i, 8);
  blake2b_32(hk, cv, 28);
  const int32_t cls = ovl_class ? ovl_class[i] : -1;
  int32_t sidx = -1;
  if (cls == -2) {
    b |= PRAOS_BIT_TP_NOT_ACTIVE;                    // NotActiveSlotOVERLAY
  } else if (cls >= 0) {                             // pbftVrfChecks vs the genesis delegate
    b |= PRAOS_BIT_TP_OVERLAY;
    const uint32_t* gd = gen + 16 * cls;
    bool cold_ok = true, vrf_ok = true;
#pragma unroll
    for (int k = 0; k < 7; k++) cold_ok &= hk[k] == gd[k];
    uint32_t vh[8];
    blake2b_32(vh, pk, 32);
#pragma unroll
    for (int k = 0; k < 8; k++) vrf_ok &= vh[k] == gd[8 + k];
    if (!cold_ok) b |= PRAOS_BIT_TP_GEN_COLD;
    if (!vrf_ok) b |= PRAOS_BIT_TP_GEN_VRF;
  } else {
    sidx = pool_search(hk, pool_hash, npools);
    if (sidx < 0) {
      b |= PRAOS_BIT_VRF_KEY_UNKNOWN;
    } else {
      uint32_t vh[8];
      blake2b_32(vh, pk, 32);
      bool same = true;
#pragma unroll
      for (int k = 0; k < 8; k++) same &= vh[k] == pool_vrf[8 * sidx + k];
      if (!same) b |= PRAOS_BIT_VRF_KEY_WRONG;
    }
  }
  const uint64_t s = slot[i];
  for (int cert = 0; cert < 2; cert++) {     // 0: eta (nonce) cert, 1: leader cert
    uint32_t pr[20], out[16], alpha[8], beta[16];
    load_words(pr, (cert ? l_proof : eta_proof) + 80 * i, 20);
    load_words(out, (cert ? l_out : eta_out) + 64 * i, 16);
    tpraos_seed(alpha, s, e0, neutral, (uint64_t)cert);
    bool gamma_ok;
    const bool ok = vrf_verify_core<false>(beta, gamma_ok, pk, pr, pr + 8, pr + 12, alpha, btab,
                                           lane_tab(tabs, i, LT_VRF));
    if (!gamma_ok) {
#pragma unroll
      for (int k = 0; k < 16; k++) beta[k] = 0;
    }
    bool eq = true;
#pragma unroll
    for (int k = 0; k < 16; k++) eq &= beta[k] == out[k];
    const uint16_t bad = cert ? PRAOS_BIT_TP_VRF_LEADER : PRAOS_BIT_TP_VRF_NONCE;
    if ((!ok || (check_output && !eq)) && cls != -2) b |= bad;
    store_words((cert ? beta_l : beta_eta) + 64 * i, beta, 16);
    if (cert == 0) {
      uint32_t nn[8];
      blake2b256_of64(nn, out);                // mkNonceFromOutputVRF
      store_words(nonce_out + 32 * i, nn, 8);
    }
  }
  pool_idx[i] = sidx < 0 ? -1 : pool_map[sidx];
  pool_sorted_idx[i] = sidx;
  bits[i] = b;
}

// ---- host launchers (kernels are only launchable from their own module)
void launch_vrf(dim3 grid, dim3 block, hipStream_t stream, size_t n, const uint32_t* list, const uint32_t* count,
                const ge_niels* gbtab, const uint8_t* cold_vk, const uint8_t* vrf_vk, const uint8_t* vrf_out,
                const uint8_t* vrf_proof, const uint64_t* slot, const uint32_t* eta0, int eta0_neutral,
                const uint8_t* eta_idx, const uint32_t* pool_hash, const uint32_t* pool_vrf, const int32_t* pool_map,
                uint32_t npools, int check_output, const uint8_t* alpha_in, uint16_t* bits, int32_t* pool_idx,
                int32_t* pool_sorted_idx, uint8_t* beta_out, uint8_t* leader_out, uint8_t* nonce_out, uint8_t* ok_out,
                ge_cached* tabs) {
  VrfIn a{cold_vk, vrf_vk, vrf_out, vrf_proof, slot, eta0, eta0_neutral, eta_idx, pool_hash, pool_vrf, pool_map, npools,
          check_output, alpha_in, bits, pool_idx, pool_sorted_idx, beta_out, leader_out, nonce_out, ok_out, tabs};
  hipLaunchKernelGGL(k_vrf, grid, block, 0, stream, n, list, count, gbtab, a);
}
void launch_vrf_ck(dim3 grid, dim3 block, hipStream_t stream, const uint32_t* list, const uint32_t* count,
                   const int32_t* item_entry, const ge_cached* ktab, const uint32_t* kinfo, const ge_niels* gbtab,
                   const uint8_t* cold_vk, const uint8_t* vrf_vk, const uint8_t* vrf_out, const uint8_t* vrf_proof,
                   const uint64_t* slot, const uint32_t* eta0, int eta0_neutral, const uint8_t* eta_idx,
                   const uint32_t* pool_hash, const uint32_t* pool_vrf, const int32_t* pool_map, uint32_t npools,
                   int check_output, const uint8_t* alpha_in, uint16_t* bits, int32_t* pool_idx,
                   int32_t* pool_sorted_idx, uint8_t* beta_out, uint8_t* leader_out, uint8_t* nonce_out,
                   uint8_t* ok_out, ge_cached* tabs) {
  VrfIn a{cold_vk, vrf_vk, vrf_out, vrf_proof, slot, eta0, eta0_neutral, eta_idx, pool_hash, pool_vrf, pool_map, npools,
          check_output, alpha_in, bits, pool_idx, pool_sorted_idx, beta_out, leader_out, nonce_out, ok_out, tabs};
  hipLaunchKernelGGL(k_vrf_ck, grid, block, 0, stream, list, count, item_entry, ktab, kinfo, gbtab, a);
}
void launch_vrf_tp(dim3 grid, dim3 block, hipStream_t stream, size_t n, const ge_niels* gbtab, const uint8_t* cold_vk,
                   const uint8_t* vrf_vk, const uint8_t* eta_out, const uint8_t* eta_proof, const uint8_t* l_out,
                   const uint8_t* l_proof, const uint64_t* slot, const uint32_t* eta0, int eta0_neutral,
                   const uint32_t* pool_hash, const uint32_t* pool_vrf, const int32_t* pool_map, uint32_t npools,
                   int check_output, uint16_t* bits, int32_t* pool_idx, int32_t* pool_sorted_idx, uint8_t* beta_eta,
                   uint8_t* beta_l, uint8_t* nonce_out, ge_cached* tabs, const int32_t* ovl_class,
                   const uint32_t* gen, const uint8_t* eta_idx) {
  hipLaunchKernelGGL(k_vrf_tp, grid, block, 0, stream, n, gbtab, cold_vk, vrf_vk, eta_out, eta_proof, l_out, l_proof,
                     slot, eta0, eta0_neutral, pool_hash, pool_vrf, pool_map, npools, check_output, bits, pool_idx,
                     pool_sorted_idx, beta_eta, beta_l, nonce_out, tabs, ovl_class, gen, eta_idx);
}
