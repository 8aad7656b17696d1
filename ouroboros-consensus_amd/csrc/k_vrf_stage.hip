// k_vrf_stage.hip -- the header pipeline's VRF verify in stages (praos_core.hpp): V over every
// header, U per key-cache partition, the join (k_vrf_join); the two-stage form (k_vrf_fin*)
// kept for A/B (PRAOS_VRF3=0).
#include "k_vrf.hpp"

// waves per SIMD the launch bounds ask for: stage V (the largest kernel, 168 VGPRs at 3) and
// the U / join kernels (at 3 they spill SHA-512 and point state to scratch)
#ifndef LB_VRF_V
#define LB_VRF_V LB_VRF
#endif
#ifndef LB_VRF_F
#define LB_VRF_F LB_VRF
#endif
// the join / U + join kernels (one batched inversion, the SHA-512 challenge and beta, the
// Blake2b range extensions): at 3 waves per SIMD they spill ~370 bytes per lane
#ifndef LB_VRF_J
#define LB_VRF_J LB_VRF_F
#endif

// ---- two-stage form of the header mode (praos_core.hpp vrf_v_core / vrf_fin_core)
// stage V over every header of the batch: no dependence on the key cache
__global__ void __launch_bounds__(NT, LB_VRF_V) k_vrf_v(size_t n, size_t i0, size_t i1, VrfIn a, uint4* __restrict__ mid) {
  const size_t i = i0 + (size_t)blockIdx.x * blockDim.x + threadIdx.x;   // headers [i0, i1), record stride n
  if (i >= i1) return;
  if (a.wave_prio) __builtin_amdgcn_s_setprio(3);
  uint32_t pk[8], pr[20], alpha[8];
  load_words(pk, a.vrf_vk + 32 * i, 8);
  load_words(pr, a.vrf_proof + 80 * i, 20);
  header_alpha(alpha, a, i);
  vrf_v_core(mid, n, i, pk, pr, pr + 8, pr + 12, alpha, lane_tab(a.tabs, i, LT_VRF));
}

// stage F: pool lookup and key hash (Praos.hs:533-541), U + challenge + beta, the output
// check and the range extension -- the same results vrf_item writes in header mode
template <bool CACHED>
__device__ __forceinline__ void vrf_fin_item(const VrfIn& a, size_t i, size_t stride, const uint4* __restrict__ mid,
                                             const ge_niels* __restrict__ btab, const ge_cached* __restrict__ ktab,
                                             const uint32_t* __restrict__ kinfo) {
  uint32_t pk[8], pr[20];
  load_words(pk, a.vrf_vk + 32 * i, 8);
  load_words(pr, a.vrf_proof + 80 * i, 20);
  uint16_t b = 0;
  int32_t sidx;
  {
    uint32_t cv[8], hk[8];
    load_words(cv, a.cold_vk + 32 * i, 8);
    blake2b_32(hk, cv, 28);
    sidx = pool_search(hk, a.pool_hash, a.npools);
    if (sidx < 0) {
      b |= PRAOS_BIT_VRF_KEY_UNKNOWN;
    } else {
      uint32_t vh[8];
      blake2b_32(vh, pk, 32);
      bool same = true;
#pragma unroll
      for (int k = 0; k < 8; k++) same &= vh[k] == a.pool_vrf[8 * sidx + k];
      if (!same) b |= PRAOS_BIT_VRF_KEY_WRONG;
    }
  }
  uint32_t beta[16];
  bool gamma_ok;
  const bool proof_ok = vrf_fin_core<CACHED>(beta, gamma_ok, mid, stride, i, pk, pr + 8, pr + 12, btab,
                                             lane_tab(a.tabs, i, LT_VRF), ktab, kinfo);
  if (!gamma_ok) {
#pragma unroll
    for (int k = 0; k < 16; k++) beta[k] = 0;
  }
  uint32_t out[16];
  load_words(out, a.vrf_out + 64 * i, 16);
  bool out_eq = true;
#pragma unroll
  for (int k = 0; k < 16; k++) out_eq &= out[k] == beta[k];
  if (!proof_ok) b |= PRAOS_BIT_VRF_PROOF;
  if (!out_eq && a.check_output) b |= PRAOS_BIT_VRF_OUTPUT;
  uint32_t lv[8], nv[8], nn[8];
  blake2b256_tag64(lv, 'L', out);
  blake2b256_tag64(nv, 'N', out);
  blake2b_32(nn, nv, 32);
  store_words(a.leader_out + 32 * i, lv, 8);
  store_words(a.nonce_out + 32 * i, nn, 8);
  store_words(a.beta_out + 64 * i, beta, 16);
  a.pool_idx[i] = sidx < 0 ? -1 : a.pool_map[sidx];
  a.pool_sorted_idx[i] = sidx;
  a.bits[i] = b;
}

// cached keys (the hit list): U from the key's tables and the radix-2^16 comb
__global__ void __launch_bounds__(NT, LB_VRF_J) k_vrf_fin(size_t stride, const uint32_t* __restrict__ list,
                                                        const uint32_t* __restrict__ count,
                                                        const int32_t* __restrict__ item_entry,
                                                        const ge_cached* __restrict__ ktab,
                                                        const uint32_t* __restrict__ kinfo,
                                                        const ge_niels* __restrict__ comb, VrfIn a,
                                                        const uint4* __restrict__ mid) {
  const size_t items = *count;
  const size_t t = (size_t)blockIdx.x * NT + threadIdx.x;
  if (t >= items) return;
  const size_t i = list[t];
  const size_t e = (size_t)item_entry[i];
  vrf_fin_item<true>(a, i, stride, mid, comb, ktab + e * KT_STRIDE, kinfo + 9 * e);
}

// uncached keys (the miss list, or every header): U on a per-lane chain
__global__ void __launch_bounds__(NT, LB_VRF_J) k_vrf_fin_nc(size_t n, const uint32_t* __restrict__ list,
                                                           const uint32_t* __restrict__ count,
                                                           const ge_niels* __restrict__ gbtab, VrfIn a,
                                                           const uint4* __restrict__ mid) {
  const size_t items = list ? (size_t)*count : n;
  if ((size_t)blockIdx.x * NT >= items) return;
  __shared__ ge_niels sbtab[2 * BTAB_N];
  const ge_niels* btab = stage_btab<5>(gbtab, sbtab);
  const size_t t = (size_t)blockIdx.x * NT + threadIdx.x;
  if (t >= items) return;
  vrf_fin_item<false>(a, list ? list[t] : t, n, mid, btab, nullptr, nullptr);
}

// ---- three-kernel form (praos_core.hpp vrf_u_core / vrf_join_core): U apart from V
// U of a cached key (the hit list): the key's tables and the radix-2^16 comb
__global__ void __launch_bounds__(NT, LB_VRF_F) k_vrf_u(size_t stride, const uint32_t* __restrict__ list,
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

// U of an uncached key (the miss list, or every header): a per-lane chain; vt = an 8-entry
// lane table region of its own (stage V runs at the same time on the 16-entry one)
__global__ void __launch_bounds__(NT, LB_VRF_F) k_vrf_u_nc(size_t n, const uint32_t* __restrict__ list,
                                                         const uint32_t* __restrict__ count,
                                                         const ge_niels* __restrict__ gbtab,
                                                         const uint8_t* __restrict__ vrf_vk,
                                                         const uint8_t* __restrict__ vrf_proof,
                                                         ge_cached* __restrict__ tabs, uint4* __restrict__ mid) {
  const size_t items = list ? (size_t)*count : n;
  if ((size_t)blockIdx.x * NT >= items) return;
  __shared__ ge_niels sbtab[2 * BTAB_N];
  const ge_niels* btab = stage_btab<5>(gbtab, sbtab);
  const size_t t = (size_t)blockIdx.x * NT + threadIdx.x;
  if (t >= items) return;
  const size_t i = list ? list[t] : t;
  uint32_t pk[8], pr[20];
  load_words(pk, vrf_vk + 32 * i, 8);
  load_words(pr, vrf_proof + 80 * i, 20);
  vrf_u_core<false>(mid, n, i, pk, pr + 8, pr + 12, btab, lane_tab(tabs, i, LT_ED), nullptr, nullptr);
}

// the header-only part of the join: pool lookup and key hash (Praos.hs:533-541), the pool
// indices and the leader / nonce values of the stated output (Praos.hs:468-502); returns the
// key bits
__device__ __forceinline__ uint16_t vrf_pool_item(const VrfIn& a, size_t i) {
  uint16_t b = 0;
  int32_t sidx;
  {
    uint32_t pk[8], cv[8], hk[8];
    load_words(cv, a.cold_vk + 32 * i, 8);
    blake2b_32(hk, cv, 28);
    sidx = pool_search(hk, a.pool_hash, a.npools);
    if (sidx < 0) {
      b |= PRAOS_BIT_VRF_KEY_UNKNOWN;
    } else {
      load_words(pk, a.vrf_vk + 32 * i, 8);
      uint32_t vh[8];
      blake2b_32(vh, pk, 32);
      bool same = true;
#pragma unroll
      for (int k = 0; k < 8; k++) same &= vh[k] == a.pool_vrf[8 * sidx + k];
      if (!same) b |= PRAOS_BIT_VRF_KEY_WRONG;
    }
  }
  uint32_t out[16], lv[8], nv[8], nn[8];
  load_words(out, a.vrf_out + 64 * i, 16);
  blake2b256_tag64(lv, 'L', out);
  blake2b256_tag64(nv, 'N', out);
  blake2b_32(nn, nv, 32);
  store_words(a.leader_out + 32 * i, lv, 8);
  store_words(a.nonce_out + 32 * i, nn, 8);
  a.pool_idx[i] = sidx < 0 ? -1 : a.pool_map[sidx];
  a.pool_sorted_idx[i] = sidx;
  return b;
}

// ... ahead of the join (small batches, on a stream with slack): the join's lanes then end
// after the inversion and the two SHA-512s (its dependent pool-search loads and five Blake2b
// compressions no longer follow stage V)
__global__ void __launch_bounds__(NT) k_vrf_pool(size_t n, VrfIn a) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  a.bits[i] = vrf_pool_item(a, i);
}

// join over every header: the pool part (vrf_pool_item, or its bits from k_vrf_pool when
// a.pre), the batched inversion, the challenge, beta and the output check
__global__ void __launch_bounds__(NT, LB_VRF_J) k_vrf_join(size_t n, VrfIn a, const uint4* __restrict__ mid) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (a.wave_prio) __builtin_amdgcn_s_setprio(3);
  uint16_t b = a.pre ? 0 : vrf_pool_item(a, i);
  uint32_t c4[4];
  {
    const uint4 q = *(const uint4*)(a.vrf_proof + 80 * i + 32);
    c4[0] = q.x; c4[1] = q.y; c4[2] = q.z; c4[3] = q.w;
  }
  uint32_t beta[16];
  bool gamma_ok;
  const bool proof_ok = vrf_join_core(beta, gamma_ok, mid, n, i, c4);
  if (!gamma_ok) {
#pragma unroll
    for (int k = 0; k < 16; k++) beta[k] = 0;
  }
  uint32_t out[16];
  load_words(out, a.vrf_out + 64 * i, 16);
  bool out_eq = true;
#pragma unroll
  for (int k = 0; k < 16; k++) out_eq &= out[k] == beta[k];
  if (!proof_ok) b |= PRAOS_BIT_VRF_PROOF;
  if (!out_eq && a.check_output) b |= PRAOS_BIT_VRF_OUTPUT;
  store_words(a.beta_out + 64 * i, beta, 16);
  a.bits[i] = a.pre ? (uint16_t)(a.bits[i] | b) : b;
}

// TPraos join of certificate `cert` (0: eta / nonce cert, 1: leader cert), the staged form of
// k_vrf_tp: cert 0 classifies the slot (overlay classes from praos_set_overlay: -2 not
// active, >= 0 a genesis delegate's slot checked against gen; else the pool lookup and VRF
// key hash, Praos.hs:533-541 as TPraos.hs:304-387 uses them) and writes beta_eta + the nonce
// (mkNonceFromOutputVRF of the stated output); cert 1 adds its bit to bits[i] and writes beta_l.
// Runs after cert 0's join on the same stream (bits read-modify-write).
__global__ void __launch_bounds__(NT, LB_VRF_J) k_vrf_join_tp(size_t n, int cert, VrfIn a,
                                                            const uint4* __restrict__ mid,
                                                            const int32_t* __restrict__ ovl_class,
                                                            const uint32_t* __restrict__ gen) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int32_t cls = ovl_class ? ovl_class[i] : -1;
  uint16_t b = 0;
  if (cert == 0) {
    uint32_t pk[8], cv[8], hk[8];
    load_words(cv, a.cold_vk + 32 * i, 8);
    blake2b_32(hk, cv, 28);
    load_words(pk, a.vrf_vk + 32 * i, 8);
    int32_t sidx = -1;
    if (cls == -2) {
      b |= PRAOS_BIT_TP_NOT_ACTIVE;                  // NotActiveSlotOVERLAY
    } else if (cls >= 0) {                           // pbftVrfChecks vs the genesis delegate
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
      sidx = pool_search(hk, a.pool_hash, a.npools);
      if (sidx < 0) {
        b |= PRAOS_BIT_VRF_KEY_UNKNOWN;
      } else {
        uint32_t vh[8];
        blake2b_32(vh, pk, 32);
        bool same = true;
#pragma unroll
        for (int k = 0; k < 8; k++) same &= vh[k] == a.pool_vrf[8 * sidx + k];
        if (!same) b |= PRAOS_BIT_VRF_KEY_WRONG;
      }
    }
    a.pool_idx[i] = sidx < 0 ? -1 : a.pool_map[sidx];
    a.pool_sorted_idx[i] = sidx;
  } else {
    b = a.bits[i];
  }
  uint32_t c4[4];
  {
    const uint4 q = *(const uint4*)(a.vrf_proof + 80 * i + 32);
    c4[0] = q.x; c4[1] = q.y; c4[2] = q.z; c4[3] = q.w;
  }
  uint32_t beta[16], out[16];
  bool gamma_ok;
  const bool ok = vrf_join_core(beta, gamma_ok, mid, n, i, c4);
  if (!gamma_ok) {
#pragma unroll
    for (int k = 0; k < 16; k++) beta[k] = 0;
  }
  load_words(out, a.vrf_out + 64 * i, 16);
  bool eq = true;
#pragma unroll
  for (int k = 0; k < 16; k++) eq &= beta[k] == out[k];
  if ((!ok || (a.check_output && !eq)) && cls != -2) b |= cert ? PRAOS_BIT_TP_VRF_LEADER : PRAOS_BIT_TP_VRF_NONCE;
  store_words(a.beta_out + 64 * i, beta, 16);
  if (cert == 0) {
    uint32_t nn[8];
    blake2b256_of64(nn, out);                        // mkNonceFromOutputVRF
    store_words(a.nonce_out + 32 * i, nn, 8);
  }
  a.bits[i] = b;
}

// ---- host launchers (kernels are only launchable from their own module)
void launch_vrf_v(hipStream_t stream, size_t n, const uint8_t* vrf_vk, const uint8_t* vrf_proof, const uint64_t* slot,
                  const uint32_t* eta0, int eta0_neutral, const uint8_t* eta_idx, ge_cached* tabs, void* mid,
                  size_t i0, size_t i1, int wave_prio, int tp_seed, int ilp4) {
  if (ilp4) {
    launch_vrf_v4(stream, n, i0, i1, vrf_vk, vrf_proof, slot, eta0, eta0_neutral, eta_idx, tabs, mid, wave_prio,
                  tp_seed, ilp4 > 1);
    return;
  }
  VrfIn a = vrf_in(nullptr, vrf_vk, nullptr, vrf_proof, slot, eta0, eta0_neutral, eta_idx, nullptr, nullptr,
                   nullptr, 0, 0, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, tabs);
  a.wave_prio = wave_prio;
  a.tp_seed = tp_seed;
  const unsigned bs = lat_block(n);
  i1 = i1 < n ? i1 : n;
  if (i1 <= i0) return;
  hipLaunchKernelGGL(k_vrf_v, dim3((unsigned)((i1 - i0 + bs - 1) / bs)), dim3(bs), 0, stream, n, i0, i1, a,
                     (uint4*)mid);
}
void launch_vrf_fin(hipStream_t stream, size_t n, const uint32_t* list, const uint32_t* count,
                    const int32_t* item_entry, const ge_cached* ktab, const uint32_t* kinfo, const ge_niels* comb,
                    const ge_niels* gbtab, const uint8_t* cold_vk, const uint8_t* vrf_vk, const uint8_t* vrf_out,
                    const uint8_t* vrf_proof, const uint32_t* pool_hash, const uint32_t* pool_vrf,
                    const int32_t* pool_map, uint32_t npools, int check_output, uint16_t* bits, int32_t* pool_idx,
                    int32_t* pool_sorted_idx, uint8_t* beta_out, uint8_t* leader_out, uint8_t* nonce_out,
                    ge_cached* tabs, const void* mid) {
  const VrfIn a = vrf_in(cold_vk, vrf_vk, vrf_out, vrf_proof, nullptr, nullptr, 0, nullptr, pool_hash, pool_vrf,
                         pool_map, npools, check_output, bits, pool_idx, pool_sorted_idx, beta_out, leader_out,
                         nonce_out, tabs);
  const dim3 g((unsigned)((n + NT - 1) / NT));
  if (ktab)
    hipLaunchKernelGGL(k_vrf_fin, g, dim3(NT), 0, stream, n, list, count, item_entry, ktab, kinfo, comb, a,
                       (const uint4*)mid);
  else
    hipLaunchKernelGGL(k_vrf_fin_nc, g, dim3(NT), 0, stream, n, list, count, gbtab, a, (const uint4*)mid);
}
void launch_vrf_u(hipStream_t stream, size_t n, const uint32_t* list, const uint32_t* count, const int32_t* item_entry,
                  const ge_cached* ktab, const uint32_t* kinfo, const ge_niels* comb, const ge_niels* gbtab,
                  const uint8_t* vrf_vk, const uint8_t* vrf_proof, ge_cached* utabs, void* mid, int ilp4,
                  int prio) {
  const dim3 g((unsigned)((n + NT - 1) / NT));
  const unsigned bs = lat_block(n);
  if (ktab && ilp4)
    launch_vrf_u4(stream, n, list, count, item_entry, ktab, kinfo, comb, vrf_proof, mid, prio);
  else if (ktab)
    hipLaunchKernelGGL(k_vrf_u, dim3((unsigned)((n + bs - 1) / bs)), dim3(bs), 0, stream, n, list, count, item_entry,
                       ktab, kinfo, comb, vrf_proof, (uint4*)mid, prio);
  else
    hipLaunchKernelGGL(k_vrf_u_nc, g, dim3(NT), 0, stream, n, list, count, gbtab, vrf_vk, vrf_proof, utabs,
                       (uint4*)mid);
}
void launch_vrf_join(hipStream_t stream, size_t n, const uint8_t* cold_vk, const uint8_t* vrf_vk,
                     const uint8_t* vrf_out, const uint8_t* vrf_proof, const uint32_t* pool_hash,
                     const uint32_t* pool_vrf, const int32_t* pool_map, uint32_t npools, int check_output,
                     uint16_t* bits, int32_t* pool_idx, int32_t* pool_sorted_idx, uint8_t* beta_out,
                     uint8_t* leader_out, uint8_t* nonce_out, const void* mid, int wave_prio, int pre) {
  VrfIn a = vrf_in(cold_vk, vrf_vk, vrf_out, vrf_proof, nullptr, nullptr, 0, nullptr, pool_hash, pool_vrf,
                   pool_map, npools, check_output, bits, pool_idx, pool_sorted_idx, beta_out, leader_out,
                   nonce_out, nullptr);
  a.wave_prio = wave_prio;
  a.pre = pre;
  const unsigned bs = lat_block(n);
  hipLaunchKernelGGL(k_vrf_join, dim3((unsigned)((n + bs - 1) / bs)), dim3(bs), 0, stream, n, a, (const uint4*)mid);
}
void launch_vrf_pool(hipStream_t stream, size_t n, const uint8_t* cold_vk, const uint8_t* vrf_vk,
                     const uint8_t* vrf_out, const uint32_t* pool_hash, const uint32_t* pool_vrf,
                     const int32_t* pool_map, uint32_t npools, uint16_t* bits, int32_t* pool_idx,
                     int32_t* pool_sorted_idx, uint8_t* leader_out, uint8_t* nonce_out) {
  const VrfIn a = vrf_in(cold_vk, vrf_vk, vrf_out, nullptr, nullptr, nullptr, 0, nullptr, pool_hash, pool_vrf,
                         pool_map, npools, 0, bits, pool_idx, pool_sorted_idx, nullptr, leader_out, nonce_out,
                         nullptr);
  hipLaunchKernelGGL(k_vrf_pool, dim3((unsigned)((n + NT - 1) / NT)), dim3(NT), 0, stream, n, a);
}
void launch_vrf_join_tp(hipStream_t stream, size_t n, int cert, const uint8_t* cold_vk, const uint8_t* vrf_vk,
                        const uint8_t* cert_out, const uint8_t* cert_proof, const uint32_t* pool_hash,
                        const uint32_t* pool_vrf, const int32_t* pool_map, uint32_t npools, int check_output,
                        uint16_t* bits, int32_t* pool_idx, int32_t* pool_sorted_idx, uint8_t* beta_out,
                        uint8_t* nonce_out, const void* mid, const int32_t* ovl_class, const uint32_t* gen) {
  const VrfIn a = vrf_in(cold_vk, vrf_vk, cert_out, cert_proof, nullptr, nullptr, 0, nullptr, pool_hash, pool_vrf,
                         pool_map, npools, check_output, bits, pool_idx, pool_sorted_idx, beta_out, nullptr,
                         nonce_out, nullptr);
  const unsigned bs = lat_block(n);
  hipLaunchKernelGGL(k_vrf_join_tp, dim3((unsigned)((n + bs - 1) / bs)), dim3(bs), 0, stream, n, cert, a,
                     (const uint4*)mid, ovl_class, gen);
}
