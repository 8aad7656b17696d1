// k_vrf.hip -- ECVRF draft-03 verify + pool lookup + range extension kernel.
#include "kcommon.hpp"

// ------------------------------------------------------------------ VRF
// Header mode: issuer hash -> pool (binary search), VRF key hash, alpha =
// mkInputVRF(slot, eta0), proof verify, beta, output check, leader/nonce values.
// Plain mode (ok_out != null): alpha given per item; ok_out, beta only.
__global__ void __launch_bounds__(NT, LB_VRF) k_vrf(size_t n, const ge_niels* __restrict__ gbtab,
                                            const uint8_t* __restrict__ cold_vk, const uint8_t* __restrict__ vrf_vk,
                                            const uint8_t* __restrict__ vrf_out, const uint8_t* __restrict__ vrf_proof,
                                            const uint64_t* __restrict__ slot, const uint32_t* __restrict__ eta0,
                                            int eta0_neutral, const uint32_t* __restrict__ pool_hash,
                                            const uint32_t* __restrict__ pool_vrf, const int32_t* __restrict__ pool_map,
                                            uint32_t npools, int check_output, const uint8_t* __restrict__ alpha_in,
                                            uint16_t* __restrict__ bits, int32_t* __restrict__ pool_idx,
                                            int32_t* __restrict__ pool_sorted_idx, uint8_t* __restrict__ beta_out,
                                            uint8_t* __restrict__ leader_out, uint8_t* __restrict__ nonce_out,
                                            uint8_t* __restrict__ ok_out) {
  __shared__ ge_niels sbtab[2 * BTAB_N];
  const ge_niels* btab = stage_btab<2>(gbtab, sbtab);
  const size_t i = (size_t)blockIdx.x * NT + threadIdx.x;
  if (i >= n) return;
  uint32_t pk[8], pr[20], alpha[8];
  load_words(pk, vrf_vk + 32 * i, 8);
  load_words(pr, vrf_proof + 80 * i, 20);
  uint16_t b = 0;
  int32_t sidx = -1;
  if (alpha_in) {
    load_words(alpha, alpha_in + 32 * i, 8);
  } else {
    uint32_t e0[8];
#pragma unroll
    for (int k = 0; k < 8; k++) e0[k] = eta0[k];
    mk_input_vrf(alpha, slot[i], e0, eta0_neutral != 0);          // Praos/VRF.hs:55-69
    // issuer pool: hashKey (Blake2b-224 of the cold vk), Praos.hs:552
    uint32_t cv[8], hk[8];
    load_words(cv, cold_vk + 32 * i, 8);
    blake2b_32(hk, cv, 28);
    int lo = 0, hi = (int)npools - 1;
    while (lo <= hi) {
      const int mid = (lo + hi) >> 1;
      const uint32_t* ph = pool_hash + 7 * mid;
      int c = 0;
      for (int k = 0; k < 7 && c == 0; k++) {
        const uint32_t a = __builtin_bswap32(ph[k]), q = __builtin_bswap32(hk[k]);   // byte order
        c = a < q ? -1 : (a > q ? 1 : 0);
      }
      if (c == 0) { sidx = mid; break; }
      if (c < 0) lo = mid + 1; else hi = mid - 1;
    }
    if (sidx < 0) {
      b |= PRAOS_BIT_VRF_KEY_UNKNOWN;                              // Praos.hs:537
    } else {
      uint32_t vh[8];
      blake2b_32(vh, pk, 32);                                      // hashVerKeyVRF
      bool same = true;
#pragma unroll
      for (int k = 0; k < 8; k++) same &= vh[k] == pool_vrf[8 * sidx + k];
      if (!same) b |= PRAOS_BIT_VRF_KEY_WRONG;                     // Praos.hs:539-541
    }
  }
  uint32_t beta[16];
  bool gamma_ok;
  const bool proof_ok = vrf_verify_core(beta, gamma_ok, pk, pr, pr + 8, pr + 12, alpha, btab);
  if (!gamma_ok) {
#pragma unroll
    for (int k = 0; k < 16; k++) beta[k] = 0;
  }
  if (ok_out) {
    ok_out[i] = proof_ok ? 1 : 0;
    if (beta_out) store_words(beta_out + 64 * i, beta, 16);
    return;
  }
  uint32_t out[16];
  load_words(out, vrf_out + 64 * i, 16);
  bool out_eq = true;
#pragma unroll
  for (int k = 0; k < 16; k++) out_eq &= out[k] == beta[k];
  if (!proof_ok) b |= PRAOS_BIT_VRF_PROOF;                         // Praos.hs:543-547
  if (!out_eq && check_output) b |= PRAOS_BIT_VRF_OUTPUT;
  // range extension of the CERTIFIED output (Praos/VRF.hs:88-131)
  uint32_t lv[8], nv[8], nn[8];
  blake2b256_tag64(lv, 'L', out);
  blake2b256_tag64(nv, 'N', out);
  blake2b_32(nn, nv, 32);
  if (leader_out) store_words(leader_out + 32 * i, lv, 8);
  if (nonce_out) store_words(nonce_out + 32 * i, nn, 8);
  if (beta_out) store_words(beta_out + 64 * i, beta, 16);
  pool_idx[i] = sidx < 0 ? -1 : pool_map[sidx];
  pool_sorted_idx[i] = sidx;
  bits[i] = b;
}


// ------------------------------------------------------------------ TPraos VRF (d = 0)
// cardano-protocol-tpraos OVERLAY.praosVrfChecks: pool lookup, VRF key hash,
// verifyCertified for the eta cert with mkSeed seedEta and for the leader cert
// with mkSeed seedL (VRFKeyBadNonce / VRFKeyBadLeaderValue); the leader value is
// the certified leader output itself (checked by k_leader with a 2^512 bound).
__global__ void __launch_bounds__(NT, LB_VRF) k_vrf_tp(
    size_t n, const ge_niels* __restrict__ gbtab, const uint8_t* __restrict__ cold_vk,
    const uint8_t* __restrict__ vrf_vk, const uint8_t* __restrict__ eta_out, const uint8_t* __restrict__ eta_proof,
    const uint8_t* __restrict__ l_out, const uint8_t* __restrict__ l_proof, const uint64_t* __restrict__ slot,
    const uint32_t* __restrict__ eta0, int eta0_neutral, const uint32_t* __restrict__ pool_hash,
    const uint32_t* __restrict__ pool_vrf, const int32_t* __restrict__ pool_map, uint32_t npools, int check_output,
    uint16_t* __restrict__ bits, int32_t* __restrict__ pool_idx, int32_t* __restrict__ pool_sorted_idx,
    uint8_t* __restrict__ beta_eta, uint8_t* __restrict__ beta_l, uint8_t* __restrict__ nonce_out) {
  __shared__ ge_niels sbtab[2 * BTAB_N];
  const ge_niels* btab = stage_btab<2>(gbtab, sbtab);
  const size_t i = (size_t)blockIdx.x * NT + threadIdx.x;
  if (i >= n) return;
  uint32_t pk[8], e0[8];
  load_words(pk, vrf_vk + 32 * i, 8);
#pragma unroll
  for (int k = 0; k < 8; k++) e0[k] = eta0[k];
  uint16_t b = 0;
  uint32_t cv[8], hk[8];
  load_words(cv, cold_vk + 32 * i, 8);
  blake2b_32(hk, cv, 28);
  int32_t sidx = -1;
  int lo = 0, hi = (int)npools - 1;
  while (lo <= hi) {
    const int mid = (lo + hi) >> 1;
    const uint32_t* ph = pool_hash + 7 * mid;
    int c = 0;
    for (int k = 0; k < 7 && c == 0; k++) {
      const uint32_t a = __builtin_bswap32(ph[k]), q = __builtin_bswap32(hk[k]);
      c = a < q ? -1 : (a > q ? 1 : 0);
    }
    if (c == 0) { sidx = mid; break; }
    if (c < 0) lo = mid + 1; else hi = mid - 1;
  }
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
  const uint64_t s = slot[i];
  for (int cert = 0; cert < 2; cert++) {     // 0: eta (nonce) cert, 1: leader cert
    uint32_t pr[20], out[16], alpha[8], beta[16];
    load_words(pr, (cert ? l_proof : eta_proof) + 80 * i, 20);
    load_words(out, (cert ? l_out : eta_out) + 64 * i, 16);
    tpraos_seed(alpha, s, e0, eta0_neutral != 0, (uint64_t)cert);
    bool gamma_ok;
    const bool ok = vrf_verify_core(beta, gamma_ok, pk, pr, pr + 8, pr + 12, alpha, btab);
    if (!gamma_ok) {
#pragma unroll
      for (int k = 0; k < 16; k++) beta[k] = 0;
    }
    bool eq = true;
#pragma unroll
    for (int k = 0; k < 16; k++) eq &= beta[k] == out[k];
    const uint16_t bad = cert ? PRAOS_BIT_TP_VRF_LEADER : PRAOS_BIT_TP_VRF_NONCE;
    if (!ok || (check_output && !eq)) b |= bad;
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
void launch_vrf(dim3 grid, dim3 block, hipStream_t stream, size_t n, const ge_niels* __restrict__ gbtab, const uint8_t* __restrict__ cold_vk, const uint8_t* __restrict__ vrf_vk, const uint8_t* __restrict__ vrf_out, const uint8_t* __restrict__ vrf_proof, const uint64_t* __restrict__ slot, const uint32_t* __restrict__ eta0, int eta0_neutral, const uint32_t* __restrict__ pool_hash, const uint32_t* __restrict__ pool_vrf, const int32_t* __restrict__ pool_map, uint32_t npools, int check_output, const uint8_t* __restrict__ alpha_in, uint16_t* __restrict__ bits, int32_t* __restrict__ pool_idx, int32_t* __restrict__ pool_sorted_idx, uint8_t* __restrict__ beta_out, uint8_t* __restrict__ leader_out, uint8_t* __restrict__ nonce_out, uint8_t* __restrict__ ok_out) {
  hipLaunchKernelGGL(k_vrf, grid, block, 0, stream, n, gbtab, cold_vk, vrf_vk, vrf_out, vrf_proof, slot, eta0, eta0_neutral, pool_hash, pool_vrf, pool_map, npools, check_output, alpha_in, bits, pool_idx, pool_sorted_idx, beta_out, leader_out, nonce_out, ok_out);
}
void launch_vrf_tp(dim3 grid, dim3 block, hipStream_t stream, size_t n, const ge_niels* gbtab, const uint8_t* cold_vk,
                   const uint8_t* vrf_vk, const uint8_t* eta_out, const uint8_t* eta_proof, const uint8_t* l_out,
                   const uint8_t* l_proof, const uint64_t* slot, const uint32_t* eta0, int eta0_neutral,
                   const uint32_t* pool_hash, const uint32_t* pool_vrf, const int32_t* pool_map, uint32_t npools,
                   int check_output, uint16_t* bits, int32_t* pool_idx, int32_t* pool_sorted_idx, uint8_t* beta_eta,
                   uint8_t* beta_l, uint8_t* nonce_out) {
  hipLaunchKernelGGL(k_vrf_tp, grid, block, 0, stream, n, gbtab, cold_vk, vrf_vk, eta_out, eta_proof, l_out, l_proof,
                     slot, eta0, eta0_neutral, pool_hash, pool_vrf, pool_map, npools, check_output, bits, pool_idx,
                     pool_sorted_idx, beta_eta, beta_l, nonce_out);
}
