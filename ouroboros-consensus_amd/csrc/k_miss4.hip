// k_miss4.hip -- the uncached OCert and KES verifies (k_ed25519.hip k_ocert / k_kes: a key
// used once in the batch, so no key tables) built with the ILP-4 group formulas
// (PRAOS_ILP4, as k_vrf_v4.hip) at 2 waves per SIMD, optionally at s_setprio 3.  In a small
// batch the misses are a few dozen waves whose full verify chain (decode, 252 doublings,
// encoding) ends the step; the wider interleave shortens each chain.  Identical operations
// and output.
#define PRAOS_ILP4 1
#include "k_ed25519.hpp"

__global__ void __launch_bounds__(NT, 2) k_ocert4(const uint32_t* __restrict__ list, const uint32_t* __restrict__ count,
                                                  const ge_niels* __restrict__ gbtab, OcertIn a, int prio) {
  const size_t items = *count;
  if ((size_t)blockIdx.x * NT >= items) return;
  __shared__ ge_niels sbtab[BTAB_N];
  const ge_niels* btab = stage_btab<1>(gbtab, sbtab);
  const size_t t = (size_t)blockIdx.x * NT + threadIdx.x;
  if (t >= items) return;
  if (prio) __builtin_amdgcn_s_setprio(3);
  const size_t i = list[t];
  uint32_t pk[8], sg[16], hram[16];
  ocert_load(a, i, sg, hram, pk);
  ocert_store(a, i, ed25519_verify_core(pk, sg, sg + 8, hram, btab, lane_tab(a.tabs, i, LT_ED)));
}

__global__ void __launch_bounds__(NT, 2) k_kes4(const uint32_t* __restrict__ list, const uint32_t* __restrict__ count,
                                                const ge_niels* __restrict__ gbtab, KesIn a, int prio) {
  const size_t items = *count;
  if ((size_t)blockIdx.x * NT >= items) return;
  __shared__ ge_niels sbtab[BTAB_N];
  const ge_niels* btab = stage_btab<1>(gbtab, sbtab);
  const size_t q = (size_t)blockIdx.x * NT + threadIdx.x;
  if (q >= items) return;
  if (prio) __builtin_amdgcn_s_setprio(3);
  const size_t i = list[q];
  uint32_t sg[16], leaf[8], hram[16];
  bool merkle_ok, in_range;
  kes_prepare(a, i, sg, leaf, hram, merkle_ok, in_range);
  const bool leaf_ok = ed25519_verify_core(leaf, sg, sg + 8, hram, btab, lane_tab(a.tabs, i, LT_ED));
  kes_store(a, i, merkle_ok, leaf_ok, in_range);
}

// The cached verifies (k_ed25519.hip k_ocert_ck / k_kes_ck, one header per lane) from the same
// ILP-4 build: in a small batch they are the last link of the cached chains
__global__ void __launch_bounds__(NT, 2) k_ocert_ck4(const uint32_t* __restrict__ list,
                                                     const uint32_t* __restrict__ count,
                                                     const int32_t* __restrict__ item_entry,
                                                     const ge_cached* __restrict__ ktab,
                                                     const uint32_t* __restrict__ kinfo,
                                                     const ge_niels* __restrict__ gbtab, OcertIn a) {
  const size_t items = *count;
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= items) return;
  const size_t i = list[t];
  const size_t e = (size_t)item_entry[i];
  uint32_t pk[8], sg[16], hram[16];
  ocert_load(a, i, sg, hram, pk);
  ocert_store(a, i, ed25519_verify_cached(sg, sg + 8, hram, kinfo[9 * e], ktab + e * KT_STRIDE, gbtab));
}

__global__ void __launch_bounds__(NT, 2) k_kes_ck4(const uint32_t* __restrict__ list,
                                                   const uint32_t* __restrict__ count,
                                                   const int32_t* __restrict__ item_entry,
                                                   const ge_cached* __restrict__ ktab,
                                                   const uint32_t* __restrict__ kinfo,
                                                   const ge_niels* __restrict__ gbtab, KesIn a) {
  const size_t items = *count;
  const size_t q = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= items) return;
  const size_t i = list[q];
  const size_t e = (size_t)item_entry[i];
  uint32_t sg[16], leaf[8], hram[16];
  bool merkle_ok, in_range;
  kes_prepare(a, i, sg, leaf, hram, merkle_ok, in_range);
  const bool leaf_ok = ed25519_verify_cached(sg, sg + 8, hram, kinfo[9 * e], ktab + e * KT_STRIDE, gbtab);
  kes_store(a, i, merkle_ok, leaf_ok, in_range);
}

void launch_ocert_ck4(hipStream_t stream, size_t n, const uint32_t* list, const uint32_t* count,
                      const int32_t* item_entry, const ge_cached* ktab, const uint32_t* kinfo, const ge_niels* gbtab,
                      const uint8_t* cold_vk, const uint8_t* hot_vk, const uint64_t* ocert_n, const uint64_t* ocert_c0,
                      const uint8_t* sig, const uint64_t* slot, uint64_t slots_per_kes_period, uint64_t max_kes_evo,
                      uint16_t* bits, uint8_t* ok_out) {
  OcertIn a{cold_vk, hot_vk, ocert_n, ocert_c0, sig, slot, slots_per_kes_period, max_kes_evo, bits, ok_out, nullptr};
  hipLaunchKernelGGL(k_ocert_ck4, dim3((unsigned)((n + NT - 1) / NT)), dim3(NT), 0, stream, list, count, item_entry,
                     ktab, kinfo, gbtab, a);
}

void launch_kes_ck4(hipStream_t stream, size_t n, const uint32_t* list, const uint32_t* count,
                    const int32_t* item_entry, const ge_cached* ktab, const uint32_t* kinfo, const ge_niels* gbtab,
                    const uint8_t* hot_vk, const uint8_t* kes_sig, const uint64_t* body_off, const uint32_t* body_len,
                    const uint8_t* body, size_t body_bytes_len, const uint64_t* slot, const uint64_t* ocert_c0,
                    uint64_t slots_per_kes_period, uint16_t* bits) {
  KesIn a{hot_vk, kes_sig, body_off, body_len, body, body_bytes_len, slot, ocert_c0, slots_per_kes_period,
          nullptr, bits, nullptr, nullptr};
  hipLaunchKernelGGL(k_kes_ck4, dim3((unsigned)((n + NT - 1) / NT)), dim3(NT), 0, stream, list, count, item_entry,
                     ktab, kinfo, gbtab, a);
}

void launch_ocert4(dim3 grid, dim3 block, hipStream_t stream, const uint32_t* list, const uint32_t* count,
                   const ge_niels* gbtab, const uint8_t* cold_vk, const uint8_t* hot_vk, const uint64_t* ocert_n,
                   const uint64_t* ocert_c0, const uint8_t* sig, const uint64_t* slot, uint64_t slots_per_kes_period,
                   uint64_t max_kes_evo, uint16_t* bits, uint8_t* ok_out, ge_cached* tabs, int prio) {
  OcertIn a{cold_vk, hot_vk, ocert_n, ocert_c0, sig, slot, slots_per_kes_period, max_kes_evo, bits, ok_out, tabs};
  hipLaunchKernelGGL(k_ocert4, grid, block, 0, stream, list, count, gbtab, a, prio);
}

void launch_kes4(dim3 grid, dim3 block, hipStream_t stream, const uint32_t* list, const uint32_t* count,
                 const ge_niels* gbtab, const uint8_t* hot_vk, const uint8_t* kes_sig, const uint64_t* body_off,
                 const uint32_t* body_len, const uint8_t* body, size_t body_bytes_len, const uint64_t* slot,
                 const uint64_t* ocert_c0, uint64_t slots_per_kes_period, uint16_t* bits, ge_cached* tabs, int prio) {
  KesIn a{hot_vk, kes_sig, body_off, body_len, body, body_bytes_len, slot, ocert_c0, slots_per_kes_period,
          nullptr, bits, nullptr, tabs};
  hipLaunchKernelGGL(k_kes4, grid, block, 0, stream, list, count, gbtab, a, prio);
}
