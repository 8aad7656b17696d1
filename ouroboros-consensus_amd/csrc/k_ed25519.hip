// k_ed25519.hip -- OCert and Sum6KES kernels (Ed25519 verify per lane).
#include "kcommon.hpp"

// ------------------------------------------------------------------ OCert + KES period checks
// bits |= KES_BEFORE_START / KES_AFTER_END / OCERT_SIG.  If ok_out != null the
// kernel is the plain praos_verify_ocert batch (ok_out[i] = 1 when valid).
// Items: i in [0, n), or list[0 .. *count) when list != null (key-cache
// partition, k_keys.hip): k_ocert takes the misses, k_ocert_ck the hits.
struct OcertIn {
  const uint8_t* __restrict__ cold_vk;
  const uint8_t* __restrict__ hot_vk;
  const uint64_t* __restrict__ ocert_n;
  const uint64_t* __restrict__ ocert_c0;
  const uint8_t* __restrict__ sig;
  const uint64_t* __restrict__ slot;
  uint64_t slots_per_kes_period, max_kes_evo;
  uint16_t* __restrict__ bits;
  uint8_t* __restrict__ ok_out;
  ge_cached* __restrict__ tabs;          // per-lane tables (LT_ED entries per item)
};

__device__ __forceinline__ void ocert_store(const OcertIn& a, size_t i, bool ok) {
  if (a.ok_out) {
    a.ok_out[i] = ok ? 1 : 0;
    return;
  }
  uint16_t b = ok ? 0 : PRAOS_BIT_OCERT_SIG;
  const uint64_t c0 = a.ocert_c0[i];
  const uint64_t kp = a.slot[i] / a.slots_per_kes_period;     // Praos.hs:596-599
  if (!(c0 <= kp)) b |= PRAOS_BIT_KES_BEFORE_START;            // Praos.hs:567
  if (!(kp < c0 + a.max_kes_evo)) b |= PRAOS_BIT_KES_AFTER_END; // Praos.hs:568
  a.bits[i] = b;
}

__device__ __forceinline__ void ocert_load(const OcertIn& a, size_t i, uint32_t sg[16], uint32_t hram[16],
                                           uint32_t pk[8]) {
  uint32_t hot[8];
  load_words(pk, a.cold_vk + 32 * i, 8);
  load_words(hot, a.hot_vk + 32 * i, 8);
  load_words(sg, a.sig + 64 * i, 16);
  ocert_hram(hram, sg, pk, hot, a.ocert_n[i], a.ocert_c0[i]);
}

__global__ void __launch_bounds__(NT, LB_ED) k_ocert(size_t n, const uint32_t* __restrict__ list,
                                                     const uint32_t* __restrict__ count,
                                                     const ge_niels* __restrict__ gbtab, OcertIn a) {
  const size_t items = list ? (size_t)*count : n;
  if ((size_t)blockIdx.x * NT >= items) return;                // whole block idle
  __shared__ ge_niels sbtab[BTAB_N];
  const ge_niels* btab = stage_btab<1>(gbtab, sbtab);
  const size_t t = (size_t)blockIdx.x * NT + threadIdx.x;
  if (t >= items) return;
  const size_t i = list ? list[t] : t;
  uint32_t pk[8], sg[16], hram[16];
  ocert_load(a, i, sg, hram, pk);
  ocert_store(a, i, ed25519_verify_core(pk, sg, sg + 8, hram, btab, lane_tab(a.tabs, i, LT_ED)));
}

__global__ void __launch_bounds__(NT, LB_ED) k_ocert_ck(const uint32_t* __restrict__ list,
                                                        const uint32_t* __restrict__ count,
                                                        const int32_t* __restrict__ item_entry,
                                                        const ge_cached* __restrict__ ktab,
                                                        const uint32_t* __restrict__ kinfo,
                                                        const ge_niels* __restrict__ gbtab, OcertIn a) {
  const size_t items = *count;
  if ((size_t)blockIdx.x * blockDim.x >= items) return;
  const ge_niels* btab = gbtab;                                 // the radix-2^16 comb, read in place
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= items) return;
  const size_t i = list[t];
  const size_t e = (size_t)item_entry[i];
  uint32_t pk[8], sg[16], hram[16];
  ocert_load(a, i, sg, hram, pk);
  ocert_store(a, i, ed25519_verify_cached(sg, sg + 8, hram, kinfo[9 * e], ktab + e * KT_STRIDE, btab));
}

// ------------------------------------------------------------------ KES
// Header mode: t = kp >= c0 ? kp - c0 : 0 (Praos.hs:570), result to bits.
// Plain mode (result != null): t = period[i], result 0 ok / 1 Reject / 2 leaf.
// Items: i in [0, n), or list[0 .. *count) (leaf-key cache partition): k_kes takes
// the misses, k_kes_ck the hits.
struct KesIn {
  const uint8_t* __restrict__ hot_vk;
  const uint8_t* __restrict__ kes_sig;
  const uint64_t* __restrict__ body_off;
  const uint32_t* __restrict__ body_len;
  const uint8_t* __restrict__ body;
  size_t body_bytes_len;
  const uint64_t* __restrict__ slot;
  const uint64_t* __restrict__ ocert_c0;
  uint64_t slots_per_kes_period;
  const uint32_t* __restrict__ period;
  uint16_t* __restrict__ bits;
  uint8_t* __restrict__ result;
  ge_cached* __restrict__ tabs;
};

__device__ __forceinline__ uint64_t kes_t(const KesIn& a, size_t i) {
  if (a.period) return a.period[i];
  const uint64_t kp = a.slot[i] / a.slots_per_kes_period, c0 = a.ocert_c0[i];
  return kp >= c0 ? kp - c0 : 0;
}

// Merkle walk + SHA-512(R || leaf || M); returns merkle_ok, in_range, the leaf
// key and the signature words.
__device__ __forceinline__ void kes_prepare(const KesIn& a, size_t i, uint32_t sg[16], uint32_t leaf[8],
                                            uint32_t hram[16], bool& merkle_ok, bool& in_range) {
  const uint8_t* sig = a.kes_sig + 448 * i;
  uint32_t vk[8];
  load_words(vk, a.hot_vk + 32 * i, 8);
  merkle_ok = kes_merkle(leaf, vk, kes_t(a, i), sig);
  load_words(sg, sig, 16);
  uint64_t off = a.body_off[i];
  uint32_t len = a.body_len[i];
  in_range = (off & 7) == 0 && off <= a.body_bytes_len && len <= a.body_bytes_len - off;
  if (!in_range) { off = 0; len = 0; }
  uint32_t pre[16];
#pragma unroll
  for (int k = 0; k < 8; k++) { pre[k] = sg[k]; pre[8 + k] = leaf[k]; }
  sha512_stream(hram, pre, 64, a.body + off, len);
}

__device__ __forceinline__ void kes_store(const KesIn& a, size_t i, bool merkle_ok, bool leaf_ok, bool in_range) {
  if (a.result) {
    a.result[i] = !in_range ? 3 : (!merkle_ok ? 1 : (leaf_ok ? 0 : 2));
    return;
  }
  uint16_t b = 0;
  if (!merkle_ok) b |= PRAOS_BIT_KES_MERKLE;
  else if (!leaf_ok) b |= PRAOS_BIT_KES_LEAF;
  if (!in_range) b |= PRAOS_BIT_INPUT;
  a.bits[i] = b;
}

__global__ void __launch_bounds__(NT, LB_ED) k_kes(size_t n, const uint32_t* __restrict__ list,
                                                   const uint32_t* __restrict__ count,
                                                   const ge_niels* __restrict__ gbtab, KesIn a) {
  const size_t items = list ? (size_t)*count : n;
  if ((size_t)blockIdx.x * NT >= items) return;
  __shared__ ge_niels sbtab[BTAB_N];
  const ge_niels* btab = stage_btab<1>(gbtab, sbtab);
  const size_t q = (size_t)blockIdx.x * NT + threadIdx.x;
  if (q >= items) return;
  const size_t i = list ? list[q] : q;
  uint32_t sg[16], leaf[8], hram[16];
  bool merkle_ok, in_range;
  kes_prepare(a, i, sg, leaf, hram, merkle_ok, in_range);
  const bool leaf_ok = ed25519_verify_core(leaf, sg, sg + 8, hram, btab, lane_tab(a.tabs, i, LT_ED));
  kes_store(a, i, merkle_ok, leaf_ok, in_range);
}

// Hits of the leaf-key cache: the leaf key's multi-power tables were built once per
// batch (k_keys.hip, kind 0), so [h]A is a 16-window chain.  The cached key is the
// same 32 bytes kes_merkle selects (k_kes_leafkeys reads them the same way).
__global__ void __launch_bounds__(NT, LB_ED) k_kes_ck(const uint32_t* __restrict__ list,
                                                      const uint32_t* __restrict__ count,
                                                      const int32_t* __restrict__ item_entry,
                                                      const ge_cached* __restrict__ ktab,
                                                      const uint32_t* __restrict__ kinfo,
                                                      const ge_niels* __restrict__ gbtab, KesIn a) {
  const size_t items = *count;
  if ((size_t)blockIdx.x * blockDim.x >= items) return;
  const ge_niels* btab = gbtab;                                 // the radix-2^16 comb, read in place
  const size_t q = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= items) return;
  const size_t i = list[q];
  const size_t e = (size_t)item_entry[i];
  uint32_t sg[16], leaf[8], hram[16];
  bool merkle_ok, in_range;
  kes_prepare(a, i, sg, leaf, hram, merkle_ok, in_range);
  const bool leaf_ok = ed25519_verify_cached(sg, sg + 8, hram, kinfo[9 * e], ktab + e * KT_STRIDE, btab);
  kes_store(a, i, merkle_ok, leaf_ok, in_range);
}

// The leaf Ed25519 key each header's KES signature selects (the depth-1 pair entry
// kes_merkle ends on), copied out densely for the key cache's hash set.
__global__ void __launch_bounds__(NT) k_kes_leafkeys(size_t n, KesIn a, uint8_t* __restrict__ keys) {
  const size_t i = (size_t)blockIdx.x * NT + threadIdx.x;
  if (i >= n) return;
  uint64_t t = kes_t(a, i);
#pragma unroll
  for (int d = 6; d >= 2; d--) {
    const uint64_t T = 1ull << (d - 1);
    t = t >= T ? t - T : t;
  }
  const uint4* src = (const uint4*)(a.kes_sig + 448 * i + 64 + (t >= 1 ? 32 : 0));
  uint4* dst = (uint4*)(keys + 32 * i);
  dst[0] = src[0];
  dst[1] = src[1];
}


// ---- host launchers (kernels are only launchable from their own module)
void launch_ocert(dim3 grid, dim3 block, hipStream_t stream, size_t n, const uint32_t* list, const uint32_t* count,
                  const ge_niels* gbtab, const uint8_t* cold_vk, const uint8_t* hot_vk, const uint64_t* ocert_n,
                  const uint64_t* ocert_c0, const uint8_t* sig, const uint64_t* slot, uint64_t slots_per_kes_period,
                  uint64_t max_kes_evo, uint16_t* bits, uint8_t* ok_out, ge_cached* tabs) {
  OcertIn a{cold_vk, hot_vk, ocert_n, ocert_c0, sig, slot, slots_per_kes_period, max_kes_evo, bits, ok_out, tabs};
  hipLaunchKernelGGL(k_ocert, grid, block, 0, stream, n, list, count, gbtab, a);
}
void launch_ocert_ck(dim3 grid, dim3 block, hipStream_t stream, const uint32_t* list, const uint32_t* count,
                     const int32_t* item_entry, const ge_cached* ktab, const uint32_t* kinfo, const ge_niels* gbtab,
                     const uint8_t* cold_vk, const uint8_t* hot_vk, const uint64_t* ocert_n, const uint64_t* ocert_c0,
                     const uint8_t* sig, const uint64_t* slot, uint64_t slots_per_kes_period, uint64_t max_kes_evo,
                     uint16_t* bits, uint8_t* ok_out) {
  OcertIn a{cold_vk, hot_vk, ocert_n, ocert_c0, sig, slot, slots_per_kes_period, max_kes_evo, bits, ok_out, nullptr};
  hipLaunchKernelGGL(k_ocert_ck, grid, block, 0, stream, list, count, item_entry, ktab, kinfo, gbtab, a);
}

void launch_kes(dim3 grid, dim3 block, hipStream_t stream, size_t n, const uint32_t* list, const uint32_t* count,
                const ge_niels* gbtab, const uint8_t* hot_vk, const uint8_t* kes_sig, const uint64_t* body_off,
                const uint32_t* body_len, const uint8_t* body, size_t body_bytes_len, const uint64_t* slot,
                const uint64_t* ocert_c0, uint64_t slots_per_kes_period, const uint32_t* period, uint16_t* bits,
                uint8_t* result, ge_cached* tabs) {
  KesIn a{hot_vk, kes_sig, body_off, body_len, body, body_bytes_len, slot, ocert_c0, slots_per_kes_period,
          period, bits, result, tabs};
  hipLaunchKernelGGL(k_kes, grid, block, 0, stream, n, list, count, gbtab, a);
}
void launch_kes_ck(dim3 grid, dim3 block, hipStream_t stream, const uint32_t* list, const uint32_t* count,
                   const int32_t* item_entry, const ge_cached* ktab, const uint32_t* kinfo, const ge_niels* gbtab,
                   const uint8_t* hot_vk, const uint8_t* kes_sig, const uint64_t* body_off, const uint32_t* body_len,
                   const uint8_t* body, size_t body_bytes_len, const uint64_t* slot, const uint64_t* ocert_c0,
                   uint64_t slots_per_kes_period, uint16_t* bits) {
  KesIn a{hot_vk, kes_sig, body_off, body_len, body, body_bytes_len, slot, ocert_c0, slots_per_kes_period,
          nullptr, bits, nullptr, nullptr};
  hipLaunchKernelGGL(k_kes_ck, grid, block, 0, stream, list, count, item_entry, ktab, kinfo, gbtab, a);
}
void launch_kes_leafkeys(dim3 grid, dim3 block, hipStream_t stream, size_t n, const uint8_t* kes_sig,
                         const uint64_t* slot, const uint64_t* ocert_c0, uint64_t slots_per_kes_period,
                         uint8_t* keys) {
  KesIn a{nullptr, kes_sig, nullptr, nullptr, nullptr, 0, slot, ocert_c0, slots_per_kes_period,
          nullptr, nullptr, nullptr, nullptr};
  hipLaunchKernelGGL(k_kes_leafkeys, grid, block, 0, stream, n, a, keys);
}
