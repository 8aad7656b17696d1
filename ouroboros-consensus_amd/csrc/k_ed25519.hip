// k_ed25519.hip -- OCert and Sum6KES kernels (Ed25519 verify per lane).
#include "k_ed25519.hpp"

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
  wave_setprio(a.wave_prio);
  const size_t i = list[t];
  const size_t e = (size_t)item_entry[i];
  uint32_t pk[8], sg[16], hram[16];
  ocert_load(a, i, sg, hram, pk);
  ocert_store(a, i, ed25519_verify_cached(sg, sg + 8, hram, kinfo[9 * e], ktab + e * KT_STRIDE, btab));
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
// k_kes_ck2, the paired form (launched when pairing is enabled, PRAOS_OPT_KES_PAIR): from
// pair_min hits on (a count the kernel reads itself) each lane takes two headers, q and
// q + lanes, and encodes both R' with one inversion of Z_a Z_b: the encoding's inversion is
// ~265 of a cached verify's ~1,000 multiplications.  Below pair_min it keeps one header per
// lane.  The first header's R' waits in LDS while the second is computed (24 words per
// lane).  Verdicts are those of ed25519_verify_cached header by header.
__global__ void __launch_bounds__(NT, LB_ED) k_kes_ck(const uint32_t* __restrict__ list,
                                                      const uint32_t* __restrict__ count,
                                                      const int32_t* __restrict__ item_entry,
                                                      const ge_cached* __restrict__ ktab,
                                                      const uint32_t* __restrict__ kinfo,
                                                      const ge_niels* __restrict__ gbtab, KesIn a,
                                                      const uint32_t* __restrict__ entry_rep,
                                                      const uint8_t* __restrict__ rep_ok) {
  const size_t items = *count;
  if ((size_t)blockIdx.x * blockDim.x >= items) return;
  const ge_niels* btab = gbtab;                                 // the radix-2^16 comb, read in place
  const size_t q = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= items) return;
  wave_setprio(a.wave_prio);
  const size_t i = list[q];
  const size_t e = (size_t)item_entry[i];
  uint32_t sg[16], leaf[8], hram[16];
  bool merkle_ok, in_range;
  kes_prepare_dd(a, i, rep_ok ? entry_rep[e] : i, rep_ok ? rep_ok + e : nullptr, sg, leaf, hram, merkle_ok,
                 in_range);
  const bool leaf_ok = ed25519_verify_cached(sg, sg + 8, hram, kinfo[9 * e], ktab + e * KT_STRIDE, btab);
  kes_store(a, i, merkle_ok, leaf_ok, in_range);
}

__global__ void __launch_bounds__(NT, LB_ED) k_kes_ck2(const uint32_t* __restrict__ list,
                                                      const uint32_t* __restrict__ count,
                                                      const int32_t* __restrict__ item_entry,
                                                      const ge_cached* __restrict__ ktab,
                                                      const uint32_t* __restrict__ kinfo,
                                                      const ge_niels* __restrict__ gbtab, KesIn a,
                                                      uint32_t pair_min, const uint32_t* __restrict__ entry_rep,
                                                      const uint8_t* __restrict__ rep_ok) {
  __shared__ uint32_t stash[24 * NT];
  const size_t items = *count;
  const size_t lanes = pair_min && items >= pair_min ? (items + 1) / 2 : items;
  if ((size_t)blockIdx.x * blockDim.x >= lanes) return;
  const ge_niels* btab = gbtab;                                 // the radix-2^16 comb, read in place
  const size_t q = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= lanes) return;
  wave_setprio(a.wave_prio);
  const bool has_b = q + lanes < items;                         // a second header (paired batches)
  const size_t ia = list[q];
  uint32_t sg[16], leaf[8], hram[16];
  uint32_t fl = 0;                                              // per header h: bits 3h.. = merkle, range, ok
  ge_p2 R;
  uint32_t* st = stash + threadIdx.x;
#pragma nounroll
  for (int h = 0; h < 2; h++) {                                 // one copy of the chain in the code
    if (h == 1 && !has_b) break;
    const size_t i = h ? list[q + lanes] : ia;
    bool merkle_ok, in_range;
    const size_t e = (size_t)item_entry[i];
    kes_prepare_dd(a, i, rep_ok ? entry_rep[e] : i, rep_ok ? rep_ok + e : nullptr, sg, leaf, hram, merkle_ok,
                   in_range);
    const bool ok = ed25519_cached_point(R, sg, sg + 8, hram, kinfo[9 * e], ktab + e * KT_STRIDE, btab);
    fl |= ((merkle_ok ? 1u : 0u) | (in_range ? 2u : 0u) | (ok ? 4u : 0u)) << (3 * h);
    if (h == 0) {
#pragma unroll
      for (int k = 0; k < 8; k++) {
        st[k * NT] = R.X.v[k];
        st[(8 + k) * NT] = R.Y.v[k];
        st[(16 + k) * NT] = R.Z.v[k];
      }
    }
  }
  // 1 / (Z_a Z_b) (Z_b = 1 without a second header); a zero Z (only from a rejected key's
  // tables) is replaced by 1 so that it cannot change the other header's encoding
  fe one, Za, Zb, zp, inv, zi;
  fe_set(one, 1);
#pragma unroll
  for (int k = 0; k < 8; k++) Za.v[k] = st[(16 + k) * NT];
  Zb = R.Z;
  fe_cmov(Za, one, fe_iszero(Za));
  fe_cmov(Zb, one, !has_b || fe_iszero(Zb));
  fe_mul(zp, Za, Zb);
  fe_invert(inv, zp);
  uint32_t enc[8];
  bool eq;
  if (has_b) {
    fe_mul(zi, inv, Za);                                       // 1 / Z_b
    ge_tobytes_zi(enc, R.X, R.Y, zi);
    eq = true;
#pragma unroll
    for (int k = 0; k < 8; k++) eq &= enc[k] == sg[k];
    kes_store(a, list[q + lanes], (fl & 8u) != 0, (fl & 32u) != 0 && eq, (fl & 16u) != 0);
  }
  fe_mul(zi, inv, Zb);                                         // 1 / Z_a
#pragma unroll
  for (int k = 0; k < 8; k++) {
    R.X.v[k] = st[k * NT];
    R.Y.v[k] = st[(8 + k) * NT];
  }
  ge_tobytes_zi(enc, R.X, R.Y, zi);
  load_words(sg, a.kes_sig + 448 * ia, 8);                     // R of header a
  eq = true;
#pragma unroll
  for (int k = 0; k < 8; k++) eq &= enc[k] == sg[k];
  kes_store(a, ia, (fl & 1u) != 0, (fl & 4u) != 0 && eq, (fl & 2u) != 0);
}

// The Merkle walk of each leaf-key cache entry's representative, for the path dedup of
// k_kes_ck / k_kes_ck2 (rep_ok[e] = the walk's verdict).
__global__ void __launch_bounds__(NT) k_kes_merkle_reps(const uint32_t* __restrict__ counters, uint32_t max_entries,
                                                        const uint32_t* __restrict__ entry_rep, KesIn a,
                                                        uint8_t* __restrict__ rep_ok) {
  const uint32_t e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= min(counters[0], max_entries)) return;
  const size_t i = entry_rep[e];
  uint32_t vk[8], leaf[8];
  load_words(vk, a.hot_vk + 32 * i, 8);
  rep_ok[e] = kes_merkle(leaf, vk, kes_t(a, i), a.kes_sig + 448 * i) ? 1 : 0;
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
                     uint16_t* bits, uint8_t* ok_out, int prio) {
  OcertIn a{cold_vk, hot_vk, ocert_n, ocert_c0, sig, slot, slots_per_kes_period, max_kes_evo, bits, ok_out, nullptr,
            prio};
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
                   uint64_t slots_per_kes_period, uint16_t* bits, uint32_t pair_min, const uint32_t* entry_rep,
                   const uint8_t* rep_ok, int prio) {
  KesIn a{hot_vk, kes_sig, body_off, body_len, body, body_bytes_len, slot, ocert_c0, slots_per_kes_period,
          nullptr, bits, nullptr, nullptr, prio};
  if (pair_min)     // (the one-header kernel keeps its registers: the paired one spills 176 bytes)
    hipLaunchKernelGGL(k_kes_ck2, grid, block, 0, stream, list, count, item_entry, ktab, kinfo, gbtab, a, pair_min,
                       entry_rep, rep_ok);
  else
    hipLaunchKernelGGL(k_kes_ck, grid, block, 0, stream, list, count, item_entry, ktab, kinfo, gbtab, a, entry_rep,
                       rep_ok);
}
void launch_kes_merkle_reps(hipStream_t stream, const uint32_t* counters, uint32_t max_entries,
                            const uint32_t* entry_rep, const uint8_t* hot_vk, const uint8_t* kes_sig,
                            const uint64_t* slot, const uint64_t* ocert_c0, uint64_t slots_per_kes_period,
                            uint8_t* rep_ok) {
  KesIn a{hot_vk, kes_sig, nullptr, nullptr, nullptr, 0, slot, ocert_c0, slots_per_kes_period, nullptr, nullptr,
          nullptr, nullptr};
  hipLaunchKernelGGL(k_kes_merkle_reps, dim3((max_entries + NT - 1) / NT), dim3(NT), 0, stream, counters, max_entries,
                     entry_rep, a, rep_ok);
}
void launch_kes_leafkeys(dim3 grid, dim3 block, hipStream_t stream, size_t n, const uint8_t* kes_sig,
                         const uint64_t* slot, const uint64_t* ocert_c0, uint64_t slots_per_kes_period,
                         uint8_t* keys) {
  KesIn a{nullptr, kes_sig, nullptr, nullptr, nullptr, 0, slot, ocert_c0, slots_per_kes_period,
          nullptr, nullptr, nullptr, nullptr};
  hipLaunchKernelGGL(k_kes_leafkeys, grid, block, 0, stream, n, a, keys);
}
