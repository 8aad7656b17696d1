// k_keys.hip -- per-batch public-key cache (cold keys, VRF keys).
//
// A Praos batch repeats the same public keys many times (each pool signs its
// OCerts with one cold key and proves leadership with one VRF key: a 432k-
// header epoch of 3000 pools has ~144 headers per key).  The cache decodes
// each recurring key once and expands it into the multi-power tables of
// scalarmult.hpp (KT_CHUNKS x {1..8} 2^(16k) (-P)), so the per-header chains
// of those headers are 4 windows long instead of 64 (straus_comb).  Keys are compared
// byte for byte (open addressing on the 32 key bytes), so a cached header
// sees exactly the point, validity flags and encoding its own bytes give.
//
//   k_key_insert     per item: insert key into the hash set, count uses
//   k_key_assign     per slot: keys used >= min_count get a cache entry and a
//                    contiguous range of the hit list (one atomic per entry)
//   k_key_partition  per item: entry id; hits go to their entry's range, so the
//                    hit list is grouped by key: the lanes of a wave mostly share
//                    one key's tables (L1/L2-resident) instead of 64 different ones;
//                    misses to the miss list in item order (wave-aggregated)
//   k_key_precompute per entry: checks, decode, tables (and Y's encoding)
//
// Pool-key store (PRAOS_OPT_POOL_KEYS, cold and VRF keys): the entries and tables persist
// across runs of a context.  k_key_insert first probes the store (keys compared byte for
// byte) and a key found there is a hit on its stored entry without entering the batch's
// set; new keys get entry ids after the store's, their tables are built once, and
// k_pkey_publish adds them to the store for the runs that follow (on the same stream).
#include "k_keys.hpp"

__device__ __forceinline__ uint32_t key_hash(const uint32_t k[8]) {
  uint32_t h = k[0] * 0x9E3779B1u;
  h ^= k[1] + 0x7F4A7C15u + (h << 6) + (h >> 2);
  h ^= k[5] + (h << 6) + (h >> 2);
  return h;
}

// Items: i in [0, n), or list[0 .. *count) (e.g. the distinct OCerts of k_ocert_dedup).
// pentry != null: the pool-key store (pkey: 8 words per slot, pentry: entry or -1); an item
// whose key is stored gets item_slot = -2 - entry and counts one use of that entry (scnt).
__global__ void k_key_insert(size_t n, const uint32_t* __restrict__ list, const uint32_t* __restrict__ count,
                             const uint8_t* __restrict__ keys, uint32_t mask, uint32_t* slot_rep,
                             uint32_t* slot_cnt, int32_t* __restrict__ item_slot, const int32_t* __restrict__ pentry,
                             const uint32_t* __restrict__ pkey, uint32_t pmask, uint32_t* __restrict__ scnt) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (list ? (size_t)*count : n)) return;
  const size_t i = list ? list[t] : t;
  uint32_t k[8];
  load_words(k, keys + 32 * i, 8);
  if (pentry) {
    uint32_t g = key_hash(k) & pmask;
    for (uint32_t probe = 0; probe <= pmask; probe++) {
      const int32_t e = pentry[g];
      if (e < 0) break;                                // not stored
      bool same = true;
#pragma unroll
      for (int q = 0; q < 8; q++) same &= pkey[8 * (size_t)g + q] == k[q];
      if (same) {
        item_slot[i] = -2 - e;
        atomicAdd(&scnt[e], 1u);
        return;
      }
      g = (g + 1u) & pmask;
    }
  }
  uint32_t h = key_hash(k) & mask;
  for (uint32_t probe = 0; probe <= mask; probe++) {
    const uint32_t cur = atomicCAS(&slot_rep[h], 0u, (uint32_t)i + 1u);
    if (cur == 0u) break;                              // new key, this item represents it
    uint32_t o[8];
    load_words(o, keys + 32 * (size_t)(cur - 1u), 8);
    bool same = true;
#pragma unroll
    for (int q = 0; q < 8; q++) same &= o[q] == k[q];
    if (same) break;
    h = (h + 1u) & mask;
  }
  atomicAdd(&slot_cnt[h], 1u);
  item_slot[i] = (int32_t)h;
}

// counters: [0] entries, [1] hits, [2] misses, [3] hit-list ranges handed out
// Wave-aggregated: the wave's new entries and the sum of their use counts are claimed with one
// atomic each (ids and hit-list ranges follow the lanes' order inside the wave).  One atomic
// per entry on the two shared counters serialised on their addresses: 0.74 ms for the 173k
// leaf keys of configs[3] (profiles/r04c4_rocprof.txt).
__global__ void k_key_assign(uint32_t cap, const uint32_t* __restrict__ slot_rep, const uint32_t* __restrict__ slot_cnt,
                             uint32_t min_count, uint32_t max_entries, int32_t* __restrict__ slot_entry,
                             uint32_t* __restrict__ entry_rep, uint32_t* __restrict__ entry_pos, uint32_t* counters) {
  const uint32_t h = blockIdx.x * blockDim.x + threadIdx.x;
  const bool in = h < cap;                           // every lane stays for the ballot and the scan
  const uint32_t rep = in ? slot_rep[h] : 0u;
  const uint32_t cnt = in ? slot_cnt[h] : 0u;
  const bool take = rep != 0u && cnt >= min_count;
  const uint64_t m = __ballot(take);
  if (m == 0) {
    if (in) slot_entry[h] = -1;
    return;
  }
  const uint32_t lane = __lane_id();
  uint32_t e_base = 0;
  if (lane == 0) e_base = atomicAdd(&counters[0], (uint32_t)__popcll(m));
  e_base = __shfl(e_base, 0);
  // entry ids past max_entries (a full pool-key store, or the per-batch cap) stay uncached:
  // only the keys that get an entry claim a range of the hit list, so it has no holes
  const uint32_t k = e_base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
  const bool got = take && k < max_entries;
  // exclusive prefix sum of the cached keys' use counts over the wave
  uint32_t incl = got ? cnt : 0u;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t v = __shfl_up(incl, d);
    if (lane >= (uint32_t)d) incl += v;
  }
  const uint32_t total = __shfl(incl, 63);
  uint32_t p_base = 0;
  if (lane == 0 && total) p_base = atomicAdd(&counters[3], total);
  p_base = __shfl(p_base, 0);
  int32_t e = -1;
  if (got) {
    e = (int32_t)k;
    entry_rep[k] = rep - 1u;
    entry_pos[k] = p_base + incl - cnt;              // this key's range of the hit list
  }
  if (in) slot_entry[h] = e;
}

// The stored entries' hit-list ranges, after the new keys' (counters[3] is their end once
// k_key_assign is done): spos[e] = the start of entry e's range (scnt[e] uses this run), so the
// stored keys' hits are grouped by key as the new keys' are.
__global__ void k_key_store_ranges(uint32_t entries, const uint32_t* __restrict__ scnt, uint32_t* __restrict__ spos,
                                   uint32_t* counters) {
  const uint32_t e = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t cnt = e < entries ? scnt[e] : 0u;   // every lane stays for the scan
  const uint32_t lane = __lane_id();
  uint32_t incl = cnt;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t v = __shfl_up(incl, d);
    if (lane >= (uint32_t)d) incl += v;
  }
  const uint32_t total = __shfl(incl, 63);
  if (total == 0) return;
  uint32_t p_base = 0;
  if (lane == 0) p_base = atomicAdd(&counters[3], total);
  p_base = __shfl(p_base, 0);
  if (cnt) spos[e] = p_base + incl - cnt;
}

// appends i to list (wave-aggregated atomic: one atomic per wave and list)
__device__ __forceinline__ void wave_append(bool pred, uint32_t value, uint32_t* counter, uint32_t* list) {
  const uint64_t m = __ballot(pred);
  if (m == 0) return;
  const int leader = __ffsll((unsigned long long)m) - 1;
  const uint32_t lane = __lane_id();
  uint32_t base = 0;
  if ((int)lane == leader) base = atomicAdd(counter, (uint32_t)__popcll(m));
  base = __shfl(base, leader);
  if (pred) {
    const uint32_t below = (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
    list[base + below] = value;
  }
}

// Stored keys' items (item_slot <= -2) are hits too; they go to their entry's range after the
// new keys' ranges (k_key_store_ranges).
__global__ void k_key_partition(size_t n, const uint32_t* __restrict__ list, const uint32_t* __restrict__ count,
                                const int32_t* __restrict__ item_slot, const int32_t* __restrict__ slot_entry,
                                int32_t* __restrict__ item_entry, uint32_t* __restrict__ entry_pos,
                                uint32_t* __restrict__ hit_list, uint32_t* __restrict__ miss_list,
                                uint32_t* counters, uint32_t* __restrict__ spos) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool in = t < (list ? (size_t)*count : n);   // every lane stays for the ballots
  const size_t i = in ? (list ? list[t] : t) : 0;
  const int32_t sl = in ? item_slot[i] : -1;
  const bool stored = sl <= -2;
  const int32_t e = !in ? -1 : (stored ? -2 - sl : slot_entry[sl]);
  if (in) item_entry[i] = e;
  if (in && e >= 0) hit_list[atomicAdd(stored ? &spos[e] : &entry_pos[e], 1u)] = (uint32_t)i;
  const uint64_t hits = __ballot(in && e >= 0);
  if (hits && __lane_id() == (uint32_t)(__ffsll((unsigned long long)hits) - 1))
    atomicAdd(&counters[1], (uint32_t)__popcll(hits));
  wave_append(in && e < 0, (uint32_t)i, &counters[2], miss_list);
}

__global__ void __launch_bounds__(64) k_key_precompute(int kind, const uint32_t* __restrict__ counters,
                                                        uint32_t max_entries, const uint32_t* __restrict__ entry_rep,
                                                        const uint8_t* __restrict__ keys, ge_cached* __restrict__ ktab,
                                                        uint32_t* __restrict__ kinfo, int wave_prio,
                                                        const uint32_t* __restrict__ base) {
  // latency-bound (a short list of long chains) and on the critical path of the cached
  // chains: raised wave priority wins the SIMD's issue arbitration against the
  // throughput kernels resident beside it
  if (wave_prio) __builtin_amdgcn_s_setprio(3);
  // grid-stride: the host sizes the grid from the previous run's entry count (a grid sized
  // for the worst case is thousands of empty blocks that wait for wave slots on a busy GPU)
  const uint32_t ne = min(counters[0], max_entries);
  for (uint32_t e = (base ? *base : 0u) + blockIdx.x * blockDim.x + threadIdx.x; e < ne; e += gridDim.x * blockDim.x)
    key_precompute_entry(kind, e, entry_rep, keys, ktab, kinfo);
}

// pass 2: lane (entry, chunk) expands the chunk base into its 8-entry table
__global__ void __launch_bounds__(256) k_key_tables(int kind, const uint32_t* __restrict__ counters,
                                                    uint32_t max_entries, ge_cached* __restrict__ ktab,
                                                    int wave_prio, const uint32_t* __restrict__ base) {
  if (wave_prio) __builtin_amdgcn_s_setprio(3);
  const uint32_t e0 = base ? *base : 0u, ne = min(counters[0], max_entries);
  const uint32_t lanes = ne > e0 ? (ne - e0) * KT_CHUNKS : 0u;
  for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < lanes; t += gridDim.x * blockDim.x) {
    const uint32_t e = e0 + t / KT_CHUNKS, k = t % KT_CHUNKS;
    if (k < (uint32_t)key_chunks(kind)) key_chunk_table(ktab + (size_t)e * KT_STRIDE + 8 * k);
  }
}

// The run's new entries [*base, min(counters[0], max_entries)) into the pool-key store
// (distinct keys, so a claimed slot needs no comparison); *count = the store's entries after.
__global__ void k_pkey_publish(const uint32_t* __restrict__ counters, const uint32_t* __restrict__ base,
                               uint32_t max_entries, const uint32_t* __restrict__ entry_rep,
                               const uint8_t* __restrict__ keys, int32_t* pentry, uint32_t* __restrict__ pkey,
                               uint32_t pmask, uint32_t* __restrict__ count) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t ne = min(counters[0], max_entries);
  if (t == 0) *count = ne;
  for (uint32_t e = *base + t; e < ne; e += gridDim.x * blockDim.x) {
    uint32_t k[8];
    load_words(k, keys + 32 * (size_t)entry_rep[e], 8);
    uint32_t g = key_hash(k) & pmask;
    for (uint32_t probe = 0; probe <= pmask; probe++) {
      if (atomicCAS(&pentry[g], -1, (int32_t)e) == -1) {
#pragma unroll
        for (int q = 0; q < 8; q++) pkey[8 * (size_t)g + q] = k[q];
        break;
      }
      g = (g + 1u) & pmask;
    }
  }
}

// Before a run that uses the store: empty it when asked (force) or when the last run left it more
// than `limit` entries.  The decision is made on the device from the count that run published
// (count[0]), into count[1], so the host never reads a count whose copy may still be in flight.
__global__ void k_pkey_decide(uint32_t* count, uint32_t limit, int force) {
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    const uint32_t r = (force || count[0] > limit) ? 1u : 0u;
    count[1] = r;
    if (r) count[0] = 0;
  }
}
__global__ void k_pkey_clear(const uint32_t* __restrict__ count, int32_t* pentry, uint32_t slots) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < slots && count[1]) pentry[i] = -1;
}

// ---- OCert signature dedup (PRAOS_OPT_DEDUP)
// The OCert signature check depends only on (cold vk, hot vk, n, c0, sigma)
// (Praos.hs:580): every header a pool forges under one operational certificate
// carries the same 144 bytes, so a mainnet-shaped epoch has ~one distinct OCert
// per pool.  k_ocert_dedup keys a hash set on the whole tuple, compared byte for
// byte; the first item of each distinct tuple (its representative) is verified
// and k_ocert_fanout copies that verdict to every item carrying identical bytes,
// adding each header's own KES-period checks (which depend on its slot).
struct OcertTuple { uint32_t w[36]; };   // cold 8 | hot 8 | n 2 | c0 2 | sigma 16
__device__ __forceinline__ void ocert_tuple(OcertTuple& t, const uint8_t* cold, const uint8_t* hot, const uint64_t* on,
                                            const uint64_t* oc, const uint8_t* sig, size_t i) {
  load_words(t.w, cold + 32 * i, 8);
  load_words(t.w + 8, hot + 32 * i, 8);
  const uint64_t n = on[i], c0 = oc[i];
  t.w[16] = (uint32_t)n; t.w[17] = (uint32_t)(n >> 32);
  t.w[18] = (uint32_t)c0; t.w[19] = (uint32_t)(c0 >> 32);
  load_words(t.w + 20, sig + 64 * i, 16);
}

// counters[0] = distinct tuples (representatives, listed in reps)
__global__ void k_ocert_dedup(size_t n, const uint8_t* __restrict__ cold, const uint8_t* __restrict__ hot,
                              const uint64_t* __restrict__ on, const uint64_t* __restrict__ oc,
                              const uint8_t* __restrict__ sig, uint32_t mask, uint32_t* slot_rep,
                              uint32_t* __restrict__ item_rep, uint32_t* __restrict__ reps, uint32_t* counters) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool in = i < n;                              // every lane stays for the ballot
  bool rep = false;
  if (in) {
    OcertTuple t;
    ocert_tuple(t, cold, hot, on, oc, sig, i);
    uint32_t h = t.w[0] * 0x9E3779B1u;
    h ^= t.w[9] + 0x7F4A7C15u + (h << 6) + (h >> 2);
    h ^= t.w[16] + (h << 6) + (h >> 2);
    h ^= t.w[20] + (h << 6) + (h >> 2);
    h ^= t.w[27] + (h << 6) + (h >> 2);
    h &= mask;
    uint32_t r = (uint32_t)i;
    for (uint32_t probe = 0; probe <= mask; probe++) {
      const uint32_t cur = atomicCAS(&slot_rep[h], 0u, (uint32_t)i + 1u);
      if (cur == 0u) { rep = true; break; }           // first of its tuple
      OcertTuple o;
      ocert_tuple(o, cold, hot, on, oc, sig, cur - 1u);
      bool same = true;
#pragma unroll
      for (int q = 0; q < 36; q++) same &= o.w[q] == t.w[q];
      if (same) { r = cur - 1u; break; }
      h = (h + 1u) & mask;
    }
    item_rep[i] = r;
  }
  wave_append(rep, (uint32_t)i, &counters[0], reps);
}

// bits[i] = verdict of i's representative (ok[rep] written by the verify kernels in
// ok_out mode) + i's own KES-period checks (Praos.hs:567-568, 596-599)
__global__ void k_ocert_fanout(size_t n, const uint32_t* __restrict__ item_rep, const uint8_t* __restrict__ ok,
                               const uint64_t* __restrict__ slot, const uint64_t* __restrict__ oc,
                               uint64_t slots_per_kes_period, uint64_t max_kes_evo, uint16_t* __restrict__ bits) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint16_t b = ok[item_rep[i]] ? 0 : PRAOS_BIT_OCERT_SIG;
  const uint64_t c0 = oc[i];
  const uint64_t kp = slot[i] / slots_per_kes_period;
  if (!(c0 <= kp)) b |= PRAOS_BIT_KES_BEFORE_START;
  if (!(kp < c0 + max_kes_evo)) b |= PRAOS_BIT_KES_AFTER_END;
  bits[i] = b;
}

// ---- host launchers
void launch_key_insert(dim3 grid, dim3 block, hipStream_t stream, size_t n, const uint32_t* list, const uint32_t* count,
                       const uint8_t* keys, uint32_t mask, uint32_t* slot_rep, uint32_t* slot_cnt, int32_t* item_slot,
                       const int32_t* pentry, const uint32_t* pkey, uint32_t pmask, uint32_t* scnt) {
  hipLaunchKernelGGL(k_key_insert, grid, block, 0, stream, n, list, count, keys, mask, slot_rep, slot_cnt, item_slot,
                     pentry, pkey, pmask, scnt);
}
void launch_key_store_ranges(hipStream_t stream, uint32_t entries, const uint32_t* scnt, uint32_t* spos,
                             uint32_t* counters) {
  hipLaunchKernelGGL(k_key_store_ranges, dim3((entries + 255) / 256), dim3(256), 0, stream, entries, scnt, spos,
                     counters);
}
void launch_key_assign(dim3 grid, dim3 block, hipStream_t stream, uint32_t cap, const uint32_t* slot_rep,
                       const uint32_t* slot_cnt, uint32_t min_count, uint32_t max_entries, int32_t* slot_entry,
                       uint32_t* entry_rep, uint32_t* entry_pos, uint32_t* counters) {
  hipLaunchKernelGGL(k_key_assign, grid, block, 0, stream, cap, slot_rep, slot_cnt, min_count, max_entries, slot_entry,
                     entry_rep, entry_pos, counters);
}
void launch_key_partition(dim3 grid, dim3 block, hipStream_t stream, size_t n, const uint32_t* list,
                          const uint32_t* count, const int32_t* item_slot, const int32_t* slot_entry,
                          int32_t* item_entry, uint32_t* entry_pos, uint32_t* hit_list, uint32_t* miss_list,
                          uint32_t* counters, uint32_t* spos) {
  hipLaunchKernelGGL(k_key_partition, grid, block, 0, stream, n, list, count, item_slot, slot_entry, item_entry,
                     entry_pos, hit_list, miss_list, counters, spos);
}
void launch_key_precompute(int kind, hipStream_t stream, const uint32_t* counters, uint32_t max_entries,
                           const uint32_t* entry_rep, const uint8_t* keys, ge_cached* ktab, uint32_t* kinfo,
                           int wave_prio, const uint32_t* base, uint32_t span, int mode) {
  if (mode == 1)
    launch_key_precompute4(kind, stream, counters, max_entries, entry_rep, keys, ktab, kinfo, wave_prio, base, span);
  else
    hipLaunchKernelGGL(k_key_precompute, dim3((span + 63) / 64), dim3(64), 0, stream, kind, counters, max_entries,
                       entry_rep, keys, ktab, kinfo, wave_prio, base);
  const size_t lanes = (size_t)span * KT_CHUNKS;
  hipLaunchKernelGGL(k_key_tables, dim3((unsigned)((lanes + 255) / 256)), dim3(256), 0, stream, kind, counters,
                     max_entries, ktab, wave_prio, base);
}
void launch_pkey_reset(hipStream_t stream, uint32_t* count, int32_t* pentry, uint32_t slots, uint32_t limit, int force) {
  hipLaunchKernelGGL(k_pkey_decide, dim3(1), dim3(64), 0, stream, count, limit, force);
  hipLaunchKernelGGL(k_pkey_clear, dim3((slots + 255) / 256), dim3(256), 0, stream, count, pentry, slots);
}
void launch_pkey_publish(hipStream_t stream, const uint32_t* counters, const uint32_t* base, uint32_t max_entries,
                         const uint32_t* entry_rep, const uint8_t* keys, int32_t* pentry, uint32_t* pkey,
                         uint32_t pmask, uint32_t* count, uint32_t span) {
  hipLaunchKernelGGL(k_pkey_publish, dim3((span + 255) / 256), dim3(256), 0, stream, counters, base, max_entries,
                     entry_rep, keys, pentry, pkey, pmask, count);
}
void launch_ocert_dedup(dim3 grid, dim3 block, hipStream_t stream, size_t n, const uint8_t* cold, const uint8_t* hot,
                        const uint64_t* on, const uint64_t* oc, const uint8_t* sig, uint32_t mask, uint32_t* slot_rep,
                        uint32_t* item_rep, uint32_t* reps, uint32_t* counters) {
  hipLaunchKernelGGL(k_ocert_dedup, grid, block, 0, stream, n, cold, hot, on, oc, sig, mask, slot_rep, item_rep, reps,
                     counters);
}
void launch_ocert_fanout(dim3 grid, dim3 block, hipStream_t stream, size_t n, const uint32_t* item_rep,
                         const uint8_t* ok, const uint64_t* slot, const uint64_t* oc, uint64_t slots_per_kes_period,
                         uint64_t max_kes_evo, uint16_t* bits) {
  hipLaunchKernelGGL(k_ocert_fanout, grid, block, 0, stream, n, item_rep, ok, slot, oc, slots_per_kes_period,
                     max_kes_evo, bits);
}
