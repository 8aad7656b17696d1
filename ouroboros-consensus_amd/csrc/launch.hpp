// launch.hpp -- host launchers exported by each kernel module (generated
// alongside the kernels; see the bottom of k_*.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <cstddef>
#include <cstdint>
// Block size of the kernels without LDS tables (V / U / join of the VRF, the cached-key
// Ed25519 chains).  1-wave blocks for small batches (so that 54k headers = 844 waves spread
// over all 256 CUs instead of 211 four-wave blocks) measured slower (k_vrf_v 2.70 -> 2.98 ms
// at 54k, profiles/r03/timeline_54k_wave_blocks.txt): 4-wave blocks everywhere.
static inline unsigned lat_block(size_t n) { (void)n; return 256u; }
struct ge_niels;
struct ge_cached;
void launch_ocert(dim3 grid, dim3 block, hipStream_t stream, size_t n, const uint32_t* list, const uint32_t* count,
                  const ge_niels* gbtab, const uint8_t* cold_vk, const uint8_t* hot_vk, const uint64_t* ocert_n,
                  const uint64_t* ocert_c0, const uint8_t* sig, const uint64_t* slot, uint64_t slots_per_kes_period,
                  uint64_t max_kes_evo, uint16_t* bits, uint8_t* ok_out, ge_cached* tabs);
void launch_ocert_ck(dim3 grid, dim3 block, hipStream_t stream, const uint32_t* list, const uint32_t* count,
                     const int32_t* item_entry, const ge_cached* ktab, const uint32_t* kinfo, const ge_niels* gbtab,
                     const uint8_t* cold_vk, const uint8_t* hot_vk, const uint64_t* ocert_n, const uint64_t* ocert_c0,
                     const uint8_t* sig, const uint64_t* slot, uint64_t slots_per_kes_period, uint64_t max_kes_evo,
                     uint16_t* bits, uint8_t* ok_out, int prio = 0);
void launch_vrf(dim3 grid, dim3 block, hipStream_t stream, size_t n, const uint32_t* list, const uint32_t* count,
                const ge_niels* gbtab, const uint8_t* cold_vk, const uint8_t* vrf_vk, const uint8_t* vrf_out,
                const uint8_t* vrf_proof, const uint64_t* slot, const uint32_t* eta0, int eta0_neutral,
                const uint8_t* eta_idx, const uint32_t* pool_hash, const uint32_t* pool_vrf, const int32_t* pool_map,
                uint32_t npools, int check_output, const uint8_t* alpha_in, uint16_t* bits, int32_t* pool_idx,
                int32_t* pool_sorted_idx, uint8_t* beta_out, uint8_t* leader_out, uint8_t* nonce_out, uint8_t* ok_out,
                ge_cached* tabs);
void launch_vrf_ck(dim3 grid, dim3 block, hipStream_t stream, const uint32_t* list, const uint32_t* count,
                   const int32_t* item_entry, const ge_cached* ktab, const uint32_t* kinfo, const ge_niels* gbtab,
                   const uint8_t* cold_vk, const uint8_t* vrf_vk, const uint8_t* vrf_out, const uint8_t* vrf_proof,
                   const uint64_t* slot, const uint32_t* eta0, int eta0_neutral, const uint8_t* eta_idx,
                   const uint32_t* pool_hash, const uint32_t* pool_vrf, const int32_t* pool_map, uint32_t npools,
                   int check_output, const uint8_t* alpha_in, uint16_t* bits, int32_t* pool_idx,
                   int32_t* pool_sorted_idx, uint8_t* beta_out, uint8_t* leader_out, uint8_t* nonce_out,
                   uint8_t* ok_out, ge_cached* tabs);
// pentry / pkey / pmask: the pool-key store probed first (null: none)
void launch_key_insert(dim3 grid, dim3 block, hipStream_t stream, size_t n, const uint32_t* list, const uint32_t* count,
                       const uint8_t* keys, uint32_t mask, uint32_t* slot_rep, uint32_t* slot_cnt, int32_t* item_slot,
                       const int32_t* pentry, const uint32_t* pkey, uint32_t pmask, uint32_t* scnt);
// stored entries' hit-list ranges (after the new keys'), from their uses this run
void launch_key_store_ranges(hipStream_t stream, uint32_t entries, const uint32_t* scnt, uint32_t* spos,
                             uint32_t* counters);
void launch_key_assign(dim3 grid, dim3 block, hipStream_t stream, uint32_t cap, const uint32_t* slot_rep,
                       const uint32_t* slot_cnt, uint32_t min_count, uint32_t max_entries, int32_t* slot_entry,
                       uint32_t* entry_rep, uint32_t* entry_pos, uint32_t* counters);
void launch_key_partition(dim3 grid, dim3 block, hipStream_t stream, size_t n, const uint32_t* list,
                          const uint32_t* count, const int32_t* item_slot, const int32_t* slot_entry,
                          int32_t* item_entry, uint32_t* entry_pos, uint32_t* hit_list, uint32_t* miss_list,
                          uint32_t* counters, uint32_t* spos);
void launch_ocert_dedup(dim3 grid, dim3 block, hipStream_t stream, size_t n, const uint8_t* cold, const uint8_t* hot,
                        const uint64_t* on, const uint64_t* oc, const uint8_t* sig, uint32_t mask, uint32_t* slot_rep,
                        uint32_t* item_rep, uint32_t* reps, uint32_t* counters);
void launch_ocert_fanout(dim3 grid, dim3 block, hipStream_t stream, size_t n, const uint32_t* item_rep,
                         const uint8_t* ok, const uint64_t* slot, const uint64_t* oc, uint64_t slots_per_kes_period,
                         uint64_t max_kes_evo, uint16_t* bits);
// entries [*base (0 when null), min(counters[0], max_entries)), at most span of them
void launch_key_precompute(int kind, hipStream_t stream, const uint32_t* counters, uint32_t max_entries,
                           const uint32_t* entry_rep, const uint8_t* keys, ge_cached* ktab, uint32_t* kinfo,
                           int wave_prio, const uint32_t* base, uint32_t span,
                           int mode);                      // 1: the chain from the ILP-4 build (k_keys4.hip)
void launch_key_precompute4(int kind, hipStream_t stream, const uint32_t* counters, uint32_t max_entries,
                            const uint32_t* entry_rep, const uint8_t* keys, ge_cached* ktab, uint32_t* kinfo,
                            int wave_prio, const uint32_t* base, uint32_t span);
void launch_pkey_reset(hipStream_t stream, uint32_t* count, int32_t* pentry, uint32_t slots, uint32_t limit, int force);
void launch_pkey_publish(hipStream_t stream, const uint32_t* counters, const uint32_t* base, uint32_t max_entries,
                         const uint32_t* entry_rep, const uint8_t* keys, int32_t* pentry, uint32_t* pkey,
                         uint32_t pmask, uint32_t* count, uint32_t span);
// the cached verifies of a small batch from the ILP-4 build (k_miss4.hip)
void launch_ocert_ck4(hipStream_t stream, size_t n, const uint32_t* list, const uint32_t* count,
                      const int32_t* item_entry, const ge_cached* ktab, const uint32_t* kinfo, const ge_niels* gbtab,
                      const uint8_t* cold_vk, const uint8_t* hot_vk, const uint64_t* ocert_n, const uint64_t* ocert_c0,
                      const uint8_t* sig, const uint64_t* slot, uint64_t slots_per_kes_period, uint64_t max_kes_evo,
                      uint16_t* bits, uint8_t* ok_out);
void launch_kes_ck4(hipStream_t stream, size_t n, const uint32_t* list, const uint32_t* count,
                    const int32_t* item_entry, const ge_cached* ktab, const uint32_t* kinfo, const ge_niels* gbtab,
                    const uint8_t* hot_vk, const uint8_t* kes_sig, const uint64_t* body_off, const uint32_t* body_len,
                    const uint8_t* body, size_t body_bytes_len, const uint64_t* slot, const uint64_t* ocert_c0,
                    uint64_t slots_per_kes_period, uint16_t* bits);
// the uncached verifies of a small batch from the ILP-4 build (k_miss4.hip), list mode only
void launch_ocert4(dim3 grid, dim3 block, hipStream_t stream, const uint32_t* list, const uint32_t* count,
                   const ge_niels* gbtab, const uint8_t* cold_vk, const uint8_t* hot_vk, const uint64_t* ocert_n,
                   const uint64_t* ocert_c0, const uint8_t* sig, const uint64_t* slot, uint64_t slots_per_kes_period,
                   uint64_t max_kes_evo, uint16_t* bits, uint8_t* ok_out, ge_cached* tabs, int prio);
void launch_kes4(dim3 grid, dim3 block, hipStream_t stream, const uint32_t* list, const uint32_t* count,
                 const ge_niels* gbtab, const uint8_t* hot_vk, const uint8_t* kes_sig, const uint64_t* body_off,
                 const uint32_t* body_len, const uint8_t* body, size_t body_bytes_len, const uint64_t* slot,
                 const uint64_t* ocert_c0, uint64_t slots_per_kes_period, uint16_t* bits, ge_cached* tabs, int prio);
void launch_kes(dim3 grid, dim3 block, hipStream_t stream, size_t n, const uint32_t* list, const uint32_t* count,
                const ge_niels* gbtab, const uint8_t* hot_vk, const uint8_t* kes_sig, const uint64_t* body_off,
                const uint32_t* body_len, const uint8_t* body, size_t body_bytes_len, const uint64_t* slot,
                const uint64_t* ocert_c0, uint64_t slots_per_kes_period, const uint32_t* period, uint16_t* bits,
                uint8_t* result, ge_cached* tabs);
void launch_kes_ck(dim3 grid, dim3 block, hipStream_t stream, const uint32_t* list, const uint32_t* count,
                   const int32_t* item_entry, const ge_cached* ktab, const uint32_t* kinfo, const ge_niels* gbtab,
                   const uint8_t* hot_vk, const uint8_t* kes_sig, const uint64_t* body_off, const uint32_t* body_len,
                   const uint8_t* body, size_t body_bytes_len, const uint64_t* slot, const uint64_t* ocert_c0,
                   uint64_t slots_per_kes_period, uint16_t* bits,
                   uint32_t pair_min,                       // two headers per lane from pair_min hits on (0: never)
                   const uint32_t* entry_rep,               // with rep_ok (k_kes_merkle_reps): the Merkle path
                   const uint8_t* rep_ok, int prio = 0);                  // dedup per cache entry (null: every item walks)
void launch_kes_merkle_reps(hipStream_t stream, const uint32_t* counters, uint32_t max_entries,
                            const uint32_t* entry_rep, const uint8_t* hot_vk, const uint8_t* kes_sig,
                            const uint64_t* slot, const uint64_t* ocert_c0, uint64_t slots_per_kes_period,
                            uint8_t* rep_ok);
void launch_kes_leafkeys(dim3 grid, dim3 block, hipStream_t stream, size_t n, const uint8_t* kes_sig,
                         const uint64_t* slot, const uint64_t* ocert_c0, uint64_t slots_per_kes_period,
                         uint8_t* keys);
void launch_init_btab(dim3 grid, dim3 block, hipStream_t stream, ge_niels* btab);
void launch_init_bcomb16(hipStream_t stream, const ge_niels* btab, ge_niels* bcomb16);
void launch_leader(dim3 grid, dim3 block, hipStream_t stream, size_t n, const uint8_t* leader_in, const int32_t* pool_sorted_idx, const uint32_t* pool_x, const uint32_t* x_item, int f_is_one, int leader_words, const uint16_t* b_ocert, const uint16_t* b_kes, const uint16_t* b_vrf, uint16_t* bits, uint8_t* is_leader, int32_t* iters, const uint16_t* dec_status);
void launch_debug_fe(dim3 grid, dim3 block, hipStream_t stream, int op, size_t n, const uint8_t* a, const uint8_t* b, uint8_t* r);
void launch_debug_sha512(dim3 grid, dim3 block, hipStream_t stream, size_t n, const uint8_t* prefix, const uint64_t* off, const uint32_t* len, const uint8_t* msg, uint8_t* out);
void launch_debug_blake2b(dim3 grid, dim3 block, hipStream_t stream, size_t n, const uint8_t* in, uint8_t* out);
void launch_debug_sc_reduce(dim3 grid, dim3 block, hipStream_t stream, size_t n, const uint8_t* in, uint8_t* out);
void launch_debug_decode(dim3 grid, dim3 block, hipStream_t stream, size_t n, const uint8_t* in, uint8_t* out, uint8_t* ok);
void launch_debug_smul_base(dim3 grid, dim3 block, hipStream_t stream, size_t n, const ge_niels* gbtab, const uint8_t* s, uint8_t* out);
void launch_debug_h2c(dim3 grid, dim3 block, hipStream_t stream, size_t n, const uint8_t* pk, const uint8_t* alpha, uint8_t* out);
void launch_synth_pools(dim3 grid, dim3 block, hipStream_t stream, uint32_t npools, const ge_niels* gbtab, const uint32_t* master, uint32_t* cold_seed, uint32_t* cold_pk, uint32_t* vrf_seed, uint32_t* vrf_pk, uint32_t* kes_seed, uint8_t* pool_hash28, uint8_t* pool_vrf32);
void launch_synth_kes_leaves(dim3 grid, dim3 block, hipStream_t stream, uint32_t npools, const ge_niels* gbtab, const uint32_t* kes_seed, uint32_t* leaf_seed, uint32_t* tree);
void launch_synth_kes_tree(dim3 grid, dim3 block, hipStream_t stream, uint32_t npools, uint32_t* tree);
void launch_synth_headers(dim3 grid, dim3 block, hipStream_t stream, size_t n, const ge_niels* gbtab, uint32_t npools, uint32_t nkes, uint64_t first_slot, uint64_t slot_stride, uint64_t slots_per_kes_period, uint32_t blen, uint64_t salt, const uint32_t* eta0, int eta0_neutral, const uint32_t* cold_seed, const uint32_t* cold_pk, const uint32_t* vrf_seed, const uint32_t* vrf_pk, const uint32_t* leaf_seed, const uint32_t* tree, uint8_t* msg_scratch, uint64_t* slot, uint8_t* cold_vk, uint8_t* vrf_vk, uint8_t* vrf_out, uint8_t* vrf_proof, uint8_t* hot_vk, uint64_t* ocert_n, uint64_t* ocert_c0, uint8_t* ocert_sig, uint8_t* kes_sig, uint64_t* body_off, uint32_t* body_len, uint8_t* body_bytes, int tpraos, uint8_t* l_out, uint8_t* l_proof, const uint8_t* body_hash_in, const uint64_t* sched_slot, const uint32_t* sched_pool, uint64_t block_no0, uint32_t* leaf_of);
void launch_synth_link(hipStream_t stream, size_t n, const ge_niels* gbtab, const uint8_t* prev0,
                       const uint32_t* leaf_seed, uint32_t nleaves, uint32_t* lkeys, const uint32_t* tree,
                       const uint32_t* leaf_of, uint8_t* body_bytes, const uint64_t* body_off, uint32_t* body_len,
                       uint8_t* kes_sig, uint8_t* header_hash, uint32_t stride);
void launch_synth_vrf_scalar(dim3 grid, dim3 block, hipStream_t stream, uint32_t npools, const uint32_t* vrf_seed,
                             uint32_t* vrf_x);
void launch_synth_leader_search(dim3 grid, dim3 block, hipStream_t stream, uint64_t first_slot, uint64_t nslots,
                                uint32_t p0, uint32_t pn, const uint32_t* vrf_x, const uint32_t* vrf_pk,
                                const uint32_t* pool_thr, const uint32_t* eta0, int eta0_neutral, int f_is_one,
                                int tpraos, int32_t* leader);
void launch_synth_corrupt(dim3 grid, dim3 block, hipStream_t stream, size_t n, uint32_t per10000, uint64_t salt, uint8_t* ocert_sig, uint8_t* kes_sig, uint8_t* vrf_proof, uint8_t* vrf_out, uint8_t* body_bytes, const uint64_t* body_off, const uint32_t* body_len, uint8_t* corrupted, uint8_t* l_proof, int cbor_body, uint32_t fields, uint8_t* cold_vk, uint8_t* hot_vk, uint64_t* ocert_n, uint64_t* ocert_c0);
// two-stage VRF of the header pipeline (k_vrf.hip): stage V over all n headers into the
// record `mid` (VRF_MID_PLANES x 16 x n bytes); stage F over list[0 .. *count) (or all n when
// list is null), cached (ktab != null: k_vrf_fin) or per-lane U (k_vrf_fin_nc)
void launch_vrf_v(hipStream_t stream, size_t n, const uint8_t* vrf_vk, const uint8_t* vrf_proof, const uint64_t* slot,
                  const uint32_t* eta0, int eta0_neutral, const uint8_t* eta_idx, ge_cached* tabs, void* mid,
                  size_t i0 = 0, size_t i1 = SIZE_MAX,    // headers [i0, min(i1, n)); mid stride n
                  int wave_prio = 0,                       // waves at s_setprio 3
                  int tp_seed = 0,                         // 1 + k: TPraos mkSeed alpha, ucNonce k
                  int ilp4 = 0);                           // 1: the ILP-4 build (k_vrf_v4.hip),
                                                           // 2: the same holding its SIMD alone

// stage V built with the ILP-4 group formulas at 2 waves per SIMD (k_vrf_v4.hip; small batches)
void launch_vrf_v4(hipStream_t stream, size_t n, size_t i0, size_t i1, const uint8_t* vrf_vk,
                   const uint8_t* vrf_proof, const uint64_t* slot, const uint32_t* eta0, int eta0_neutral,
                   const uint8_t* eta_idx, ge_cached* tabs, void* mid, int wave_prio, int tp_seed, int excl);
void launch_vrf_fin(hipStream_t stream, size_t n, const uint32_t* list, const uint32_t* count,
                    const int32_t* item_entry, const ge_cached* ktab, const uint32_t* kinfo, const ge_niels* comb,
                    const ge_niels* gbtab, const uint8_t* cold_vk, const uint8_t* vrf_vk, const uint8_t* vrf_out,
                    const uint8_t* vrf_proof, const uint32_t* pool_hash, const uint32_t* pool_vrf,
                    const int32_t* pool_map, uint32_t npools, int check_output, uint16_t* bits, int32_t* pool_idx,
                    int32_t* pool_sorted_idx, uint8_t* beta_out, uint8_t* leader_out, uint8_t* nonce_out,
                    ge_cached* tabs, const void* mid);
// three-kernel VRF: stage U (cached: ktab != null, k_vrf_u over the hit list; uncached: k_vrf_u_nc
// over list[0 .. *count) or all n, 8-entry lane tables utabs) and the join over all n
void launch_vrf_u(hipStream_t stream, size_t n, const uint32_t* list, const uint32_t* count, const int32_t* item_entry,
                  const ge_cached* ktab, const uint32_t* kinfo, const ge_niels* comb, const ge_niels* gbtab,
                  const uint8_t* vrf_vk, const uint8_t* vrf_proof, ge_cached* utabs, void* mid,
                  int ilp4 = 0,                            // cached keys: the ILP-4 build (k_vrf_v4.hip k_vrf_u4)
                  int prio = 0);                           // cached keys: waves at s_setprio <prio>
void launch_vrf_u4(hipStream_t stream, size_t n, const uint32_t* list, const uint32_t* count, const int32_t* item_entry,
                   const ge_cached* ktab, const uint32_t* kinfo, const ge_niels* comb, const uint8_t* vrf_proof,
                   void* mid, int prio = 0);
void launch_vrf_join(hipStream_t stream, size_t n, const uint8_t* cold_vk, const uint8_t* vrf_vk,
                     const uint8_t* vrf_out, const uint8_t* vrf_proof, const uint32_t* pool_hash,
                     const uint32_t* pool_vrf, const int32_t* pool_map, uint32_t npools, int check_output,
                     uint16_t* bits, int32_t* pool_idx, int32_t* pool_sorted_idx, uint8_t* beta_out,
                     uint8_t* leader_out, uint8_t* nonce_out, const void* mid, int wave_prio = 0,
                     int pre = 0);                         // pre: launch_vrf_pool ran before (bits, pool, leader, nonce)
// the join's pool part ahead of it (k_vrf_stage.hip k_vrf_pool): key bits, pool indices, leader / nonce
void launch_vrf_pool(hipStream_t stream, size_t n, const uint8_t* cold_vk, const uint8_t* vrf_vk,
                     const uint8_t* vrf_out, const uint32_t* pool_hash, const uint32_t* pool_vrf,
                     const int32_t* pool_map, uint32_t npools, uint16_t* bits, int32_t* pool_idx,
                     int32_t* pool_sorted_idx, uint8_t* leader_out, uint8_t* nonce_out);
// TPraos join of certificate cert (0: eta, 1: leader; k_vrf_stage.hip k_vrf_join_tp), after
// stage V (tp_seed 1 + cert) and U of that certificate into `mid`
void launch_vrf_join_tp(hipStream_t stream, size_t n, int cert, const uint8_t* cold_vk, const uint8_t* vrf_vk,
                        const uint8_t* cert_out, const uint8_t* cert_proof, const uint32_t* pool_hash,
                        const uint32_t* pool_vrf, const int32_t* pool_map, uint32_t npools, int check_output,
                        uint16_t* bits, int32_t* pool_idx, int32_t* pool_sorted_idx, uint8_t* beta_out,
                        uint8_t* nonce_out, const void* mid, const int32_t* ovl_class, const uint32_t* gen);
void launch_vrf_tp(dim3 grid, dim3 block, hipStream_t stream, size_t n, const ge_niels* gbtab, const uint8_t* cold_vk, const uint8_t* vrf_vk, const uint8_t* eta_out, const uint8_t* eta_proof, const uint8_t* l_out, const uint8_t* l_proof, const uint64_t* slot, const uint32_t* eta0, int eta0_neutral, const uint32_t* pool_hash, const uint32_t* pool_vrf, const int32_t* pool_map, uint32_t npools, int check_output, uint16_t* bits, int32_t* pool_idx, int32_t* pool_sorted_idx, uint8_t* beta_eta, uint8_t* beta_l, uint8_t* nonce_out, ge_cached* tabs,
                   const int32_t* ovl_class, const uint32_t* gen, const uint8_t* eta_idx = nullptr);
void launch_decode_praos(dim3 grid, dim3 block, hipStream_t stream, size_t n, const uint8_t* arena, uint64_t arena_len,
                         const uint64_t* hoff, const uint32_t* hlen, uint64_t* slot, uint8_t* cold_vk, uint8_t* vrf_vk,
                         uint8_t* vrf_out, uint8_t* vrf_proof, uint8_t* hot_vk, uint8_t* ocert_sig, uint8_t* kes_sig,
                         uint64_t* ocert_n, uint64_t* ocert_c0, uint64_t* body_off, uint32_t* body_len,
                         uint8_t* signed_body, uint64_t* block_no, uint8_t* prev_hash, uint8_t* prev_genesis,
                         uint32_t* body_size, uint8_t* body_hash, uint64_t* prot_major, uint64_t* prot_minor,
                         uint8_t* header_hash, uint16_t* status, int allow_tp, uint32_t stride, uint8_t* lead_out = nullptr, uint8_t* lead_proof = nullptr,
                         size_t i0 = 0);   // headers [i0, n); grid covers n - i0
void launch_block_split(dim3 grid, dim3 block, hipStream_t stream, size_t n, const uint8_t* arena,
                        uint64_t arena_len, uint64_t* off_io, uint32_t* len_io, uint64_t* seg_off, uint32_t* seg_len,
                        uint8_t* nseg, uint8_t* status);
void launch_seg_hash(dim3 grid, dim3 block, hipStream_t stream, size_t n, const uint8_t* arena,
                     const uint64_t* seg_off, const uint32_t* seg_len, const uint8_t* nseg, uint8_t* seg_hash);
void launch_block_join(dim3 grid, dim3 block, hipStream_t stream, size_t n, const uint8_t* nseg,
                       const uint8_t* split_status, const uint16_t* dec_status, const uint16_t* kes_bits,
                       const uint8_t* seg_hash, const uint8_t* body_hash, uint8_t* result, uint8_t* calc_hash);
// replay: nonce contribution of each header's certified VRF output (k_misc.hip)
void launch_vrf_nonce(hipStream_t stream, size_t n, const uint8_t* vrf_out, int tpraos, uint8_t* nonce_out);
