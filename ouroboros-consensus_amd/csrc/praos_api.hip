// praos_api.hip -- host side of libpraos_hip: context, device buffers, launches
// and the sequential part of Praos.updateChainDepState (C++).
// Single translation unit with the kernels (no relocatable device code).
#include "praos_hip.h"
#include "launch.hpp"
#include "host_util.hpp"
#include "replay_internal.hpp"

static constexpr size_t NT = 256;                  // threads per block of the crypto kernels
static constexpr size_t NIELS_BYTES = 3 * 32;      // sizeof(ge_niels)
static constexpr size_t BTAB_N = 128;              // entries per fixed-base table (scalarmult.hpp)
static constexpr size_t BCOMB_TABLES = 32;         // fixed-base comb: 256^j B, j < 32 (scalarmult.hpp BCOMB_T)
static constexpr size_t C16_TABLES = 16, C16_ENTRIES = 32768;   // radix-2^16 comb (scalarmult.hpp C16_T, C16_N)
static constexpr size_t CACHED_BYTES = 4 * 32;     // sizeof(ge_cached)
static constexpr size_t LT_ED_B = 8 * CACHED_BYTES, LT_VRF_B = 16 * CACHED_BYTES;   // per-lane tables (kcommon.hpp)
static constexpr size_t VRF_MID_BYTES = 28 * 16;    // per-header records of the staged VRF (praos_core.hpp)
static constexpr uint32_t TP_SIGNED_STRIDE = 640;   // max canonical TPraos BHBody: 598 bytes (k_decode.hip)

#include <pthread.h>
#include <sched.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <functional>
#include <map>
#include <set>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

// A small persistent pool of host threads for the staging copies (pageable caller
// memory <-> pinned buffers): one job at a time, each worker takes its share.
class CopyPool {
 public:
  explicit CopyPool(unsigned n) : nt_(n) {
    for (unsigned t = 0; t < nt_; t++) th_.emplace_back([this, t] { loop(t); });
  }
  ~CopyPool() {
    { std::lock_guard<std::mutex> g(m_); stop_ = true; }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  unsigned size() const { return nt_; }
  void run(const std::function<void(unsigned)>& f) {
    std::unique_lock<std::mutex> g(m_);
    job_ = &f;
    pending_ = nt_;
    gen_++;
    cv_.notify_all();
    done_.wait(g, [this] { return pending_ == 0; });
    job_ = nullptr;
  }
  // every worker onto the given CPUs (empty: back to the process's own mask)
  void pin(const std::vector<int>& cpus) {
    cpu_set_t set;
    CPU_ZERO(&set);
    if (cpus.empty()) {
      if (sched_getaffinity(0, sizeof set, &set) != 0) return;
    } else {
      for (int c : cpus) CPU_SET(c, &set);
    }
    run([&](unsigned) { (void)pthread_setaffinity_np(pthread_self(), sizeof set, &set); });
  }
  // dst[0, n) = src[0, n), split over the workers
  void copy(void* dst, const void* src, size_t n) {
    if (n < (1u << 20)) { std::memcpy(dst, src, n); return; }
    run([&](unsigned t) {
      const size_t a = n * t / nt_, b = n * (t + 1) / nt_;
      std::memcpy((uint8_t*)dst + a, (const uint8_t*)src + a, b - a);
    });
  }

 private:
  void loop(unsigned t) {
    uint64_t seen = 0;
    for (;;) {
      const std::function<void(unsigned)>* f;
      {
        std::unique_lock<std::mutex> g(m_);
        cv_.wait(g, [&] { return stop_ || gen_ != seen; });
        if (stop_) return;
        seen = gen_;
        f = job_;
      }
      (*f)(t);
      std::lock_guard<std::mutex> g(m_);
      if (--pending_ == 0) done_.notify_all();
    }
  }
  unsigned nt_;
  std::vector<std::thread> th_;
  std::mutex m_;
  std::condition_variable cv_, done_;
  const std::function<void(unsigned)>* job_ = nullptr;
  unsigned pending_ = 0;
  uint64_t gen_ = 0;
  bool stop_ = false;
};

static constexpr size_t STAGE_PIECE = 16u << 20;    // pinned staging buffers: 2 x 16 MB per context
static constexpr int PIPE_MAX = 8;                  // chunks of the stored-bytes pipeline
static constexpr int PIPE_CALLS = 3;                // submitted stored-bytes calls in flight (pipe[0 .. 3))
static constexpr size_t PIPE_MIN_CHUNK = 49152;     // headers per chunk at least (auto mode)
// Batches below this many headers (a strong-scaling shard of an epoch over 8 GPUs is 54k) leave
// most wave slots empty and run latency-bound (PRAOS_VRF_PRIO = -1 raises stage V there)
static constexpr size_t SMALL_BATCH = 80000;
// below this many headers the key precomputes run at raised wave priority (PRAOS_KEY_PRIO -1):
// they head the cached chains (profiles/r04/bb: 96k 3.66 -> 3.57 ms, 108k 4.14 -> 3.83, 160k
// 5.19 -> 4.88, 300k 8.83 -> 8.67; 432k within noise)
static constexpr size_t KEY_PRIO_BATCH = 400000;
// below this many headers stage V, the uncached verifies and the key precompute come from their
// ILP-4 builds (k_vrf_v4 / k_miss4 / k_keys4): a step's chains are latency-bound there
// (profiles/r04/y: 96k 4.06 -> 3.64 ms, 108k 4.25 -> 4.10, 112k 4.39 -> 4.15; equal at 120k,
// slower at 128k)
static constexpr size_t ILP4_BATCH = 120000;
// below this many headers the KES leaf keys are not cached (every KES check uncached, from the
// ILP-4 build, beside stage V): a 54k-header shard's stage V and uncached KES waves fit in one
// round of wave slots (2 per SIMD), and the leaf-key chain -- lists, precompute, tables, k_kes_ck,
// the step's longest after stage V + join -- is gone (54k 2.44-2.49 -> 2.29-2.37 ms; at 64k the
// waves no longer fit and it is slower, 2.53 -> 3.05; 80k 2.97 -> 3.47; 108k 3.41 -> 4.59;
// profiles/r06/i_kes_nocache).  PRAOS_OPT_KES_NOCACHE / PRAOS_KES_NOCACHE=<headers> override it
// (0: always cached).
static constexpr size_t KES_NOCACHE_BATCH = 58000;
// below this many headers (the 1/8-epoch shard of a 432k epoch is 54k) stage V's join runs on the
// main stream after it waits for U itself (PRAOS_V_MAIN 2) and the uncached verifies keep normal
// wave priority
static constexpr size_t SHARD_SMALL = 60000;
static constexpr int PIPE_AUTO = 8;                 // chunks in auto mode (round 3, equal chunks: 4 -> 21.9M,
                                                    // 6 -> 23.0M, 8 -> 22.1M headers/s, profiles/r03/e2e_chunks.txt;
                                                    // round 5 with the first chunk at 1/4 of the others: 6 ->
                                                    // 25.3-25.6M, 8 -> 26.4-26.6M, profiles/r05/c8_pipe_head)
struct praos_batch;

// The context's last error.  The replay's worker threads (reader, nonce chain, launcher,
// fold) can fail at the same time, so every assignment takes a lock; while a replay runs
// (first_only) only the first message of the call is kept -- the one that stopped it.
class ErrMsg {
 public:
  ErrMsg& operator=(const std::string& m) {
    std::lock_guard<std::mutex> g(mu_);
    if (!(first_ && held_)) s_ = m;
    held_ = true;
    return *this;
  }
  ErrMsg& operator=(const char* m) { return *this = std::string(m); }
  const char* c_str() {
    std::lock_guard<std::mutex> g(mu_);
    return s_.c_str();
  }
  void first_only(bool on) {
    std::lock_guard<std::mutex> g(mu_);
    first_ = on;
    held_ = false;
  }

 private:
  std::mutex mu_;
  std::string s_;
  bool first_ = false, held_ = false;
};

struct praos_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  hipStream_t side[3] = {nullptr, nullptr, nullptr};   // concurrent crypto kernels
  hipStream_t mside[3] = {nullptr, nullptr, nullptr};  // their key-cache misses (uncached verifies)
  hipEvent_t mdone_ev[3] = {};
  hipStream_t vstream = nullptr;                       // VRF stage V (no key-cache dependence)
  hipStream_t vstream2 = nullptr;                      // the odd chunks' stage V of the stored-bytes pipeline
  hipEvent_t v_ev = nullptr, v2_ev = nullptr;
  hipEvent_t v0_ev = nullptr, v1_ev = nullptr;         // timing of k_vrf_v on its stream (kernel_ms[6])
  hipEvent_t kc0_ev = nullptr, kc1_ev = nullptr;       // timing of k_kes_ck on its stream (kernel_ms[7])
  hipEvent_t u_ev = nullptr;                           // stage U of the uncached VRF keys done
  int tp_staged = 1;                                  // TPraos VRF through the staged kernels + VRF key cache
                                                       // (PRAOS_TP_STAGED=0: the one-kernel k_vrf_tp)
  int vrf_prio = 0;                                   // stage V and join waves at s_setprio 3 (PRAOS_VRF_PRIO 1 / 0;
                                                       // -1: batches below SMALL_BATCH headers).  Off: with the
                                                       // uncached verifies raised instead a 54k-header step takes
                                                       // 2.83 ms against 3.16 (profiles/r04/i, r04/j)
  int vrf_ilp4 = (int)ILP4_BATCH;                    // stage V from the ILP-4 build (k_vrf_v4.hip): PRAOS_VRF_ILP4
                                                       // 1 always, 0 never, N > 1: batches below N headers
                                                       // (profiles/r04/b: V alone 1.71 -> 1.51 ms at 54k; alone
                                                       // at 108k the step was slower, 4.25 -> 4.37, but with the
                                                       // ILP-4 uncached verifies and precompute beside it faster,
                                                       // profiles/r04/y)
  int v_excl = 0;                                      // the ILP-4 stage V holding its SIMDs alone (k_vrf_v4x):
                                                       // PRAOS_V_EXCL (54k: 3.30 -> 3.46 ms, off)
  int miss4 = -1;                                      // uncached OCert / KES verifies from the ILP-4 build
                                                       // (k_miss4.hip): PRAOS_MISS4 1 / 0, -1 below ILP4_BATCH
                                                       // (54k: 3.33 -> 3.09 ms; 108k: 4.26 -> 4.66, so not there)
  int miss_prio = -1;                                  // ... at s_setprio 3: PRAOS_MISS_PRIO 1 / 0, -1 with miss4
                                                       // from SHARD_SMALL headers on (below it, beside the GCD
                                                       // inversion's shorter join, normal priority with
                                                       // v_main 1 was faster: profiles/r06/s_retune)
  int miss_prio_for(size_t n) const { return miss_prio >= 0 ? miss_prio : (n < SHARD_SMALL ? 0 : 1); }
  long kes_pair = -1;                                  // k_kes_ck two headers per lane from this many hits on
                                                       // (PRAOS_KES_PAIR, 0 = never; -1: from 196,608 when the
                                                       // KES pass runs alone -- beside the OCert / VRF passes
                                                       // the longer paired waves cost the C5 step 2 %,
                                                       // profiles/r04/i: 12.15 -> 12.40 ms, C4 6.43 -> 6.10 ms)
  uint32_t kes_pair_min() const {
    return kes_pair >= 0 ? (uint32_t)kes_pair : ((kernels & 5) ? 0u : 196608u);
  }
  int kes_dedup = 0;                                   // KES Merkle path dedup per leaf-key entry (PRAOS_KES_DEDUP):
                                                       // off, measured slower (C4 10.7 -> 11.2 ms: the
                                                       // representatives' walks lengthen the KES chain more than
                                                       // the skipped walks save; C5 unchanged, profiles/r04/r)
  int v_main = -1;                                     // stage V on the main stream (PRAOS_V_MAIN; 0 off): no
                                                       // cross-stream wait between the previous run's end and V;
                                                       // the join after U and V on the VRF stream (3), or on the
                                                       // main stream after a wait for U (1; 2: U's two streams
                                                       // waited for separately).  54k headers (C5 1/8 shard):
                                                       // 2.354-2.380 ms off, 2.284-2.330 (1), 2.315-2.332 (2),
                                                       // 2.267-2.297 (3); 108k: 3.418-3.443 off, 3.36-3.42 on
                                                       // (profiles/r06/k_vmain); -1: 2 below ILP4_BATCH
                                                       // headers, 3 from it (with the GCD inversion, mode 1 +
                                                       // normal-priority misses below SHARD_SMALL: 54k
                                                       // 2.18-2.22 -> 2.17-2.19 ms, 40k 2.19-2.21 -> 2.08; then
                                                       // mode 2 over mode 1 at 54k 2.16-2.19 -> 2.15, 40k equal
                                                       // or 2 % faster; over mode 3 at 80k 2.78-2.80 -> 2.76,
                                                       // 108k 3.24-3.26 -> 3.21-3.22, 216k 5.63-5.70 -> 5.70-5.71;
                                                       // profiles/r06/s_retune)
  int vmain_mode(size_t n) const { return v_main >= 0 ? v_main : (n < ILP4_BATCH ? 2 : 3); }
  int pre_join = -1;                                   // the join's pool part (lookup, key hash, leader / nonce
                                                       // values) as k_vrf_pool on the VRF miss stream before the
                                                       // uncached U, off the chain after stage V (PRAOS_PRE_JOIN
                                                       // 1 / 0, -1 below SMALL_BATCH)
  int vrf_keys_first = 0;                              // PRAOS_VRF_KEYS_FIRST (see batch_run_impl; 54k: 2.80 ->
                                                       // 2.85 ms, 108k 4.24 -> 4.27: off, profiles/r04/k)
  int key4 = -1;                                       // key precompute from the ILP-4 build (k_keys4.hip):
                                                       // PRAOS_KEY4 1 / 0, -1 below ILP4_BATCH (54k: 2.78-2.84
                                                       // -> 2.76-2.77 ms; 108k 4.17 -> 4.21, profiles/r04/n)
  bool use_key4(size_t n) const { return key4 > 0 || (key4 < 0 && n < ILP4_BATCH); }
  // (round 5 also measured a key precompute with four lanes per key, DPP quad broadcasts: inside a
  // step its chains were about as long as the ILP-4 build's and its four lanes per key took issue
  // slots from the rest, 54k 2.72-2.75 -> 2.84-2.88 ms, 108k 3.79-3.84 -> 4.00,
  // profiles/r05/c11_keyq_nobranch; removed in round 6)
  int key_mode(size_t n) const { return use_key4(n) ? 1 : 0; }
  int u4 = -1;                                         // cached stage U from the ILP-4 build (PRAOS_U4 1 / 0,
                                                       // -1 below ILP4_BATCH; 54k 2.79 -> 2.75 ms, 108k 3.87-3.92
                                                       // -> 3.81-3.83, profiles/r04/hh)
  int ck4 = 0;                                         // cached OCert / KES verifies from the ILP-4 build
                                                       // (PRAOS_CK4 1 / 0, -1 below ILP4_BATCH)
  bool use_ck4(size_t n) const { return ck4 > 0 || (ck4 < 0 && n < ILP4_BATCH); }
  bool use_u4(size_t n) const { return u4 > 0 || (u4 < 0 && n < ILP4_BATCH); }
  bool use_miss4(size_t n) const { return miss4 > 0 || (miss4 < 0 && n < ILP4_BATCH); }
  int v_ilp4(size_t n) const {
    const bool on = vrf_ilp4 == 1 || (vrf_ilp4 > 1 && n < (size_t)vrf_ilp4);
    return on ? (v_excl ? 2 : 1) : 0;
  }
  int vrf3 = -1;                                       // VRF as V | U | join (1), V | U + join (0), -1 auto:
                                                       // the three-kernel form below 300k headers (latency)
  // chunked stored-bytes pipeline (praos_verify_header_bytes): a copy stream, per-chunk
  // events and persistent chunk batches (reused while they are large enough)
  int pipeline = 0;                                    // PRAOS_OPT_PIPELINE (0 = auto)
  hipStream_t cstream = nullptr;
  hipStream_t dstream = nullptr;                       // replay: result downloads (rp_download_results)
  hipStream_t decstream = nullptr;                     // submitted calls: each landed chunk's decode (off the
                                                       // copy stream, whose next upload must not wait for it)
  praos_batch* rp_keep[RP_SLOTS] = {};                 // replay batches kept between calls
  hipEvent_t up_ev[PIPE_MAX] = {}, done_ev[PIPE_MAX] = {};
  praos_batch* pipe[PIPE_MAX] = {};
  // praos_verify_header_bytes_submit: up to PIPE_CALLS calls in flight, on pipe[0 .. PIPE_CALLS) in turn
  struct PipeCall {
    bool active = false;
    praos_out out{};
    praos_decoded* dec = nullptr;
    hipEvent_t ev = nullptr;                           // the call's run has ended (ctx stream)
    uint64_t* off_h = nullptr;                         // pinned: its rebased offsets and lengths (async H2D:
    uint32_t* len_h = nullptr;                         // a pageable copy would wait for the copy stream)
    size_t cap = 0;
  } pcall[PIPE_CALLS];
  int pcall_next = 0;                                  // the slot the next submit takes: the oldest call's
  int stream_chunk_v = 1;                              // submitted calls: stage V per landed chunk (1) or in the
                                                       // run over the whole batch (0); PRAOS_STREAM_CHUNK_V.  C5,
                                                       // 432k headers, three calls in flight: 13.2-13.4 ms per
                                                       // call (1) against 15.3-17.6 (0), profiles/r06/l_stream
  size_t pipe_n[PIPE_MAX] = {}, pipe_bytes[PIPE_MAX] = {};
  int concurrent = 1;                                  // PRAOS_OPT_CONCURRENT
  int kernels = 7;                                     // PRAOS_OPT_KERNELS
  int keycache = 2;                                    // PRAOS_OPT_KEYCACHE (min uses; 0 = off)
  size_t kes_nocache = KES_NOCACHE_BATCH;              // PRAOS_KES_NOCACHE (see KES_NOCACHE_BATCH)
  int kc_min[3] = {0, 0, 0};                           // per cache (cold, VRF, KES leaf) min uses overriding
                                                       // keycache when > 0 (PRAOS_KC_MIN="c,v,k")
  int dedup = 1;                                       // PRAOS_OPT_DEDUP
  // (round 5 measured the cached chains' last kernels -- cached U, the join, the cached OCert /
  // KES verifies -- at s_setprio 2 / 3 below ILP4_BATCH: U shortened (54k 0.71 -> 0.43 ms) but
  // stage V stretched past it and the step with it, 54k 2.74-2.76 -> 2.89-2.95 ms,
  // profiles/r05/c14_ckprio; the option was removed in round 6)
  int key_wave_prio = -1;                              // key precompute waves at s_setprio 3 (PRAOS_KEY_PRIO 1 / 0;
                                                       // -1: batches below KEY_PRIO_BATCH headers)
  hipEvent_t ev[6] = {};
  hipEvent_t side_ev[4] = {};
  hipEvent_t miss_ev[4] = {};                          // miss lists ready (OCert, KES, VRF), OCert misses done
  float kernel_ms[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  bool last_from_bytes = false;
  bool v_timed = false;                                // the last run launched k_vrf_v
  bool kes_ck_timed = false;                           // ... and k_kes_ck
  ErrMsg err;
  ge_niels* btab = nullptr;
  ge_niels* bcomb16 = nullptr;                         // radix-2^16 comb of the cached-key chains (48 MB)
  // pool-key store (PRAOS_OPT_POOL_KEYS, k_keys.hip): cold [0] and VRF [1] key entries and
  // tables kept across runs; allocated on first use (256 MB of tables each)
  struct PoolKeyStore {
    uint32_t slots = 0, cap = 0;
    uint32_t *pkey = nullptr, *count = nullptr, *base = nullptr, *entry_rep = nullptr, *entry_pos = nullptr;
    uint32_t* kinfo = nullptr;
    int32_t* pentry = nullptr;
    ge_cached* ktab = nullptr;
    uint32_t *scnt = nullptr, *spos = nullptr;           // per entry: uses this run, start of its hit range
  } pks[2];                                            // [0] cold keys, [1] VRF keys
  int pool_keys = -1;                                  // 1 on, 0 off, -1 on inside praos_replay_immutable*
  bool replaying = false;
  bool pk_on = false;                                  // this run uses the store
  bool pk_reset[2] = {false, false};                   // empty store t before the next run that uses it
  // (round 6 measured key hints for the stored-bytes pipeline -- each header's cold, VRF and KES
  // leaf keys read on the host while the chunks upload, the key stores filled from them on the
  // side streams before the last chunk lands -- bit-exact and slower, 432k e2e 15.7 -> 18.4 ms:
  // the fill shares the GPU with the chunks' stage V and the tail stays throughput-bound;
  // profiles/r06/h_e2e_hints.  Removed.)
  // (round 5 measured a per-chunk key prefill in the stored-bytes pipeline -- the landed chunks'
  // cold, KES leaf and VRF keys stored and their tables built while later chunks upload -- in two
  // forms, both slower: the GPU is busy with the chunks' stage V during the upload, so the
  // prefill only moves work there, and a key first seen in the last chunk still needs a
  // latency-bound chain after it lands (432k, 8 chunks: 16.3-16.4 -> 18.2-18.5 ms,
  // profiles/r05/c12_prefill_v3; 16.9 -> 19.2 ms, c7_e2e_timeline_pf{0,1}.txt).  Removed in round 6.)
  // stored-bytes pipeline: the first chunk's size in percent of the others' (PRAOS_PIPE_HEAD):
  // nothing runs on the GPU until it has landed and been decoded
  int pipe_head = 25;                                  // (432k headers, 8 chunks: 100 -> 16.9-17.0 ms,
                                                       // 50 -> 16.5, 25 -> 16.3-16.4, 12 -> 16.2-16.4)
  // (round 6 measured the KES checks queued while later chunks upload, in two forms, both slower:
  // uncached per landed chunk, 432k e2e 15.5-16.0 -> 18.2-18.9 ms; with the leaf-key cache over 1,
  // 2 or 4 groups of landed chunks, 15.8 / 17.0 / 18.2-18.7 ms: the GPU runs the chunks' stage V
  // during the upload, so the KES work there only stretches V; profiles/r06/g_e2e_kes.  Removed.)
  int pipe_tail = 100;                                 // ... and the last chunk's (PRAOS_PIPE_TAIL): the run after it
                                                       // waits for its decode, but a smaller one leaves more of the
                                                       // batch's stage V after the upload (432k, 8 chunks: 100 ->
                                                       // 16.4-16.7 ms, 50 -> 17.1-17.3, 25 -> 18.5-18.8;
                                                       // profiles/r05/c16_pipe_tail)
  // epoch
  bool have_epoch = false;
  std::vector<praos_pool> epoch_pools;                 // praos_set_epoch's inputs as installed (a call
  praos_params epoch_params{};                         // with the same pools and parameters only swaps eta0)
  praos_params params{};
  uint32_t eta0[8] = {0};
  int eta0_neutral = 1;
  uint32_t npools = 0;
  uint32_t* d_pool_hash = nullptr;   // sorted, 7 words each
  uint32_t* d_pool_vrf = nullptr;    // 8 words
  uint32_t* d_pool_x = nullptr;      // 4 words
  int32_t* d_pool_map = nullptr;     // sorted idx -> caller idx
  uint32_t* d_eta0 = nullptr;
  std::vector<praos_pool> pools;     // caller order
  std::map<std::string, int32_t> pool_by_hash;
  // TPraos overlay schedule (praos_set_overlay): d, ascInv, epochs, genesis delegates
  // sorted by genesis key hash; device table: delegate hash (7 words + 0) | VRF hash (8)
  bool ovl_on = false;
  uint64_t ovl_d_num = 0, ovl_d_den = 1, ovl_asc_inv = 1, ovl_base = 0, ovl_len = 1;
  std::vector<praos_gen_deleg> gen_delegs;
  std::set<std::string> gen_delegate_hashes;
  uint32_t* d_gen = nullptr;
  // caller ranges page-locked with praos_host_register: uploads from them skip the staging
  std::mutex reg_mu;
  std::vector<std::pair<uintptr_t, size_t>> registered;
  // host <-> device staging for large transfers from pageable caller memory
  uint8_t* pin[2] = {nullptr, nullptr};
  uint8_t* zero_h = nullptr;                           // pinned zeros: an arena's tail padding by DMA (a fill
                                                       // kernel on the copy stream could wait behind another
                                                       // stream's kernels on a shared hardware queue)
  hipEvent_t pin_ev[2] = {};
  std::unique_ptr<CopyPool> pool;
  // device buffers of the last freed batch, reused by the next one in allocation
  // order (hipMalloc / hipFree of ~40 buffers cost ~20 ms per 432k batch)
  std::vector<void*> spare;
  std::vector<size_t> spare_sz;
  // host-side repack arena of praos_batch_upload, kept across calls (a fresh 170 MB
  // allocation per 432k batch cost its page faults and its unmapping on every call)
  std::unique_ptr<uint8_t[]> h_arena;
  size_t h_arena_cap = 0;
  std::vector<uint64_t> h_off;
  std::vector<uint32_t> h_len;
};

static void free_spare(praos_ctx* c) {
  for (void* p : c->spare)
    if (p) (void)hipFree(p);
  c->spare.clear();
  c->spare_sz.clear();
}

// Large H2D / D2H copies through two pinned buffers: the host threads fill (drain) one
// piece while the DMA engine moves the other, so pageable caller memory moves at PCIe
// speed instead of through the runtime's own pageable path.  Small copies go direct.
// the arena's zero padding after its last byte (< 64 bytes), copied from pinned zeros on st
static hipError_t zero_pad(praos_ctx* c, uint8_t* dst, size_t pad, hipStream_t st) {
  if (!c->zero_h) {
    if (hipHostMalloc((void**)&c->zero_h, 64, hipHostMallocDefault) != hipSuccess) return hipErrorOutOfMemory;
    std::memset(c->zero_h, 0, 64);
  }
  return hipMemcpyAsync(dst, c->zero_h, pad, hipMemcpyHostToDevice, st);
}

static bool stage_init(praos_ctx* c) {
  if (c->pin[0]) return true;
  for (int k = 0; k < 2; k++) {
    if (hipHostMalloc((void**)&c->pin[k], STAGE_PIECE, hipHostMallocDefault) != hipSuccess) return false;
    if (hipEventCreateWithFlags(&c->pin_ev[k], hipEventDisableTiming) != hipSuccess) return false;
  }
  const unsigned hw = std::thread::hardware_concurrency();
  unsigned nt = std::max(1u, std::min(16u, hw ? hw : 1u));      // the box's CPU share per GPU
  if (const char* e = std::getenv("PRAOS_COPY_THREADS")) nt = (unsigned)std::max(1, std::min(64, std::atoi(e)));
  c->pool.reset(new CopyPool(nt));
  return true;
}

static bool is_registered(praos_ctx* c, const void* p, size_t len) {
  std::lock_guard<std::mutex> g(c->reg_mu);
  const uintptr_t a = (uintptr_t)p;
  for (const auto& r : c->registered)
    if (a >= r.first && len <= r.second && a - r.first <= r.second - len) return true;
  return false;
}

static hipError_t h2d_on(praos_ctx* c, void* dst, const void* src, size_t bytes, hipStream_t st) {
  if (bytes < (4u << 20) || is_registered(c, src, bytes) || !stage_init(c))
    return hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, st);   // registered memory: direct DMA
  for (size_t off = 0, k = 0; off < bytes; off += STAGE_PIECE, k++) {
    const size_t len = std::min(STAGE_PIECE, bytes - off);
    hipError_t e = hipEventSynchronize(c->pin_ev[k & 1]);    // the DMA that last used this buffer
    if (e != hipSuccess) return e;
    c->pool->copy(c->pin[k & 1], (const uint8_t*)src + off, len);
    e = hipMemcpyAsync((uint8_t*)dst + off, c->pin[k & 1], len, hipMemcpyHostToDevice, st);
    if (e == hipSuccess) e = hipEventRecord(c->pin_ev[k & 1], st);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}
// D2H on stream st, whose producers the caller has ordered before (an event wait); returns
// when the bytes are in dst
static hipError_t d2h_on(praos_ctx* c, void* dst, const void* src, size_t bytes, hipStream_t st) {
  if (bytes < (4u << 20) || is_registered(c, dst, bytes) || !stage_init(c)) {
    hipError_t e = hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, st);
    return e == hipSuccess ? hipStreamSynchronize(st) : e;
  }
  const size_t np = (bytes + STAGE_PIECE - 1) / STAGE_PIECE;
  hipError_t e = hipSuccess;
  for (size_t k = 0; k <= np && e == hipSuccess; k++) {
    if (k < np) {
      const size_t off = k * STAGE_PIECE, len = std::min(STAGE_PIECE, bytes - off);
      e = hipEventSynchronize(c->pin_ev[k & 1]);
      if (e == hipSuccess) e = hipMemcpyAsync(c->pin[k & 1], (const uint8_t*)src + off, len, hipMemcpyDeviceToHost, st);
      if (e == hipSuccess) e = hipEventRecord(c->pin_ev[k & 1], st);
    }
    if (e == hipSuccess && k > 0) {
      const size_t j = k - 1, off = j * STAGE_PIECE, len = std::min(STAGE_PIECE, bytes - off);
      e = hipEventSynchronize(c->pin_ev[j & 1]);
      if (e == hipSuccess) c->pool->copy((uint8_t*)dst + off, c->pin[j & 1], len);
    }
  }
  return e;
}

static hipError_t h2d(praos_ctx* c, void* dst, const void* src, size_t bytes) {
  if (bytes < (4u << 20) || !stage_init(c)) return hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, c->stream);
  for (size_t off = 0, k = 0; off < bytes; off += STAGE_PIECE, k++) {
    const size_t len = std::min(STAGE_PIECE, bytes - off);
    hipError_t e = hipEventSynchronize(c->pin_ev[k & 1]);    // the DMA that last read this buffer
    if (e != hipSuccess) return e;
    c->pool->copy(c->pin[k & 1], (const uint8_t*)src + off, len);
    e = hipMemcpyAsync((uint8_t*)dst + off, c->pin[k & 1], len, hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess) e = hipEventRecord(c->pin_ev[k & 1], c->stream);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

// blocking: the stream is drained first (the producer kernels), then piecewise
static hipError_t d2h(praos_ctx* c, void* dst, const void* src, size_t bytes) {
  if (bytes < (4u << 20) || !stage_init(c)) return hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost);
  hipError_t e = hipStreamSynchronize(c->stream);
  const size_t np = (bytes + STAGE_PIECE - 1) / STAGE_PIECE;
  for (size_t k = 0; k <= np && e == hipSuccess; k++) {
    if (k < np) {     // start piece k, then drain piece k - 1 while it moves
      const size_t off = k * STAGE_PIECE, len = std::min(STAGE_PIECE, bytes - off);
      e = hipMemcpyAsync(c->pin[k & 1], (const uint8_t*)src + off, len, hipMemcpyDeviceToHost, c->stream);
      if (e == hipSuccess) e = hipEventRecord(c->pin_ev[k & 1], c->stream);
    }
    if (e == hipSuccess && k > 0) {
      const size_t j = k - 1, off = j * STAGE_PIECE, len = std::min(STAGE_PIECE, bytes - off);
      e = hipEventSynchronize(c->pin_ev[j & 1]);
      if (e == hipSuccess) c->pool->copy((uint8_t*)dst + off, c->pin[j & 1], len);
    }
  }
  return e;
}

struct praos_batch {
  size_t n = 0;
  size_t body_bytes_len = 0;
  uint64_t *slot = nullptr, *ocert_n = nullptr, *ocert_c0 = nullptr, *body_off = nullptr;
  uint32_t* body_len = nullptr;
  uint8_t *cold_vk = nullptr, *vrf_vk = nullptr, *vrf_out = nullptr, *vrf_proof = nullptr, *hot_vk = nullptr,
          *ocert_sig = nullptr, *kes_sig = nullptr, *body = nullptr;
  uint16_t* bits = nullptr;
  uint16_t* bits3 = nullptr;   // per-kernel bits: ocert | kes | vrf
  int32_t *pool_idx = nullptr, *pool_sorted = nullptr;
  uint8_t *beta = nullptr, *leader = nullptr, *nonce = nullptr;
  // per-lane point tables of the three crypto kernels (kcommon.hpp lane_tab)
  ge_cached *tab_ocert = nullptr, *tab_kes = nullptr, *tab_vrf = nullptr;
  ge_cached* tab_vrfu = nullptr;   // 8-entry lane tables of stage U on uncached VRF keys
  bool v_done = false;             // stage V already queued on ctx->vstream (stored-bytes pipeline)
  uint8_t* vrf_mid = nullptr;   // stage V -> stage F record of the two-stage VRF
  uint8_t* vrf_mid2 = nullptr;  // TPraos: the leader certificate's record (allocated on first use)
  ge_cached* tab_vrf2 = nullptr; // TPraos: the leader certificate's stage-V lane tables
  size_t vrf_mid2_n = 0;
  // TPraos overlay classes of the batch's slots (praos_set_overlay): device copy sized once
  // per capacity, host arrays kept with the batch (the async upload reads them)
  int32_t* dcls = nullptr;
  size_t dcls_n = 0;
  std::vector<uint64_t> slots_h;
  std::vector<int32_t> cls_h;
  // per-run public-key cache (k_keys.hip): [0] cold keys (OCert), [1] VRF keys, [2] KES leaf keys
  struct KeyCache {
    uint32_t cap = 0, max_entries = 0;
    uint32_t *slot_rep = nullptr, *slot_cnt = nullptr, *entry_rep = nullptr, *entry_pos = nullptr, *kinfo = nullptr;
    int32_t *slot_entry = nullptr, *item_slot = nullptr, *item_entry = nullptr;
    uint32_t *counters = nullptr, *hit = nullptr, *miss = nullptr;   // counters: entries, hits, misses
    ge_cached* ktab = nullptr;
    uint8_t* rep_ok = nullptr;   // KES leaf keys: the Merkle walk verdict of each entry's representative
    // this run's entry space: the arrays above, or the context's pool-key store
    ge_cached* kt = nullptr;
    uint32_t *ki = nullptr, *erep = nullptr, *epos = nullptr;
    const uint32_t* ebase = nullptr;
    uint32_t emax = 0;
    int store = -1;
  } kc[3];                       // [2] KES leaf keys
  uint8_t* kes_leaf = nullptr;   // n*32: the leaf key of each header's KES signature
  bool kc_used = false;
  // OCert dedup (k_keys.hip k_ocert_dedup): hash set over the 144-byte OCert tuple,
  // representative per item, list of representatives, their verify results
  uint32_t dd_cap = 0;
  uint32_t *dd_slot = nullptr, *dd_item_rep = nullptr, *dd_reps = nullptr, *dd_counters = nullptr;
  uint8_t* dd_ok = nullptr;
  bool dd_used = false;
  // batches from stored bytes (praos_batch_upload_bytes): the arena and the
  // decoded HeaderBody fields beyond the SoA above (k_decode.hip)
  bool from_bytes = false;
  uint32_t signed_stride = PRAOS_SIGNED_STRIDE;   // bytes per signed body (block batches: TP_SIGNED_STRIDE)
  uint8_t* arena = nullptr;
  size_t arena_len = 0;
  uint64_t *hoff = nullptr, *block_no = nullptr, *prot_major = nullptr, *prot_minor = nullptr;
  uint32_t *hlen = nullptr, *body_size = nullptr;
  uint8_t *prev_hash = nullptr, *prev_genesis = nullptr, *body_hash = nullptr, *header_hash = nullptr;
  uint16_t* dec_status = nullptr;
  // block-integrity batches (k_block.hip): stored block spans, segment spans
  // (segment-major [k][i]), per-segment hashes, results
  bool is_block = false;
  // several epoch nonces in one batch (praos_batch_set_nonces): device table of 9-word
  // entries (nonce, neutral flag) and per-header index; host copies for the fold
  uint32_t* eta_tab = nullptr;
  uint8_t* eta_idx = nullptr;
  bool decoded = false;          // praos_batch_decode ran: praos_batch_run skips the decode
  // TPraos header batches from stored bytes (praos_verify_tpraos_header_bytes): the
  // decoded leader certificate and its beta
  bool tp_only = false;
  uint8_t *lead_out = nullptr, *lead_proof = nullptr, *beta_l = nullptr;
  uint64_t *blk_off = nullptr, *seg_off = nullptr;
  uint32_t *blk_len = nullptr, *seg_len = nullptr;
  uint8_t *nseg = nullptr, *split_status = nullptr, *seg_hash = nullptr, *blk_result = nullptr, *blk_hash = nullptr;
  std::vector<void*> owned;
  std::vector<size_t> owned_sz;
  praos_ctx* owner = nullptr;
  // replay batches (rp_batch_alloc): capacity, decode / run events, pinned nonce table
  size_t cap_n = 0, cap_bytes = 0;
  hipEvent_t dec_ev = nullptr, run_ev = nullptr;
  uint32_t* eta_h = nullptr;       // pinned: 9-word entries (nonce, neutral flag)
  uint8_t* eidx_h = nullptr;       // pinned: per-header index
  uint16_t* res_bits_h = nullptr;  // pinned: the replay's result downloads (bits, pool index), cap_n each
  int32_t* res_pidx_h = nullptr;
  uint8_t* dec_h = nullptr;        // pinned: the replay's decoded-field downloads (DEC_H_BYTES per header)
};

static constexpr size_t KT_BYTES = 16 * 8 * 4 * 32; // per cached key: 16 tables x 8 cached points
static constexpr uint32_t KC_MAX_ENTRIES = 1u << 20;   // a key used twice already pays for its tables

#define HIPCHK(ctx, x)                                                                    \
  do {                                                                                    \
    if ((ctx)->device < 0) {                                                              \
      (ctx)->err = "host-only context: no HIP device";                                    \
      return PRAOS_E_STATE;                                                               \
    }                                                                                     \
    hipError_t e_ = (x);                                                                  \
    if (e_ != hipSuccess) {                                                               \
      (ctx)->err = std::string(#x) + ": " + hipGetErrorString(e_);                        \
      return PRAOS_E_HIP;                                                                 \
    }                                                                                     \
  } while (0)

static inline unsigned nblocks(size_t n, unsigned bs) { return (unsigned)((n + bs - 1) / bs); }

template <typename T>
static hipError_t dalloc(praos_batch* b, T** p, size_t bytes) {
  void* q = nullptr;
  size_t sz = bytes ? bytes : 16;
  const size_t k = b->owned.size();
  praos_ctx* c = b->owner;
  hipError_t e = hipSuccess;
  if (c && k < c->spare.size() && c->spare[k] && c->spare_sz[k] >= sz && c->spare_sz[k] <= 2 * sz + 4096) {
    q = c->spare[k];                 // the previous batch's buffer at the same position
    sz = c->spare_sz[k];
    c->spare[k] = nullptr;
  } else {
    e = hipMalloc(&q, sz);
  }
  if (e == hipSuccess) { b->owned.push_back(q); b->owned_sz.push_back(sz); *p = (T*)q; }
  return e;
}

extern "C" {

int praos_abi_version(void) { return PRAOS_ABI_VERSION; }

int praos_host_register(praos_ctx* c, void* p, size_t len) {
  if (!c || !p || len == 0) return PRAOS_E_ARG;
  if (c->device < 0) return PRAOS_E_STATE;
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipHostRegister(p, len, hipHostRegisterDefault));
  std::lock_guard<std::mutex> g(c->reg_mu);
  c->registered.emplace_back((uintptr_t)p, len);
  return PRAOS_OK;
}

int praos_host_unregister(praos_ctx* c, void* p) {
  if (!c || !p) return PRAOS_E_ARG;
  {
    std::lock_guard<std::mutex> g(c->reg_mu);
    auto it = std::find_if(c->registered.begin(), c->registered.end(),
                           [&](const std::pair<uintptr_t, size_t>& r) { return r.first == (uintptr_t)p; });
    if (it == c->registered.end()) return PRAOS_E_ARG;
    c->registered.erase(it);
  }
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipHostUnregister(p));
  return PRAOS_OK;
}

const char* praos_last_error(praos_ctx* ctx) { return ctx ? ctx->err.c_str() : "no context"; }

// streams and events of a context (praos_open, and the pipeline's second engine)
static bool open_streams(praos_ctx* c) {
  if (const char* kp = std::getenv("PRAOS_KEY_PRIO")) c->key_wave_prio = std::atoi(kp);
  if (hipSetDevice(c->device) != hipSuccess || hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
    c->stream = nullptr;
    return false;
  }
  for (auto& e : c->ev) (void)hipEventCreate(&e);
  for (auto& e : c->side_ev) (void)hipEventCreate(&e);
  for (auto& e : c->miss_ev) (void)hipEventCreateWithFlags(&e, hipEventDisableTiming);
  for (auto& e : c->mdone_ev) (void)hipEventCreateWithFlags(&e, hipEventDisableTiming);
  (void)hipEventCreateWithFlags(&c->v_ev, hipEventDisableTiming);
  (void)hipEventCreateWithFlags(&c->v2_ev, hipEventDisableTiming);
  (void)hipEventCreate(&c->v0_ev);
  (void)hipEventCreateWithFlags(&c->u_ev, hipEventDisableTiming);
  if (const char* e = std::getenv("PRAOS_VRF3")) c->vrf3 = std::atoi(e) != 0;
  if (const char* e = std::getenv("PRAOS_VRF_PRIO")) c->vrf_prio = std::atoi(e);
  if (const char* e = std::getenv("PRAOS_VRF_ILP4")) c->vrf_ilp4 = std::atoi(e);
  if (const char* e = std::getenv("PRAOS_V_EXCL")) c->v_excl = std::atoi(e);
  if (const char* e = std::getenv("PRAOS_MISS4")) c->miss4 = std::atoi(e);
  if (const char* e = std::getenv("PRAOS_KEY4")) c->key4 = std::atoi(e);
  if (const char* e = std::getenv("PRAOS_U4")) c->u4 = std::atoi(e);
  if (const char* e = std::getenv("PRAOS_CK4")) c->ck4 = std::atoi(e);
  if (const char* e = std::getenv("PRAOS_KES_DEDUP")) c->kes_dedup = std::atoi(e);
  if (const char* e = std::getenv("PRAOS_POOL_KEYS")) (void)praos_set_option(c, PRAOS_OPT_POOL_KEYS, std::atoi(e));
  if (const char* e = std::getenv("PRAOS_VRF_KEYS_FIRST")) c->vrf_keys_first = std::atoi(e);
  if (const char* e = std::getenv("PRAOS_PRE_JOIN")) c->pre_join = std::atoi(e);
  if (const char* e = std::getenv("PRAOS_V_MAIN")) c->v_main = std::atoi(e);
  if (const char* e = std::getenv("PRAOS_STREAM_CHUNK_V")) c->stream_chunk_v = std::atoi(e);
  if (const char* e = std::getenv("PRAOS_KES_NOCACHE")) c->kes_nocache = (size_t)std::atoll(e);
  if (const char* e = std::getenv("PRAOS_MISS_PRIO")) c->miss_prio = std::atoi(e);
  if (const char* e = std::getenv("PRAOS_KES_PAIR")) c->kes_pair = std::atol(e);
  if (const char* e = std::getenv("PRAOS_KC_MIN")) (void)std::sscanf(e, "%d,%d,%d", &c->kc_min[0], &c->kc_min[1], &c->kc_min[2]);
  if (const char* e = std::getenv("PRAOS_TP_STAGED")) c->tp_staged = std::atoi(e) != 0;
  if (const char* e = std::getenv("PRAOS_PIPE_HEAD")) c->pipe_head = std::max(5, std::min(100, std::atoi(e)));
  if (const char* e = std::getenv("PRAOS_PIPE_TAIL")) c->pipe_tail = std::max(5, std::min(100, std::atoi(e)));
  (void)hipEventCreate(&c->v1_ev);
  (void)hipEventCreate(&c->kc0_ev);
  (void)hipEventCreate(&c->kc1_ev);
  for (auto& e : c->up_ev) (void)hipEventCreateWithFlags(&e, hipEventDisableTiming);
  for (auto& e : c->done_ev) (void)hipEventCreateWithFlags(&e, hipEventDisableTiming);
  for (auto& p : c->pcall) (void)hipEventCreateWithFlags(&p.ev, hipEventDisableTiming);
  // side streams: [0] OCert, [1] KES, [2] VRF.  The VRF stream (the longest chain of
  // work) gets the device's greatest priority, so its waves dispatch first and the
  // KES / OCert / miss kernels fill the remaining slots and its tail (C5: 15.8 ->
  // 14.3 ms per 432k-header step, round-2 A/B).  PRAOS_SIDE_PRIO = three
  // digits overriding that (1 = greatest, 0 = default priority), an A/B knob.
  {
    int least = 0, greatest = 0;
    (void)hipDeviceGetStreamPriorityRange(&least, &greatest);
    const char* pe = std::getenv("PRAOS_SIDE_PRIO");
    if (!pe || std::strlen(pe) != 3) pe = "001";
    for (int k = 0; k < 3; k++) {
      const bool hi = pe && std::strlen(pe) == 3 && pe[k] == '1';
      (void)hipStreamCreateWithPriority(&c->side[k], hipStreamNonBlocking, hi ? greatest : least);
      // each kind's misses get a stream of their own at the same priority: a handful of
      // uncached verifies is one full-length chain of latency, and three of them in a
      // row on one stream were the critical path of small batches (54k headers: k_kes
      // 2.1 ms -> k_vrf 3.4 ms -> k_ocert 1.6 ms, profiles/r03b/timeline.txt)
      (void)hipStreamCreateWithPriority(&c->mside[k], hipStreamNonBlocking, hi ? greatest : least);
    }
    // the VRF's stage V is the longest chain of a batch and starts at once: greatest priority
    // (PRAOS_V_PRIO=0: least, an A/B knob)
    const char* vp = std::getenv("PRAOS_V_PRIO");
    const int vprio = (vp && std::atoi(vp) == 0) ? least : greatest;
    (void)hipStreamCreateWithPriority(&c->vstream, hipStreamNonBlocking, vprio);
    (void)hipStreamCreateWithPriority(&c->vstream2, hipStreamNonBlocking, vprio);
    // the copy stream (uploads; the replay's decode): PRAOS_CSTREAM_PRIO=1 at the greatest priority
    const char* cp = std::getenv("PRAOS_CSTREAM_PRIO");
    // (the copy / decode / download streams on hardware queues of their own -- CU-masked streams,
    // every CU enabled -- or GPU_MAX_HW_QUEUES=16 were measured for the streaming form: no gain,
    // 13.2-13.4 -> 13.5-13.7 ms per call, profiles/r06/l_stream)
    (void)hipStreamCreateWithPriority(&c->cstream, hipStreamNonBlocking, (cp && std::atoi(cp) == 1) ? greatest : least);
    (void)hipStreamCreateWithFlags(&c->dstream, hipStreamNonBlocking);
    (void)hipStreamCreateWithFlags(&c->decstream, hipStreamNonBlocking);
  }
  return true;
}

praos_ctx* praos_open(int device) {
  if (device == PRAOS_HOST_ONLY) {
    praos_ctx* c = new praos_ctx();
    c->device = -1;
    return c;
  }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0 || device < 0 || device >= ndev) {
    fprintf(stderr, "praos_open: no HIP device %d (count %d)\n", device, ndev);
    return nullptr;
  }
  praos_ctx* c = new praos_ctx();
  c->device = device;
  if (!open_streams(c)) {
    praos_close(c);
    return nullptr;
  }
  if (hipMalloc(&c->btab, BCOMB_TABLES * BTAB_N * NIELS_BYTES) != hipSuccess) {
    c->btab = nullptr;
    praos_close(c);
    return nullptr;
  }
  launch_init_btab(dim3(BCOMB_TABLES * BTAB_N / 256), dim3(256), c->stream, c->btab);
  if (hipStreamSynchronize(c->stream) != hipSuccess || hipGetLastError() != hipSuccess) {
    fprintf(stderr, "praos_open: init kernel failed\n");
    praos_close(c);
    return nullptr;
  }
  return c;
}

// The radix-2^16 comb of the cached-key chains (48 MB, scalarmult.hpp C16_T x C16_N):
// built on the first run that uses a key cache, on the ctx stream (the kernels that
// read it are ordered after it), then kept for the context's lifetime.
static int ensure_bcomb16(praos_ctx* c) {
  if (c->bcomb16) return PRAOS_OK;
  ge_niels* t = nullptr;
  if (hipMalloc(&t, C16_TABLES * C16_ENTRIES * NIELS_BYTES) != hipSuccess) {
    c->err = "praos: radix-2^16 comb allocation (48 MB) failed";
    return PRAOS_E_OOM;
  }
  launch_init_bcomb16(c->stream, c->btab, t);
  if (hipGetLastError() != hipSuccess) {
    (void)hipStreamSynchronize(c->stream);
    (void)hipFree(t);
    c->err = "praos: comb init launch failed";
    return PRAOS_E_HIP;
  }
  c->bcomb16 = t;
  return PRAOS_OK;
}

static void free_epoch(praos_ctx* c) {
  (void)hipFree(c->d_pool_hash); (void)hipFree(c->d_pool_vrf); (void)hipFree(c->d_pool_x);
  (void)hipFree(c->d_pool_map); (void)hipFree(c->d_eta0);
  c->d_pool_hash = nullptr; c->d_pool_vrf = nullptr; c->d_pool_x = nullptr; c->d_pool_map = nullptr; c->d_eta0 = nullptr;
}

void praos_close(praos_ctx* c) {
  if (!c) return;
  if (c->device < 0) { delete c; return; }
  (void)hipSetDevice(c->device);
  (void)praos_verify_drain(c);                 // submitted calls' outputs are written before the close
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  free_epoch(c);
  (void)hipFree(c->d_gen);
  (void)hipFree(c->btab);
  (void)hipFree(c->bcomb16);
  for (auto& ps : c->pks) {
    for (void* q : {(void*)ps.pkey, (void*)ps.count, (void*)ps.base, (void*)ps.entry_rep, (void*)ps.entry_pos,
                    (void*)ps.kinfo, (void*)ps.pentry, (void*)ps.ktab, (void*)ps.scnt, (void*)ps.spos})
      (void)hipFree(q);
  }
  free_spare(c);
  c->pool.reset();
  for (int k = 0; k < 2; k++) {
    if (c->pin[k]) (void)hipHostFree(c->pin[k]);
    if (c->pin_ev[k]) (void)hipEventDestroy(c->pin_ev[k]);
  }
  if (c->zero_h) (void)hipHostFree(c->zero_h);
  for (auto& e : c->ev) if (e) (void)hipEventDestroy(e);
  for (auto& e : c->side_ev) if (e) (void)hipEventDestroy(e);
  for (auto& e : c->miss_ev) if (e) (void)hipEventDestroy(e);
  for (auto& e : c->mdone_ev) if (e) (void)hipEventDestroy(e);
  for (auto& st : c->side) if (st) (void)hipStreamDestroy(st);
  for (auto& st : c->mside) if (st) (void)hipStreamDestroy(st);
  if (c->vstream) (void)hipStreamDestroy(c->vstream);
  if (c->vstream2) (void)hipStreamDestroy(c->vstream2);
  if (c->v2_ev) (void)hipEventDestroy(c->v2_ev);
  if (c->v_ev) (void)hipEventDestroy(c->v_ev);
  if (c->v0_ev) (void)hipEventDestroy(c->v0_ev);
  if (c->u_ev) (void)hipEventDestroy(c->u_ev);
  if (c->v1_ev) (void)hipEventDestroy(c->v1_ev);
  if (c->kc0_ev) (void)hipEventDestroy(c->kc0_ev);
  if (c->kc1_ev) (void)hipEventDestroy(c->kc1_ev);
  if (c->cstream) (void)hipStreamSynchronize(c->cstream);
  for (int k = 0; k < RP_SLOTS; k++) rp_batch_destroy(c, c->rp_keep[k]);
  for (int k = 0; k < PIPE_MAX; k++) {
    if (c->pipe[k]) {
      for (void* p : c->pipe[k]->owned) (void)hipFree(p);
      delete c->pipe[k];
    }
    if (c->up_ev[k]) (void)hipEventDestroy(c->up_ev[k]);
    if (c->done_ev[k]) (void)hipEventDestroy(c->done_ev[k]);
  }
  for (auto& p : c->pcall) {
    if (p.ev) (void)hipEventDestroy(p.ev);
    if (p.off_h) (void)hipHostFree(p.off_h);
    if (p.len_h) (void)hipHostFree(p.len_h);
  }
  if (c->cstream) (void)hipStreamDestroy(c->cstream);
  if (c->dstream) (void)hipStreamDestroy(c->dstream);
  if (c->decstream) (void)hipStreamDestroy(c->decstream);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

}  // extern "C"

// The pool part of a ledger view (lvPoolDistr): the caller's pools, the map hash28 -> caller
// index (OCert counter slots), and on a device the tables the VRF join and the leader test read
// (hashes sorted, 7 words each | VRF key hashes, 8 | x = -(sigma * c) in Fixed E34, 4 | sorted
// index -> caller index).  praos_set_epoch installs one in the context; the per-epoch replay
// (praos_replay_immutable_views) keeps one per view and swaps its device tables in between batches.
struct rp_view {
  int device = -1;
  uint32_t npools = 0;
  std::vector<praos_pool> pools;
  std::map<std::string, int32_t> by_hash;
  uint32_t *d_hash = nullptr, *d_vrf = nullptr, *d_x = nullptr;
  int32_t* d_map = nullptr;
};

static void pool_tables_free(rp_view* v) {
  if (!v || v->device < 0) return;
  (void)hipFree(v->d_hash); (void)hipFree(v->d_vrf); (void)hipFree(v->d_x); (void)hipFree(v->d_map);
  v->d_hash = v->d_vrf = v->d_x = nullptr;
  v->d_map = nullptr;
}

// Builds v's host map and, for device >= 0, its device tables (on the current device).  On
// failure nothing is left allocated and err says why.
static int pool_tables_build(rp_view* v, int device, const praos_pool* pools, uint32_t npools,
                             const praos_params* params, std::string* err) {
  std::vector<int32_t> order(npools);
  for (uint32_t i = 0; i < npools; i++) order[i] = (int32_t)i;
  std::sort(order.begin(), order.end(), [&](int32_t a, int32_t b) {
    return std::memcmp(pools[a].hash28, pools[b].hash28, 28) < 0;
  });
  std::vector<uint32_t> h(7 * (size_t)std::max(1u, npools)), vr(8 * (size_t)std::max(1u, npools)),
      x(4 * (size_t)std::max(1u, npools));
  std::map<std::string, int32_t> by_hash;
  for (uint32_t s = 0; s < npools; s++) {
    const praos_pool& p = pools[order[s]];
    std::memcpy(&h[7 * s], p.hash28, 28);
    std::memcpy(&vr[8 * s], p.vrf_hash32, 32);
    uint8_t xr[16];
    if (!praos_host::leader_x_raw(xr, p.sigma_fp, params->c_raw)) {
      *err = "sigma * activeSlotLog out of range (x_raw > 16 * 10^34)";
      return PRAOS_E_ARG;
    }
    std::memcpy(&x[4 * s], xr, 16);
    by_hash[std::string((const char*)p.hash28, 28)] = order[s];
  }
  v->device = device;
  if (device >= 0) {
    bool ok = hipMalloc(&v->d_hash, h.size() * 4) == hipSuccess && hipMalloc(&v->d_vrf, vr.size() * 4) == hipSuccess &&
              hipMalloc(&v->d_x, x.size() * 4) == hipSuccess &&
              hipMalloc(&v->d_map, std::max<size_t>(1, npools) * 4) == hipSuccess;
    ok = ok && hipMemcpy(v->d_hash, h.data(), h.size() * 4, hipMemcpyHostToDevice) == hipSuccess &&
         hipMemcpy(v->d_vrf, vr.data(), vr.size() * 4, hipMemcpyHostToDevice) == hipSuccess &&
         hipMemcpy(v->d_x, x.data(), x.size() * 4, hipMemcpyHostToDevice) == hipSuccess &&
         (!npools || hipMemcpy(v->d_map, order.data(), npools * 4, hipMemcpyHostToDevice) == hipSuccess);
    if (!ok) {
      pool_tables_free(v);
      *err = "pool tables: device allocation / copy failed";
      return PRAOS_E_OOM;
    }
  }
  v->npools = npools;
  v->pools.assign(pools, pools + npools);
  v->by_hash.swap(by_hash);
  return PRAOS_OK;
}

rp_view* rp_view_make(praos_ctx* c, const praos_pool* pools, uint32_t npools, const praos_params* params,
                      bool device) {
  if (!c || !params || (npools && !pools)) return nullptr;
  if (device && c->device < 0) return nullptr;
  if (device) (void)hipSetDevice(c->device);
  rp_view* v = new rp_view;
  std::string err;
  if (pool_tables_build(v, device ? c->device : -1, pools, npools, params, &err) != PRAOS_OK) {
    c->err = err;
    delete v;
    return nullptr;
  }
  return v;
}

void rp_view_free(praos_ctx* c, rp_view* v) {
  if (!v) return;
  if (c && v->device >= 0) (void)hipSetDevice(v->device);
  pool_tables_free(v);
  delete v;
}

rp_tables rp_tables_get(const praos_ctx* c) {
  return {c->npools, c->d_pool_hash, c->d_pool_vrf, c->d_pool_x, c->d_pool_map};
}

void rp_tables_set(praos_ctx* c, const rp_tables& t) {
  c->npools = t.npools;
  c->d_pool_hash = t.hash; c->d_pool_vrf = t.vrf; c->d_pool_x = t.x; c->d_pool_map = t.map;
}

rp_tables rp_view_tables(const rp_view* v) { return {v->npools, v->d_hash, v->d_vrf, v->d_x, v->d_map}; }

extern "C" {

int praos_set_epoch(praos_ctx* c, const uint8_t eta0[32], const praos_pool* pools, uint32_t npools,
                    const praos_params* params) {
  if (!c || !params || (npools && !pools) || params->slots_per_kes_period == 0) return PRAOS_E_ARG;
  // The installed ledger view again (a replay call per batch of epochs, db-analyser's per-epoch
  // calls under an unchanged PoolDistr): only the epoch nonce changes
  if (c->have_epoch && c->device >= 0 && npools == c->epoch_pools.size() &&
      std::memcmp(params, &c->epoch_params, sizeof *params) == 0 &&
      (npools == 0 || std::memcmp(pools, c->epoch_pools.data(), npools * sizeof *pools) == 0)) {
    if ((eta0 == nullptr) == c->eta0_neutral && (eta0 == nullptr || std::memcmp(eta0, c->eta0, 32) == 0))
      return PRAOS_OK;                            // the same nonce too: nothing to change
  }
  if (std::any_of(std::begin(c->pcall), std::end(c->pcall), [](const praos_ctx::PipeCall& p) { return p.active; })) {
    // submitted calls (praos_verify_header_bytes_submit) read the installed view and nonce until
    // they end: their outputs first
    const int r = praos_verify_drain(c);
    if (r != PRAOS_OK) return r;
  }
  if (c->have_epoch && c->device >= 0 && npools == c->epoch_pools.size() &&
      std::memcmp(params, &c->epoch_params, sizeof *params) == 0 &&
      (npools == 0 || std::memcmp(pools, c->epoch_pools.data(), npools * sizeof *pools) == 0)) {
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipStreamSynchronize(c->stream));   // no run in flight reads the old nonce
    uint32_t e0[8] = {0};
    if (eta0) std::memcpy(e0, eta0, 32);
    HIPCHK(c, hipMemcpy(c->d_eta0, e0, 32, hipMemcpyHostToDevice));
    c->eta0_neutral = eta0 == nullptr;
    std::memset(c->eta0, 0, 32);
    if (eta0) std::memcpy(c->eta0, eta0, 32);
    return PRAOS_OK;
  }
  // Validate and build every table first; the context is only touched once all of it
  // succeeded (a failed call leaves NO epoch: runs return PRAOS_E_STATE until the next
  // successful praos_set_epoch).
  if (c->device >= 0) {
    HIPCHK(c, hipSetDevice(c->device));
    (void)hipStreamSynchronize(c->stream);      // no run in flight reads the old tables
    free_epoch(c);
  }
  c->have_epoch = false;
  c->npools = 0;
  c->pools.clear();
  c->pool_by_hash.clear();
  rp_view v;
  std::string err;
  int r = pool_tables_build(&v, c->device, pools, npools, params, &err);
  if (r != PRAOS_OK) { c->err = err; return r; }
  if (c->device >= 0) {
    uint32_t e0[8] = {0};
    if (eta0) std::memcpy(e0, eta0, 32);
    if (hipMalloc(&c->d_eta0, 32) != hipSuccess ||
        hipMemcpy(c->d_eta0, e0, 32, hipMemcpyHostToDevice) != hipSuccess) {
      pool_tables_free(&v);
      (void)hipFree(c->d_eta0);
      c->d_eta0 = nullptr;
      c->err = "praos_set_epoch: device allocation / copy failed";
      return PRAOS_E_OOM;
    }
    c->d_pool_hash = v.d_hash; c->d_pool_vrf = v.d_vrf; c->d_pool_x = v.d_x; c->d_pool_map = v.d_map;
  }
  c->params = *params;
  c->eta0_neutral = eta0 == nullptr;
  std::memset(c->eta0, 0, 32);
  if (eta0) std::memcpy(c->eta0, eta0, 32);
  c->npools = npools;
  c->pools.swap(v.pools);
  c->pool_by_hash.swap(v.by_hash);
  c->epoch_pools.assign(pools, pools + npools);
  c->epoch_params = *params;
  c->have_epoch = true;
  return PRAOS_OK;
}

void praos_batch_free(praos_ctx* c, praos_batch* b) {
  if (!b) return;
  if (c && c->device >= 0 && b->owner == c) {
    // keep the buffers for the next batch (its kernels are ordered after this one's on
    // the ctx stream, so no wait is needed); drop the older spares it did not take
    (void)hipSetDevice(c->device);
    free_spare(c);
    c->spare.swap(b->owned);
    c->spare_sz.swap(b->owned_sz);
    delete b;
    return;
  }
  if (c) (void)hipSetDevice(c->device);
  for (void* p : b->owned) (void)hipFree(p);
  delete b;
}

// one public-key cache (k_keys.hip) for batches of up to n items
static bool alloc_keycache(praos_batch* b, praos_batch::KeyCache& k, size_t n) {
  bool ok = true;
  k.cap = 256;
  while (k.cap < 2 * n) k.cap <<= 1;
  k.max_entries = (uint32_t)std::min<size_t>(n / 2 + 1, KC_MAX_ENTRIES);
  ok &= dalloc(b, &k.slot_rep, 4 * (size_t)k.cap) == hipSuccess;
  ok &= dalloc(b, &k.slot_cnt, 4 * (size_t)k.cap) == hipSuccess;
  ok &= dalloc(b, &k.slot_entry, 4 * (size_t)k.cap) == hipSuccess;
  ok &= dalloc(b, &k.item_slot, 4 * n) == hipSuccess;
  ok &= dalloc(b, &k.item_entry, 4 * n) == hipSuccess;
  ok &= dalloc(b, &k.hit, 4 * n) == hipSuccess;
  ok &= dalloc(b, &k.miss, 4 * n) == hipSuccess;
  ok &= dalloc(b, &k.counters, 16) == hipSuccess;
  ok &= dalloc(b, &k.entry_rep, 4 * (size_t)k.max_entries) == hipSuccess;
  ok &= dalloc(b, &k.entry_pos, 4 * (size_t)k.max_entries) == hipSuccess;
  ok &= dalloc(b, &k.kinfo, 36 * (size_t)k.max_entries) == hipSuccess;
  ok &= dalloc(b, (uint8_t**)&k.ktab, KT_BYTES * k.max_entries) == hipSuccess;
  ok &= dalloc(b, &k.rep_ok, (size_t)k.max_entries) == hipSuccess;
  return ok;
}

// device buffers of a batch: header SoA, body arena, outputs, key caches
static bool alloc_soa(praos_batch* b, size_t n, size_t body_arena_bytes) {
  bool ok = true;
  ok &= dalloc(b, &b->slot, 8 * n) == hipSuccess;
  ok &= dalloc(b, &b->ocert_n, 8 * n) == hipSuccess;
  ok &= dalloc(b, &b->ocert_c0, 8 * n) == hipSuccess;
  ok &= dalloc(b, &b->body_off, 8 * n) == hipSuccess;
  ok &= dalloc(b, &b->body_len, 4 * n) == hipSuccess;
  ok &= dalloc(b, &b->cold_vk, 32 * n) == hipSuccess;
  ok &= dalloc(b, &b->vrf_vk, 32 * n) == hipSuccess;
  ok &= dalloc(b, &b->vrf_out, 64 * n) == hipSuccess;
  ok &= dalloc(b, &b->vrf_proof, 80 * n) == hipSuccess;
  ok &= dalloc(b, &b->hot_vk, 32 * n) == hipSuccess;
  ok &= dalloc(b, &b->ocert_sig, 64 * n) == hipSuccess;
  ok &= dalloc(b, &b->kes_sig, 448 * n) == hipSuccess;
  ok &= dalloc(b, &b->body, body_arena_bytes) == hipSuccess;
  ok &= dalloc(b, &b->bits, 2 * n) == hipSuccess;
  ok &= dalloc(b, &b->bits3, 6 * n) == hipSuccess;
  ok &= dalloc(b, &b->pool_idx, 4 * n) == hipSuccess;
  ok &= dalloc(b, &b->pool_sorted, 4 * n) == hipSuccess;
  ok &= dalloc(b, &b->beta, 64 * n) == hipSuccess;
  ok &= dalloc(b, &b->leader, 32 * n) == hipSuccess;
  ok &= dalloc(b, &b->nonce, 32 * n) == hipSuccess;
  ok &= dalloc(b, (uint8_t**)&b->tab_ocert, LT_ED_B * n) == hipSuccess;
  ok &= dalloc(b, (uint8_t**)&b->tab_kes, LT_ED_B * n) == hipSuccess;
  ok &= dalloc(b, (uint8_t**)&b->tab_vrf, LT_VRF_B * n) == hipSuccess;
  ok &= dalloc(b, (uint8_t**)&b->tab_vrfu, LT_ED_B * n) == hipSuccess;
  ok &= dalloc(b, &b->vrf_mid, VRF_MID_BYTES * n) == hipSuccess;
  ok &= dalloc(b, &b->kes_leaf, 32 * n) == hipSuccess;
  b->dd_cap = 256;
  while (b->dd_cap < 2 * n) b->dd_cap <<= 1;
  ok &= dalloc(b, &b->dd_slot, 4 * (size_t)b->dd_cap) == hipSuccess;
  ok &= dalloc(b, &b->dd_item_rep, 4 * n) == hipSuccess;
  ok &= dalloc(b, &b->dd_reps, 4 * n) == hipSuccess;
  ok &= dalloc(b, &b->dd_counters, 16) == hipSuccess;
  ok &= dalloc(b, &b->dd_ok, n) == hipSuccess;
  for (auto& k : b->kc) ok &= alloc_keycache(b, k, n);
  return ok;
}

praos_batch* praos_batch_upload(praos_ctx* c, const praos_headers* h) {
  if (!c || !h) return nullptr;
  if (hipSetDevice(c->device) != hipSuccess) return nullptr;
  praos_batch* b = new praos_batch();
  b->owner = c;
  const size_t n = h->n;
  b->n = n;
  // repack bodies 8-byte aligned (the SHA-512 feeder reads 64-bit words)
  std::vector<uint64_t>& off = c->h_off;
  off.resize(n);
  size_t total = 0;
  bool bad_range = false;
  for (size_t i = 0; i < n; i++) {
    off[i] = total;
    if (h->body_off[i] > h->body_bytes_len || h->body_len[i] > h->body_bytes_len - h->body_off[i]) bad_range = true;
    total += (h->body_len[i] + 7) & ~(size_t)7;
  }
  auto tr0 = std::chrono::steady_clock::now();
  if (c->h_arena_cap < total + 16) {
    c->h_arena.reset(new uint8_t[total + 16]);
    c->h_arena_cap = total + 16;
  }
  uint8_t* const arena = c->h_arena.get();
  std::vector<uint32_t>& len = c->h_len;
  len.resize(n);
  auto repack = [&](size_t i0, size_t i1) {
    for (size_t i = i0; i < i1; i++) {
      const bool ok = h->body_off[i] <= h->body_bytes_len && h->body_len[i] <= h->body_bytes_len - h->body_off[i];
      len[i] = ok ? h->body_len[i] : 0xffffffffu;  // marks out-of-range (kernel flags PRAOS_BIT_INPUT)
      const size_t pad = ((size_t)h->body_len[i] + 7) & ~(size_t)7;
      uint8_t* d = arena + off[i];
      if (ok) std::memcpy(d, h->body_bytes + h->body_off[i], h->body_len[i]);
      if (pad > (ok ? (size_t)h->body_len[i] : 0)) std::memset(d + (ok ? h->body_len[i] : 0), 0, pad - (ok ? h->body_len[i] : 0));
    }
  };
  if (n >= 65536 && stage_init(c)) {
    const unsigned nt = c->pool->size();
    c->pool->run([&](unsigned t) { repack(n * t / nt, n * (t + 1) / nt); });
  } else {
    repack(0, n);
  }
  std::memset(arena + total, 0, 16);
  if (std::getenv("PRAOS_TRACE_UPLOAD"))
    fprintf(stderr, "upload: repack %.2f ms\n",
            std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tr0).count());
  (void)bad_range;
  b->body_bytes_len = total;
  static const bool trace = std::getenv("PRAOS_TRACE_UPLOAD") != nullptr;
  auto now = [] { return std::chrono::steady_clock::now(); };
  auto t0 = now();
  bool ok = alloc_soa(b, n, total + 16);
  if (!ok) { c->err = "device allocation failed"; praos_batch_free(c, b); return nullptr; }
  if (trace) fprintf(stderr, "upload: alloc %.2f ms\n", std::chrono::duration<double, std::milli>(now() - t0).count());
  auto up = [&](void* d, const void* s, size_t bytes) {
    auto t = now();
    if (bytes) ok &= h2d(c, d, s, bytes) == hipSuccess;
    if (trace) fprintf(stderr, "upload: %zu bytes %.2f ms\n", bytes, std::chrono::duration<double, std::milli>(now() - t).count());
  };
  up(b->slot, h->slot, 8 * n);
  up(b->ocert_n, h->ocert_n, 8 * n);
  up(b->ocert_c0, h->ocert_c0, 8 * n);
  up(b->body_off, off.data(), 8 * n);
  up(b->body_len, len.data(), 4 * n);
  up(b->cold_vk, h->cold_vk, 32 * n);
  up(b->vrf_vk, h->vrf_vk, 32 * n);
  up(b->vrf_out, h->vrf_out, 64 * n);
  up(b->vrf_proof, h->vrf_proof, 80 * n);
  up(b->hot_vk, h->hot_vk, 32 * n);
  up(b->ocert_sig, h->ocert_sig, 64 * n);
  up(b->kes_sig, h->kes_sig, 448 * n);
  up(b->body, arena, total + 16);
  auto ts = now();
  ok &= hipStreamSynchronize(c->stream) == hipSuccess;
  if (trace) fprintf(stderr, "upload: final sync %.2f ms, from the repack %.2f ms\n",
                     std::chrono::duration<double, std::milli>(now() - ts).count(),
                     std::chrono::duration<double, std::milli>(now() - tr0).count());
  if (!ok) { c->err = "upload failed"; praos_batch_free(c, b); return nullptr; }
  return b;
}

static praos_batch* upload_bytes_impl(praos_ctx* c, const praos_header_bytes* in, bool tpraos);

praos_batch* praos_batch_upload_bytes(praos_ctx* c, const praos_header_bytes* in) {
  return upload_bytes_impl(c, in, false);
}

// device buffers of a from-bytes batch of n headers over an arena of bytes_len bytes
// (owner == nullptr: fresh allocations, not taken from / given back to the spare list)
static praos_batch* bytes_batch_alloc(praos_ctx* c, size_t n, size_t bytes_len, bool tpraos, praos_ctx* owner) {
  praos_batch* b = new praos_batch();
  b->owner = owner;
  b->n = n;
  b->from_bytes = true;
  b->arena_len = bytes_len;
  b->tp_only = tpraos;
  b->signed_stride = tpraos ? TP_SIGNED_STRIDE : PRAOS_SIGNED_STRIDE;
  b->body_bytes_len = (size_t)b->signed_stride * n;
  bool ok = alloc_soa(b, n, b->body_bytes_len + 16);
  if (tpraos) {
    ok &= dalloc(b, &b->lead_out, 64 * n) == hipSuccess;
    ok &= dalloc(b, &b->lead_proof, 80 * n) == hipSuccess;
    ok &= dalloc(b, &b->beta_l, 64 * n) == hipSuccess;
  }
  ok &= dalloc(b, &b->arena, ((bytes_len + 7) & ~(size_t)7) + 16) == hipSuccess;  // +16: ld64u pad
  ok &= dalloc(b, &b->hoff, 8 * n) == hipSuccess;
  ok &= dalloc(b, &b->hlen, 4 * n) == hipSuccess;
  ok &= dalloc(b, &b->block_no, 8 * n) == hipSuccess;
  ok &= dalloc(b, &b->prot_major, 8 * n) == hipSuccess;
  ok &= dalloc(b, &b->prot_minor, 8 * n) == hipSuccess;
  ok &= dalloc(b, &b->body_size, 4 * n) == hipSuccess;
  ok &= dalloc(b, &b->prev_hash, 32 * n) == hipSuccess;
  ok &= dalloc(b, &b->prev_genesis, n) == hipSuccess;
  ok &= dalloc(b, &b->body_hash, 32 * n) == hipSuccess;
  ok &= dalloc(b, &b->header_hash, 32 * n) == hipSuccess;
  ok &= dalloc(b, &b->dec_status, 2 * n) == hipSuccess;
  if (!ok) {
    c->err = "device allocation failed";
    for (void* p : b->owned) (void)hipFree(p);
    delete b;
    return nullptr;
  }
  return b;
}

static praos_batch* upload_bytes_impl(praos_ctx* c, const praos_header_bytes* in, bool tpraos) {
  if (!c || !in || (in->n && (!in->off || !in->len || (!in->bytes && in->bytes_len)))) return nullptr;
  if (c->device < 0) { c->err = "host-only context: no HIP device"; return nullptr; }
  if (hipSetDevice(c->device) != hipSuccess) return nullptr;
  praos_batch* b = new praos_batch();
  b->owner = c;
  const size_t n = in->n;
  b->n = n;
  b->from_bytes = true;
  b->arena_len = in->bytes_len;
  b->tp_only = tpraos;
  b->signed_stride = tpraos ? TP_SIGNED_STRIDE : PRAOS_SIGNED_STRIDE;
  b->body_bytes_len = (size_t)b->signed_stride * n;
  bool ok = alloc_soa(b, n, b->body_bytes_len + 16);
  if (tpraos) {
    ok &= dalloc(b, &b->lead_out, 64 * n) == hipSuccess;
    ok &= dalloc(b, &b->lead_proof, 80 * n) == hipSuccess;
    ok &= dalloc(b, &b->beta_l, 64 * n) == hipSuccess;
  }
  ok &= dalloc(b, &b->arena, ((in->bytes_len + 7) & ~(size_t)7) + 16) == hipSuccess;  // +16: ld64u pad
  ok &= dalloc(b, &b->hoff, 8 * n) == hipSuccess;
  ok &= dalloc(b, &b->hlen, 4 * n) == hipSuccess;
  ok &= dalloc(b, &b->block_no, 8 * n) == hipSuccess;
  ok &= dalloc(b, &b->prot_major, 8 * n) == hipSuccess;
  ok &= dalloc(b, &b->prot_minor, 8 * n) == hipSuccess;
  ok &= dalloc(b, &b->body_size, 4 * n) == hipSuccess;
  ok &= dalloc(b, &b->prev_hash, 32 * n) == hipSuccess;
  ok &= dalloc(b, &b->prev_genesis, n) == hipSuccess;
  ok &= dalloc(b, &b->body_hash, 32 * n) == hipSuccess;
  ok &= dalloc(b, &b->header_hash, 32 * n) == hipSuccess;
  ok &= dalloc(b, &b->dec_status, 2 * n) == hipSuccess;
  if (!ok) { c->err = "device allocation failed"; praos_batch_free(c, b); return nullptr; }
  const size_t pad = ((in->bytes_len + 7) & ~(size_t)7) + 16 - in->bytes_len;
  ok &= hipMemsetAsync(b->arena + in->bytes_len, 0, pad, c->stream) == hipSuccess;
  if (in->bytes_len)
    ok &= h2d(c, b->arena, in->bytes, in->bytes_len) == hipSuccess;
  if (n) {
    ok &= hipMemcpyAsync(b->hoff, in->off, 8 * n, hipMemcpyHostToDevice, c->stream) == hipSuccess;
    ok &= hipMemcpyAsync(b->hlen, in->len, 4 * n, hipMemcpyHostToDevice, c->stream) == hipSuccess;
  }
  ok &= hipStreamSynchronize(c->stream) == hipSuccess;
  if (!ok) { c->err = "upload failed"; praos_batch_free(c, b); return nullptr; }
  return b;
}

// k_decode_praos over a from-bytes batch, on the ctx stream
static int batch_decode(praos_ctx* c, praos_batch* b) {
  if (b->n == 0) return PRAOS_OK;
  launch_decode_praos(dim3(nblocks(b->n, NT)), dim3(NT), c->stream, b->n, b->arena, b->arena_len, b->hoff, b->hlen,
                      b->slot, b->cold_vk, b->vrf_vk, b->vrf_out, b->vrf_proof, b->hot_vk, b->ocert_sig, b->kes_sig,
                      b->ocert_n, b->ocert_c0, b->body_off, b->body_len, b->body, b->block_no, b->prev_hash,
                      b->prev_genesis, b->body_size, b->body_hash, b->prot_major, b->prot_minor, b->header_hash,
                      b->dec_status, b->is_block ? 1 : (b->tp_only ? 2 : 0), b->signed_stride, b->lead_out,
                      b->lead_proof);
  return hipGetLastError() == hipSuccess ? PRAOS_OK : PRAOS_E_HIP;
}

static int32_t overlay_class(const praos_ctx* c, uint64_t slot);
static int batch_run_impl(praos_ctx* c, praos_batch* b);
static int tpraos_download(praos_ctx* c, praos_batch* b, const uint8_t* dbeta_l, praos_tpraos_out* out);

int praos_batch_run(praos_ctx* c, praos_batch* b) {
  if (!c || !b) return PRAOS_E_ARG;
  if (!c->have_epoch) return PRAOS_E_STATE;
  HIPCHK(c, hipSetDevice(c->device));
  if (b->n == 0) return PRAOS_OK;
  const int r = batch_run_impl(c, b);
  if (r != PRAOS_OK && c->concurrent) {
    // work already queued on the side streams must be ordered before anything the ctx
    // stream runs next (praos_batch_free hands this batch's buffers to the next upload)
    for (int k = 0; k < 3; k++) {
      if (hipEventRecord(c->side_ev[k], c->side[k]) != hipSuccess ||
          hipStreamWaitEvent(c->stream, c->side_ev[k], 0) != hipSuccess)
        (void)hipStreamSynchronize(c->side[k]);
      if (hipEventRecord(c->mdone_ev[k], c->mside[k]) != hipSuccess ||
          hipStreamWaitEvent(c->stream, c->mdone_ev[k], 0) != hipSuccess)
        (void)hipStreamSynchronize(c->mside[k]);
    }
    if (hipEventRecord(c->v_ev, c->vstream) != hipSuccess || hipStreamWaitEvent(c->stream, c->v_ev, 0) != hipSuccess)
      (void)hipStreamSynchronize(c->vstream);
    if (hipEventRecord(c->v2_ev, c->vstream2) != hipSuccess || hipStreamWaitEvent(c->stream, c->v2_ev, 0) != hipSuccess)
      (void)hipStreamSynchronize(c->vstream2);
  }
  return r;
}

// key cache prepass over items [0, n) (or list[0 .. *count)): hash set, entries, hit/miss lists
// the pool-key store t (cold 0, VRF 1): 32,768 slots, 16,384 entries.  Allocated on first use
// and initialised on st, the stream every later use of store t is ordered after (the cache's
// own stream; the context's other streams join it at the end of a run): no device-wide sync.
static bool ensure_pks(praos_ctx* c, int t, hipStream_t st) {
  praos_ctx::PoolKeyStore& s = c->pks[t];
  if (s.ktab) return true;
  praos_ctx::PoolKeyStore z;
  z.slots = 1u << 15;
  z.cap = 1u << 14;
  bool ok = hipMalloc(&z.pkey, 32 * (size_t)z.slots) == hipSuccess;
  ok = ok && hipMalloc(&z.pentry, 4 * (size_t)z.slots) == hipSuccess;
  ok = ok && hipMalloc(&z.count, 8) == hipSuccess;
  ok = ok && hipMalloc(&z.base, 8) == hipSuccess;
  ok = ok && hipMalloc(&z.entry_rep, 4 * (size_t)z.cap) == hipSuccess;
  ok = ok && hipMalloc(&z.entry_pos, 4 * (size_t)z.cap) == hipSuccess;
  ok = ok && hipMalloc(&z.kinfo, 36 * (size_t)z.cap) == hipSuccess;
  ok = ok && hipMalloc(&z.ktab, KT_BYTES * (size_t)z.cap) == hipSuccess;
  ok = ok && hipMalloc(&z.scnt, 4 * (size_t)z.cap) == hipSuccess;
  ok = ok && hipMalloc(&z.spos, 4 * (size_t)z.cap) == hipSuccess;
  ok = ok && hipMemsetAsync(z.pentry, 0xff, 4 * (size_t)z.slots, st) == hipSuccess;
  ok = ok && hipMemsetAsync(z.count, 0, 8, st) == hipSuccess;
  ok = ok && hipMemsetAsync(z.base, 0, 8, st) == hipSuccess;
  if (!ok) {
    (void)hipStreamSynchronize(st);              // (the memsets queued so far) before the frees
    for (void* q : {(void*)z.pkey, (void*)z.count, (void*)z.base, (void*)z.entry_rep, (void*)z.entry_pos,
                    (void*)z.kinfo, (void*)z.pentry, (void*)z.ktab, (void*)z.scnt, (void*)z.spos})
      (void)hipFree(q);
    return false;
  }
  s = z;
  return true;
}

static int kc_lists(praos_ctx* c, praos_batch::KeyCache& k, size_t n, const uint8_t* keys, hipStream_t st,
                    const uint32_t* list, const uint32_t* count, int which) {
  int min_uses = c->kc_min[which] > 0 ? c->kc_min[which] : c->keycache;
  // small batches: no KES leaf key is cached (every item a miss, KES_NOCACHE_BATCH); the batch size
  // is the caller's n (the lists of the KES pass run over every header)
  if (which == 2 && c->kc_min[2] <= 0 && n < c->kes_nocache) min_uses = INT32_MAX;
  const dim3 g(nblocks(n, NT)), blk(NT);
  k.kt = k.ktab; k.ki = k.kinfo; k.erep = k.entry_rep; k.epos = k.entry_pos; k.emax = k.max_entries;
  k.ebase = nullptr; k.store = -1;
  HIPCHK(c, hipMemsetAsync(k.slot_rep, 0, 4 * (size_t)k.cap, st));
  HIPCHK(c, hipMemsetAsync(k.slot_cnt, 0, 4 * (size_t)k.cap, st));
  HIPCHK(c, hipMemsetAsync(k.counters, 0, 16, st));
  praos_ctx::PoolKeyStore* ps = nullptr;
  if (c->pk_on && which < 2 && ensure_pks(c, which, st)) {
    // pool keys: entries continue the store's, every new key is cached (it recurs in the runs
    // that follow); a store more than 3/4 full (decided on the device, from the count the last
    // run left: no host read of a count still in flight) or one asked to be emptied is emptied
    ps = &c->pks[which];
    launch_pkey_reset(st, ps->count, ps->pentry, ps->slots, ps->cap / 4 * 3, c->pk_reset[which] ? 1 : 0);
    c->pk_reset[which] = false;
    HIPCHK(c, hipMemsetAsync(ps->scnt, 0, 4 * (size_t)ps->cap, st));
    HIPCHK(c, hipMemcpyAsync(k.counters, ps->count, 4, hipMemcpyDeviceToDevice, st));
    HIPCHK(c, hipMemcpyAsync(ps->base, ps->count, 4, hipMemcpyDeviceToDevice, st));
    k.kt = ps->ktab; k.ki = ps->kinfo; k.erep = ps->entry_rep; k.epos = ps->entry_pos; k.emax = ps->cap;
    k.ebase = ps->base; k.store = which;
    min_uses = 1;
  }
  launch_key_insert(g, blk, st, n, list, count, keys, k.cap - 1, k.slot_rep, k.slot_cnt, k.item_slot,
                    ps ? ps->pentry : nullptr, ps ? ps->pkey : nullptr, ps ? ps->slots - 1 : 0u,
                    ps ? ps->scnt : nullptr);
  launch_key_assign(dim3(nblocks(k.cap, NT)), blk, st, k.cap, k.slot_rep, k.slot_cnt, (uint32_t)min_uses,
                    k.emax, k.slot_entry, k.erep, k.epos, k.counters);
  if (ps) launch_key_store_ranges(st, ps->cap, ps->scnt, ps->spos, k.counters);
  launch_key_partition(g, blk, st, n, list, count, k.item_slot, k.slot_entry, k.item_entry, k.epos, k.hit, k.miss,
                       k.counters, ps ? ps->spos : nullptr);
  return PRAOS_OK;
}
static void kc_precompute(praos_ctx* c, praos_batch::KeyCache& k, const uint8_t* keys, int kind, hipStream_t st, size_t n) {
  const int prio = c->key_wave_prio > 0 || (c->key_wave_prio < 0 && n < KEY_PRIO_BATCH);
  if (k.store < 0) {
    launch_key_precompute(kind, st, k.counters, k.max_entries, k.entry_rep, keys, k.ktab, k.kinfo, prio, nullptr,
                          k.max_entries, c->key_mode(n));
    return;
  }
  praos_ctx::PoolKeyStore& ps = c->pks[k.store];
  const uint32_t span = (uint32_t)std::min<size_t>(n, ps.cap);   // new entries of this run, at most
  launch_key_precompute(kind, st, k.counters, ps.cap, ps.entry_rep, keys, ps.ktab, ps.kinfo, prio, ps.base, span,
                        c->key_mode(n));
  launch_pkey_publish(st, k.counters, ps.base, ps.cap, ps.entry_rep, keys, ps.pentry, ps.pkey, ps.slots - 1, ps.count,
                      span);
}

static int batch_run_impl(praos_ctx* c, praos_batch* b) {
  const size_t n = b->n;
  const praos_params& P = c->params;
  uint16_t* bo = b->bits3;
  uint16_t* bk = b->bits3 + n;
  uint16_t* bv = b->bits3 + 2 * n;
  const dim3 g(nblocks(n, NT)), blk(NT);
  const dim3 gl(nblocks(n, lat_block(n))), bl(lat_block(n));     // kernels without LDS tables
  // The three crypto kernels are independent; run concurrently they fill each
  // other's tail waves (one launch of 432k headers is ~3.3 rounds of resident
  // waves).  Each writes its own bit array; k_leader joins and combines.
  hipStream_t so = c->concurrent ? c->side[0] : c->stream;
  hipStream_t sk = c->concurrent ? c->side[1] : c->stream;
  hipStream_t sv = c->concurrent ? c->side[2] : c->stream;
  c->last_from_bytes = b->from_bytes;
  c->v_timed = false;
  c->kes_ck_timed = false;
  c->pk_on = c->keycache > 0 && (c->pool_keys > 0 || (c->pool_keys < 0 && c->replaying));
  if (b->from_bytes) {
    // stored bytes -> SoA (k_decode.hip); the crypto kernels read its output
    HIPCHK(c, hipEventRecord(c->ev[5], c->stream));
    if (!b->decoded) {
      const int rd = batch_decode(c, b);
      if (rd != PRAOS_OK) { c->err = "decode launch failed"; return rd; }
    }
  }
  if (c->keycache > 0 && n >= 2) {     // the comb is read by the cached chains: built before ev[0]
    const int rc = ensure_bcomb16(c);
    if (rc != PRAOS_OK) return rc;
  }
  // TPraos (b->tp_only): the same OCert and KES passes (dedup, key caches, side streams); the
  // VRF pass is the two-certificate k_vrf_tp (overlay classes from the host slots when
  // praos_set_overlay is on) and the leader test takes the certified L output, 2^512 bound
  int32_t* dcls = nullptr;
  if (b->tp_only && c->ovl_on) {
    // the slots come from the decode on this stream; the sync also retires the previous
    // run's upload of cls_h before it is rewritten
    b->slots_h.resize(n);
    b->cls_h.resize(n);
    HIPCHK(c, hipMemcpyAsync(b->slots_h.data(), b->slot, 8 * n, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    for (size_t i = 0; i < n; i++) b->cls_h[i] = overlay_class(c, b->slots_h[i]);
    if (!b->dcls || b->dcls_n < n) {
      const size_t cap = std::max(n, b->cap_n);
      if (dalloc(b, &b->dcls, 4 * cap) != hipSuccess) return PRAOS_E_OOM;
      b->dcls_n = cap;
    }
    dcls = b->dcls;
    HIPCHK(c, hipMemcpyAsync(dcls, b->cls_h.data(), 4 * n, hipMemcpyHostToDevice, c->stream));
  }
  HIPCHK(c, hipEventRecord(c->ev[0], c->stream));
  if (c->concurrent)
    for (int k = 0; k < 3; k++) HIPCHK(c, hipStreamWaitEvent(c->side[k], c->ev[0], 0));
  // Stage V of the VRF needs nothing but the decoded header (no key table, no list), and it is
  // the longest chain of the step: with concurrent streams it is queued first, so its waves
  // are dispatched before the key-cache passes' (queued after it, it started ~0.3 ms into a
  // 54k-header step, behind a dozen list kernels on the other streams)
  const bool do_vrf = (c->kernels & 4) != 0;
  const bool tp_staged = do_vrf && b->tp_only && c->tp_staged;
  // PRAOS_V_MAIN: the three-kernel Praos VRF with stage V and the join on the main stream (the
  // step's critical path then crosses streams once, U -> join, instead of at ev[0] -> V, V -> join
  // and join -> leader)
  const int vm_mode = c->vmain_mode(n);
  const bool v_main = vm_mode > 0 && c->concurrent && do_vrf && !b->tp_only && !b->v_done &&
                      (c->vrf3 > 0 || (c->vrf3 < 0 && n < 300000));
  const int wprio_v = c->vrf_prio > 0 || (c->vrf_prio < 0 && n < SMALL_BATCH);
  bool v_queued = false;
  if (tp_staged) {
    const size_t cap = std::max(n, b->cap_n);
    if (!b->vrf_mid2 || b->vrf_mid2_n < n) {
      if (dalloc(b, &b->vrf_mid2, VRF_MID_BYTES * cap) != hipSuccess ||
          dalloc(b, (uint8_t**)&b->tab_vrf2, LT_VRF_B * cap) != hipSuccess)
        return PRAOS_E_OOM;
      b->vrf_mid2_n = cap;
    }
  }
  auto queue_stage_v = [&]() -> int {
    const uint32_t* eta = b->eta_tab ? b->eta_tab : c->d_eta0;
    if (tp_staged) {
      // the two certificates' stage V side by side (own lane tables, mkSeed alphas): a batch
      // below ~300k headers leaves most wave slots empty with one V at a time
      hipStream_t sVk[2] = {c->concurrent ? c->vstream : c->stream, c->concurrent ? c->vstream2 : c->stream};
      const uint8_t* proof[2] = {b->vrf_proof, b->lead_proof};
      uint8_t* mid[2] = {b->vrf_mid, b->vrf_mid2};
      ge_cached* vtab[2] = {b->tab_vrf, b->tab_vrf2};
      for (int k = 0; k < 2; k++) {
        if (sVk[k] != c->stream) HIPCHK(c, hipStreamWaitEvent(sVk[k], c->ev[0], 0));
        if (k == 0) HIPCHK(c, hipEventRecord(c->v0_ev, sVk[0]));
        launch_vrf_v(sVk[k], n, b->vrf_vk, proof[k], b->slot, eta, c->eta0_neutral, b->eta_idx, vtab[k], mid[k], 0,
                     SIZE_MAX, wprio_v, 1 + k, c->v_ilp4(n));
      }
      HIPCHK(c, hipEventRecord(c->v1_ev, sVk[0]));
      HIPCHK(c, hipEventRecord(c->v_ev, sVk[0]));
      HIPCHK(c, hipEventRecord(c->v2_ev, sVk[1]));
    } else {
      hipStream_t sV = c->concurrent && !v_main ? c->vstream : c->stream;
      if (sV != c->stream) HIPCHK(c, hipStreamWaitEvent(sV, c->ev[0], 0));
      HIPCHK(c, hipEventRecord(c->v0_ev, sV));
      launch_vrf_v(sV, n, b->vrf_vk, b->vrf_proof, b->slot, eta, c->eta0_neutral, b->eta_idx, b->tab_vrf,
                   b->vrf_mid, 0, SIZE_MAX, wprio_v, 0, c->v_ilp4(n));
      HIPCHK(c, hipEventRecord(c->v1_ev, sV));
    }
    c->v_timed = true;
    v_queued = true;
    return PRAOS_OK;
  };
  // (serial runs keep the OCert | KES | VRF order: their per-stream spans are measured in turn)
  if (c->concurrent && do_vrf && (tp_staged || (!b->tp_only && !b->v_done))) {
    const int r = queue_stage_v();
    if (r != PRAOS_OK) return r;
  }
  const bool kc = c->keycache > 0 && n >= 2;
  b->kc_used = kc;
  // key cache prepass on the kernel's own stream: hash set, entries, hit/miss lists, tables
  // (items: all n, or list[0 .. *count) when list != null)
  // Each miss list goes to its own stream as soon as its partition is known, so the
  // uncached verifies run during the latency-bound key precompute, beside each other,
  // instead of trailing the cached chains (miss_ev[t]: the partition of cache t is done).
  hipStream_t sm_[3] = {c->concurrent ? c->mside[0] : c->stream, c->concurrent ? c->mside[1] : c->stream,
                        c->concurrent ? c->mside[2] : c->stream};
  auto to_main = [&](int t, hipStream_t st) -> int {
    if (st == sm_[t]) return PRAOS_OK;
    HIPCHK(c, hipEventRecord(c->miss_ev[t], st));
    HIPCHK(c, hipStreamWaitEvent(sm_[t], c->miss_ev[t], 0));
    return PRAOS_OK;
  };
  auto keycache_lists = [&](praos_batch::KeyCache& k, const uint8_t* keys, hipStream_t st,
                            const uint32_t* list = nullptr, const uint32_t* count = nullptr) -> int {
    return kc_lists(c, k, n, keys, st, list, count, (int)(&k - b->kc));
  };
  auto keycache_precompute = [&](praos_batch::KeyCache& k, const uint8_t* keys, int kind, hipStream_t st) {
    kc_precompute(c, k, keys, kind, st, n);
  };
  // Praos VRF in three kernels (below 300k headers): the VRF key lists, the uncached U and the
  // key precompute + cached U are queued ahead of the OCert and KES passes when the streams
  // run concurrently (PRAOS_VRF_KEYS_FIRST): after stage V, the VRF key chain -- lists,
  // precompute, tables, U, join -- is a small batch's longest (profiles/r04/i: its lists
  // started 0.33 ms into a 54k-header step, behind the OCert and KES lists)
  const bool vrf3 = do_vrf && !b->tp_only && (c->vrf3 > 0 || (c->vrf3 < 0 && n < 300000));
  bool vrf_keys_queued = false;
  const bool pre_join = vrf3 && kc && (c->pre_join > 0 || (c->pre_join < 0 && n < SMALL_BATCH));
  auto vrf_keys = [&]() -> int {
    praos_batch::KeyCache& k = b->kc[1];
    int r = keycache_lists(k, b->vrf_vk, sv);
    if (r == PRAOS_OK) r = to_main(2, sv);
    if (r != PRAOS_OK) return r;
    if (pre_join)
      launch_vrf_pool(sm_[2], n, b->cold_vk, b->vrf_vk, b->vrf_out, c->d_pool_hash, c->d_pool_vrf, c->d_pool_map,
                      c->npools, bv, b->pool_idx, b->pool_sorted, b->leader, b->nonce);
    launch_vrf_u(sm_[2], n, k.miss, k.counters + 2, nullptr, nullptr, nullptr, c->bcomb16, c->btab, b->vrf_vk,
                 b->vrf_proof, b->tab_vrfu, b->vrf_mid);
    if (sm_[2] != sv) HIPCHK(c, hipEventRecord(c->u_ev, sm_[2]));
    keycache_precompute(k, b->vrf_vk, 1, sv);
    launch_vrf_u(sv, n, k.hit, k.counters + 1, k.item_entry, k.kt, k.ki, c->bcomb16, c->btab, b->vrf_vk,
                 b->vrf_proof, b->tab_vrfu, b->vrf_mid, c->use_u4(n), 0);
    // (v_main 2: the main stream waits for u_ev itself, before the join)
    if (sm_[2] != sv && !(v_main && vm_mode == 2)) HIPCHK(c, hipStreamWaitEvent(sv, c->u_ev, 0));
    vrf_keys_queued = true;
    return PRAOS_OK;
  };
  if (vrf3 && kc && c->concurrent && c->vrf_keys_first) {
    const int r = vrf_keys();
    if (r != PRAOS_OK) return r;
  }
  b->dd_used = false;
  std::function<void()> ocert_miss;
  if ((c->kernels & 1) && c->dedup && n >= 2) {
    // distinct OCert tuples only; their verdicts fan out to every header carrying them
    b->dd_used = true;
    HIPCHK(c, hipMemsetAsync(b->dd_slot, 0, 4 * (size_t)b->dd_cap, so));
    HIPCHK(c, hipMemsetAsync(b->dd_counters, 0, 16, so));
    launch_ocert_dedup(g, blk, so, n, b->cold_vk, b->hot_vk, b->ocert_n, b->ocert_c0, b->ocert_sig, b->dd_cap - 1,
                       b->dd_slot, b->dd_item_rep, b->dd_reps, b->dd_counters);
    if (kc) {
      praos_batch::KeyCache& k = b->kc[0];
      int r = keycache_lists(k, b->cold_vk, so, b->dd_reps, b->dd_counters);
      if (r == PRAOS_OK) r = to_main(0, so);
      if (r != PRAOS_OK) return r;
      ocert_miss = [&, k]() {
        if (c->use_miss4(n))
          launch_ocert4(g, blk, sm_[0], k.miss, k.counters + 2, c->btab, b->cold_vk, b->hot_vk, b->ocert_n,
                        b->ocert_c0, b->ocert_sig, b->slot, P.slots_per_kes_period, P.max_kes_evo, bo, b->dd_ok,
                        b->tab_ocert, c->miss_prio_for(n));
        else
          launch_ocert(g, blk, sm_[0], n, k.miss, k.counters + 2, c->btab, b->cold_vk, b->hot_vk, b->ocert_n,
                       b->ocert_c0, b->ocert_sig, b->slot, P.slots_per_kes_period, P.max_kes_evo, bo, b->dd_ok,
                       b->tab_ocert);
      };
      keycache_precompute(k, b->cold_vk, 0, so);
      if (c->use_ck4(n))
        launch_ocert_ck4(so, n, k.hit, k.counters + 1, k.item_entry, k.kt, k.ki, c->bcomb16, b->cold_vk, b->hot_vk,
                         b->ocert_n, b->ocert_c0, b->ocert_sig, b->slot, P.slots_per_kes_period, P.max_kes_evo, bo,
                         b->dd_ok);
      else
        launch_ocert_ck(gl, bl, so, k.hit, k.counters + 1, k.item_entry, k.kt, k.ki, c->bcomb16, b->cold_vk,
                        b->hot_vk, b->ocert_n, b->ocert_c0, b->ocert_sig, b->slot, P.slots_per_kes_period,
                        P.max_kes_evo, bo, b->dd_ok, 0);
    } else {
      launch_ocert(g, blk, so, n, b->dd_reps, b->dd_counters, c->btab, b->cold_vk, b->hot_vk, b->ocert_n,
                   b->ocert_c0, b->ocert_sig, b->slot, P.slots_per_kes_period, P.max_kes_evo, bo, b->dd_ok,
                   b->tab_ocert);
    }
    // the fanout reads dd_ok of the misses (main stream) and of the hits (this stream)
    auto fan = ocert_miss;
    ocert_miss = [&, fan, kc]() {
      if (fan) fan();
      if (kc && so != sm_[0]) {
        (void)hipEventRecord(c->miss_ev[3], sm_[0]);
        (void)hipStreamWaitEvent(so, c->miss_ev[3], 0);
      }
      launch_ocert_fanout(g, blk, so, n, b->dd_item_rep, b->dd_ok, b->slot, b->ocert_c0, P.slots_per_kes_period,
                          P.max_kes_evo, bo);
    };
  } else if (c->kernels & 1) {
    if (kc) {
      praos_batch::KeyCache& k = b->kc[0];
      int r = keycache_lists(k, b->cold_vk, so);
      if (r == PRAOS_OK) r = to_main(0, so);
      if (r != PRAOS_OK) return r;
      ocert_miss = [&, k]() {
        if (c->use_miss4(n))
          launch_ocert4(g, blk, sm_[0], k.miss, k.counters + 2, c->btab, b->cold_vk, b->hot_vk, b->ocert_n,
                        b->ocert_c0, b->ocert_sig, b->slot, P.slots_per_kes_period, P.max_kes_evo, bo,
                        (uint8_t*)nullptr, b->tab_ocert, c->miss_prio_for(n));
        else
          launch_ocert(g, blk, sm_[0], n, k.miss, k.counters + 2, c->btab, b->cold_vk, b->hot_vk, b->ocert_n,
                       b->ocert_c0, b->ocert_sig, b->slot, P.slots_per_kes_period, P.max_kes_evo, bo,
                       (uint8_t*)nullptr, b->tab_ocert);
      };
      keycache_precompute(k, b->cold_vk, 0, so);
      if (c->use_ck4(n))
        launch_ocert_ck4(so, n, k.hit, k.counters + 1, k.item_entry, k.kt, k.ki, c->bcomb16, b->cold_vk, b->hot_vk,
                         b->ocert_n, b->ocert_c0, b->ocert_sig, b->slot, P.slots_per_kes_period, P.max_kes_evo, bo,
                         (uint8_t*)nullptr);
      else
        launch_ocert_ck(gl, bl, so, k.hit, k.counters + 1, k.item_entry, k.kt, k.ki, c->bcomb16, b->cold_vk,
                        b->hot_vk, b->ocert_n, b->ocert_c0, b->ocert_sig, b->slot, P.slots_per_kes_period,
                        P.max_kes_evo, bo, (uint8_t*)nullptr, 0);
    } else {
      launch_ocert(g, blk, so, n, (const uint32_t*)nullptr, (const uint32_t*)nullptr, c->btab, b->cold_vk,
                   b->hot_vk, b->ocert_n, b->ocert_c0, b->ocert_sig, b->slot, P.slots_per_kes_period, P.max_kes_evo,
                   bo, (uint8_t*)nullptr, b->tab_ocert);
    }
  } else {
    HIPCHK(c, hipMemsetAsync(bo, 0, 2 * n, so));
  }
  if (ocert_miss) ocert_miss();
  HIPCHK(c, hipEventRecord(c->side_ev[0], so));
  if (c->kernels & 2) {
    if (kc) {
      // leaf-key cache: the Ed25519 key a Sum6KES signature ends on repeats for every
      // header a pool signs in one KES period
      praos_batch::KeyCache& k = b->kc[2];
      launch_kes_leafkeys(g, blk, sk, n, b->kes_sig, b->slot, b->ocert_c0, P.slots_per_kes_period, b->kes_leaf);
      int r = keycache_lists(k, b->kes_leaf, sk);
      if (r == PRAOS_OK) r = to_main(1, sk);
      if (r != PRAOS_OK) return r;
      if (c->use_miss4(n))
        launch_kes4(g, blk, sm_[1], k.miss, k.counters + 2, c->btab, b->hot_vk, b->kes_sig, b->body_off, b->body_len,
                    b->body, b->body_bytes_len, b->slot, b->ocert_c0, P.slots_per_kes_period, bk, b->tab_kes,
                    c->miss_prio_for(n));
      else
        launch_kes(g, blk, sm_[1], n, k.miss, k.counters + 2, c->btab, b->hot_vk, b->kes_sig, b->body_off,
                   b->body_len, b->body, b->body_bytes_len, b->slot, b->ocert_c0, P.slots_per_kes_period,
                   (const uint32_t*)nullptr, bk, (uint8_t*)nullptr, b->tab_kes);
      // Merkle path dedup: a pool's headers of one KES period carry the same hot key, period and
      // six vk pairs, so each cache entry's representative walks once and equal paths reuse it
      if (c->kes_dedup)
        launch_kes_merkle_reps(sk, k.counters, k.max_entries, k.entry_rep, b->hot_vk, b->kes_sig, b->slot,
                               b->ocert_c0, P.slots_per_kes_period, k.rep_ok);
      keycache_precompute(k, b->kes_leaf, 0, sk);
      HIPCHK(c, hipEventRecord(c->kc0_ev, sk));
      if (c->use_ck4(n) && !c->kes_pair_min() && !c->kes_dedup)
        launch_kes_ck4(sk, n, k.hit, k.counters + 1, k.item_entry, k.kt, k.ki, c->bcomb16, b->hot_vk, b->kes_sig,
                       b->body_off, b->body_len, b->body, b->body_bytes_len, b->slot, b->ocert_c0,
                       P.slots_per_kes_period, bk);
      else
        launch_kes_ck(gl, bl, sk, k.hit, k.counters + 1, k.item_entry, k.kt, k.ki, c->bcomb16, b->hot_vk, b->kes_sig,
                      b->body_off, b->body_len, b->body, b->body_bytes_len, b->slot, b->ocert_c0,
                      P.slots_per_kes_period, bk, c->kes_pair_min(), c->kes_dedup ? k.entry_rep : nullptr,
                      c->kes_dedup ? k.rep_ok : nullptr, 0);
      HIPCHK(c, hipEventRecord(c->kc1_ev, sk));
      c->kes_ck_timed = true;
    } else {
      launch_kes(g, blk, sk, n, (const uint32_t*)nullptr, (const uint32_t*)nullptr, c->btab, b->hot_vk, b->kes_sig,
                 b->body_off, b->body_len, b->body, b->body_bytes_len, b->slot, b->ocert_c0, P.slots_per_kes_period,
                 (const uint32_t*)nullptr, bk, (uint8_t*)nullptr, b->tab_kes);
    }
  } else
    HIPCHK(c, hipMemsetAsync(bk, 0, 2 * n, sk));
  HIPCHK(c, hipEventRecord(c->side_ev[1], sk));
  if (tp_staged) {
    // TPraos, staged: stage V of both certificates (mkSeed alphas) on the V streams from ev[0]
    // on (queue_stage_v), U of both against the VRF key cache (misses on the miss stream at
    // once, hits after the key tables), then the two joins in order on the VRF stream
    if (!v_queued) {
      const int r = queue_stage_v();
      if (r != PRAOS_OK) return r;
    }
    const uint8_t* proof[2] = {b->vrf_proof, b->lead_proof};
    const uint8_t* outv[2] = {b->vrf_out, b->lead_out};
    uint8_t* mid[2] = {b->vrf_mid, b->vrf_mid2};
    uint8_t* beta[2] = {b->beta, b->beta_l};
    hipStream_t sVk[2] = {c->concurrent ? c->vstream : c->stream, c->concurrent ? c->vstream2 : c->stream};
    if (kc) {
      praos_batch::KeyCache& k = b->kc[1];
      int r = keycache_lists(k, b->vrf_vk, sv);
      if (r == PRAOS_OK) r = to_main(2, sv);
      if (r != PRAOS_OK) return r;
      for (int q = 0; q < 2; q++)
        launch_vrf_u(sm_[2], n, k.miss, k.counters + 2, nullptr, nullptr, nullptr, c->bcomb16, c->btab, b->vrf_vk,
                     proof[q], b->tab_vrfu, mid[q]);
      if (sm_[2] != sv) HIPCHK(c, hipEventRecord(c->u_ev, sm_[2]));
      keycache_precompute(k, b->vrf_vk, 1, sv);
      for (int q = 0; q < 2; q++)
        launch_vrf_u(sv, n, k.hit, k.counters + 1, k.item_entry, k.kt, k.ki, c->bcomb16, c->btab, b->vrf_vk,
                     proof[q], b->tab_vrfu, mid[q], c->use_u4(n));
      if (sm_[2] != sv) HIPCHK(c, hipStreamWaitEvent(sv, c->u_ev, 0));
    } else {
      for (int q = 0; q < 2; q++)
        launch_vrf_u(sv, n, nullptr, nullptr, nullptr, nullptr, nullptr, c->bcomb16, c->btab, b->vrf_vk, proof[q],
                     b->tab_vrfu, mid[q]);
    }
    if (sv != sVk[0]) HIPCHK(c, hipStreamWaitEvent(sv, c->v_ev, 0));
    if (sv != sVk[1]) HIPCHK(c, hipStreamWaitEvent(sv, c->v2_ev, 0));
    for (int q = 0; q < 2; q++)
      launch_vrf_join_tp(sv, n, q, b->cold_vk, b->vrf_vk, outv[q], proof[q], c->d_pool_hash, c->d_pool_vrf,
                         c->d_pool_map, c->npools, (int)P.vrf_check_output, bv, b->pool_idx, b->pool_sorted, beta[q],
                         b->nonce, mid[q], dcls, c->d_gen);
  } else if (do_vrf && b->tp_only) {
    launch_vrf_tp(g, blk, sv, n, c->btab, b->cold_vk, b->vrf_vk, b->vrf_out, b->vrf_proof, b->lead_out, b->lead_proof,
                  b->slot, b->eta_tab ? b->eta_tab : c->d_eta0, c->eta0_neutral, c->d_pool_hash, c->d_pool_vrf,
                  c->d_pool_map, c->npools, (int)P.vrf_check_output, bv, b->pool_idx, b->pool_sorted, b->beta, b->beta_l,
                  b->nonce, b->tab_vrf, dcls, c->d_gen, b->eta_idx);
  } else if (do_vrf) {
    // two stages (k_vrf_stage.hip): V over every header on its own stream, from ev[0] on (it
    // needs no key); F after it -- the hits on sv once their key tables exist, the misses
    // on their miss stream (per-lane U)
    const uint32_t* eta = b->eta_tab ? b->eta_tab : c->d_eta0;
    // (stored-bytes pipeline: stage V was queued chunk by chunk on vstream while the later
    // chunks were still uploading; b->v_done)
    hipStream_t sV = v_main ? c->stream : (c->concurrent || b->v_done) ? c->vstream : c->stream;
    const int wprio = wprio_v;
    if (!b->v_done && !v_queued) {
      const int r = queue_stage_v();
      if (r != PRAOS_OK) return r;
    }
    HIPCHK(c, hipEventRecord(c->v_ev, sV));
    if (b->v_done) HIPCHK(c, hipEventRecord(c->v2_ev, c->vstream2));
    auto after_v = [&](hipStream_t st) -> int {
      if (st != sV) HIPCHK(c, hipStreamWaitEvent(st, c->v_ev, 0));
      if (b->v_done) HIPCHK(c, hipStreamWaitEvent(st, c->v2_ev, 0));
      return PRAOS_OK;
    };
    auto fin = [&](hipStream_t st, const uint32_t* list, const uint32_t* count, const praos_batch::KeyCache* k) {
      launch_vrf_fin(st, n, list, count, k ? k->item_entry : nullptr, k ? k->kt : nullptr, k ? k->ki : nullptr,
                     c->bcomb16, c->btab, b->cold_vk, b->vrf_vk, b->vrf_out, b->vrf_proof, c->d_pool_hash,
                     c->d_pool_vrf, c->d_pool_map, c->npools, (int)P.vrf_check_output, bv, b->pool_idx,
                     b->pool_sorted, b->beta, b->leader, b->nonce, b->tab_vrf, b->vrf_mid);
    };
    auto stage_u = [&](hipStream_t st, const uint32_t* list, const uint32_t* count, const praos_batch::KeyCache* k) {
      launch_vrf_u(st, n, list, count, k ? k->item_entry : nullptr, k ? k->kt : nullptr, k ? k->ki : nullptr,
                   c->bcomb16, c->btab, b->vrf_vk, b->vrf_proof, b->tab_vrfu, b->vrf_mid);
    };
    auto join = [&](hipStream_t st) {
      launch_vrf_join(st, n, b->cold_vk, b->vrf_vk, b->vrf_out, b->vrf_proof, c->d_pool_hash, c->d_pool_vrf,
                      c->d_pool_map, c->npools, (int)P.vrf_check_output, bv, b->pool_idx, b->pool_sorted, b->beta,
                      b->leader, b->nonce, b->vrf_mid, wprio, pre_join ? 1 : 0);
    };
    if (vrf3) {
      // three kernels: U runs beside V (uncached keys at once on the miss stream, cached keys
      // once their tables exist), the join after both
      int r;
      if (kc) {
        if (!vrf_keys_queued && (r = vrf_keys()) != PRAOS_OK) return r;
      } else {
        stage_u(sv, nullptr, nullptr, nullptr);
      }
      if (v_main && vm_mode == 3) {  // V on the main stream, the join on the VRF stream after U
        HIPCHK(c, hipEventRecord(c->v_ev, c->stream));
        HIPCHK(c, hipStreamWaitEvent(sv, c->v_ev, 0));
        join(sv);
      } else if (v_main) {             // V is on the main stream: the join follows it there, after U
        if (vm_mode == 2 && kc) HIPCHK(c, hipStreamWaitEvent(c->stream, c->u_ev, 0));
        HIPCHK(c, hipEventRecord(c->side_ev[2], sv));
        HIPCHK(c, hipStreamWaitEvent(c->stream, c->side_ev[2], 0));
        join(c->stream);
      } else {
        if ((r = after_v(sv)) != PRAOS_OK) return r;
        join(sv);
      }
    } else if (kc) {
      praos_batch::KeyCache& k = b->kc[1];
      int r = keycache_lists(k, b->vrf_vk, sv);
      if (r == PRAOS_OK) r = to_main(2, sv);
      if (r == PRAOS_OK) r = after_v(sm_[2]);
      if (r != PRAOS_OK) return r;
      fin(sm_[2], k.miss, k.counters + 2, nullptr);
      keycache_precompute(k, b->vrf_vk, 1, sv);
      if ((r = after_v(sv)) != PRAOS_OK) return r;
      fin(sv, k.hit, k.counters + 1, &k);
    } else {
      const int r = after_v(sv);
      if (r != PRAOS_OK) return r;
      fin(sv, nullptr, nullptr, nullptr);
    }
  }
  else {
    HIPCHK(c, hipMemsetAsync(bv, 0, 2 * n, sv));
    HIPCHK(c, hipMemsetAsync(b->pool_sorted, 0xff, 4 * n, sv));   // no pool -> leader kernel skips
  }
  HIPCHK(c, hipEventRecord(c->side_ev[2], sv));
  if (c->concurrent) {
    // (v_main: the VRF stream and its miss stream -- u_ev -- were waited for before the join)
    const bool sv_done = v_main && vm_mode != 3;
    for (int k = 0; k < 3; k++)
      if (!(sv_done && k == 2)) HIPCHK(c, hipStreamWaitEvent(c->stream, c->side_ev[k], 0));
    for (int k = 0; k < 3; k++) {
      if (sv_done && k == 2) continue;
      HIPCHK(c, hipEventRecord(c->mdone_ev[k], c->mside[k]));
      HIPCHK(c, hipStreamWaitEvent(c->stream, c->mdone_ev[k], 0));
    }
  }
  launch_leader(g, blk, c->stream, n, b->tp_only ? b->lead_out : b->leader, b->pool_sorted, c->d_pool_x,
                (const uint32_t*)nullptr, (int)P.f_is_one, b->tp_only ? 16 : 8, bo, bk, bv, b->bits, (uint8_t*)nullptr,
                (int32_t*)nullptr, b->from_bytes ? b->dec_status : (const uint16_t*)nullptr);
  HIPCHK(c, hipEventRecord(c->ev[4], c->stream));
  HIPCHK(c, hipGetLastError());
  return PRAOS_OK;
}

// ---- block-integrity batch (k_block.hip + k_decode + k_kes header mode)
praos_batch* praos_block_batch_upload(praos_ctx* c, const praos_header_bytes* blocks) {
  praos_batch* b = praos_batch_upload_bytes(c, blocks);
  if (!b) return nullptr;
  const size_t n = b->n;
  b->is_block = true;
  bool ok = dalloc(b, &b->blk_off, 8 * n) == hipSuccess;
  ok &= dalloc(b, &b->blk_len, 4 * n) == hipSuccess;
  ok &= dalloc(b, &b->seg_off, 8 * 4 * n) == hipSuccess;
  ok &= dalloc(b, &b->seg_len, 4 * 4 * n) == hipSuccess;
  ok &= dalloc(b, &b->nseg, n) == hipSuccess;
  ok &= dalloc(b, &b->split_status, n) == hipSuccess;
  ok &= dalloc(b, &b->seg_hash, 32 * 4 * n) == hipSuccess;
  ok &= dalloc(b, &b->blk_result, n) == hipSuccess;
  ok &= dalloc(b, &b->blk_hash, 32 * n) == hipSuccess;
  // TPraos BHBody signed bodies are up to 598 bytes: a wider stride than header batches
  b->signed_stride = TP_SIGNED_STRIDE;
  b->body_bytes_len = (size_t)TP_SIGNED_STRIDE * n;
  ok &= dalloc(b, &b->body, b->body_bytes_len + 16) == hipSuccess;
  if (!ok) { c->err = "device allocation failed"; praos_batch_free(c, b); return nullptr; }
  // the uploaded spans are whole blocks; k_block_split rewrites hoff/hlen to the header spans
  if (n) {
    ok &= hipMemcpyAsync(b->blk_off, b->hoff, 8 * n, hipMemcpyDeviceToDevice, c->stream) == hipSuccess;
    ok &= hipMemcpyAsync(b->blk_len, b->hlen, 4 * n, hipMemcpyDeviceToDevice, c->stream) == hipSuccess;
  }
  ok &= hipStreamSynchronize(c->stream) == hipSuccess;
  if (!ok) { c->err = "upload failed"; praos_batch_free(c, b); return nullptr; }
  return b;
}

int praos_block_batch_run(praos_ctx* c, praos_batch* b, uint64_t slots_per_kes_period) {
  if (!c || !b || !b->is_block || slots_per_kes_period == 0) return PRAOS_E_ARG;
  HIPCHK(c, hipSetDevice(c->device));
  const size_t n = b->n;
  if (n == 0) return PRAOS_OK;
  const dim3 g(nblocks(n, NT)), blk(NT);
  uint16_t* bk = b->bits3 + n;
  HIPCHK(c, hipEventRecord(c->ev[0], c->stream));
  HIPCHK(c, hipMemcpyAsync(b->hoff, b->blk_off, 8 * n, hipMemcpyDeviceToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(b->hlen, b->blk_len, 4 * n, hipMemcpyDeviceToDevice, c->stream));
  (void)hipGetLastError();   // clear a stale error of an earlier, already-reported runtime call
  launch_block_split(g, blk, c->stream, n, b->arena, b->arena_len, b->hoff, b->hlen, b->seg_off, b->seg_len, b->nseg,
                     b->split_status);
  HIPCHK(c, hipGetLastError());
  const int rd = batch_decode(c, b);
  if (rd != PRAOS_OK) { c->err = "decode launch failed"; return rd; }
  HIPCHK(c, hipEventRecord(c->ev[1], c->stream));
  // segment hashes on a side stream, concurrent with the KES verify
  HIPCHK(c, hipStreamWaitEvent(c->side[0], c->ev[1], 0));
  launch_seg_hash(dim3(nblocks(4 * n, NT)), blk, c->side[0], n, b->arena, b->seg_off, b->seg_len, b->nseg,
                  b->seg_hash);
  HIPCHK(c, hipEventRecord(c->side_ev[0], c->side[0]));
  launch_kes(g, blk, c->stream, n, (const uint32_t*)nullptr, (const uint32_t*)nullptr, c->btab, b->hot_vk, b->kes_sig, b->body_off, b->body_len, b->body,
             b->body_bytes_len, b->slot, b->ocert_c0, slots_per_kes_period, (const uint32_t*)nullptr, bk,
             (uint8_t*)nullptr, b->tab_kes);
  HIPCHK(c, hipEventRecord(c->ev[2], c->stream));
  HIPCHK(c, hipStreamWaitEvent(c->stream, c->side_ev[0], 0));
  launch_block_join(g, blk, c->stream, n, b->nseg, b->split_status, b->dec_status, bk, b->seg_hash, b->body_hash,
                    b->blk_result, b->blk_hash);
  HIPCHK(c, hipEventRecord(c->ev[4], c->stream));
  HIPCHK(c, hipGetLastError());
  return PRAOS_OK;
}

int praos_block_batch_download(praos_ctx* c, praos_batch* b, uint8_t* result, uint8_t* body_hash) {
  if (!c || !b || !b->is_block || (b->n && !result)) return PRAOS_E_ARG;
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  if (b->n == 0) return PRAOS_OK;
  HIPCHK(c, hipMemcpy(result, b->blk_result, b->n, hipMemcpyDeviceToHost));
  if (body_hash) HIPCHK(c, hipMemcpy(body_hash, b->blk_hash, 32 * b->n, hipMemcpyDeviceToHost));
  return PRAOS_OK;
}

int praos_verify_block_integrity(praos_ctx* c, const praos_header_bytes* blocks, uint64_t slots_per_kes_period,
                                 uint8_t* result, uint8_t* body_hash) {
  if (!c || !blocks || (blocks->n && !result) || slots_per_kes_period == 0) return PRAOS_E_ARG;
  if (c->device < 0) { c->err = "host-only context: no HIP device"; return PRAOS_E_STATE; }
  if (blocks->n == 0) return PRAOS_OK;
  praos_batch* b = praos_block_batch_upload(c, blocks);
  if (!b) return PRAOS_E_OOM;
  int r = praos_block_batch_run(c, b, slots_per_kes_period);
  if (r == PRAOS_OK) r = praos_block_batch_download(c, b, result, body_hash);
  praos_batch_free(c, b);
  return r;
}

int praos_batch_stats(praos_ctx* c, praos_batch* b, uint32_t out[9]) {
  if (!c || !b || !out) return PRAOS_E_ARG;
  for (int k = 0; k < 9; k++) out[k] = 0;
  if (!b->kc_used) return PRAOS_OK;
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  for (int t = 0; t < 3; t++) {
    uint32_t cnt[4] = {0, 0, 0, 0};
    HIPCHK(c, hipMemcpy(cnt, b->kc[t].counters, 16, hipMemcpyDeviceToHost));
    out[3 * t] = std::min(cnt[0], b->kc[t].emax ? b->kc[t].emax : b->kc[t].max_entries);
    out[3 * t + 1] = cnt[1];
    out[3 * t + 2] = cnt[2];
  }
  return PRAOS_OK;
}

int praos_batch_dedup_stats(praos_ctx* c, praos_batch* b, uint32_t out[2]) {
  if (!c || !b || !out) return PRAOS_E_ARG;
  out[0] = 0;
  out[1] = (uint32_t)b->n;
  if (!b->dd_used) return PRAOS_OK;
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  HIPCHK(c, hipMemcpy(out, b->dd_counters, 4, hipMemcpyDeviceToHost));
  return PRAOS_OK;
}

int praos_set_option(praos_ctx* c, int opt, int value) {
  if (!c) return PRAOS_E_ARG;
  if (opt == PRAOS_OPT_CONCURRENT) { c->concurrent = value != 0; return PRAOS_OK; }
  if (opt == PRAOS_OPT_KERNELS) { c->kernels = value & 7; return PRAOS_OK; }
  if (opt == PRAOS_OPT_KEYCACHE) { c->keycache = value < 0 ? 0 : value; return PRAOS_OK; }
  if (opt == PRAOS_OPT_DEDUP) { c->dedup = value != 0; return PRAOS_OK; }
  if (opt == PRAOS_OPT_PIPELINE) { c->pipeline = value < 0 ? 0 : std::min(value, PIPE_MAX); return PRAOS_OK; }
  if (opt == PRAOS_OPT_KES_PAIR) { c->kes_pair = value < 0 ? -1 : value; return PRAOS_OK; }
  if (opt == PRAOS_OPT_KES_NOCACHE) { c->kes_nocache = value < 0 ? KES_NOCACHE_BATCH : (size_t)value; return PRAOS_OK; }
  if (opt == PRAOS_OPT_POOL_KEYS) {
    c->pool_keys = value < 0 ? -1 : (value != 0);
    if (value == 2) c->pk_reset[0] = c->pk_reset[1] = true;
    return PRAOS_OK;
  }
  return PRAOS_E_ARG;
}

int praos_batch_sync(praos_ctx* c) {
  if (!c) return PRAOS_E_ARG;
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  // per-kernel: from the common start event to each kernel's end event (with
  // concurrent streams these overlap; which = 4 is the whole run)
  float t[3] = {0, 0, 0};
  for (int k = 0; k < 3; k++) (void)hipEventElapsedTime(&t[k], c->ev[0], c->side_ev[k]);
  if (c->concurrent) {
    for (int k = 0; k < 3; k++) c->kernel_ms[k] = t[k];
  } else {
    c->kernel_ms[0] = t[0];
    c->kernel_ms[1] = t[1] - t[0];
    c->kernel_ms[2] = t[2] - t[1];
  }
  float all = 0, dec = 0;
  (void)hipEventElapsedTime(&all, c->ev[0], c->ev[4]);
  if (c->last_from_bytes) (void)hipEventElapsedTime(&dec, c->ev[5], c->ev[0]);
  c->kernel_ms[3] = all - (c->concurrent ? std::max(t[0], std::max(t[1], t[2])) : t[2]);
  c->kernel_ms[4] = all + dec;
  c->kernel_ms[5] = dec;
  c->kernel_ms[6] = 0;
  if (c->v_timed) (void)hipEventElapsedTime(&c->kernel_ms[6], c->v0_ev, c->v1_ev);
  c->kernel_ms[7] = 0;
  if (c->kes_ck_timed) (void)hipEventElapsedTime(&c->kernel_ms[7], c->kc0_ev, c->kc1_ev);
  return PRAOS_OK;
}

float praos_batch_kernel_ms(praos_ctx* c, int which) {
  if (!c || which < 0 || which > 7) return -1.f;
  return c->kernel_ms[which];
}

int praos_batch_download(praos_ctx* c, praos_batch* b, praos_out* out) {
  if (!c || !b || !out || !out->bits) return PRAOS_E_ARG;
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  const size_t n = b->n;
  if (n == 0) return PRAOS_OK;
  HIPCHK(c, d2h(c, out->bits, b->bits, 2 * n));
  if (out->pool_idx) HIPCHK(c, d2h(c, out->pool_idx, b->pool_idx, 4 * n));
  if (out->beta) HIPCHK(c, d2h(c, out->beta, b->beta, 64 * n));
  if (out->leader) HIPCHK(c, d2h(c, out->leader, b->leader, 32 * n));
  if (out->nonce) HIPCHK(c, d2h(c, out->nonce, b->nonce, 32 * n));
  return PRAOS_OK;
}

int praos_verify_headers(praos_ctx* c, const praos_headers* h, praos_out* out) {
  if (!c || !h || !out || !out->bits) return PRAOS_E_ARG;
  if (!c->have_epoch) return PRAOS_E_STATE;
  if (h->n == 0) return PRAOS_OK;
  praos_batch* b = praos_batch_upload(c, h);
  if (!b) return PRAOS_E_OOM;
  int r = praos_batch_run(c, b);
  if (r == PRAOS_OK) r = praos_batch_sync(c);
  if (r == PRAOS_OK) r = praos_batch_download(c, b, out);
  praos_batch_free(c, b);
  return r;
}

int praos_batch_decode(praos_ctx* c, praos_batch* b) {
  if (!c || !b || !b->from_bytes) return PRAOS_E_ARG;
  HIPCHK(c, hipSetDevice(c->device));
  const int r = batch_decode(c, b);
  if (r != PRAOS_OK) { c->err = "decode launch failed"; return r; }
  b->decoded = true;
  return PRAOS_OK;
}

int praos_batch_set_nonces(praos_ctx* c, praos_batch* b, const praos_nonce* etas, uint32_t k, const uint8_t* eta_idx) {
  if (!c || !b || (b->n && (!etas || !eta_idx)) || k == 0 || k > 256) return PRAOS_E_ARG;
  for (size_t i = 0; i < b->n; i++)
    if (eta_idx[i] >= k) { c->err = "eta_idx out of range"; return PRAOS_E_ARG; }
  HIPCHK(c, hipSetDevice(c->device));
  std::vector<uint32_t> tab(9 * (size_t)k, 0);
  for (uint32_t e = 0; e < k; e++) {
    if (!etas[e].neutral) std::memcpy(&tab[9 * e], etas[e].hash, 32);
    tab[9 * e + 8] = etas[e].neutral ? 1u : 0u;
  }
  if (!b->eta_tab) {
    if (dalloc(b, &b->eta_tab, 9 * 4 * 256) != hipSuccess || dalloc(b, &b->eta_idx, std::max<size_t>(b->n, 1)) != hipSuccess) {
      c->err = "device allocation failed";
      return PRAOS_E_OOM;
    }
  }
  HIPCHK(c, hipMemcpyAsync(b->eta_tab, tab.data(), 4 * tab.size(), hipMemcpyHostToDevice, c->stream));
  if (b->n) HIPCHK(c, hipMemcpyAsync(b->eta_idx, eta_idx, b->n, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return PRAOS_OK;
}

int praos_batch_download_decoded(praos_ctx* c, praos_batch* b, praos_decoded* d) {
  if (!c || !b || !d || !b->from_bytes) return PRAOS_E_ARG;
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  const size_t n = b->n;
  if (n == 0) return PRAOS_OK;
  auto dn = [&](void* dst, const void* src, size_t bytes) -> hipError_t {
    return dst ? d2h(c, dst, src, bytes) : hipSuccess;
  };
  HIPCHK(c, dn(d->status, b->dec_status, 2 * n));
  HIPCHK(c, dn(d->block_no, b->block_no, 8 * n));
  HIPCHK(c, dn(d->slot, b->slot, 8 * n));
  HIPCHK(c, dn(d->prev_hash, b->prev_hash, 32 * n));
  HIPCHK(c, dn(d->prev_is_genesis, b->prev_genesis, n));
  HIPCHK(c, dn(d->cold_vk, b->cold_vk, 32 * n));
  HIPCHK(c, dn(d->vrf_vk, b->vrf_vk, 32 * n));
  HIPCHK(c, dn(d->vrf_out, b->vrf_out, 64 * n));
  HIPCHK(c, dn(d->vrf_proof, b->vrf_proof, 80 * n));
  HIPCHK(c, dn(d->body_size, b->body_size, 4 * n));
  HIPCHK(c, dn(d->body_hash, b->body_hash, 32 * n));
  HIPCHK(c, dn(d->hot_vk, b->hot_vk, 32 * n));
  HIPCHK(c, dn(d->ocert_n, b->ocert_n, 8 * n));
  HIPCHK(c, dn(d->ocert_c0, b->ocert_c0, 8 * n));
  HIPCHK(c, dn(d->ocert_sig, b->ocert_sig, 64 * n));
  HIPCHK(c, dn(d->prot_major, b->prot_major, 8 * n));
  HIPCHK(c, dn(d->prot_minor, b->prot_minor, 8 * n));
  HIPCHK(c, dn(d->kes_sig, b->kes_sig, 448 * n));
  HIPCHK(c, dn(d->signed_len, b->body_len, 4 * n));
  HIPCHK(c, dn(d->signed_body, b->body, (size_t)b->signed_stride * n));
  HIPCHK(c, dn(d->header_hash, b->header_hash, 32 * n));
  return PRAOS_OK;
}

int praos_decode_headers(praos_ctx* c, const praos_header_bytes* in, praos_decoded* out) {
  if (!c || !in || !out) return PRAOS_E_ARG;
  if (c->device < 0) { c->err = "host-only context: no HIP device"; return PRAOS_E_STATE; }
  if (in->n == 0) return PRAOS_OK;
  praos_batch* b = praos_batch_upload_bytes(c, in);
  if (!b) return PRAOS_E_OOM;
  int r = batch_decode(c, b);
  if (r == PRAOS_OK) r = praos_batch_download_decoded(c, b, out);
  praos_batch_free(c, b);
  return r;
}

}  // extern "C"

// ---------------------------------------------------------------- replay pipeline (internal, C++ linkage)
// A batch the context keeps between calls (the replay's RP_SLOTS batches, the stored-bytes
// pipeline's batch) goes through here every time it is taken for another run: every per-run field
// back to the state of a fresh batch, so nothing one call set (its header count, "decoded",
// "stage V queued", the key-cache / dedup use of its last run, the nonce table's use) can reach
// the next call, whichever entry point made either.  Buffers, capacities and events stay.
static void batch_reuse_reset(praos_batch* b) {
  b->n = 0;
  b->arena_len = 0;
  b->body_bytes_len = 0;
  b->decoded = false;
  b->v_done = false;
  b->kc_used = false;
  b->dd_used = false;
  for (auto& k : b->kc) {            // this run's entry space (set again by the run's key lists)
    k.kt = nullptr; k.ki = nullptr; k.erep = nullptr; k.epos = nullptr; k.ebase = nullptr;
    k.emax = 0; k.store = -1;
  }
}

praos_batch* rp_batch_alloc(praos_ctx* c, size_t n_cap, size_t bytes_cap, bool tpraos) {
  if (!c || c->device < 0) return nullptr;
  (void)hipSetDevice(c->device);
  praos_batch* b = bytes_batch_alloc(c, std::max<size_t>(n_cap, 1), std::max<size_t>(bytes_cap, 8), tpraos, nullptr);
  if (!b) return nullptr;
  b->cap_n = std::max<size_t>(n_cap, 1);
  b->cap_bytes = std::max<size_t>(bytes_cap, 8);
  bool ok = dalloc(b, &b->eta_tab, 9 * 4 * 256) == hipSuccess && dalloc(b, &b->eta_idx, b->cap_n) == hipSuccess;
  ok = ok && hipEventCreateWithFlags(&b->dec_ev, hipEventDisableTiming) == hipSuccess;
  ok = ok && hipEventCreateWithFlags(&b->run_ev, hipEventDisableTiming) == hipSuccess;
  ok = ok && hipEventRecord(b->run_ev, c->stream) == hipSuccess;     // recorded once: waits on it are defined
  ok = ok && hipHostMalloc((void**)&b->eta_h, 9 * 4 * 256, hipHostMallocDefault) == hipSuccess;
  ok = ok && hipHostMalloc((void**)&b->eidx_h, b->cap_n, hipHostMallocDefault) == hipSuccess;
  ok = ok && hipHostMalloc((void**)&b->res_bits_h, 2 * b->cap_n, hipHostMallocDefault) == hipSuccess;
  ok = ok && hipHostMalloc((void**)&b->res_pidx_h, 4 * b->cap_n, hipHostMallocDefault) == hipSuccess;
  ok = ok && hipHostMalloc((void**)&b->dec_h, DEC_H_BYTES * b->cap_n, hipHostMallocDefault) == hipSuccess;
  if (!ok) { rp_batch_destroy(c, b); return nullptr; }
  return b;
}

// the batch's pinned result buffers (kept with it between calls: no page-locking per call)
void rp_batch_results(praos_batch* b, uint16_t** bits, int32_t** pidx) {
  *bits = b->res_bits_h;
  *pidx = b->res_pidx_h;
}

void rp_batch_destroy(praos_ctx* c, praos_batch* b) {
  if (!b) return;
  if (c) (void)hipSetDevice(c->device);
  if (b->dec_ev) (void)hipEventSynchronize(b->dec_ev);
  if (b->run_ev) (void)hipEventSynchronize(b->run_ev);
  if (b->dec_ev) (void)hipEventDestroy(b->dec_ev);
  if (b->run_ev) (void)hipEventDestroy(b->run_ev);
  if (b->eta_h) (void)hipHostFree(b->eta_h);
  if (b->eidx_h) (void)hipHostFree(b->eidx_h);
  if (b->res_bits_h) (void)hipHostFree(b->res_bits_h);
  if (b->res_pidx_h) (void)hipHostFree(b->res_pidx_h);
  if (b->dec_h) (void)hipHostFree(b->dec_h);
  for (void* p : b->owned) (void)hipFree(p);
  delete b;
}

bool rp_batch_fits(const praos_batch* b, size_t n, size_t bytes) { return b && n <= b->cap_n && bytes <= b->cap_bytes; }

praos_batch* rp_batch_take(praos_ctx* c, int k, size_t n, size_t bytes, bool tpraos) {
  if (!c || k < 0 || k >= RP_SLOTS) return nullptr;
  praos_batch* b = c->rp_keep[k];
  c->rp_keep[k] = nullptr;
  if (b && rp_batch_fits(b, n, bytes) && b->tp_only == tpraos) {
    batch_reuse_reset(b);
    return b;
  }
  rp_batch_destroy(c, b);
  return rp_batch_alloc(c, n + n / 8 + 64, bytes + bytes / 8 + 4096, tpraos);
}

void rp_batch_quiesce(praos_batch* b) {
  if (!b) return;
  if (b->dec_ev) (void)hipEventSynchronize(b->dec_ev);
  if (b->run_ev) (void)hipEventSynchronize(b->run_ev);
}

void rp_batch_keep(praos_ctx* c, int k, praos_batch* b) {
  if (!c || k < 0 || k >= RP_SLOTS) { rp_batch_destroy(c, b); return; }
  if (c->rp_keep[k] && c->rp_keep[k] != b) rp_batch_destroy(c, c->rp_keep[k]);
  c->rp_keep[k] = b;
}

// H2D of the concatenation of spans through the two pinned staging buffers: the pool's
// threads gather each 16 MB piece (many small spans or a few large ones) while the DMA
// engine moves the previous piece
static hipError_t h2d_gather(praos_ctx* c, uint8_t* dst, const praos_span* sp, size_t ns, size_t total,
                             hipStream_t st) {
  if (!stage_init(c)) return hipErrorOutOfMemory;
  std::vector<size_t> pre(ns + 1, 0);
  for (size_t j = 0; j < ns; j++) pre[j + 1] = pre[j] + sp[j].len;
  for (size_t off = 0, k = 0; off < total; off += STAGE_PIECE, k++) {
    const size_t len = std::min(STAGE_PIECE, total - off);
    hipError_t e = hipEventSynchronize(c->pin_ev[k & 1]);    // the DMA that last read this buffer
    if (e != hipSuccess) return e;
    uint8_t* pin = c->pin[k & 1];
    const unsigned nt = c->pool->size();
    c->pool->run([&](unsigned t) {
      size_t a = off + len * t / nt;
      const size_t b_ = off + len * (t + 1) / nt;
      size_t j = (size_t)(std::upper_bound(pre.begin(), pre.end(), a) - pre.begin()) - 1;
      while (a < b_ && j < ns) {
        const size_t in = a - pre[j], m = std::min(b_ - a, sp[j].len - in);
        std::memcpy(pin + (a - off), sp[j].p + in, m);
        a += m;
        j++;
      }
    });
    e = hipMemcpyAsync(dst + off, pin, len, hipMemcpyHostToDevice, st);
    if (e == hipSuccess) e = hipEventRecord(c->pin_ev[k & 1], st);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

int rp_upload_decode(praos_ctx* c, praos_batch* b, size_t n, const praos_span* spans, size_t nspans,
                     const uint64_t* hoff, const uint32_t* hlen) {
  size_t bytes = 0;
  for (size_t j = 0; j < nspans; j++) bytes += spans[j].len;
  if (!c || !b || !rp_batch_fits(b, n, bytes) || (n && (!hoff || !hlen))) return PRAOS_E_ARG;
  HIPCHK(c, hipSetDevice(c->device));
  // the batch's previous crypto run (ctx stream) reads the buffers rewritten below
  HIPCHK(c, hipStreamWaitEvent(c->cstream, b->run_ev, 0));
  b->n = n;
  b->arena_len = bytes;
  b->body_bytes_len = (size_t)b->signed_stride * n;
  b->decoded = true;                               // praos_batch_run skips the decode
  const size_t pad = ((bytes + 7) & ~(size_t)7) + 16 - bytes;
  HIPCHK(c, zero_pad(c, b->arena + bytes, pad, c->cstream));
  if (bytes) HIPCHK(c, h2d_gather(c, b->arena, spans, nspans, bytes, c->cstream));
  if (n) {
    HIPCHK(c, h2d_on(c, b->hoff, hoff, 8 * n, c->cstream));
    HIPCHK(c, h2d_on(c, b->hlen, hlen, 4 * n, c->cstream));
    launch_decode_praos(dim3(nblocks(n, NT)), dim3(NT), c->cstream, n, b->arena, bytes, b->hoff, b->hlen, b->slot,
                        b->cold_vk, b->vrf_vk, b->vrf_out, b->vrf_proof, b->hot_vk, b->ocert_sig, b->kes_sig,
                        b->ocert_n, b->ocert_c0, b->body_off, b->body_len, b->body, b->block_no, b->prev_hash,
                        b->prev_genesis, b->body_size, b->body_hash, b->prot_major, b->prot_minor, b->header_hash,
                        b->dec_status, b->tp_only ? 2 : 0, b->signed_stride, b->lead_out, b->lead_proof);
    launch_vrf_nonce(c->cstream, n, b->vrf_out, b->tp_only ? 1 : 0, b->nonce);
    HIPCHK(c, hipGetLastError());
  }
  HIPCHK(c, hipEventRecord(b->dec_ev, c->cstream));
  return PRAOS_OK;
}

// The decoded fields into the batch's pinned area (direct DMA, one sync: ten pageable copies
// with a sync each took ~2-3 ms of the replay's per-batch decode stage); d's pointers and
// *nonce point into it until the batch's next download
int rp_download_decoded(praos_ctx* c, praos_batch* b, praos_decoded* d, uint8_t** nonce) {
  if (!c || !b || !d || !nonce || !b->dec_h) return PRAOS_E_ARG;
  HIPCHK(c, hipSetDevice(c->device));
  const size_t n = b->n;
  uint8_t* h = b->dec_h;                          // 8-byte fields first, then 32-byte, 4, 2, 1
  *d = praos_decoded{};
  d->block_no = (uint64_t*)h; h += 8 * n;
  d->slot = (uint64_t*)h; h += 8 * n;
  d->ocert_n = (uint64_t*)h; h += 8 * n;
  d->prev_hash = h; h += 32 * n;
  d->cold_vk = h; h += 32 * n;
  d->header_hash = h; h += 32 * n;
  *nonce = h; h += 32 * n;
  d->body_size = (uint32_t*)h; h += 4 * n;
  d->status = (uint16_t*)h; h += 2 * n;
  d->prev_is_genesis = h;
  if (n == 0) return PRAOS_OK;
  auto dn = [&](void* dst, const void* src, size_t bytes) {
    return hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, c->cstream);
  };
  HIPCHK(c, dn(d->block_no, b->block_no, 8 * n));
  HIPCHK(c, dn(d->slot, b->slot, 8 * n));
  HIPCHK(c, dn(d->ocert_n, b->ocert_n, 8 * n));
  HIPCHK(c, dn(d->prev_hash, b->prev_hash, 32 * n));
  HIPCHK(c, dn(d->cold_vk, b->cold_vk, 32 * n));
  HIPCHK(c, dn(d->header_hash, b->header_hash, 32 * n));
  HIPCHK(c, dn(*nonce, b->nonce, 32 * n));
  HIPCHK(c, dn(d->body_size, b->body_size, 4 * n));
  HIPCHK(c, dn(d->status, b->dec_status, 2 * n));
  HIPCHK(c, dn(d->prev_is_genesis, b->prev_genesis, n));
  HIPCHK(c, hipStreamSynchronize(c->cstream));
  return PRAOS_OK;
}

int rp_run(praos_ctx* c, praos_batch* b, const praos_nonce* etas, uint32_t k, const uint8_t* eta_idx) {
  if (!c || !b || (b->n && (!etas || !eta_idx)) || k == 0 || k > 256) return PRAOS_E_ARG;
  HIPCHK(c, hipSetDevice(c->device));
  for (uint32_t e = 0; e < k; e++) {
    std::memset(b->eta_h + 9 * e, 0, 36);
    if (!etas[e].neutral) std::memcpy(b->eta_h + 9 * e, etas[e].hash, 32);
    b->eta_h[9 * e + 8] = etas[e].neutral ? 1u : 0u;
  }
  std::memcpy(b->eidx_h, eta_idx, b->n);
  // the pinned host buffers are reused by the next batch on this slot only after this run
  HIPCHK(c, hipStreamWaitEvent(c->stream, b->dec_ev, 0));
  HIPCHK(c, hipMemcpyAsync(b->eta_tab, b->eta_h, 36 * (size_t)k, hipMemcpyHostToDevice, c->stream));
  if (b->n) HIPCHK(c, hipMemcpyAsync(b->eta_idx, b->eidx_h, b->n, hipMemcpyHostToDevice, c->stream));
  const int r = praos_batch_run(c, b);
  if (r != PRAOS_OK) return r;
  HIPCHK(c, hipEventRecord(b->run_ev, c->stream));
  return PRAOS_OK;
}

int rp_download_results(praos_ctx* c, praos_batch* b, uint16_t* bits, int32_t* pool_idx) {
  if (!c || !b || !bits) return PRAOS_E_ARG;
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipStreamWaitEvent(c->dstream, b->run_ev, 0));
  if (b->n) {
    HIPCHK(c, hipMemcpyAsync(bits, b->bits, 2 * b->n, hipMemcpyDeviceToHost, c->dstream));
    if (pool_idx) HIPCHK(c, hipMemcpyAsync(pool_idx, b->pool_idx, 4 * b->n, hipMemcpyDeviceToHost, c->dstream));
  }
  HIPCHK(c, hipStreamSynchronize(c->dstream));
  return PRAOS_OK;
}

extern "C" {

// Stored-bytes verification with the upload in K chunks (contiguous runs of headers) and
// the batch's largest kernel run under it: chunk k's bytes move H2D on the copy stream
// (pinned staging, host threads) while, on the GPU, chunk k-1 is decoded (ctx stream) and
// its VRF stage V (H, Gamma, V = [s]H - [c]Gamma: over half of a header's work, and it needs
// nothing but the header) runs on vstream.  After the last chunk the rest of the batch --
// key caches, OCert, KES, U, the join, the leader test -- runs once over the whole batch, as
// praos_batch_run does (full-batch key caches, no small-batch tails).  One batch for the whole
// input, kept in the context (device buffers allocated once for a given size).
//
// async (praos_verify_header_bytes_submit): the call on pipe[slot], queued and not waited for:
// each chunk is decoded on the copy stream right after its upload (on the ctx stream the decode
// would queue behind the previous call's run), the run's end is recorded in pcall[slot].ev and the
// outputs come back in pipe_finish.  The next call's uploads, decodes and stage V then overlap this
// call's key chains, as back-to-back resident runs overlap.
static int verify_bytes_pipelined(praos_ctx* c, const praos_header_bytes* in, praos_out* out, praos_decoded* dec,
                                  int K, int slot = 0, bool async = false) {
  const auto t_entry = std::chrono::steady_clock::now();
  HIPCHK(c, hipSetDevice(c->device));
  const size_t n = in->n;
  // the arena span of the in-range headers, and offsets rebased to it
  uint64_t base = UINT64_MAX, end = 0;
  for (size_t i = 0; i < n; i++) {
    if (in->off[i] > in->bytes_len || in->len[i] > in->bytes_len - in->off[i]) continue;
    base = std::min<uint64_t>(base, in->off[i]);
    end = std::max<uint64_t>(end, in->off[i] + in->len[i]);
  }
  if (base == UINT64_MAX) base = end = 0;
  praos_ctx::PipeCall& pc = c->pcall[slot];
  if (pc.cap < n) {                     // (the slot's previous call has finished: its H2D is done)
    if (pc.off_h) (void)hipHostFree(pc.off_h);
    if (pc.len_h) (void)hipHostFree(pc.len_h);
    pc.off_h = nullptr;
    pc.len_h = nullptr;
    pc.cap = 0;
    const size_t cap = n + n / 8 + 64;
    if (hipHostMalloc((void**)&pc.off_h, 8 * cap, hipHostMallocDefault) != hipSuccess ||
        hipHostMalloc((void**)&pc.len_h, 4 * cap, hipHostMallocDefault) != hipSuccess) {
      c->err = "pinned offsets";
      return PRAOS_E_OOM;
    }
    pc.cap = cap;
  }
  uint64_t* off = pc.off_h;
  std::memcpy(pc.len_h, in->len, 4 * n);
  for (size_t i = 0; i < n; i++) {   // a span outside the caller's arena stays outside
    const bool in_range = in->off[i] <= in->bytes_len && in->len[i] <= in->bytes_len - in->off[i];
    off[i] = in_range ? in->off[i] - base : UINT64_MAX / 2;
  }
  // chunk k = headers [lo_k, hi_k) and the byte range [b0_k, b1_k) of the arena its headers
  // need (relative to base); chunk k's upload covers what earlier chunks did not
  std::vector<size_t> lo(K + 1);
  std::vector<uint64_t> need(K);
  {
    // weights: head / 100 for chunk 0, tail / 100 for chunk K-1, 1 for the others
    std::vector<size_t> w(K, 100);
    w[0] = (size_t)c->pipe_head;
    if (K > 2) w[K - 1] = (size_t)c->pipe_tail;
    size_t W = 0, acc = 0;
    for (int k = 0; k < K; k++) W += w[k];
    lo[0] = 0;
    for (int k = 1; k <= K; k++) { acc += w[k - 1]; lo[k] = n * acc / W; }
  }
  uint64_t hw = 0;
  for (int k = 0; k < K; k++) {
    for (size_t i = lo[k]; i < lo[k + 1]; i++)
      if (off[i] != UINT64_MAX / 2) hw = std::max<uint64_t>(hw, off[i] + in->len[i]);
    need[k] = hw;                                 // bytes [0, need[k]) cover chunks 0..k
  }
  const uint64_t bytes = end - base;
  if (!c->pipe[slot] || c->pipe_n[slot] < n || c->pipe_bytes[slot] < bytes) {
    if (c->pipe[slot]) {
      HIPCHK(c, hipDeviceSynchronize());
      for (void* q : c->pipe[slot]->owned) (void)hipFree(q);
      delete c->pipe[slot];
      c->pipe[slot] = nullptr;
    }
    const size_t mc = n + n / 8 + 64, bc = bytes + bytes / 8 + 4096;   // headroom for the next call
    c->pipe[slot] = bytes_batch_alloc(c, mc, bc, false, nullptr);
    if (!c->pipe[slot]) return PRAOS_E_OOM;
    c->pipe_n[slot] = mc;
    c->pipe_bytes[slot] = bc;
  }
  praos_batch* b = c->pipe[slot];
  batch_reuse_reset(b);
  b->n = n;
  b->arena_len = bytes;
  b->body_bytes_len = (size_t)b->signed_stride * n;
  const size_t pad = ((bytes + 7) & ~(size_t)7) + 16 - bytes;
  HIPCHK(c, zero_pad(c, b->arena + bytes, pad, c->cstream));
  HIPCHK(c, hipMemcpyAsync(b->hoff, off, 8 * n, hipMemcpyHostToDevice, c->cstream));
  HIPCHK(c, hipMemcpyAsync(b->hlen, pc.len_h, 4 * n, hipMemcpyHostToDevice, c->cstream));
  if (c->keycache > 0 && n >= 2) {               // the comb the cached chains read (built once)
    const int rc = ensure_bcomb16(c);
    if (rc != PRAOS_OK) return rc;
  }
  const uint32_t* eta = b->eta_tab ? b->eta_tab : c->d_eta0;
  // stage V chunk by chunk under the upload, or (submitted calls, PRAOS_STREAM_CHUNK_V=0) in the
  // run over the whole batch
  const bool vrf = (c->kernels & 4) != 0 && (!async || c->stream_chunk_v);
  uint64_t sent = 0;
  for (int k = 0; k < K; k++) {
    if (need[k] > sent) {
      HIPCHK(c, h2d_on(c, b->arena + sent, in->bytes + base + sent, need[k] - sent, c->cstream));
      sent = need[k];
    }
    hipStream_t sd = async ? c->decstream : c->stream;    // the chunk's decode
    HIPCHK(c, hipEventRecord(c->up_ev[k], c->cstream));
    HIPCHK(c, hipStreamWaitEvent(sd, c->up_ev[k], 0));
    const size_t m = lo[k + 1] - lo[k];
    if (m) {
      launch_decode_praos(dim3(nblocks(m, NT)), dim3(NT), sd, lo[k + 1], b->arena, bytes, b->hoff, b->hlen,
                          b->slot, b->cold_vk, b->vrf_vk, b->vrf_out, b->vrf_proof, b->hot_vk, b->ocert_sig,
                          b->kes_sig, b->ocert_n, b->ocert_c0, b->body_off, b->body_len, b->body, b->block_no,
                          b->prev_hash, b->prev_genesis, b->body_size, b->body_hash, b->prot_major, b->prot_minor,
                          b->header_hash, b->dec_status, 0, b->signed_stride, nullptr, nullptr, lo[k]);
      HIPCHK(c, hipGetLastError());
    }
    HIPCHK(c, hipEventRecord(c->done_ev[k], sd));
    if (m && vrf) {
      // the chunks' stage V alternate between two streams: on one they would queue behind
      // each other (a chunk's V alone is latency-bound)
      hipStream_t sv = (k & 1) ? c->vstream2 : c->vstream;
      HIPCHK(c, hipStreamWaitEvent(sv, c->done_ev[k], 0));
      launch_vrf_v(sv, n, b->vrf_vk, b->vrf_proof, b->slot, eta, c->eta0_neutral, b->eta_idx, b->tab_vrf,
                   b->vrf_mid, lo[k], lo[k + 1], 0, 0, c->v_ilp4(n));
      HIPCHK(c, hipGetLastError());
    }
  }
  if (async) HIPCHK(c, hipStreamWaitEvent(c->stream, c->done_ev[K - 1], 0));   // every chunk decoded
  const auto t_chunks = std::chrono::steady_clock::now();
  b->decoded = true;
  b->v_done = vrf;
  int r = praos_batch_run(c, b);
  if (async && std::getenv("PRAOS_SUBMIT_TRACE"))
    std::fprintf(stderr, "submit: chunks queued %.3f ms after entry, run queued %.3f ms\n",
                 std::chrono::duration<double, std::milli>(t_chunks - t_entry).count(),
                 std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_chunks).count());
  b->decoded = false;                // (the downloads below still read b->n; the next call resets
  b->v_done = false;                 // every per-run field when it takes the batch: batch_reuse_reset)
  if (async) {
    if (r != PRAOS_OK) {             // nothing of this call is left running when it reports an error
      (void)hipDeviceSynchronize();
      return r;
    }
    praos_ctx::PipeCall& p = c->pcall[slot];
    HIPCHK(c, hipEventRecord(p.ev, c->stream));
    p.out = *out;
    p.dec = dec;
    p.active = true;
    return PRAOS_OK;
  }
  // the VRF outputs (pool index, beta, leader and nonce values: 132 of the 134 bytes per
  // header) are final once the VRF stream is done: they come back while KES still runs
  if (r == PRAOS_OK && c->concurrent) {
    HIPCHK(c, hipStreamWaitEvent(c->cstream, c->side_ev[2], 0));
    auto dn = [&](void* dst, const void* src, size_t nb) -> hipError_t {
      return dst && nb ? d2h_on(c, dst, src, nb, c->cstream) : hipSuccess;
    };
    HIPCHK(c, dn(out->pool_idx, b->pool_idx, 4 * n));
    HIPCHK(c, dn(out->beta, b->beta, 64 * n));
    HIPCHK(c, dn(out->leader, b->leader, 32 * n));
    HIPCHK(c, dn(out->nonce, b->nonce, 32 * n));
    if (r == PRAOS_OK) r = praos_batch_sync(c);
    if (r == PRAOS_OK) HIPCHK(c, d2h(c, out->bits, b->bits, 2 * n));
  } else {
    if (r == PRAOS_OK) r = praos_batch_sync(c);
    if (r == PRAOS_OK) r = praos_batch_download(c, b, out);
  }
  if (r == PRAOS_OK && dec) r = praos_batch_download_decoded(c, b, dec);
  (void)hipStreamSynchronize(c->cstream);
  (void)hipStreamSynchronize(c->vstream);
  (void)hipStreamSynchronize(c->vstream2);
  return r;
}

// the outputs of submitted call `slot` (waits for its run): on the download stream, which the
// calls queued after it do not use
static int pipe_finish(praos_ctx* c, int slot) {
  praos_ctx::PipeCall& p = c->pcall[slot];
  if (!p.active) return PRAOS_OK;
  p.active = false;
  HIPCHK(c, hipSetDevice(c->device));
  const praos_batch* b = c->pipe[slot];
  const size_t n = b->n;
  HIPCHK(c, hipStreamWaitEvent(c->dstream, p.ev, 0));
  auto dn = [&](void* dst, const void* src, size_t nb) -> hipError_t {
    return dst && nb ? d2h_on(c, dst, src, nb, c->dstream) : hipSuccess;
  };
  HIPCHK(c, dn(p.out.bits, b->bits, 2 * n));
  HIPCHK(c, dn(p.out.pool_idx, b->pool_idx, 4 * n));
  HIPCHK(c, dn(p.out.beta, b->beta, 64 * n));
  HIPCHK(c, dn(p.out.leader, b->leader, 32 * n));
  HIPCHK(c, dn(p.out.nonce, b->nonce, 32 * n));
  if (praos_decoded* d = p.dec) {
    HIPCHK(c, dn(d->status, b->dec_status, 2 * n));
    HIPCHK(c, dn(d->block_no, b->block_no, 8 * n));
    HIPCHK(c, dn(d->slot, b->slot, 8 * n));
    HIPCHK(c, dn(d->prev_hash, b->prev_hash, 32 * n));
    HIPCHK(c, dn(d->prev_is_genesis, b->prev_genesis, n));
    HIPCHK(c, dn(d->cold_vk, b->cold_vk, 32 * n));
    HIPCHK(c, dn(d->vrf_vk, b->vrf_vk, 32 * n));
    HIPCHK(c, dn(d->vrf_out, b->vrf_out, 64 * n));
    HIPCHK(c, dn(d->vrf_proof, b->vrf_proof, 80 * n));
    HIPCHK(c, dn(d->body_size, b->body_size, 4 * n));
    HIPCHK(c, dn(d->body_hash, b->body_hash, 32 * n));
    HIPCHK(c, dn(d->hot_vk, b->hot_vk, 32 * n));
    HIPCHK(c, dn(d->ocert_n, b->ocert_n, 8 * n));
    HIPCHK(c, dn(d->ocert_c0, b->ocert_c0, 8 * n));
    HIPCHK(c, dn(d->ocert_sig, b->ocert_sig, 64 * n));
    HIPCHK(c, dn(d->prot_major, b->prot_major, 8 * n));
    HIPCHK(c, dn(d->prot_minor, b->prot_minor, 8 * n));
    HIPCHK(c, dn(d->header_hash, b->header_hash, 32 * n));
    HIPCHK(c, dn(d->kes_sig, b->kes_sig, 448 * n));
    HIPCHK(c, dn(d->signed_body, b->body, (size_t)b->signed_stride * n));
    HIPCHK(c, dn(d->signed_len, b->body_len, 4 * n));
  }
  HIPCHK(c, hipStreamSynchronize(c->dstream));
  return PRAOS_OK;
}

int praos_verify_drain(praos_ctx* c) {
  if (!c) return PRAOS_E_ARG;
  if (c->device < 0) return PRAOS_OK;
  int r = PRAOS_OK;
  for (int j = 0; j < PIPE_CALLS; j++) {       // oldest first: the slot the next submit reuses
    const int rj = pipe_finish(c, (c->pcall_next + j) % PIPE_CALLS);
    if (r == PRAOS_OK) r = rj;
  }
  return r;
}

int praos_verify_header_bytes_submit(praos_ctx* c, const praos_header_bytes* in, praos_out* out, praos_decoded* dec) {
  if (!c || !in || !out || !out->bits) return PRAOS_E_ARG;
  if (!c->have_epoch) return PRAOS_E_STATE;
  if (in->n && (!in->off || !in->len || (!in->bytes && in->bytes_len))) return PRAOS_E_ARG;
  int K = c->pipeline;
  if (K == 0) K = (int)std::min<size_t>(PIPE_AUTO, in->n / PIPE_MIN_CHUNK);
  K = std::min<int>(K, (int)std::min<size_t>(PIPE_MAX, in->n));
  if (in->n == 0 || K < 2 || c->device < 0) {  // too small to pipeline: the blocking call, in order
    const int r = praos_verify_drain(c);
    return r != PRAOS_OK ? r : praos_verify_header_bytes(c, in, out, dec);
  }
  const int slot = c->pcall_next;
  const auto t0 = std::chrono::steady_clock::now();
  int r = pipe_finish(c, slot);                // PIPE_CALLS in flight: the oldest one's outputs first
  if (r != PRAOS_OK) return r;
  if (std::getenv("PRAOS_SUBMIT_TRACE"))
    std::fprintf(stderr, "submit: finish of the oldest call %.3f ms\n",
                 std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
  r = verify_bytes_pipelined(c, in, out, dec, K, slot, true);
  if (r == PRAOS_OK) c->pcall_next = (slot + 1) % PIPE_CALLS;
  return r;
}

int praos_verify_header_bytes(praos_ctx* c, const praos_header_bytes* in, praos_out* out, praos_decoded* dec) {
  if (!c || !in || !out || !out->bits) return PRAOS_E_ARG;
  if (!c->have_epoch) return PRAOS_E_STATE;
  if (in->n == 0) return PRAOS_OK;
  if (in->n && (!in->off || !in->len || (!in->bytes && in->bytes_len))) return PRAOS_E_ARG;
  {
    const int rd = praos_verify_drain(c);     // submitted calls use pipe[0] / pipe[1]: finished first
    if (rd != PRAOS_OK) return rd;
  }
  {
    // chunked pipeline (PRAOS_OPT_PIPELINE: chunks; 0 = auto: up to PIPE_AUTO chunks of >= PIPE_MIN_CHUNK)
    int K = c->pipeline;
    if (K == 0) K = (int)std::min<size_t>(PIPE_AUTO, in->n / PIPE_MIN_CHUNK);
    K = std::min<int>(K, (int)std::min<size_t>(PIPE_MAX, in->n));
    if (K >= 2 && c->device >= 0) return verify_bytes_pipelined(c, in, out, dec, K);
  }
  praos_batch* b = praos_batch_upload_bytes(c, in);
  if (!b) return PRAOS_E_OOM;
  int r = praos_batch_run(c, b);
  if (r == PRAOS_OK) r = praos_batch_sync(c);
  if (r == PRAOS_OK) r = praos_batch_download(c, b, out);
  if (r == PRAOS_OK && dec) r = praos_batch_download_decoded(c, b, dec);
  praos_batch_free(c, b);
  return r;
}

// ---------------------------------------------------------------- single-primitive batches
}  // extern "C"
namespace {
struct Scratch {
  praos_ctx* c;
  std::vector<void*> ptrs;
  bool ok = true;
  explicit Scratch(praos_ctx* cc) : c(cc) {}
  ~Scratch() { for (void* p : ptrs) (void)hipFree(p); }
  template <typename T>
  T* up(const T* src, size_t bytes) {
    void* d = nullptr;
    if (hipMalloc(&d, bytes ? bytes : 16) != hipSuccess) { ok = false; return nullptr; }
    ptrs.push_back(d);
    if (src && bytes && hipMemcpy(d, src, bytes, hipMemcpyHostToDevice) != hipSuccess) ok = false;
    return (T*)d;
  }
  template <typename T>
  T* zeros(size_t bytes) {
    T* d = up<T>(nullptr, bytes);
    // on the ctx stream: a null-stream hipMemset is not ordered with the (non-blocking)
    // stream the kernel runs on and could land after the kernel's writes
    if (d && hipMemsetAsync(d, 0, bytes ? bytes : 16, c->stream) != hipSuccess) ok = false;
    return d;
  }
};
}  // namespace
extern "C" {

int praos_verify_ocert(praos_ctx* c, size_t n, const uint8_t* cold_vk, const uint8_t* hot_vk, const uint64_t* ocert_n,
                       const uint64_t* ocert_c0, const uint8_t* sig, uint8_t* ok) {
  if (!c || (n && (!cold_vk || !hot_vk || !ocert_n || !ocert_c0 || !sig || !ok))) return PRAOS_E_ARG;
  if (n == 0) return PRAOS_OK;
  HIPCHK(c, hipSetDevice(c->device));
  Scratch s(c);
  auto dv = s.up(cold_vk, 32 * n);
  auto dh = s.up(hot_vk, 32 * n);
  auto dn = s.up(ocert_n, 8 * n);
  auto dc = s.up(ocert_c0, 8 * n);
  auto ds = s.up(sig, 64 * n);
  auto dok = s.zeros<uint8_t>(n);
  auto dtab = s.up<ge_cached>(nullptr, LT_ED_B * n);
  if (!s.ok) { c->err = "alloc/copy"; return PRAOS_E_OOM; }
  HIPCHK(c, hipEventRecord(c->ev[0], c->stream));
  launch_ocert(dim3(nblocks(n, NT)), dim3(NT), c->stream, n, nullptr, nullptr, c->btab, dv, dh, dn, dc, ds,
                     (const uint64_t*)nullptr, (uint64_t)1, (uint64_t)0, (uint16_t*)nullptr, dok, dtab);
  HIPCHK(c, hipEventRecord(c->ev[1], c->stream));
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipStreamSynchronize(c->stream));
  (void)hipEventElapsedTime(&c->kernel_ms[0], c->ev[0], c->ev[1]);
  HIPCHK(c, hipMemcpy(ok, dok, n, hipMemcpyDeviceToHost));
  return PRAOS_OK;
}

int praos_verify_kes(praos_ctx* c, size_t n, const uint8_t* vk, const uint32_t* period, const uint8_t* sig,
                     const uint64_t* msg_off, const uint32_t* msg_len, const uint8_t* msg_bytes, size_t msg_bytes_len,
                     uint8_t* result) {
  if (!c || (n && (!vk || !period || !sig || !msg_off || !msg_len || !result))) return PRAOS_E_ARG;
  if (n == 0) return PRAOS_OK;
  HIPCHK(c, hipSetDevice(c->device));
  std::vector<uint64_t> off(n);
  std::vector<uint32_t> len(n);
  size_t total = 0;
  for (size_t i = 0; i < n; i++) { off[i] = total; total += (msg_len[i] + 7) & ~(size_t)7; }
  std::vector<uint8_t> arena(total + 16, 0);
  for (size_t i = 0; i < n; i++) {
    const bool okr = msg_off[i] <= msg_bytes_len && msg_len[i] <= msg_bytes_len - msg_off[i];
    len[i] = okr ? msg_len[i] : 0xffffffffu;
    if (okr && msg_len[i]) std::memcpy(arena.data() + off[i], msg_bytes + msg_off[i], msg_len[i]);
  }
  Scratch s(c);
  auto dvk = s.up(vk, 32 * n);
  auto dp = s.up(period, 4 * n);
  auto dsig = s.up(sig, 448 * n);
  auto doff = s.up(off.data(), 8 * n);
  auto dlen = s.up(len.data(), 4 * n);
  auto dmsg = s.up(arena.data(), arena.size());
  auto dres = s.zeros<uint8_t>(n);
  auto dtab = s.up<ge_cached>(nullptr, LT_ED_B * n);
  if (!s.ok) { c->err = "alloc/copy"; return PRAOS_E_OOM; }
  HIPCHK(c, hipEventRecord(c->ev[0], c->stream));
  launch_kes(dim3(nblocks(n, NT)), dim3(NT), c->stream, n, (const uint32_t*)nullptr, (const uint32_t*)nullptr,
             c->btab, dvk, dsig, doff, dlen, dmsg,
                     total, (const uint64_t*)nullptr, (const uint64_t*)nullptr, (uint64_t)1, dp, (uint16_t*)nullptr,
                     dres, dtab);
  HIPCHK(c, hipEventRecord(c->ev[1], c->stream));
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipStreamSynchronize(c->stream));
  (void)hipEventElapsedTime(&c->kernel_ms[1], c->ev[0], c->ev[1]);
  HIPCHK(c, hipMemcpy(result, dres, n, hipMemcpyDeviceToHost));
  return PRAOS_OK;
}

int praos_verify_vrf(praos_ctx* c, size_t n, const uint8_t* vk, const uint8_t* proof, const uint8_t* alpha,
                     uint8_t* ok, uint8_t* beta) {
  if (!c || (n && (!vk || !proof || !alpha || !ok))) return PRAOS_E_ARG;
  if (n == 0) return PRAOS_OK;
  HIPCHK(c, hipSetDevice(c->device));
  Scratch s(c);
  auto dvk = s.up(vk, 32 * n);
  auto dpr = s.up(proof, 80 * n);
  auto dal = s.up(alpha, 32 * n);
  auto dok = s.zeros<uint8_t>(n);
  auto dbeta = s.zeros<uint8_t>(64 * n);
  auto dtab = s.up<ge_cached>(nullptr, LT_VRF_B * n);
  if (!s.ok) { c->err = "alloc/copy"; return PRAOS_E_OOM; }
  HIPCHK(c, hipEventRecord(c->ev[0], c->stream));
  launch_vrf(dim3(nblocks(n, NT)), dim3(NT), c->stream, n, nullptr, nullptr, c->btab, (const uint8_t*)nullptr, dvk,
                     (const uint8_t*)nullptr, dpr, (const uint64_t*)nullptr, (const uint32_t*)nullptr, 1,
                     (const uint8_t*)nullptr,
                     (const uint32_t*)nullptr, (const uint32_t*)nullptr, (const int32_t*)nullptr, 0u, 0, dal,
                     (uint16_t*)nullptr, (int32_t*)nullptr, (int32_t*)nullptr, dbeta, (uint8_t*)nullptr,
                     (uint8_t*)nullptr, dok, dtab);
  HIPCHK(c, hipEventRecord(c->ev[1], c->stream));
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipStreamSynchronize(c->stream));
  (void)hipEventElapsedTime(&c->kernel_ms[2], c->ev[0], c->ev[1]);
  HIPCHK(c, hipMemcpy(ok, dok, n, hipMemcpyDeviceToHost));
  if (beta) HIPCHK(c, hipMemcpy(beta, dbeta, 64 * n, hipMemcpyDeviceToHost));
  return PRAOS_OK;
}

int praos_check_leader(praos_ctx* c, size_t n, const uint8_t* leader, const uint8_t* sigma_fp,
                       const praos_params* params, uint8_t* is_leader) {
  if (!c || !params || (n && (!leader || !sigma_fp || !is_leader))) return PRAOS_E_ARG;
  if (n == 0) return PRAOS_OK;
  HIPCHK(c, hipSetDevice(c->device));
  std::vector<uint32_t> x(4 * n);
  for (size_t i = 0; i < n; i++) {
    uint8_t xr[16];
    if (!praos_host::leader_x_raw(xr, sigma_fp + 16 * i, params->c_raw)) { c->err = "x out of range"; return PRAOS_E_ARG; }
    std::memcpy(&x[4 * i], xr, 16);
  }
  Scratch s(c);
  auto dl = s.up(leader, 32 * n);
  auto dx = s.up(x.data(), 16 * n);
  auto dres = s.zeros<uint8_t>(n);
  if (!s.ok) { c->err = "alloc/copy"; return PRAOS_E_OOM; }
  HIPCHK(c, hipEventRecord(c->ev[0], c->stream));
  launch_leader(dim3(nblocks(n, NT)), dim3(NT), c->stream, n, dl, (const int32_t*)nullptr,
                (const uint32_t*)nullptr, dx, (int)params->f_is_one, 8, (const uint16_t*)nullptr,
                (const uint16_t*)nullptr, (const uint16_t*)nullptr, (uint16_t*)nullptr, dres, (int32_t*)nullptr, (const uint16_t*)nullptr);
  HIPCHK(c, hipEventRecord(c->ev[1], c->stream));
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipStreamSynchronize(c->stream));
  (void)hipEventElapsedTime(&c->kernel_ms[3], c->ev[0], c->ev[1]);
  HIPCHK(c, hipMemcpy(is_leader, dres, n, hipMemcpyDeviceToHost));
  return PRAOS_OK;
}

// ---------------------------------------------------------------- sequential part (host)
// First-error-wins order of Praos.updateChainDepState (Praos.hs:441-459):
// validateKESSignature (:567 c0<=kp, :568 kp<c0+maxKESEvo, :580 OCert, :582 KES,
// :584-590 counter), then validateVRFSignature (:537 unknown, :539 vrf key,
// :543 proof, :549 leader).  Counter source (:601-606): the counter map, else
// 0 if the issuer is in the pool distribution, else missing.
}  // extern "C"

// First failing check of one header in the reference order (Praos.hs:449-455 with
// validateKESSignature :558-606 and validateVRFSignature :528-556).  has_counter / m
// = the counter-map lookup of :601-606 (PoolDistr membership counts as m = 0).
static uint8_t header_verdict(uint16_t b, bool have, uint64_t m, uint64_t n) {
  if (b & PRAOS_BIT_INPUT) return PRAOS_V_INPUT;
  if (b & PRAOS_BIT_KES_BEFORE_START) return PRAOS_V_KES_BEFORE_START;
  if (b & PRAOS_BIT_KES_AFTER_END) return PRAOS_V_KES_AFTER_END;
  if (b & PRAOS_BIT_OCERT_SIG) return PRAOS_V_OCERT_SIG;
  if (b & (PRAOS_BIT_KES_MERKLE | PRAOS_BIT_KES_LEAF)) return PRAOS_V_KES_SIG;
  if (!have) return PRAOS_V_COUNTER_MISSING;
  if (!(m <= n)) return PRAOS_V_COUNTER_TOO_SMALL;
  if (!(n <= m + 1)) return PRAOS_V_COUNTER_OVER_INC;
  if (b & PRAOS_BIT_VRF_KEY_UNKNOWN) return PRAOS_V_VRF_KEY_UNKNOWN;
  if (b & PRAOS_BIT_VRF_KEY_WRONG) return PRAOS_V_VRF_KEY_WRONG;
  if (b & (PRAOS_BIT_VRF_PROOF | PRAOS_BIT_VRF_OUTPUT)) return PRAOS_V_VRF_BAD_PROOF;
  if (b & PRAOS_BIT_LEADER) return PRAOS_V_LEADER_TOO_BIG;
  return PRAOS_V_OK;
}

// TPraos predicate failures of one header (PRAOS_TPF_*), as PRTCL collects them
// (small-steps ValidateAll: every `?!` of OVERLAY and OCERT is recorded):
//   OVERLAY (cardano-protocol-tpraos Rules/Overlay.hs): NotActiveSlotOVERLAY; or, in an
//     active overlay slot, WrongGenesisColdKeyOVERLAY (?!) and pbftVrfChecks (an Either:
//     its first failure -- WrongGenesisVRFKey, BadNonce, BadLeaderValue); or, outside the
//     overlay, praosVrfChecks (an Either: VRFKeyUnknown, VRFKeyWrongVRFKey, BadNonce,
//     BadLeaderValue, VRFLeaderValueTooBig -- first failure);
//   OCERT (Rules/OCert.hs): KESBeforeStart, KESAfterEnd, InvalidSignature, InvalidKesSignature,
//     then the counter (currentIssueNo: Nothing -> NoCounterForKeyHash; else CounterTooSmall,
//     CounterOverIncremented).
static uint16_t tpraos_failures(uint16_t b, bool have, uint64_t m, uint64_t n) {
  uint16_t f = 0;
  if (b & PRAOS_BIT_TP_NOT_ACTIVE) {
    f |= PRAOS_TPF_NOT_ACTIVE;
  } else if (b & PRAOS_BIT_TP_OVERLAY) {
    if (b & PRAOS_BIT_TP_GEN_COLD) f |= PRAOS_TPF_GEN_COLD;
    if (b & PRAOS_BIT_TP_GEN_VRF) f |= PRAOS_TPF_GEN_VRF;
    else if (b & PRAOS_BIT_TP_VRF_NONCE) f |= PRAOS_TPF_BAD_NONCE;
    else if (b & PRAOS_BIT_TP_VRF_LEADER) f |= PRAOS_TPF_BAD_LEADER;
  } else {
    if (b & PRAOS_BIT_VRF_KEY_UNKNOWN) f |= PRAOS_TPF_VRF_KEY_UNKNOWN;
    else if (b & PRAOS_BIT_VRF_KEY_WRONG) f |= PRAOS_TPF_VRF_KEY_WRONG;
    else if (b & PRAOS_BIT_TP_VRF_NONCE) f |= PRAOS_TPF_BAD_NONCE;
    else if (b & PRAOS_BIT_TP_VRF_LEADER) f |= PRAOS_TPF_BAD_LEADER;
    else if (b & PRAOS_BIT_LEADER) f |= PRAOS_TPF_LEADER_TOO_BIG;
  }
  if (b & PRAOS_BIT_KES_BEFORE_START) f |= PRAOS_TPF_KES_BEFORE_START;
  if (b & PRAOS_BIT_KES_AFTER_END) f |= PRAOS_TPF_KES_AFTER_END;
  if (b & PRAOS_BIT_OCERT_SIG) f |= PRAOS_TPF_OCERT_SIG;
  if (b & (PRAOS_BIT_KES_MERKLE | PRAOS_BIT_KES_LEAF)) f |= PRAOS_TPF_KES_SIG;
  if (!have) {
    f |= PRAOS_TPF_COUNTER_MISSING;
  } else {
    if (!(m <= n)) f |= PRAOS_TPF_COUNTER_TOO_SMALL;
    if (!(n <= m + 1)) f |= PRAOS_TPF_COUNTER_OVER_INC;
  }
  return f;
}

static std::string issuer_hash(const praos_ctx* c, const praos_headers* h, const praos_out* crypto, size_t i) {
  const int32_t pidx = crypto->pool_idx ? crypto->pool_idx[i] : -1;
  if (pidx >= 0 && (size_t)pidx < c->pools.size()) return std::string((const char*)c->pools[pidx].hash28, 28);
  uint8_t hh[28];
  praos_host::blake2b(hh, 28, h->cold_vk + 32 * i, 32);
  return std::string((const char*)hh, 28);
}

using praos_host::nonce_combine;
using praos_host::nonce_eq;

// the staging copy threads of a context onto the given CPUs (the replay's thread placement)
void rp_copy_pin(praos_ctx* c, const std::vector<int>& cpus) {
  if (c && c->device >= 0 && stage_init(c)) c->pool->pin(cpus);
}

// error text for the other host modules of the library (praos_replay.hip)
void praos_set_error_(praos_ctx* c, const std::string& m) { if (c) c->err = m; }
// the group's page-locked ranges (praos_group_host_register: pinned once, known to every member)
int praos_ctx_note_registered_(praos_ctx* c, void* p, size_t len, bool add) {
  if (!c) return PRAOS_E_ARG;
  std::lock_guard<std::mutex> g(c->reg_mu);
  if (add) {
    c->registered.emplace_back((uintptr_t)p, len);
    return PRAOS_OK;
  }
  auto it = std::find_if(c->registered.begin(), c->registered.end(),
                         [&](const std::pair<uintptr_t, size_t>& r) { return r.first == (uintptr_t)p; });
  if (it == c->registered.end()) return PRAOS_E_ARG;
  c->registered.erase(it);
  return PRAOS_OK;
}
int praos_ctx_device_(praos_ctx* c) { return c ? c->device : -1; }
void praos_replay_scope_(praos_ctx* c, bool on) {
  if (!c) return;
  c->err.first_only(on);
  c->replaying = on;                                   // (set for the length of a replay call)
}

extern "C" {

int praos_apply_batch(praos_ctx* c, const praos_headers* h, const praos_out* crypto, praos_counters* counters,
                      uint8_t* verdict, size_t* chain_stop) {
  if (!c || !h || !crypto || !crypto->bits || !verdict) return PRAOS_E_ARG;
  if (!c->have_epoch) return PRAOS_E_STATE;
  std::map<std::string, uint64_t> cmap;
  if (counters)
    for (size_t k = 0; k < counters->m; k++)
      cmap[std::string((const char*)counters->hash28 + 28 * k, 28)] = counters->counter[k];
  size_t stop = h->n;
  for (size_t i = 0; i < h->n; i++) {
    const std::string hk = issuer_hash(c, h, crypto, i);
    const uint64_t n = h->ocert_n[i];
    auto it = cmap.find(hk);
    const bool have = it != cmap.end() || c->pool_by_hash.count(hk);
    const uint8_t v = header_verdict(crypto->bits[i], have, it != cmap.end() ? it->second : 0, n);
    verdict[i] = v;
    if (v == PRAOS_V_OK) cmap[hk] = n;               // reupdateChainDepState, Praos.hs:484-485
    else if (stop == h->n) stop = i;
  }
  if (chain_stop) *chain_stop = stop;
  if (counters)
    for (size_t k = 0; k < counters->m; k++)
      counters->counter[k] = cmap[std::string((const char*)counters->hash28 + 28 * k, 28)];
  return PRAOS_OK;
}

}  // extern "C"

// validateEnvelope (HeaderValidation.hs:297-344) with the Praos additionalEnvelopeChecks
// (envelopeChecks, Shelley/Protocol/Praos.hs:66-80), against the tip the chain has
// reached (AnnTip: slot, block number, header hash).  First failure in that order.
struct EnvTip {
  int32_t origin;
  uint64_t slot, block_no;
  uint8_t hash[32];
};
static uint8_t envelope_verdict(const praos_envelope* e, const EnvTip& tip, const praos_headers* h,
                                const uint8_t* prev_hash, const uint8_t* prev_is_genesis, size_t i) {
  const uint64_t expected_block = tip.origin ? 0 : tip.block_no + 1;     // expectedFirstBlockNo / succ
  if (e->block_no[i] != expected_block) return PRAOS_V_ENV_BLOCK_NO;
  const uint64_t min_slot = tip.origin ? 0 : tip.slot + 1;                // minimumPossibleSlotNo / succ
  if (!(h->slot[i] >= min_slot)) return PRAOS_V_ENV_SLOT_NO;
  const bool genesis = prev_is_genesis && prev_is_genesis[i];
  const bool prev_ok = tip.origin ? genesis : (!genesis && std::memcmp(prev_hash + 32 * i, tip.hash, 32) == 0);
  if (!prev_ok) return PRAOS_V_ENV_PREV_HASH;                             // checkPrevHash'
  if (!(e->lv_prot_major <= e->max_major_pv)) return PRAOS_V_ENV_OBSOLETE_NODE;
  if (!((uint64_t)e->header_size[i] <= e->max_header_size)) return PRAOS_V_ENV_HEADER_SIZE;
  if (!((uint64_t)e->body_size[i] <= e->max_body_size)) return PRAOS_V_ENV_BLOCK_SIZE;
  return PRAOS_V_OK;
}

// OCert counters of the fold, indexed densely: slot k < npools is pool k of the epoch's
// distribution (caller order, found through the device's pool_idx), slots >= npools
// hold issuers outside it (keys from the incoming state, or headers whose issuer the
// distribution lacks).  has[k] = the praosStateOCertCounters map has the key.
struct CounterTab {
  std::vector<uint64_t> ctr;
  std::vector<uint8_t> has;
  std::vector<std::string> extra_keys;
  std::map<std::string, uint32_t> extra;
};

static uint32_t counter_slot(const std::map<std::string, int32_t>& by_hash, CounterTab& T, const uint8_t* hash28) {
  const std::string k((const char*)hash28, 28);
  auto p = by_hash.find(k);
  if (p != by_hash.end()) return (uint32_t)p->second;
  auto e = T.extra.find(k);
  if (e != T.extra.end()) return e->second;
  const uint32_t slot = (uint32_t)T.ctr.size();
  T.extra.emplace(k, slot);
  T.extra_keys.push_back(k);
  T.ctr.push_back(0);
  T.has.push_back(0);
  return slot;
}

static int fold_impl(praos_ctx* c, const praos_headers* h, const uint8_t* prev_hash, const uint8_t* prev_is_genesis,
                     const praos_out* crypto, praos_envelope* env, const praos_epoch_info* ei,
                     praos_chain_state* st, uint8_t* verdict, size_t* chain_stop, size_t* processed,
                     const praos_nonce* etas = nullptr, uint32_t netas = 0, const uint8_t* eta_idx = nullptr,
                     bool tpraos = false, const praos_nonce* extra_entropy = nullptr, uint16_t* failures = nullptr,
                     const praos_nonce* evol_after = nullptr, const rp_view* view = nullptr) {
  if (!c) return PRAOS_E_ARG;
  if (!h || !crypto || !crypto->bits || !crypto->nonce || !verdict || !ei || !st || !prev_hash) {
    c->err = "fold: a required pointer is NULL (headers, crypto bits / nonce, verdict, epoch info, state, prev_hash)";
    return PRAOS_E_ARG;
  }
  if (ei->epoch_length == 0 || st->m > st->cap || (st->cap && (!st->counter_hash28 || !st->counter))) {
    c->err = "fold: epoch_length 0 or a counter map without room";
    return PRAOS_E_ARG;
  }
  if (env && h->n && (!env->block_no || !env->header_hash || !env->header_size || !env->body_size)) {
    c->err = "fold: the envelope needs block_no, header_hash, header_size and body_size";
    return PRAOS_E_ARG;
  }
  if (!c->have_epoch) { c->err = "fold: no epoch installed (praos_set_epoch)"; return PRAOS_E_STATE; }
  if (eta_idx && (!etas || netas == 0)) { c->err = "fold: eta_idx without etas"; return PRAOS_E_ARG; }
  praos_nonce eta0{};
  eta0.neutral = c->eta0_neutral;
  if (!c->eta0_neutral) std::memcpy(eta0.hash, c->eta0, 32);
  auto epoch_of = [&](uint64_t s, bool* ok) -> uint64_t {
    *ok = s >= ei->epoch_base_slot;
    return ei->epoch_base_no + (*ok ? (s - ei->epoch_base_slot) / ei->epoch_length : 0);
  };
  // Working state W (the fold) and the returned state: the reference stops the
  // chain at the first invalid header, so *st is the state after the last valid
  // header before chain_stop.  Later headers keep being judged (would-be
  // verdicts) against W, which carries on as if the failing header were absent.
  struct Work {
    int32_t origin;
    uint64_t last_slot;
    praos_nonce evolving, candidate, epoch_nonce, lab, leb;
    EnvTip tip;
  };
  // the ledger view's pools: the batch's own (per-epoch replay) or the context's praos_set_epoch
  const uint32_t np = view ? view->npools : (uint32_t)c->pools.size();
  const praos_pool* vpools = view ? view->pools.data() : c->pools.data();
  const std::map<std::string, int32_t>& by_hash = view ? view->by_hash : c->pool_by_hash;
  CounterTab T;
  T.ctr.assign(np, 0);
  T.has.assign(np, 0);
  for (size_t k = 0; k < st->m; k++) {
    const uint32_t slot = counter_slot(by_hash, T, st->counter_hash28 + 28 * k);
    T.ctr[slot] = st->counter[k];
    T.has[slot] = 1;
  }
  Work W;
  if (env) {
    W.tip.origin = env->tip_is_origin;
    W.tip.slot = env->tip_slot;
    W.tip.block_no = env->tip_block_no;
    std::memcpy(W.tip.hash, env->tip_hash, 32);
  }
  W.origin = st->last_slot_origin;
  W.last_slot = st->last_slot;
  W.evolving = st->evolving; W.candidate = st->candidate; W.epoch_nonce = st->epoch_nonce;
  W.lab = st->lab; W.leb = st->last_epoch_block;
  bool frozen = false;
  Work F;                                            // state at the chain stop
  std::vector<uint64_t> Fctr;                        // and its counters (T is W's)
  std::vector<uint8_t> Fhas;
  size_t stop = h->n, i = 0;
  for (; i < h->n; i++) {
    const uint64_t slot = h->slot[i];
    bool ok = true;
    const uint64_t e_new = epoch_of(slot, &ok);
    if (!ok) { c->err = "slot before the epoch base"; return PRAOS_E_ARG; }
    // tickChainDepState (Praos.hs:407-431) with isNewEpoch (Ledger/Util.hs:27-40)
    const uint64_t e_old = W.origin ? 0 : epoch_of(W.last_slot, &ok);
    praos_nonce tick_epoch = W.epoch_nonce, tick_leb = W.leb;
    if (e_new > e_old) {
      tick_epoch = nonce_combine(W.candidate, W.leb);
      if (tpraos && extra_entropy) tick_epoch = nonce_combine(tick_epoch, *extra_entropy);   // TICKN
      tick_leb = W.lab;
    }
    // the crypto outputs of header i were computed for this nonce: a tick to another one
    // ends the fold (the caller re-verifies from here under the right nonce)
    if (eta_idx && eta_idx[i] >= netas) { c->err = "eta_idx out of range"; return PRAOS_E_ARG; }
    if (!nonce_eq(tick_epoch, eta_idx ? etas[eta_idx[i]] : eta0)) break;
    // the issuer's counter slot (hashKey of the cold key, Praos.hs:595-606)
    const int32_t pidx = crypto->pool_idx ? crypto->pool_idx[i] : -1;
    uint32_t k;
    if (pidx >= 0 && (uint32_t)pidx < np) {
      k = (uint32_t)pidx;
    } else {
      uint8_t hh[28];
      praos_host::blake2b(hh, 28, h->cold_vk + 32 * i, 32);
      k = counter_slot(by_hash, T, hh);
    }
    const uint64_t n = h->ocert_n[i];
    const bool has = T.has[k];
    uint8_t v;
    if (tpraos) {
      // currentIssueNo: the counter map, else 0 for a pool or a genesis delegate
      const bool known = has || k < np || c->gen_delegate_hashes.count(T.extra_keys[k - np]) > 0;
      const uint16_t f = (crypto->bits[i] & PRAOS_BIT_INPUT) ? 0 : tpraos_failures(crypto->bits[i], known,
                                                                                    has ? T.ctr[k] : 0, n);
      if (failures) failures[i] = f;
      v = (crypto->bits[i] & PRAOS_BIT_INPUT) ? PRAOS_V_INPUT : (f ? PRAOS_V_TPRAOS : PRAOS_V_OK);
    } else {
      v = header_verdict(crypto->bits[i], has || k < np, has ? T.ctr[k] : 0, n);
    }
    // validateHeader (HeaderValidation.hs:419-428): the envelope before the protocol checks
    if (env && v != PRAOS_V_INPUT) {
      const uint8_t ve = envelope_verdict(env, W.tip, h, prev_hash, prev_is_genesis, i);
      if (ve != PRAOS_V_OK) {
        v = ve;
        if (failures) failures[i] = 0;               // validateEnvelope failed: PRTCL does not run
      }
    }
    verdict[i] = v;
    if (v != PRAOS_V_OK) {
      if (!frozen) {
        F = W;
        Fctr = T.ctr;
        Fhas = T.has;
        frozen = true;
        stop = i;
      }
      continue;
    }
    // reupdateChainDepState (Praos.hs:468-502)
    W.epoch_nonce = tick_epoch;
    W.leb = tick_leb;
    W.origin = 0;
    W.last_slot = slot;
    W.lab.neutral = prev_is_genesis && prev_is_genesis[i];
    std::memset(W.lab.hash, 0, 32);
    if (!W.lab.neutral) std::memcpy(W.lab.hash, prev_hash + 32 * i, 32);
    praos_nonce eta{};
    std::memcpy(eta.hash, crypto->nonce + 32 * i, 32);
    eta.neutral = 0;
    // evol_after (the replay's nonce chain, run ahead as if every header were valid) equals
    // this chain up to the first invalid header; from there W skips the failed headers
    W.evolving = (evol_after && !frozen) ? evol_after[i] : nonce_combine(W.evolving, eta);
    const uint64_t first_next = ei->epoch_base_slot + (e_new - ei->epoch_base_no + 1) * ei->epoch_length;
    if (slot + ei->stability_window < first_next) W.candidate = W.evolving;
    T.ctr[k] = n;
    T.has[k] = 1;
    if (env) {                                       // HeaderState tip := getAnnTip hdr
      W.tip.origin = 0;
      W.tip.slot = slot;
      W.tip.block_no = env->block_no[i];
      std::memcpy(W.tip.hash, env->header_hash + 32 * i, 32);
    }
  }
  const Work& R = frozen ? F : W;
  const std::vector<uint64_t>& Rctr = frozen ? Fctr : T.ctr;
  const std::vector<uint8_t>& Rhas = frozen ? Fhas : T.has;
  size_t m = 0;
  for (size_t k = 0; k < Rhas.size(); k++) m += Rhas[k];
  if (m > st->cap) { c->err = "counter map capacity exceeded"; return PRAOS_E_ARG; }
  size_t j = 0;
  for (size_t k = 0; k < Rhas.size(); k++) {
    if (!Rhas[k]) continue;
    const uint8_t* key = k < np ? vpools[k].hash28 : (const uint8_t*)T.extra_keys[k - np].data();
    std::memcpy(st->counter_hash28 + 28 * j, key, 28);
    st->counter[j++] = Rctr[k];
  }
  st->m = m;
  st->last_slot_origin = R.origin;
  st->last_slot = R.last_slot;
  st->evolving = R.evolving; st->candidate = R.candidate; st->epoch_nonce = R.epoch_nonce;
  st->lab = R.lab; st->last_epoch_block = R.leb;
  if (env) {
    env->tip_is_origin = R.tip.origin;
    env->tip_slot = R.tip.slot;
    env->tip_block_no = R.tip.block_no;
    std::memcpy(env->tip_hash, R.tip.hash, 32);
  }
  if (chain_stop) *chain_stop = std::min(stop, i);
  if (processed) *processed = i;
  return PRAOS_OK;
}

int rp_fold(praos_ctx* c, const praos_headers* h, const uint8_t* prev_hash, const uint8_t* prev_is_genesis,
            const praos_out* crypto, praos_envelope* env, const praos_epoch_info* ei, praos_chain_state* st,
            const praos_nonce* etas, uint32_t k, const uint8_t* eta_idx, const praos_nonce* evolving_after,
            bool tpraos, const praos_nonce* extra_entropy, uint8_t* verdict, uint16_t* failures, size_t* chain_stop,
            size_t* processed, const rp_view* view) {
  if (!etas || !eta_idx || k == 0) return PRAOS_E_ARG;
  return fold_impl(c, h, prev_hash, prev_is_genesis, crypto, env, ei, st, verdict, chain_stop, processed, etas, k,
                   eta_idx, tpraos, extra_entropy, failures, evolving_after, view);
}

extern "C" {

int praos_update_chain_dep_state(praos_ctx* c, const praos_headers* h, const uint8_t* prev_hash,
                                 const uint8_t* prev_is_genesis, const praos_out* crypto,
                                 const praos_epoch_info* ei, praos_chain_state* st, uint8_t* verdict,
                                 size_t* chain_stop, size_t* processed) {
  return fold_impl(c, h, prev_hash, prev_is_genesis, crypto, nullptr, ei, st, verdict, chain_stop, processed);
}

int praos_ticked_epoch_nonce(const praos_chain_state* st, const praos_epoch_info* ei, uint64_t slot,
                             praos_nonce* out) {
  if (!st || !ei || !out || ei->epoch_length == 0 || slot < ei->epoch_base_slot) return PRAOS_E_ARG;
  auto epoch_of = [&](uint64_t s) {
    return ei->epoch_base_no + (s < ei->epoch_base_slot ? 0 : (s - ei->epoch_base_slot) / ei->epoch_length);
  };
  const uint64_t e_old = st->last_slot_origin ? 0 : epoch_of(st->last_slot);
  *out = epoch_of(slot) > e_old ? nonce_combine(st->candidate, st->last_epoch_block) : st->epoch_nonce;
  return PRAOS_OK;
}

int praos_tpraos_ticked_epoch_nonce(const praos_chain_state* st, const praos_epoch_info* ei, uint64_t slot,
                                    const praos_nonce* extra_entropy, praos_nonce* out) {
  if (!st || !ei || !out || ei->epoch_length == 0 || slot < ei->epoch_base_slot) return PRAOS_E_ARG;
  auto epoch_of = [&](uint64_t s) {
    return ei->epoch_base_no + (s < ei->epoch_base_slot ? 0 : (s - ei->epoch_base_slot) / ei->epoch_length);
  };
  const uint64_t e_old = st->last_slot_origin ? 0 : epoch_of(st->last_slot);
  if (epoch_of(slot) > e_old) {        // TICKN: eta_c ⭒ eta_h ⭒ extraEntropy
    *out = nonce_combine(st->candidate, st->last_epoch_block);
    if (extra_entropy) *out = nonce_combine(*out, *extra_entropy);
  } else {
    *out = st->epoch_nonce;
  }
  return PRAOS_OK;
}

int praos_validate_headers(praos_ctx* c, const praos_headers* h, const uint8_t* prev_hash,
                           const uint8_t* prev_is_genesis, const praos_out* crypto, praos_envelope* env,
                           const praos_epoch_info* ei, praos_chain_state* st, uint8_t* verdict, size_t* chain_stop,
                           size_t* processed) {
  if (!env) return PRAOS_E_ARG;
  return fold_impl(c, h, prev_hash, prev_is_genesis, crypto, env, ei, st, verdict, chain_stop, processed);
}

int praos_validate_headers_nonces(praos_ctx* c, const praos_headers* h, const uint8_t* prev_hash,
                                  const uint8_t* prev_is_genesis, const praos_out* crypto, praos_envelope* env,
                                  const praos_epoch_info* ei, praos_chain_state* st, const praos_nonce* etas,
                                  uint32_t k, const uint8_t* eta_idx, uint8_t* verdict, size_t* chain_stop,
                                  size_t* processed) {
  if (!eta_idx || !etas || k == 0) return PRAOS_E_ARG;
  return fold_impl(c, h, prev_hash, prev_is_genesis, crypto, env, ei, st, verdict, chain_stop, processed, etas, k,
                   eta_idx);
}

int praos_tpraos_update_chain_dep_state(praos_ctx* c, const praos_tpraos_headers* th, const uint8_t* prev_hash,
                                        const uint8_t* prev_is_genesis, const praos_tpraos_out* crypto,
                                        praos_envelope* env, const praos_epoch_info* ei,
                                        const praos_nonce* extra_entropy, praos_chain_state* st, uint8_t* verdict,
                                        uint16_t* failures, size_t* chain_stop, size_t* processed) {
  if (!th || !crypto) return PRAOS_E_ARG;
  praos_out o{};
  o.bits = crypto->bits;
  o.pool_idx = crypto->pool_idx;
  o.nonce = crypto->nonce;                           // mkNonceFromOutputVRF of the eta certificate
  return fold_impl(c, &th->h, prev_hash, prev_is_genesis, &o, env, ei, st, verdict, chain_stop, processed, nullptr, 0,
                   nullptr, true, extra_entropy, failures);
}



// ---------------------------------------------------------------- PraosState CBOR
// Serialise (PraosState c) (Praos.hs:274-310): encodeVersion 0 [lastSlot, counters,
// evolving, candidate, epoch, lab, lastEpochBlock]; WithOrigin: Origin = [0], At s =
// [1, s]; Nonce: NeutralNonce = [0], Nonce h = [1, bytes(32)]; counters = CBOR map
// KeyHash (bytes 28) -> Word64 in ascending key order (Data.Map).  Shortest-form heads.
namespace {
struct CborW {
  uint8_t* out;
  size_t cap, n;
  void byte(uint32_t b) { if (n < cap) out[n] = (uint8_t)b; n++; }
  void head(uint32_t mt, uint64_t v) {
    if (v < 24) { byte((mt << 5) | (uint32_t)v); return; }
    const int nb = v < 256 ? 1 : v < 65536 ? 2 : v < (1ull << 32) ? 4 : 8;
    byte((mt << 5) | (nb == 1 ? 24u : nb == 2 ? 25u : nb == 4 ? 26u : 27u));
    for (int k = nb - 1; k >= 0; k--) byte((uint32_t)(v >> (8 * k)));
  }
  void bytes(const uint8_t* p, size_t len) { head(2, len); for (size_t k = 0; k < len; k++) byte(p[k]); }
  void nonce(const praos_nonce& x) {
    if (x.neutral) { head(4, 1); head(0, 0); }
    else { head(4, 2); head(0, 1); bytes(x.hash, 32); }
  }
};
struct CborR {
  const uint8_t* p;
  size_t len, pos;
  bool ok = true;
  bool head(uint32_t want_mt, uint64_t* v) {
    if (!ok || pos >= len) return ok = false;
    const uint32_t ib = p[pos++], mt = ib >> 5, ai = ib & 31;
    if (mt != want_mt) return ok = false;
    if (ai < 24) { *v = ai; return true; }
    if (ai > 27) return ok = false;
    const int nb = 1 << (ai - 24);
    if (pos + nb > len) return ok = false;
    uint64_t x = 0;
    for (int k = 0; k < nb; k++) x = (x << 8) | p[pos++];
    *v = x;
    return true;
  }
  bool expect(uint32_t mt, uint64_t want) { uint64_t v; return head(mt, &v) && (v == want || (ok = false)); }
  bool bytes(uint8_t* dst, size_t n) {
    uint64_t l;
    if (!head(2, &l) || l != n || pos + n > len) return ok = false;
    std::memcpy(dst, p + pos, n);
    pos += n;
    return true;
  }
  bool nonce(praos_nonce& x) {
    uint64_t l, tag;
    if (!head(4, &l) || !head(0, &tag)) return false;
    std::memset(&x, 0, sizeof x);
    if (l == 1 && tag == 0) { x.neutral = 1; return true; }
    if (l == 2 && tag == 1) { x.neutral = 0; return bytes(x.hash, 32); }
    return ok = false;
  }
};
}  // namespace

extern "C" {

int praos_state_encode(const praos_chain_state* st, uint8_t* out, size_t cap, size_t* len) {
  if (!st || !len || (cap && !out) || (st->m && (!st->counter_hash28 || !st->counter))) return PRAOS_E_ARG;
  std::vector<size_t> order(st->m);
  for (size_t k = 0; k < st->m; k++) order[k] = k;
  std::sort(order.begin(), order.end(), [&](size_t a, size_t b) {
    return std::memcmp(st->counter_hash28 + 28 * a, st->counter_hash28 + 28 * b, 28) < 0;
  });
  for (size_t k = 1; k < order.size(); k++)
    if (!std::memcmp(st->counter_hash28 + 28 * order[k - 1], st->counter_hash28 + 28 * order[k], 28))
      return PRAOS_E_ARG;                                   // duplicate key: not a Map
  CborW w{out, cap, 0};
  w.head(4, 2); w.head(0, 0);                               // encodeVersion 0
  w.head(4, 7);
  if (st->last_slot_origin) { w.head(4, 1); w.head(0, 0); }
  else { w.head(4, 2); w.head(0, 1); w.head(0, st->last_slot); }
  w.head(5, st->m);
  for (size_t k : order) { w.bytes(st->counter_hash28 + 28 * k, 28); w.head(0, st->counter[k]); }
  w.nonce(st->evolving); w.nonce(st->candidate); w.nonce(st->epoch_nonce); w.nonce(st->lab);
  w.nonce(st->last_epoch_block);
  *len = w.n;
  return w.n <= cap ? PRAOS_OK : PRAOS_E_ARG;
}

int praos_state_decode(const uint8_t* in, size_t len, praos_chain_state* st) {
  if (!in || !st || (st->cap && (!st->counter_hash28 || !st->counter))) return PRAOS_E_ARG;
  CborR r{in, len, 0};
  uint64_t v, tag, m;
  r.expect(4, 2); r.expect(0, 0); r.expect(4, 7);
  if (!r.ok) return PRAOS_E_ARG;
  if (!r.head(4, &v) || !r.head(0, &tag)) return PRAOS_E_ARG;
  if (v == 1 && tag == 0) { st->last_slot_origin = 1; st->last_slot = 0; }
  else if (v == 2 && tag == 1 && r.head(0, &st->last_slot)) st->last_slot_origin = 0;
  else return PRAOS_E_ARG;
  if (!r.head(5, &m) || m > st->cap) return PRAOS_E_ARG;
  for (size_t k = 0; k < m; k++) {
    if (!r.bytes(st->counter_hash28 + 28 * k, 28) || !r.head(0, &st->counter[k])) return PRAOS_E_ARG;
    if (k && std::memcmp(st->counter_hash28 + 28 * (k - 1), st->counter_hash28 + 28 * k, 28) >= 0)
      return PRAOS_E_ARG;                                   // Data.Map decoding wants ascending keys
  }
  st->m = m;
  if (!r.nonce(st->evolving) || !r.nonce(st->candidate) || !r.nonce(st->epoch_nonce) || !r.nonce(st->lab) ||
      !r.nonce(st->last_epoch_block))
    return PRAOS_E_ARG;
  return r.pos == len ? PRAOS_OK : PRAOS_E_ARG;
}

}  // extern "C"

// ---------------------------------------------------------------- generator
}  // extern "C"
static int synthesize_impl(praos_ctx* c, const praos_synth_params* sp, const praos_params* params,
                           const uint8_t eta0[32], praos_pool* pools_out, uint64_t* slot, uint8_t* cold_vk,
                           uint8_t* vrf_vk, uint8_t* vrf_out, uint8_t* vrf_proof, uint8_t* hot_vk, uint64_t* ocert_n,
                           uint64_t* ocert_c0, uint8_t* ocert_sig, uint8_t* kes_sig, uint64_t* body_off,
                           uint32_t* body_len, uint8_t* body_bytes, uint8_t* corrupted, int tpraos,
                           uint8_t* leader_out, uint8_t* leader_proof) {
  if (!c || !sp || !params || sp->npools == 0 || params->slots_per_kes_period == 0) return PRAOS_E_ARG;
  HIPCHK(c, hipSetDevice(c->device));
  const size_t n = sp->n, np = sp->npools;
  // body_len 0: genuine CBOR bodies, PRAOS_SIGNED_STRIDE (Praos HeaderBody) or
  // TP_SIGNED_STRIDE (TPraos BHBody) bytes per header
  const size_t bstride = sp->body_len ? (((size_t)sp->body_len + 7) & ~(size_t)7)
                                      : (size_t)(tpraos ? TP_SIGNED_STRIDE : PRAOS_SIGNED_STRIDE);
  Scratch s(c);
  uint32_t master[8], e0[8] = {0};
  std::memcpy(master, sp->seed, 32);
  if (eta0) std::memcpy(e0, eta0, 32);
  auto dmaster = s.up(master, 32);
  auto de0 = s.up(e0, 32);
  auto cold_seed = s.zeros<uint32_t>(32 * np);
  auto cold_pk = s.zeros<uint32_t>(32 * np);
  auto vrf_seed = s.zeros<uint32_t>(32 * np);
  auto vrf_pk = s.zeros<uint32_t>(32 * np);
  auto kes_seed = s.zeros<uint32_t>(32 * np);
  auto ph = s.zeros<uint8_t>(28 * np);
  auto pv = s.zeros<uint8_t>(32 * np);
  const size_t nk = sp->nkes ? std::min<size_t>(sp->nkes, np) : np;
  auto leaf_seed = s.zeros<uint32_t>(32 * nk * 64);
  auto tree = s.zeros<uint32_t>(32 * nk * 128);
  auto scratch = s.zeros<uint8_t>(48 * n);
  auto dslot = s.zeros<uint64_t>(8 * n);
  auto dcold = s.zeros<uint8_t>(32 * n);
  auto dvrfvk = s.zeros<uint8_t>(32 * n);
  auto dvout = s.zeros<uint8_t>(64 * n);
  auto dproof = s.zeros<uint8_t>(80 * n);
  auto dhot = s.zeros<uint8_t>(32 * n);
  auto dn = s.zeros<uint64_t>(8 * n);
  auto dc0 = s.zeros<uint64_t>(8 * n);
  auto dosig = s.zeros<uint8_t>(64 * n);
  auto dksig = s.zeros<uint8_t>(448 * n);
  auto doff = s.zeros<uint64_t>(8 * n);
  auto dlen = s.zeros<uint32_t>(4 * n);
  auto dbody = s.zeros<uint8_t>(bstride * n + 8);
  auto dcor = s.zeros<uint8_t>(n);
  auto dlout = s.zeros<uint8_t>(tpraos ? 64 * n : 16);
  auto dlproof = s.zeros<uint8_t>(tpraos ? 80 * n : 16);
  const uint8_t* dbh = sp->body_hash ? s.up(sp->body_hash, 32 * n) : nullptr;   // caller's hbBodyHash values
  if ((sp->sched_slot == nullptr) != (sp->sched_pool == nullptr)) return PRAOS_E_ARG;
  if (sp->sched_pool)
    for (size_t i = 0; i < n; i++)
      if (sp->sched_pool[i] >= np) { c->err = "sched_pool out of range"; return PRAOS_E_ARG; }
  const uint64_t* dss = sp->sched_slot ? s.up(sp->sched_slot, 8 * n) : nullptr;
  const uint32_t* dsp = sp->sched_pool ? s.up(sp->sched_pool, 4 * n) : nullptr;
  const bool link = sp->link_prev != 0;
  if (link && sp->body_len != 0) { c->err = "link_prev needs CBOR bodies (body_len 0)"; return PRAOS_E_ARG; }
  auto dleaf = s.zeros<uint32_t>(4 * n);
  auto dprev0 = link && sp->prev0 ? s.up(sp->prev0, 32) : nullptr;
  auto dlkeys = s.zeros<uint32_t>(link ? 4 * 24 * (size_t)nk * 64 : 16);   // per KES leaf: a, r, R (k_synth_link_keys)
  auto dhh = s.zeros<uint8_t>(link ? 32 * n : 16);
  if (!s.ok) { c->err = "alloc"; return PRAOS_E_OOM; }
  uint64_t salt = 0;
  std::memcpy(&salt, sp->seed, 8);
  launch_synth_pools(dim3(nblocks(np, NT)), dim3(NT), c->stream, (uint32_t)np, c->btab, dmaster,
                     cold_seed, cold_pk, vrf_seed, vrf_pk, kes_seed, ph, pv);
  launch_synth_kes_leaves(dim3(nblocks(nk * 64, NT)), dim3(NT), c->stream, (uint32_t)nk, c->btab,
                     kes_seed, leaf_seed, tree);
  launch_synth_kes_tree(dim3(nblocks(nk, 64)), dim3(64), c->stream, (uint32_t)nk, tree);
  if (n) {
    launch_synth_headers(dim3(nblocks(n, NT)), dim3(NT), c->stream, n, c->btab, (uint32_t)np,
                       (uint32_t)nk, sp->first_slot, sp->slot_stride, params->slots_per_kes_period, sp->body_len, salt, de0,
                       eta0 ? 0 : 1, cold_seed, cold_pk, vrf_seed, vrf_pk, leaf_seed, tree, scratch, dslot, dcold,
                       dvrfvk, dvout, dproof, dhot, dn, dc0, dosig, dksig, doff, dlen, dbody, tpraos, dlout, dlproof,
                       sp->body_len == 0 ? dbh : nullptr, dss, dsp, sp->block_no0, dleaf);
    if (link)
      launch_synth_link(c->stream, n, c->btab, dprev0, leaf_seed, (uint32_t)(nk * 64), dlkeys, tree, dleaf, dbody, doff,
                        dlen, dksig, dhh, (uint32_t)bstride);
    launch_synth_corrupt(dim3(nblocks(n, 256)), dim3(256), c->stream, n, sp->corrupt_per_10000,
                       salt, dosig, dksig, dproof, dvout, dbody, doff, dlen, dcor, tpraos ? dlproof : nullptr,
                       sp->body_len == 0 ? (tpraos ? 2 : 1) : 0, sp->corrupt_fields ? sp->corrupt_fields : 0x1fu, dcold, dhot, dn,
                       dc0);
  }
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipStreamSynchronize(c->stream));
  std::vector<uint8_t> hh(28 * np), vv(32 * np);
  HIPCHK(c, hipMemcpy(hh.data(), ph, 28 * np, hipMemcpyDeviceToHost));
  HIPCHK(c, hipMemcpy(vv.data(), pv, 32 * np, hipMemcpyDeviceToHost));
  if (pools_out)
    for (size_t p = 0; p < np; p++) {
      std::memcpy(pools_out[p].hash28, &hh[28 * p], 28);
      std::memcpy(pools_out[p].vrf_hash32, &vv[32 * p], 32);
    }
  if (n) {
    auto dn2h = [&](void* h, const void* d, size_t bytes) -> int {
      if (h) HIPCHK(c, hipMemcpy(h, d, bytes, hipMemcpyDeviceToHost));
      return PRAOS_OK;
    };
    int r = PRAOS_OK;
    r |= dn2h(slot, dslot, 8 * n); r |= dn2h(cold_vk, dcold, 32 * n); r |= dn2h(vrf_vk, dvrfvk, 32 * n);
    r |= dn2h(vrf_out, dvout, 64 * n); r |= dn2h(vrf_proof, dproof, 80 * n); r |= dn2h(hot_vk, dhot, 32 * n);
    r |= dn2h(ocert_n, dn, 8 * n); r |= dn2h(ocert_c0, dc0, 8 * n); r |= dn2h(ocert_sig, dosig, 64 * n);
    r |= dn2h(kes_sig, dksig, 448 * n); r |= dn2h(body_off, doff, 8 * n); r |= dn2h(body_len, dlen, 4 * n);
    r |= dn2h(body_bytes, dbody, bstride * n + 8); r |= dn2h(corrupted, dcor, n);
    if (tpraos) { r |= dn2h(leader_out, dlout, 64 * n); r |= dn2h(leader_proof, dlproof, 80 * n); }
    if (link) r |= dn2h(sp->header_hash, dhh, 32 * n);
    if (r != PRAOS_OK) return PRAOS_E_HIP;
  }
  return PRAOS_OK;
}
extern "C" {

int praos_synthesize(praos_ctx* c, const praos_synth_params* sp, const praos_params* params, const uint8_t eta0[32],
                     praos_pool* pools_out, uint64_t* slot, uint8_t* cold_vk, uint8_t* vrf_vk, uint8_t* vrf_out,
                     uint8_t* vrf_proof, uint8_t* hot_vk, uint64_t* ocert_n, uint64_t* ocert_c0, uint8_t* ocert_sig,
                     uint8_t* kes_sig, uint64_t* body_off, uint32_t* body_len, uint8_t* body_bytes,
                     uint8_t* corrupted) {
  return synthesize_impl(c, sp, params, eta0, pools_out, slot, cold_vk, vrf_vk, vrf_out, vrf_proof, hot_vk, ocert_n,
                         ocert_c0, ocert_sig, kes_sig, body_off, body_len, body_bytes, corrupted, 0, nullptr, nullptr);
}

int praos_synthesize_tpraos(praos_ctx* c, const praos_synth_params* sp, const praos_params* params,
                            const uint8_t eta0[32], praos_pool* pools_out, uint64_t* slot, uint8_t* cold_vk,
                            uint8_t* vrf_vk, uint8_t* vrf_out, uint8_t* vrf_proof, uint8_t* hot_vk, uint64_t* ocert_n,
                            uint64_t* ocert_c0, uint8_t* ocert_sig, uint8_t* kes_sig, uint64_t* body_off,
                            uint32_t* body_len, uint8_t* body_bytes, uint8_t* leader_out, uint8_t* leader_proof,
                            uint8_t* corrupted) {
  if (!leader_out || !leader_proof) return PRAOS_E_ARG;
  return synthesize_impl(c, sp, params, eta0, pools_out, slot, cold_vk, vrf_vk, vrf_out, vrf_proof, hot_vk, ocert_n,
                         ocert_c0, ocert_sig, kes_sig, body_off, body_len, body_bytes, corrupted, 1, leader_out,
                         leader_proof);
}

int praos_leader_schedule(praos_ctx* c, const uint8_t seed[32], uint32_t npools, const uint8_t* sigma_fp,
                          const praos_params* params, const uint8_t eta0[32], uint64_t first_slot, uint64_t nslots,
                          int tpraos, int32_t* leader) {
  if (!c || !seed || npools == 0 || !sigma_fp || !params || (nslots && !leader)) return PRAOS_E_ARG;
  if (nslots > (1ull << 32)) { c->err = "nslots > 2^32: split the range"; return PRAOS_E_ARG; }
  HIPCHK(c, hipSetDevice(c->device));
  if (nslots == 0) return PRAOS_OK;
  std::vector<uint32_t> thr(4 * (size_t)npools);
  for (uint32_t p = 0; p < npools; p++)
    if (!praos_host::leader_x_raw((uint8_t*)&thr[4 * p], sigma_fp + 16 * (size_t)p, params->c_raw)) {
      c->err = "sigma * activeSlotLog out of range";
      return PRAOS_E_ARG;
    }
  Scratch s(c);
  uint32_t master[8], e0[8] = {0};
  std::memcpy(master, seed, 32);
  if (eta0) std::memcpy(e0, eta0, 32);
  const size_t np = npools;
  auto dmaster = s.up(master, 32);
  auto de0 = s.up(e0, 32);
  auto cold_seed = s.zeros<uint32_t>(32 * np);
  auto cold_pk = s.zeros<uint32_t>(32 * np);
  auto vrf_seed = s.zeros<uint32_t>(32 * np);
  auto vrf_pk = s.zeros<uint32_t>(32 * np);
  auto kes_seed = s.zeros<uint32_t>(32 * np);
  auto vrf_x = s.zeros<uint32_t>(32 * np);
  auto ph = s.zeros<uint8_t>(28 * np);
  auto pv = s.zeros<uint8_t>(32 * np);
  auto dthr = s.up(thr.data(), 16 * np);
  auto dlead = s.up<int32_t>(nullptr, 4 * nslots);
  if (!s.ok) { c->err = "alloc"; return PRAOS_E_OOM; }
  launch_synth_pools(dim3(nblocks(np, NT)), dim3(NT), c->stream, (uint32_t)np, c->btab, dmaster, cold_seed, cold_pk,
                     vrf_seed, vrf_pk, kes_seed, ph, pv);
  launch_synth_vrf_scalar(dim3(nblocks(np, 64)), dim3(64), c->stream, (uint32_t)np, vrf_seed, vrf_x);
  HIPCHK(c, hipMemsetD32Async((hipDeviceptr_t)dlead, 0x7fffffff, nslots, c->stream));
  // pool chunks in forger order; a slot led by an earlier chunk is skipped by later ones
  constexpr uint32_t CH = 32;
  for (uint32_t p0 = 0; p0 < npools; p0 += CH) {
    const uint32_t pn = std::min(CH, npools - p0);
    const uint64_t lanes = nslots * pn;
    if (lanes / NT + 1 > 0x7fffffffull) { c->err = "range too large"; return PRAOS_E_ARG; }
    launch_synth_leader_search(dim3((unsigned)((lanes + NT - 1) / NT)), dim3(NT), c->stream, first_slot, nslots, p0,
                               pn, vrf_x, vrf_pk, dthr, de0, eta0 ? 0 : 1, (int)params->f_is_one, tpraos, dlead);
  }
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipStreamSynchronize(c->stream));
  HIPCHK(c, hipMemcpy(leader, dlead, 4 * nslots, hipMemcpyDeviceToHost));
  for (uint64_t k = 0; k < nslots; k++)
    if (leader[k] == 0x7fffffff) leader[k] = -1;
  return PRAOS_OK;
}

// ---- TPraos overlay schedule (cardano-protocol-tpraos Rules/Overlay.hs, restated):
//   isOverlaySlot firstSlotNo d slot = step s < step (s + 1), step x = ceiling (x * d),
//     s = slot - firstSlotNo;
//   classifyOverlaySlot: position = ceiling (s * d); active iff position mod ascInv == 0,
//     ascInv = floor (1 / activeSlotVal f); genesis key = Set.elemAt ((position div ascInv)
//     mod |gkeys|) gkeys (ascending byte order of the 28-byte key hashes).
int praos_set_overlay(praos_ctx* c, const praos_overlay* ov) {
  if (!c) return PRAOS_E_ARG;
  if (!ov) {
    c->ovl_on = false;
    c->gen_delegs.clear();
    c->gen_delegate_hashes.clear();
    return PRAOS_OK;
  }
  // d = 0 keeps the genesis delegates for the OCERT counter rule only (currentIssueNo)
  if (ov->d_den == 0 || ov->d_num > ov->d_den || ov->asc_num == 0 || ov->asc_den == 0 || ov->asc_num > ov->asc_den ||
      ov->epoch_length == 0 || (ov->n_gen_delegs && !ov->gen_delegs) || (ov->d_num && ov->n_gen_delegs == 0))
    return PRAOS_E_ARG;
  std::vector<praos_gen_deleg> g(ov->gen_delegs, ov->gen_delegs + ov->n_gen_delegs);
  std::sort(g.begin(), g.end(), [](const praos_gen_deleg& a, const praos_gen_deleg& b) {
    return std::memcmp(a.genesis_hash28, b.genesis_hash28, 28) < 0;
  });
  for (size_t k = 1; k < g.size(); k++)
    if (std::memcmp(g[k - 1].genesis_hash28, g[k].genesis_hash28, 28) == 0) return PRAOS_E_ARG;   // a Map
  if (c->device >= 0 && ov->d_num) {
    std::vector<uint32_t> t(16 * g.size(), 0);
    for (size_t k = 0; k < g.size(); k++) {
      std::memcpy(&t[16 * k], g[k].delegate_hash28, 28);
      std::memcpy(&t[16 * k + 8], g[k].vrf_hash32, 32);
    }
    HIPCHK(c, hipSetDevice(c->device));
    (void)hipStreamSynchronize(c->stream);
    (void)hipFree(c->d_gen);
    c->d_gen = nullptr;
    c->ovl_on = false;
    HIPCHK(c, hipMalloc(&c->d_gen, 4 * t.size()));
    HIPCHK(c, hipMemcpy(c->d_gen, t.data(), 4 * t.size(), hipMemcpyHostToDevice));
  }
  c->ovl_d_num = ov->d_num;
  c->ovl_d_den = ov->d_den;
  c->ovl_asc_inv = ov->asc_den / ov->asc_num;          // floor (1 / f), >= 1
  c->ovl_base = ov->epoch_base_slot;
  c->ovl_len = ov->epoch_length;
  c->gen_delegs.swap(g);
  c->gen_delegate_hashes.clear();
  for (const auto& e : c->gen_delegs) c->gen_delegate_hashes.insert(std::string((const char*)e.delegate_hash28, 28));
  c->ovl_on = ov->d_num != 0;
  return PRAOS_OK;
}

static int32_t overlay_class(const praos_ctx* c, uint64_t slot) {
  if (!c->ovl_on || slot < c->ovl_base) return -1;
  const uint64_t first = c->ovl_base + (slot - c->ovl_base) / c->ovl_len * c->ovl_len;
  const unsigned __int128 x = slot - first;
  auto step = [&](unsigned __int128 v) {             // ceiling (v * d), v * d_num < 2^128
    const unsigned __int128 num = v * c->ovl_d_num;
    return (num + c->ovl_d_den - 1) / c->ovl_d_den;
  };
  const unsigned __int128 position = step(x);
  if (!(position < step(x + 1))) return -1;
  if (position % c->ovl_asc_inv != 0) return -2;
  return (int32_t)((position / c->ovl_asc_inv) % c->gen_delegs.size());
}

int praos_overlay_classify(praos_ctx* c, size_t n, const uint64_t* slots, int32_t* cls) {
  if (!c || (n && (!slots || !cls))) return PRAOS_E_ARG;
  for (size_t i = 0; i < n; i++) cls[i] = overlay_class(c, slots[i]);
  return PRAOS_OK;
}

static int tpraos_download(praos_ctx* c, praos_batch* b, const uint8_t* dbeta_l, praos_tpraos_out* out) {
  const size_t n = b->n;
  HIPCHK(c, hipStreamSynchronize(c->stream));
  HIPCHK(c, d2h(c, out->bits, b->bits, 2 * n));
  if (out->pool_idx) HIPCHK(c, d2h(c, out->pool_idx, b->pool_idx, 4 * n));
  if (out->beta_eta) HIPCHK(c, d2h(c, out->beta_eta, b->beta, 64 * n));
  if (out->beta_leader) HIPCHK(c, d2h(c, out->beta_leader, dbeta_l, 64 * n));
  if (out->nonce) HIPCHK(c, d2h(c, out->nonce, b->nonce, 32 * n));
  return PRAOS_OK;
}

int praos_verify_tpraos_headers(praos_ctx* c, const praos_tpraos_headers* th, praos_tpraos_out* out) {
  if (!c || !th || !out || !out->bits || !th->leader_out || !th->leader_proof) return PRAOS_E_ARG;
  if (!c->have_epoch) return PRAOS_E_STATE;
  const size_t n = th->h.n;
  if (n == 0) return PRAOS_OK;
  praos_batch* b = praos_batch_upload(c, &th->h);
  if (!b) return PRAOS_E_OOM;
  uint8_t *dlout = nullptr, *dlproof = nullptr, *dbeta_l = nullptr;
  int rc = PRAOS_OK;
  if (dalloc(b, &dlout, 64 * n) != hipSuccess || dalloc(b, &dlproof, 80 * n) != hipSuccess ||
      dalloc(b, &dbeta_l, 64 * n) != hipSuccess) {
    praos_batch_free(c, b);
    return PRAOS_E_OOM;
  }
  auto body = [&]() -> int {
    HIPCHK(c, hipMemcpy(dlout, th->leader_out, 64 * n, hipMemcpyHostToDevice));
    HIPCHK(c, hipMemcpy(dlproof, th->leader_proof, 80 * n, hipMemcpyHostToDevice));
    b->tp_only = true;
    b->lead_out = dlout;
    b->lead_proof = dlproof;
    b->beta_l = dbeta_l;
    const int r = praos_batch_run(c, b);
    return r == PRAOS_OK ? tpraos_download(c, b, dbeta_l, out) : r;
  };
  rc = body();
  praos_batch_free(c, b);
  return rc;
}

praos_batch* praos_batch_upload_tpraos_bytes(praos_ctx* c, const praos_header_bytes* in) {
  return upload_bytes_impl(c, in, true);
}

int praos_batch_download_tpraos(praos_ctx* c, praos_batch* b, praos_tpraos_out* out) {
  if (!c || !b || !out || !out->bits || !b->tp_only) return PRAOS_E_ARG;
  HIPCHK(c, hipSetDevice(c->device));
  if (b->n == 0) return PRAOS_OK;
  return tpraos_download(c, b, b->beta_l, out);
}

int praos_tpraos_validate_headers_nonces(praos_ctx* c, const praos_tpraos_headers* th, const uint8_t* prev_hash,
                                         const uint8_t* prev_is_genesis, const praos_tpraos_out* crypto,
                                         praos_envelope* env, const praos_epoch_info* ei,
                                         const praos_nonce* extra_entropy, praos_chain_state* st,
                                         const praos_nonce* etas, uint32_t k, const uint8_t* eta_idx,
                                         uint8_t* verdict, uint16_t* failures, size_t* chain_stop,
                                         size_t* processed) {
  if (!th || !crypto || !etas || !eta_idx || k == 0) return PRAOS_E_ARG;
  praos_out o{};
  o.bits = crypto->bits;
  o.pool_idx = crypto->pool_idx;
  o.nonce = crypto->nonce;
  return fold_impl(c, &th->h, prev_hash, prev_is_genesis, &o, env, ei, st, verdict, chain_stop, processed, etas, k,
                   eta_idx, true, extra_entropy, failures);
}

int praos_verify_tpraos_header_bytes(praos_ctx* c, const praos_header_bytes* in, praos_tpraos_out* out,
                                     praos_decoded* dec, uint8_t* leader_out, uint8_t* leader_proof) {
  if (!c || !in || !out || !out->bits) return PRAOS_E_ARG;
  if (!c->have_epoch) return PRAOS_E_STATE;
  const size_t n = in->n;
  if (n == 0) return PRAOS_OK;
  praos_batch* b = upload_bytes_impl(c, in, true);
  if (!b) return PRAOS_E_OOM;
  auto body = [&]() -> int {
    int r = praos_batch_run(c, b);             // decode, then the TPraos passes
    if (r == PRAOS_OK) r = tpraos_download(c, b, b->beta_l, out);
    if (r == PRAOS_OK && dec) r = praos_batch_download_decoded(c, b, dec);
    if (r == PRAOS_OK && leader_out) HIPCHK(c, d2h(c, leader_out, b->lead_out, 64 * n));
    if (r == PRAOS_OK && leader_proof) HIPCHK(c, d2h(c, leader_proof, b->lead_proof, 80 * n));
    return r;
  };
  const int rc = body();
  praos_batch_free(c, b);
  return rc;
}

// ---------------------------------------------------------------- debug entry points
int praos_debug_fe(praos_ctx* c, int op, size_t n, const uint8_t* a, const uint8_t* b, uint8_t* r) {
  if (!c || !a || !r) return PRAOS_E_ARG;
  HIPCHK(c, hipSetDevice(c->device));
  Scratch s(c);
  auto da = s.up(a, 32 * n);
  auto db = s.up(b ? b : a, 32 * n);
  auto dr = s.zeros<uint8_t>(32 * n);
  if (!s.ok) return PRAOS_E_OOM;
  launch_debug_fe(dim3(nblocks(n, 64)), dim3(64), c->stream, op, n, da, db, dr);
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipStreamSynchronize(c->stream));
  HIPCHK(c, hipMemcpy(r, dr, 32 * n, hipMemcpyDeviceToHost));
  return PRAOS_OK;
}

int praos_debug_sha512(praos_ctx* c, size_t n, const uint8_t* prefix, const uint64_t* msg_off, const uint32_t* msg_len,
                       const uint8_t* msg_bytes, size_t msg_bytes_len, uint8_t* out) {
  if (!c) return PRAOS_E_ARG;
  HIPCHK(c, hipSetDevice(c->device));
  std::vector<uint64_t> off(n);
  size_t total = 0;
  for (size_t i = 0; i < n; i++) { off[i] = total; total += (msg_len[i] + 7) & ~(size_t)7; }
  std::vector<uint8_t> arena(total + 16, 0);
  for (size_t i = 0; i < n; i++)
    if (msg_len[i]) std::memcpy(arena.data() + off[i], msg_bytes + msg_off[i], msg_len[i]);
  (void)msg_bytes_len;
  Scratch s(c);
  auto dp = s.up(prefix, 64 * n);
  auto doff = s.up(off.data(), 8 * n);
  auto dlen = s.up(msg_len, 4 * n);
  auto dmsg = s.up(arena.data(), arena.size());
  auto dout = s.zeros<uint8_t>(64 * n);
  if (!s.ok) return PRAOS_E_OOM;
  launch_debug_sha512(dim3(nblocks(n, 64)), dim3(64), c->stream, n, dp, doff, dlen, dmsg, dout);
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipStreamSynchronize(c->stream));
  HIPCHK(c, hipMemcpy(out, dout, 64 * n, hipMemcpyDeviceToHost));
  return PRAOS_OK;
}

int praos_debug_blake2b(praos_ctx* c, size_t n, const uint8_t* in64, uint8_t* out) {
  if (!c) return PRAOS_E_ARG;
  HIPCHK(c, hipSetDevice(c->device));
  Scratch s(c);
  auto di = s.up(in64, 64 * n);
  auto dout = s.zeros<uint8_t>(32 * n);
  if (!s.ok) return PRAOS_E_OOM;
  launch_debug_blake2b(dim3(nblocks(n, 64)), dim3(64), c->stream, n, di, dout);
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipStreamSynchronize(c->stream));
  HIPCHK(c, hipMemcpy(out, dout, 32 * n, hipMemcpyDeviceToHost));
  return PRAOS_OK;
}

int praos_debug_sc_reduce(praos_ctx* c, size_t n, const uint8_t* in64, uint8_t* out) {
  if (!c) return PRAOS_E_ARG;
  HIPCHK(c, hipSetDevice(c->device));
  Scratch s(c);
  auto di = s.up(in64, 64 * n);
  auto dout = s.zeros<uint8_t>(32 * n);
  if (!s.ok) return PRAOS_E_OOM;
  launch_debug_sc_reduce(dim3(nblocks(n, 64)), dim3(64), c->stream, n, di, dout);
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipStreamSynchronize(c->stream));
  HIPCHK(c, hipMemcpy(out, dout, 32 * n, hipMemcpyDeviceToHost));
  return PRAOS_OK;
}

int praos_debug_decode(praos_ctx* c, size_t n, const uint8_t* in32, uint8_t* out, uint8_t* ok) {
  if (!c) return PRAOS_E_ARG;
  HIPCHK(c, hipSetDevice(c->device));
  Scratch s(c);
  auto di = s.up(in32, 32 * n);
  auto dout = s.zeros<uint8_t>(32 * n);
  auto dok = s.zeros<uint8_t>(n);
  if (!s.ok) return PRAOS_E_OOM;
  launch_debug_decode(dim3(nblocks(n, 64)), dim3(64), c->stream, n, di, dout, dok);
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipStreamSynchronize(c->stream));
  HIPCHK(c, hipMemcpy(out, dout, 32 * n, hipMemcpyDeviceToHost));
  HIPCHK(c, hipMemcpy(ok, dok, n, hipMemcpyDeviceToHost));
  return PRAOS_OK;
}

int praos_debug_scalarmult_base(praos_ctx* c, size_t n, const uint8_t* sc, uint8_t* out) {
  if (!c) return PRAOS_E_ARG;
  HIPCHK(c, hipSetDevice(c->device));
  Scratch s(c);
  auto di = s.up(sc, 32 * n);
  auto dout = s.zeros<uint8_t>(32 * n);
  if (!s.ok) return PRAOS_E_OOM;
  launch_debug_smul_base(dim3(nblocks(n, NT)), dim3(NT), c->stream, n, c->btab, di, dout);
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipStreamSynchronize(c->stream));
  HIPCHK(c, hipMemcpy(out, dout, 32 * n, hipMemcpyDeviceToHost));
  return PRAOS_OK;
}

int praos_debug_leader(praos_ctx* c, size_t n, const uint8_t* leader, const uint8_t* x_raw16, uint8_t* is_leader,
                       int32_t* iters) {
  if (!c) return PRAOS_E_ARG;
  HIPCHK(c, hipSetDevice(c->device));
  Scratch s(c);
  auto dl = s.up(leader, 32 * n);
  auto dx = s.up(x_raw16, 16 * n);
  auto dres = s.zeros<uint8_t>(n);
  auto dit = s.zeros<int32_t>(4 * n);
  if (!s.ok) return PRAOS_E_OOM;
  launch_leader(dim3(nblocks(n, NT)), dim3(NT), c->stream, n, dl, (const int32_t*)nullptr, (const uint32_t*)nullptr,
                (const uint32_t*)dx, 0, 8, (const uint16_t*)nullptr, (const uint16_t*)nullptr,
                (const uint16_t*)nullptr, (uint16_t*)nullptr, dres, dit, (const uint16_t*)nullptr);
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipStreamSynchronize(c->stream));
  HIPCHK(c, hipMemcpy(is_leader, dres, n, hipMemcpyDeviceToHost));
  HIPCHK(c, hipMemcpy(iters, dit, 4 * n, hipMemcpyDeviceToHost));
  return PRAOS_OK;
}

int praos_debug_leader512(praos_ctx* c, size_t n, const uint8_t* leader64, const uint8_t* x_raw16, uint8_t* is_leader,
                          int32_t* iters) {
  if (!c) return PRAOS_E_ARG;
  HIPCHK(c, hipSetDevice(c->device));
  Scratch s(c);
  auto dl = s.up(leader64, 64 * n);
  auto dx = s.up(x_raw16, 16 * n);
  auto dres = s.zeros<uint8_t>(n);
  auto dit = s.zeros<int32_t>(4 * n);
  if (!s.ok) return PRAOS_E_OOM;
  launch_leader(dim3(nblocks(n, NT)), dim3(NT), c->stream, n, dl, (const int32_t*)nullptr, (const uint32_t*)nullptr,
                (const uint32_t*)dx, 0, 16, (const uint16_t*)nullptr, (const uint16_t*)nullptr,
                (const uint16_t*)nullptr, (uint16_t*)nullptr, dres, dit, (const uint16_t*)nullptr);
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipStreamSynchronize(c->stream));
  HIPCHK(c, hipMemcpy(is_leader, dres, n, hipMemcpyDeviceToHost));
  HIPCHK(c, hipMemcpy(iters, dit, 4 * n, hipMemcpyDeviceToHost));
  return PRAOS_OK;
}

int praos_debug_hash_to_curve(praos_ctx* c, size_t n, const uint8_t* pk, const uint8_t* alpha, uint8_t* out) {
  if (!c) return PRAOS_E_ARG;
  HIPCHK(c, hipSetDevice(c->device));
  Scratch s(c);
  auto dpk = s.up(pk, 32 * n);
  auto dal = s.up(alpha, 32 * n);
  auto dout = s.zeros<uint8_t>(32 * n);
  if (!s.ok) return PRAOS_E_OOM;
  launch_debug_h2c(dim3(nblocks(n, 64)), dim3(64), c->stream, n, dpk, dal, dout);
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipStreamSynchronize(c->stream));
  HIPCHK(c, hipMemcpy(out, dout, 32 * n, hipMemcpyDeviceToHost));
  return PRAOS_OK;
}

}  // extern "C"
