// praos_replay.hip -- db-analyser-style chain replay over an ImmutableDB directory
// (SURVEY.md sec. 8 row N3): host C++ on top of the library (its C ABI and the internal
// pipeline entry points of replay_internal.hpp).
//
// Mirrors the reference's streaming loop (DBAnalyser/Analysis.hs:815-847,
// processAllImmutableDB: ImmutableDB.streamAll, one iteratorNext per block) and its
// header-validation pass (benchmarkLedgerOps, :479-607: tick, then validateHeader),
// in batches: headers are read through the secondary index into batches of up to
// batch_max headers (any number of epochs, up to 256), decoded on the device, given their
// epoch nonces -- the nonce tickChainDepState (Praos.hs:407-431) reaches at each header,
// computed on the host from the certified VRF outputs as if every header were valid --
// crypto-checked under those nonces, and folded on the host (envelope, then
// updateChainDepState), which accepts a header only if the nonce its crypto ran with is the
// one the real fold ticks to.  One ledger view (pools, parameters) for the whole replay.
// Like the reference, the replay ends at the first invalid header.
//
// Host threads, up to RP_SLOTS (4) batches in flight per context:
//   reader (this thread): chunk files are memory-mapped; a batch is the secondary index's spans
//     of header bytes (coalesced, no host copy of the chunk);
//   parser: the chain's inputs of each header -- slot, prev hash, the nonce value of its
//     certified VRF output -- read on the host by a few workers (chain_fields), so the chain
//     never waits for the device;
//   uploader: the spans go from the mappings into the pinned staging buffers, H2D on the copy
//     stream, decode on the device and the decoded fields back (the fold's; the chain's only
//     for a batch the parser could not read);
//   nonce chain: the evolving-nonce Blake2b chain in header order (the one sequential piece
//     of work of the replay) and the per-header epoch nonces;
//   launcher: the batch's crypto run once it is decoded and its nonces are known;
//   fold: waits for the crypto bits, folds envelope + updateChainDepState reusing the nonce
//     chain's evolving nonces (no second Blake2b chain), writes the verdicts (after checking
//     that the host's reading of every decoded header is the device's).
//
// On-disk format (ImmutableDB, Storage/ImmutableDB/Impl): NNNNN.chunk holds the
// stored blocks back to back; NNNNN.secondary one 56-byte Entry per block
// (Impl/Index/Secondary.hs:93-128): blockOffset u64 BE, headerOffset u16 BE,
// headerSize u16 BE, checksum u32 BE, headerHash 32 bytes, blockOrEBB (slot) u64 BE.
// The primary index maps relative slots to entries and is not needed for a full
// sequential replay.  Chunks are read from 00000 upwards until one is missing.
#include <hip/hip_runtime.h>

#include "praos_hip.h"
#include "host_util.hpp"
#include "replay_internal.hpp"

#include <fcntl.h>
#include <pthread.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

void praos_set_error_(praos_ctx* c, const std::string& m);   // praos_api.hip
void rp_copy_pin(praos_ctx* c, const std::vector<int>& cpus);  // praos_api.hip
void praos_replay_scope_(praos_ctx* c, bool on);   // replay call scope: first error kept, pool-key store on

namespace {

bool read_file(const std::string& path, std::vector<uint8_t>& out) {
  FILE* f = std::fopen(path.c_str(), "rb");
  if (!f) return false;
  std::fseek(f, 0, SEEK_END);
  const long sz = std::ftell(f);
  std::fseek(f, 0, SEEK_SET);
  out.resize(sz > 0 ? (size_t)sz : 0);
  const bool ok = sz >= 0 && (out.empty() || std::fread(out.data(), 1, out.size(), f) == out.size());
  std::fclose(f);
  return ok;
}

uint64_t be(const uint8_t* p, int n) {
  uint64_t v = 0;
  for (int k = 0; k < n; k++) v = (v << 8) | p[k];
  return v;
}

double ms_since(std::chrono::steady_clock::time_point t0) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

// one chunk: its data file memory-mapped (read-only), its secondary index in memory
struct Chunk {
  const uint8_t* data = nullptr;
  size_t len = 0;
  void* map = nullptr;
  std::vector<uint8_t> sec;
  ~Chunk() {
    if (map) munmap(map, len);
  }
};

bool map_chunk(const std::string& path, Chunk& ch) {
  const int fd = open(path.c_str(), O_RDONLY);
  if (fd < 0) return false;
  struct stat st;
  if (fstat(fd, &st) != 0) { close(fd); return false; }
  ch.len = (size_t)st.st_size;
  if (ch.len) {
    void* m = mmap(nullptr, ch.len, PROT_READ, MAP_PRIVATE | MAP_POPULATE, fd, 0);
    if (m == MAP_FAILED) { close(fd); return false; }
    ch.map = m;
    ch.data = (const uint8_t*)m;
  }
  close(fd);
  return true;
}

// Streams (header bytes, slot) out of the chunk files, one chunk mapped at a time (a batch
// keeps the chunks it points into alive until its upload has read them).
struct ChunkReader {
  std::string dir, err;
  int chunk = 0;
  bool done = false;
  std::shared_ptr<Chunk> cur;
  size_t entry = 0, nentries = 0;
  void load_next() {
    char name[32];
    std::snprintf(name, sizeof name, "/%05d.chunk", chunk);
    auto ch = std::make_shared<Chunk>();
    if (!map_chunk(dir + name, *ch)) { done = true; cur.reset(); return; }
    std::snprintf(name, sizeof name, "/%05d.secondary", chunk);
    if (!read_file(dir + name, ch->sec) || ch->sec.size() % 56 != 0) {
      err = std::string("missing or malformed secondary index ") + (name + 1);
      done = true;
      cur.reset();
      return;
    }
    cur = ch;
    chunk++;
    entry = 0;
    nentries = cur->sec.size() / 56;
  }
  // the next entry, without consuming it; false at the end of the database
  bool peek(const uint8_t** hdr, uint32_t* len, uint64_t* slot, const uint8_t** hash = nullptr) {
    while (!done && entry >= nentries) load_next();
    if (done) return false;
    const uint8_t* e = cur->sec.data() + 56 * entry;
    const uint64_t boff = be(e, 8), hoff = be(e + 8, 2), hsz = be(e + 10, 2);
    if (boff > cur->len || hoff + hsz > cur->len - boff) {
      err = "secondary index entry outside its chunk (chunk " + std::to_string(chunk - 1) + ", entry " +
            std::to_string(entry) + ")";
      done = true;
      return false;
    }
    *hdr = cur->data + boff + hoff;
    *len = (uint32_t)hsz;
    *slot = be(e + 48, 8);
    if (hash) *hash = e + 16;
    return true;
  }
  void pop() { entry++; }
};

constexpr int SLOTS = RP_SLOTS;               // batches in flight (kept by the context between calls)

// Batch k's size cap (PRAOS_REPLAY_RAMP): ramp 1 = batch_max / 4, / 2, then batch_max; ramp 2 =
// batch_max / 8, / 4, / 2, 3/4, then batch_max.  (A geometric ramp from batch_max / 8 up by 1.4x
// per batch was measured slower before the host parse and the pinned decode downloads, 84 ->
// 132 ms on the C5 chain: many small device steps, profiles/r06/g_replay.)
constexpr int RP_RAMP_DEFAULT = 1;
size_t rp_ramp_cap(int ramp, uint64_t k, size_t batch_max) {
  static const size_t r1[][2] = {{1, 4}, {1, 2}}, r2[][2] = {{1, 8}, {1, 4}, {1, 2}, {3, 4}};
  const size_t (*r)[2] = ramp == 2 ? r2 : r1;
  const uint64_t nr = ramp == 2 ? 4 : ramp == 1 ? 2 : 0;
  return k < nr ? std::max<size_t>(1, batch_max * r[k][0] / r[k][1]) : batch_max;
}

// The nonce chain's inputs of a stored Praos header, read on the host (Praos/Header.hs HeaderRaw
// [body, kesSig], the 10-field HeaderBody as k_decode_praos reads it): the slot, the prev hash
// (or the genesis flag) and the header's nonce value, Blake2b-256(Blake2b-256("N" || certified
// VRF output)) as k_vrf_nonce computes it.  false: the header does not start the usual way (the
// batch's chain then waits for the device decode).  A header whose bytes go wrong further on is
// rejected by the device decode and the fold stops at it, whatever the chain assumed after it.
bool chain_fields(const uint8_t* h, uint32_t len, uint64_t* slot, uint8_t* prev, uint8_t* gen, uint8_t* nonce) {
  size_t pos = 0;
  auto head = [&](int want, uint64_t* v) -> bool {
    if (pos >= len) return false;
    const uint8_t ib = h[pos++];
    if ((ib >> 5) != want) return false;
    const int ai = ib & 31;
    if (ai < 24) { *v = (uint64_t)ai; return true; }
    if (ai > 27) return false;
    const int nb = 1 << (ai - 24);
    if (pos + (size_t)nb > len) return false;
    uint64_t x = 0;
    for (int k = 0; k < nb; k++) x = (x << 8) | h[pos++];
    *v = x;
    return true;
  };
  uint64_t v;
  auto bytes = [&](uint64_t n) -> const uint8_t* {
    if (!head(2, &v) || v != n || pos + n > len) return nullptr;
    const uint8_t* q = h + pos;
    pos += n;
    return q;
  };
  if (!head(4, &v) || v != 2 || !head(4, &v) || v != 10 || !head(0, &v) || !head(0, slot)) return false;
  if (pos < len && h[pos] == 0xF6) {
    pos++;
    *gen = 1;
    std::memset(prev, 0, 32);
  } else {
    const uint8_t* q = bytes(32);
    if (!q) return false;
    *gen = 0;
    std::memcpy(prev, q, 32);
  }
  if (!bytes(32) || !bytes(32) || !head(4, &v) || v != 2) return false;
  const uint8_t* out = bytes(64);
  if (!out) return false;
  uint8_t msg[65], nv[32];
  msg[0] = 'N';
  std::memcpy(msg + 1, out, 64);
  praos_host::blake2b(nv, 32, msg, 65);
  praos_host::blake2b(nonce, 32, nv, 32);
  return true;
}

// a few persistent workers for the host parse of a batch (run: f(t) on every worker, returns
// when all are done)
class ParPool {
 public:
  explicit ParPool(unsigned n) : nt_(n) {
    for (unsigned t = 0; t < nt_; t++) th_.emplace_back([this, t] { loop(t); });
  }
  ~ParPool() {
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

// Thread placement (PRAOS_REPLAY_PIN, read per call: 1 on, 0 off, unset = on for batches of
// 64k headers or more): the nonce chain -- the replay's one sequential piece of work, one
// Blake2b compression per header in order -- on a CPU of its own, the launcher, the fold and the
// reader on one each, and the contexts' staging copy threads on the rest, so the chain is never
// descheduled by the copies of the next batch.  Only with at least 8 CPUs in the process's mask.
// Measured on the C5 chain (863,780 headers, 2 epochs; profiles/r06/c_replay): the chain thread
// 62-65 ms pinned against 62-105 ms unpinned; 96k-header batches 9.6-9.8 -> 10.0-10.1 M headers/s
// on one context and 7.3-8.0 -> 9.0-9.3 M on a 2-member group; 48k-header batches slower pinned
// (5.4-5.5 vs 5.9-8.7 M: the device stage of the many small batches, cause not isolated), hence
// the size threshold.
struct Placement {
  bool on = false;
  std::vector<int> cpus;                      // the process's CPUs, in order
  cpu_set_t reader_was;
  bool reader_saved = false;
  static void pin_self(int cpu) {
    cpu_set_t set;
    CPU_ZERO(&set);
    CPU_SET(cpu, &set);
    (void)pthread_setaffinity_np(pthread_self(), sizeof set, &set);
  }
  void init(size_t batch_max) {
    const char* e = std::getenv("PRAOS_REPLAY_PIN");
    const bool want = e ? std::atoi(e) != 0 : batch_max >= 65536;
    if (!want) return;
    cpu_set_t set;
    CPU_ZERO(&set);
    if (sched_getaffinity(0, sizeof set, &set) != 0) return;
    for (int c = 0; c < CPU_SETSIZE; c++)
      if (CPU_ISSET(c, &set)) cpus.push_back(c);
    if (cpus.size() < 8) { cpus.clear(); return; }
    on = true;
  }
  int chain() const { return cpus[0]; }
  int launcher() const { return cpus[1]; }
  int folder() const { return cpus[2]; }         // (and the parse pool's coordinating thread)
  int reader() const { return cpus[3]; }
  int uploader() const { return cpus[4]; }       // its device syncs spin: a CPU of its own
  std::vector<int> copies() const { return std::vector<int>(cpus.begin() + 5, cpus.end()); }
};
constexpr size_t SPAN_GAP = 4096;             // headers this close share one uploaded span

}  // namespace

// TPraos mode (eras Shelley..Alonzo, HFEras.hs:43-49; TPraos.hs:361-387): stored BHeaders,
// the TPraos nonce rules -- the header's nonce is mkNonceFromOutputVRF of its eta
// certificate (Blake2b-256 of the output, no range extension) and TICKN adds the extra
// entropy (eta0 := eta_c ⭒ eta_h ⭒ extraEntropy) -- and the TPraos fold (PRTCL
// predicate-failure sets into failures[]).
//
// Several contexts (a praos_group, praos_group.hip): consecutive batches are dealt to the
// members in turn (batch k to member k mod m, each member with its own slots and copy /
// compute streams), the nonce chain and the fold stay single and in chain order (the fold
// on member 0's context), so the result is the one-context replay's, bit for bit.
int rp_replay(praos_ctx* const* mem, int m, const char* dir, const praos_pool* pools, uint32_t npools,
              const praos_params* params, const praos_epoch_info* ei, praos_envelope* env, praos_chain_state* st,
              size_t batch_max, uint8_t* verdicts, uint16_t* failures, size_t verdicts_cap,
              praos_replay_stats* stats, bool tpraos, const praos_nonce* extra_entropy,
              const praos_ledger_view* views, uint32_t nviews) {
  const auto t_base = std::chrono::steady_clock::now();   // (the stage trace's origin)
  praos_ctx* const ctx = m > 0 && mem ? mem[0] : nullptr;
  for (int q = 0; q < m; q++)
    if (!mem[q]) return PRAOS_E_ARG;
  for (int q = 0; q < m; q++) {     // submitted stored-bytes calls read the tables the replay swaps
    const int rd = praos_verify_drain(mem[q]);
    if (rd != PRAOS_OK) return rd;
  }
  if (!ctx || !dir || !params || (npools && !pools) || !ei || !env || !st || !stats || batch_max == 0 ||
      ei->epoch_length == 0 || (verdicts_cap && !verdicts) || (views && (nviews == 0 || tpraos)))
    return PRAOS_E_ARG;
  // The ledger views: one for the whole replay (pools + env's limits), or one per epoch range
  // (praos_replay_immutable_views: the LedgerView db-analyser forecasts for each epoch).
  struct View {
    uint64_t first_epoch;
    const praos_pool* pools;
    uint32_t npools;
    uint64_t prot, maxh, maxb;
  };
  std::vector<View> V;
  if (views) {
    for (uint32_t j = 0; j < nviews; j++) {
      const praos_ledger_view& w = views[j];
      if ((w.npools && !w.pools) || (j && w.first_epoch <= views[j - 1].first_epoch)) {
        praos_set_error_(ctx, "replay: ledger views must have pools and strictly increasing first_epoch");
        return PRAOS_E_ARG;
      }
      V.push_back({w.first_epoch, w.pools, w.npools, w.lv_prot_major, w.max_header_size, w.max_body_size});
    }
  } else {
    V.push_back({0, pools, npools, env->lv_prot_major, env->max_header_size, env->max_body_size});
  }
  auto view_of = [&](uint64_t e) -> int {     // the last view with first_epoch <= e, or -1
    int lo = -1;
    for (int a = 0, b = (int)V.size() - 1; a <= b;) {
      const int mid = (a + b) / 2;
      if (V[mid].first_epoch <= e) { lo = mid; a = mid + 1; } else { b = mid - 1; }
    }
    return lo;
  };
  // the fold's pools per view (host maps; the context's praos_set_epoch tables when one view)
  std::vector<std::unique_ptr<rp_view, std::function<void(rp_view*)>>> hv;
  if (views)
    for (const View& w : V) {
      rp_view* v = rp_view_make(ctx, w.pools, w.npools, params, false);
      if (!v) return PRAOS_E_ARG;
      hv.emplace_back(v, [ctx](rp_view* p) { rp_view_free(ctx, p); });
    }
  std::memset(stats, 0, sizeof *stats);
  ChunkReader rd;
  rd.dir = dir;
  auto epoch_of = [&](uint64_t s) {
    return s < ei->epoch_base_slot ? ei->epoch_base_no : ei->epoch_base_no + (s - ei->epoch_base_slot) / ei->epoch_length;
  };
  // resume (db-analyser --analyse-from a snapshot): a tip that is not Origin must be a
  // block of the database; replay starts right after it
  if (!env->tip_is_origin) {
    const uint8_t *p, *hash;
    uint32_t l;
    uint64_t s;
    bool found = false;
    while (rd.peek(&p, &l, &s, &hash) && s <= env->tip_slot) {
      rd.pop();
      stats->skipped++;
      if (s == env->tip_slot && std::memcmp(hash, env->tip_hash, 32) == 0) { found = true; break; }
    }
    if (!found) {
      praos_set_error_(ctx, rd.err.empty() ? "replay: the tip is not a block of the database" : rd.err);
      return PRAOS_E_ARG;
    }
  }
  // The ledger view (pools, parameters) is installed once (per view with views); the epoch
  // nonces travel with each batch, so a batch may span many epochs and stay large enough to fill
  // the device even when epochs are short.
  int v0 = 0;
  std::chrono::steady_clock::time_point t_peek0 = t_base, t_epoch0 = t_base;   // (setup's parts, traced)
  {
    praos_nonce eta0{};
    uint32_t l;
    uint64_t s0 = 0;
    const uint8_t* p;
    t_peek0 = std::chrono::steady_clock::now();
    if (rd.peek(&p, &l, &s0) && praos_ticked_epoch_nonce(st, ei, s0, &eta0) != PRAOS_OK) {
      praos_set_error_(ctx, "replay: first slot before the epoch base");
      return PRAOS_E_ARG;
    }
    // (the installed nonce only seeds praos_set_epoch: every batch carries its own nonces)
    if (!rd.err.empty()) { praos_set_error_(ctx, rd.err); return PRAOS_E_ARG; }
    v0 = rd.peek(&p, &l, &s0) ? view_of(epoch_of(s0)) : 0;
    if (v0 < 0) {
      praos_set_error_(ctx, "replay: no ledger view for epoch " + std::to_string(epoch_of(s0)));
      return PRAOS_E_ARG;
    }
    for (int q = 0; q < m; q++) {
      if (q == 0) t_epoch0 = std::chrono::steady_clock::now();
      const int r = praos_set_epoch(mem[q], eta0.neutral ? nullptr : eta0.hash, V[v0].pools, V[v0].npools, params);
      if (r != PRAOS_OK) {
        if (q) praos_set_error_(ctx, std::string("member ") + std::to_string(q) + ": " + praos_last_error(mem[q]));
        return r;
      }
    }
  }
  struct Slot {
    praos_batch* b = nullptr;
    int state = 0;                            // 0 free, 1 read (spans, offsets; the host parse)
    uint64_t batch = UINT64_MAX;              // the batch it holds (state 1)
    bool parsed = false;                      // the host parse is done (host_ok: it read every header)
    bool host_ok = false;                     // the chain's inputs read on the host (hslot, hprev, ...)
    bool decoded = false;                     // uploaded and decoded on the device, fields downloaded
    bool chained = false;                     // the nonce chain has been over it (etas, eidx, evol)
    bool launched = false;                    // its crypto is queued
    bool early = false;                       // ... with the launcher's etas_l / eidx_l (PRAOS_REPLAY_EARLY)
    size_t n = 0;
    int view = 0;                             // its ledger view (a batch never spans two)
    uint64_t index0 = 0;
    std::vector<praos_span> spans;
    std::vector<std::shared_ptr<Chunk>> chunks;
    std::vector<uint64_t> off;
    std::vector<uint32_t> len;
    std::vector<uint8_t> v, eidx;
    std::vector<uint16_t> fails;
    // the device decode's fields (the batch's pinned area, rp_download_decoded)
    const uint64_t *slot = nullptr, *block_no = nullptr, *ocn = nullptr;
    const uint32_t* bsize = nullptr;
    const uint8_t *prev = nullptr, *gen = nullptr, *cold = nullptr, *hh = nullptr;
    uint8_t* nonce = nullptr;
    const uint16_t* dstat = nullptr;
    std::vector<praos_nonce> etas, evol, etas_l;
    std::vector<uint8_t> eidx_l;
    std::vector<const uint8_t*> hptr;         // each header's bytes (the mapped chunk)
    std::vector<uint64_t> hslot;
    std::vector<uint8_t> hprev, hgen, hnonce;
    uint16_t* bits = nullptr;                 // pinned (the batch's: rp_batch_results)
    int32_t* pidx = nullptr;
  };
  // batch k: slot k mod T (T = m x SLOTS), member k mod m, that member's kept slot (k mod T) / m
  const int T = m * SLOTS;
  std::vector<Slot> S(T);
  auto member = [&](uint64_t k) { return mem[k % (uint64_t)m]; };
  auto member_slot = [&](uint64_t k) { return (int)((k % (uint64_t)T) / (uint64_t)m); };
  std::mutex mu;
  std::condition_variable cv;
  std::atomic<bool> stop{false};
  int first_rc = PRAOS_OK;
  uint64_t nbatches = UINT64_MAX;             // set by the reader at the end of the database
  bool stopped = false;
  auto fail = [&](int rc) {
    std::lock_guard<std::mutex> g(mu);
    if (first_rc == PRAOS_OK) first_rc = rc;
    stop = true;
    cv.notify_all();
  };
  double t_io = 0, t_dev = 0, t_wait = 0, t_nonce = 0, t_fold = 0;   // per thread: reader | fold
  // per-batch stage timeline (PRAOS_REPLAY_TRACE=<file>: one line per stage of each batch, "batch
  // stage start_ms end_ms headers", appended when the replay ends); one event list per thread
  struct Ev { uint64_t k; const char* what; double t0, t1; size_t n; };
  const char* trace_path = std::getenv("PRAOS_REPLAY_TRACE");
  std::vector<Ev> ev_reader, ev_chain, ev_launch, ev_fold;
  auto ev_add = [&](std::vector<Ev>& v, uint64_t k, const char* what, std::chrono::steady_clock::time_point t0,
                    size_t n) {
    if (trace_path)
      v.push_back({k, what, std::chrono::duration<double, std::milli>(t0 - t_base).count(), ms_since(t_base), n});
  };
  uint64_t epochs_seen = 0, batches = 0;
  if (trace_path) {
    const auto ms = [&](std::chrono::steady_clock::time_point t) {
      return std::chrono::duration<double, std::milli>(t - t_base).count();
    };
    ev_reader.push_back({0, "first_chunk", ms(t_peek0), ms(t_epoch0), 0});
  }
  ev_add(ev_reader, 0, "setup", t_base, 0);
  Placement pl;
  pl.init(batch_max);
  const char* ramp_env = std::getenv("PRAOS_REPLAY_RAMP");
  const int ramp = ramp_env ? std::atoi(ramp_env) : RP_RAMP_DEFAULT;
  if (pl.on) {
    for (int q = 0; q < m; q++) rp_copy_pin(mem[q], pl.copies());
    pl.reader_saved = pthread_getaffinity_np(pthread_self(), sizeof pl.reader_was, &pl.reader_was) == 0;
  }
  // the host parse of the chain's inputs (Praos; PRAOS_PARSE_THREADS workers, 0 = off: the chain
  // then waits for each batch's device decode)
  std::unique_ptr<ParPool> parse;
  {
    const char* e = std::getenv("PRAOS_PARSE_THREADS");
    const int np = e ? std::atoi(e) : 6;
    if (!tpraos && np > 0) {
      parse.reset(new ParPool((unsigned)std::min(np, 32)));
      if (pl.on) {
        const std::vector<int> cp = pl.copies();
        parse->run([&](unsigned t) { Placement::pin_self(cp[t % cp.size()]); });
      }
    }
  }
  const bool parse_on = parse != nullptr;
  // ---- nonce chain (speculative tick + reupdate as if every header were valid)
  struct Spec {
    int32_t origin;
    uint64_t last;
    praos_nonce evolving, candidate, epoch_nonce, lab, leb;
    bool dead;
  } sp{st->last_slot_origin, st->last_slot, st->evolving, st->candidate, st->epoch_nonce, st->lab,
       st->last_epoch_block, false};
  praos_nonce last_eta{};
  bool have_last = false;
  uint64_t sp_epoch = sp.origin ? 0 : epoch_of(sp.last);
  // Early launches (PRAOS_REPLAY_EARLY=1): the chain publishes each epoch nonce when it reaches the
  // epoch's first header (the tick that fixes it), and a decoded batch whose headers all lie in
  // epochs up to the last published one has its crypto queued at once, beside the chain's pass
  // over it, instead of after it.  The fold checks every header's nonce against its own tick
  // (fold_impl), so the launcher's nonces are the chain's or the replay stops.
  // PRAOS_REPLAY_EARLY=2: only once the reader has decoded the next batch (or there is none), so
  // the early crypto does not share the GPU with the decode the chain waits for next
  const char* early_env = std::getenv("PRAOS_REPLAY_EARLY");
  const int early_mode = early_env ? std::atoi(early_env) : (pl.on ? 2 : 0);
  const bool early_on = early_mode != 0;
  std::vector<std::pair<uint64_t, praos_nonce>> pubs{{sp_epoch, sp.epoch_nonce}};   // (epoch, nonce), mu
  uint64_t pub_epoch = sp_epoch;                                                      // mu
  std::thread chain([&] {
    if (pl.on) Placement::pin_self(pl.chain());
    for (uint64_t k = 0;; k++) {
      Slot& C = S[k % T];
      {
        std::unique_lock<std::mutex> g(mu);
        cv.wait(g, [&] { return stop || k >= nbatches || (C.state == 1 && C.batch == k && ((C.parsed && C.host_ok) || C.decoded)); });
        if (stop || k >= nbatches) return;
      }
      auto t0 = std::chrono::steady_clock::now();
      const size_t n = C.n;
      // the chain's inputs: read on the host (no wait for the device), or the device decode's
      const bool host = C.host_ok;
      const uint64_t* c_slot = host ? C.hslot.data() : C.slot;
      const uint8_t* c_prev = host ? C.hprev.data() : C.prev;
      const uint8_t* c_gen = host ? C.hgen.data() : C.gen;
      const uint8_t* c_nonce = host ? C.hnonce.data() : C.nonce;
      const uint16_t* c_dstat = host ? nullptr : C.dstat;
      C.etas.clear();
      C.eidx.resize(n);
      C.evol.resize(n);
      // epoch bounds cached: a division per epoch, not per header (the loop is the replay's
      // one sequential piece of work; one Blake2b compression per header is its floor)
      uint64_t ep_lo = 1, ep_hi = 0, ep_no = 0, ep_cut = 0;     // [ep_lo, ep_hi): epoch ep_no
      size_t lab_i = SIZE_MAX, cand_i = SIZE_MAX;   // headers whose prev hash / evolving nonce are the
                                                    // current labNonce / candidate (copied when needed)
      bool fresh = true;
      auto set_lab = [&](size_t j) {
        sp.lab.neutral = c_gen[j] ? 1 : 0;
        std::memset(sp.lab.hash, 0, 32);
        if (!c_gen[j]) std::memcpy(sp.lab.hash, c_prev + 32 * j, 32);
      };
      for (size_t i = 0; i < n; i++) {
        const uint64_t slot_i = c_slot[i];
        if (slot_i < ep_lo || slot_i >= ep_hi) {
          ep_no = epoch_of(slot_i);
          ep_lo = slot_i < ei->epoch_base_slot ? 0 : ei->epoch_base_slot + (ep_no - ei->epoch_base_no) * ei->epoch_length;
          ep_hi = slot_i < ei->epoch_base_slot ? ei->epoch_base_slot : ep_lo + ei->epoch_length;
          const uint64_t first_next = ei->epoch_base_slot + (ep_no - ei->epoch_base_no + 1) * ei->epoch_length;
          ep_cut = first_next > ei->stability_window ? first_next - ei->stability_window : 0;
        }
        const uint64_t e_new = ep_no;
        if (!sp.dead && e_new > (sp.origin ? 0 : sp_epoch)) {
          if (lab_i != SIZE_MAX) set_lab(lab_i);
          lab_i = SIZE_MAX;
          if (cand_i != SIZE_MAX) sp.candidate = C.evol[cand_i];
          cand_i = SIZE_MAX;
          sp.epoch_nonce = praos_host::nonce_combine(sp.candidate, sp.leb);
          if (tpraos && extra_entropy) sp.epoch_nonce = praos_host::nonce_combine(sp.epoch_nonce, *extra_entropy);
          sp.leb = sp.lab;
          fresh = true;
          if (early_on) {
            std::lock_guard<std::mutex> g(mu);
            pubs.push_back({e_new, sp.epoch_nonce});
            pub_epoch = e_new;
            cv.notify_all();
          }
        }
        if (fresh) {                              // the epoch nonce changes only at a tick
          if (C.etas.empty() || !praos_host::nonce_eq(C.etas.back(), sp.epoch_nonce)) C.etas.push_back(sp.epoch_nonce);
          fresh = false;
        }
        C.eidx[i] = (uint8_t)std::min<size_t>(C.etas.size() - 1, 255);
        if (sp.dead || (c_dstat && (c_dstat[i] & PRAOS_DEC_FAILED))) { sp.dead = true; C.evol[i] = sp.evolving; continue; }
        sp.origin = 0;
        sp.last = slot_i;
        sp_epoch = e_new;
        lab_i = i;                                // labNonce: the prev hash of this header (copied when needed)
        praos_nonce eta;
        std::memcpy(eta.hash, c_nonce + 32 * i, 32);
        eta.neutral = 0;
        sp.evolving = praos_host::nonce_combine(sp.evolving, eta);
        C.evol[i] = sp.evolving;
        if (slot_i < ep_cut) cand_i = i;          // slot + window < first slot of the next epoch: candidate := evolving
      }
      if (lab_i != SIZE_MAX) set_lab(lab_i);
      if (cand_i != SIZE_MAX) sp.candidate = C.evol[cand_i];
      if (C.etas.size() > 256) { praos_set_error_(ctx, "replay: > 256 epochs in a batch"); fail(PRAOS_E_STATE); return; }
      t_nonce += ms_since(t0);
      ev_add(ev_chain, k, "chain", t0, n);
      std::lock_guard<std::mutex> g(mu);
      C.chained = true;
      cv.notify_all();
    }
  });
  // per member: its own (praos_set_epoch) tables, the view they hold now, the other views' tables
  std::vector<rp_tables> own(m);
  std::vector<int> cur_view(m, v0);
  std::vector<std::vector<rp_view*>> dev_views(m, std::vector<rp_view*>(V.size(), nullptr));
  for (int q = 0; q < m; q++) own[q] = rp_tables_get(mem[q]);
  // ---- launcher: queues each batch's crypto (~30 launches: 1-2 ms of host time per batch,
  // kept off the nonce chain's thread)
  std::thread launcher([&] {
    if (pl.on) Placement::pin_self(pl.launcher());
    for (uint64_t k = 0;; k++) {
      Slot& C = S[k % T];
      {
        std::unique_lock<std::mutex> g(mu);
        cv.wait(g, [&] { return stop || k >= nbatches || (C.state == 1 && C.batch == k && C.decoded); });
        if (stop || k >= nbatches) return;
      }
      // the batch's last epoch (decoded slots; a header that did not decode may carry any slot:
      // the batch then waits for the chain)
      uint64_t e_max = 0;
      if (early_on) {
        uint64_t lo = 1, hi = 0;
        for (size_t i = 0; i < C.n; i++) {
          const uint64_t s = C.slot[i];
          if (s < lo || s >= hi) {
            const uint64_t e = epoch_of(s);
            e_max = std::max(e_max, e);
            lo = s < ei->epoch_base_slot ? 0 : ei->epoch_base_slot + (e - ei->epoch_base_no) * ei->epoch_length;
            hi = s < ei->epoch_base_slot ? ei->epoch_base_slot : lo + ei->epoch_length;
          }
        }
      }
      std::vector<std::pair<uint64_t, praos_nonce>> pub;
      {
        std::unique_lock<std::mutex> g(mu);
        auto next_decoded = [&] {
          if (early_mode != 2) return true;
          if (nbatches != UINT64_MAX && k + 1 >= nbatches) return true;
          const Slot& N = S[(k + 1) % T];
          return T > 1 && N.state == 1 && N.batch == k + 1 && N.decoded;
        };
        cv.wait(g, [&] { return stop || C.chained || (early_on && e_max <= pub_epoch && next_decoded()); });
        if (stop) return;
        C.early = !C.chained;
        if (C.early) pub = pubs;
      }
      if (C.early) {
        // each header's nonce: the last one published for an epoch <= its own (the nonce changes
        // only at the tick into an epoch that has headers)
        C.etas_l.clear();
        C.eidx_l.resize(C.n);
        size_t j = 0;
        uint64_t lo = 1, hi = 0, e = 0;
        for (size_t i = 0; i < C.n; i++) {
          const uint64_t s = C.slot[i];
          if (s < lo || s >= hi) {
            e = epoch_of(s);
            lo = s < ei->epoch_base_slot ? 0 : ei->epoch_base_slot + (e - ei->epoch_base_no) * ei->epoch_length;
            hi = s < ei->epoch_base_slot ? ei->epoch_base_slot : lo + ei->epoch_length;
          }
          while (j + 1 < pub.size() && pub[j + 1].first <= e) j++;
          while (j > 0 && pub[j].first > e) j--;
          const praos_nonce& eta = pub[j].second;
          if (C.etas_l.empty() || !praos_host::nonce_eq(C.etas_l.back(), eta)) C.etas_l.push_back(eta);
          C.eidx_l[i] = (uint8_t)std::min<size_t>(C.etas_l.size() - 1, 255);
        }
        if (C.etas_l.size() > 256) {
          praos_set_error_(ctx, "replay: > 256 epochs in a batch");
          fail(PRAOS_E_STATE);
          return;
        }
      }
      if (views && cur_view[k % (uint64_t)m] != C.view) {
        // the member's launches from here on read this view's pool tables (queued kernels of
        // earlier batches keep the tables they were launched with; all are freed at the end)
        const int q = (int)(k % (uint64_t)m);
        if (C.view == v0) {
          rp_tables_set(mem[q], own[q]);
        } else {
          rp_view*& t = dev_views[q][C.view];
          if (!t) t = rp_view_make(mem[q], V[C.view].pools, V[C.view].npools, params, true);
          if (!t) {
            if (mem[q] != ctx) praos_set_error_(ctx, praos_last_error(mem[q]));
            fail(PRAOS_E_OOM);
            return;
          }
          rp_tables_set(mem[q], rp_view_tables(t));
        }
        cur_view[q] = C.view;
      }
      const auto t0 = std::chrono::steady_clock::now();
      const std::vector<praos_nonce>& etas = C.early ? C.etas_l : C.etas;
      const int rc = rp_run(member(k), C.b, etas.data(), (uint32_t)etas.size(), (C.early ? C.eidx_l : C.eidx).data());
      ev_add(ev_launch, k, "launch", t0, C.n);
      if (rc != PRAOS_OK && member(k) != ctx) praos_set_error_(ctx, praos_last_error(member(k)));
      if (rc != PRAOS_OK) { fail(rc); return; }
      std::lock_guard<std::mutex> g(mu);
      C.launched = true;
      batches++;
      cv.notify_all();
    }
  });
  // ---- fold (envelope + updateChainDepState over each verified batch, in order)
  uint64_t validated = 0, headers_done = 0, stop_index = 0;
  uint8_t stop_verdict = 0;
  std::thread folder([&] {
    if (pl.on) Placement::pin_self(pl.folder());
    for (uint64_t k = 0;; k++) {
      Slot& C = S[k % T];
      {
        std::unique_lock<std::mutex> g(mu);
        cv.wait(g, [&] { return stop || k >= nbatches || (C.state == 1 && C.batch == k && C.chained && C.launched &&
                                                        (C.parsed || !parse_on)); });
        if (stop || k >= nbatches) return;
      }
      auto t0 = std::chrono::steady_clock::now();
      int rc = rp_download_results(member(k), C.b, C.bits, C.pidx);
      if (rc != PRAOS_OK) {
        if (member(k) != ctx) praos_set_error_(ctx, praos_last_error(member(k)));
        fail(rc);
        return;
      }
      t_wait += ms_since(t0);
      ev_add(ev_fold, k, "wait", t0, C.n);
      t0 = std::chrono::steady_clock::now();
      const size_t n = C.n;
      if (C.host_ok &&
          (std::memcmp(C.hslot.data(), C.slot, 8 * n) || std::memcmp(C.hgen.data(), C.gen, n) ||
           std::memcmp(C.hprev.data(), C.prev, 32 * n) || std::memcmp(C.hnonce.data(), C.nonce, 32 * n))) {
        // the chain ran on the host's reading of the headers: it must be the device decode's for
        // every header that decodes (the fold stops at the first that does not)
        for (size_t i = 0; i < n && !(C.dstat[i] & PRAOS_DEC_FAILED); i++)
          if (C.hslot[i] != C.slot[i] || C.hgen[i] != C.gen[i] ||
              std::memcmp(&C.hprev[32 * i], &C.prev[32 * i], 32) || std::memcmp(&C.hnonce[32 * i], &C.nonce[32 * i], 32)) {
            praos_set_error_(ctx, "replay: host and device read header " + std::to_string(C.index0 + i) + " differently");
            fail(PRAOS_E_STATE);
            return;
          }
      }
      C.v.resize(n);
      C.fails.resize(n);
      praos_out out{C.bits, C.pidx, nullptr, nullptr, C.nonce};
      praos_headers h{};
      h.n = n;
      h.slot = C.slot;
      h.cold_vk = C.cold;
      h.ocert_n = C.ocn;
      env->block_no = C.block_no;
      env->header_hash = C.hh;
      env->header_size = C.len.data();
      env->body_size = C.bsize;
      size_t stp = 0, done = 0;
      if (views) {                            // the envelope limits of the batch's ledger view
        env->lv_prot_major = V[C.view].prot;
        env->max_header_size = V[C.view].maxh;
        env->max_body_size = V[C.view].maxb;
      }
      const std::vector<praos_nonce>& etas = C.early ? C.etas_l : C.etas;   // the nonces its crypto ran with
      rc = rp_fold(ctx, &h, C.prev, C.gen, &out, env, ei, st, etas.data(), (uint32_t)etas.size(),
                   (C.early ? C.eidx_l : C.eidx).data(), C.evol.data(), tpraos, extra_entropy, C.v.data(),
                   C.fails.data(), &stp, &done, views ? hv[C.view].get() : nullptr);
      env->block_no = nullptr;
      env->header_hash = nullptr;
      env->header_size = nullptr;
      env->body_size = nullptr;
      t_fold += ms_since(t0);
      ev_add(ev_fold, k, "fold", t0, C.n);
      if (rc != PRAOS_OK) { fail(rc); return; }
      {
        // epoch nonces the folded headers ran under (up to and including a stopping header: the
        // count does not depend on how far the chain or the reader got before the stop)
        const std::vector<uint8_t>& ix = C.early ? C.eidx_l : C.eidx;
        const size_t upto = stp < done ? stp + 1 : done;
        for (size_t j = 0; j < upto; j++) {
          const praos_nonce& e = etas[ix[j]];
          if (!have_last || !praos_host::nonce_eq(e, last_eta)) { epochs_seen++; last_eta = e; have_last = true; }
        }
      }
      for (size_t j = 0; j < done && C.index0 + j < verdicts_cap; j++) {
        verdicts[C.index0 + j] = C.v[j];
        if (failures) failures[C.index0 + j] = tpraos ? C.fails[j] : 0;
      }
      std::lock_guard<std::mutex> g(mu);
      if (stp < done) {          // the chain stops at the first invalid header
        validated += stp;
        stop_index = C.index0 + stp;
        stop_verdict = C.v[stp];
        headers_done = C.index0 + stp + 1;
        stopped = true;
        stop = true;
      } else if (done < n) {     // every header valid so far, yet a nonce the fold disagrees with
        praos_set_error_(ctx, "replay: epoch nonce of header " + std::to_string(C.index0 + done) + " diverged");
        if (first_rc == PRAOS_OK) first_rc = PRAOS_E_STATE;
        stop = true;
      } else {
        validated += n;
        headers_done = C.index0 + n;
      }
      C.state = 0;
      C.chained = C.launched = C.early = C.decoded = C.host_ok = C.parsed = false;
      cv.notify_all();
    }
  });
  // ---- uploader: H2D + device decode of each batch the reader has built, then the decoded
  // fields back (the launcher and the fold wait for them; the chain only when the host parse
  // could not read the batch)
  std::vector<Ev> ev_up;
  std::thread uploader([&] {
    if (pl.on) Placement::pin_self(pl.uploader());
    for (uint64_t k = 0;; k++) {
      Slot& C = S[k % T];
      {
        std::unique_lock<std::mutex> g(mu);
        cv.wait(g, [&] { return stop || k >= nbatches || (C.state == 1 && C.batch == k); });
        if (stop || k >= nbatches) return;
      }
      const auto t0 = std::chrono::steady_clock::now();
      praos_ctx* const mc = member(k);
      const size_t n = C.n;
      int rc = rp_upload_decode(mc, C.b, n, C.spans.data(), C.spans.size(), C.off.data(), C.len.data());
      ev_add(ev_up, k, "gather", t0, n);        // the bytes staged and queued (host side)
      praos_decoded dec{};
      if (rc == PRAOS_OK) rc = rp_download_decoded(mc, C.b, &dec, &C.nonce);   // into the batch's pinned area
      if (rc == PRAOS_OK) {
        C.dstat = dec.status; C.block_no = dec.block_no; C.slot = dec.slot; C.ocn = dec.ocert_n;
        C.bsize = dec.body_size; C.prev = dec.prev_hash; C.gen = dec.prev_is_genesis; C.cold = dec.cold_vk;
        C.hh = dec.header_hash;
      }
      t_dev += ms_since(t0);
      ev_add(ev_up, k, "decode", t0, n);
      if (rc != PRAOS_OK) {
        if (mc != ctx) praos_set_error_(ctx, praos_last_error(mc));
        fail(rc);
        return;
      }
      std::lock_guard<std::mutex> g(mu);
      if (C.parsed || !parse_on) C.chunks.clear();   // the mappings have been read (the last reader drops them)
      C.decoded = true;
      cv.notify_all();
    }
  });
  // ---- parser: the chain's inputs of each batch read on the host (the pool's workers), beside
  // the reader's next batch and the uploader
  std::vector<Ev> ev_parse;
  std::thread parser([&] {
    if (!parse_on) return;
    if (pl.on) Placement::pin_self(pl.folder());
    for (uint64_t k = 0;; k++) {
      Slot& C = S[k % T];
      {
        std::unique_lock<std::mutex> g(mu);
        cv.wait(g, [&] { return stop || k >= nbatches || (C.state == 1 && C.batch == k); });
        if (stop || k >= nbatches) return;
      }
      const auto t0 = std::chrono::steady_clock::now();
      const size_t n = C.n;
      C.hslot.resize(n); C.hprev.resize(32 * n); C.hgen.resize(n); C.hnonce.resize(32 * n);
      std::atomic<bool> ok{true};
      const unsigned np = parse->size();
      parse->run([&](unsigned t) {
        for (size_t i = n * t / np; i < n * (t + 1) / np; i++)
          if (!chain_fields(C.hptr[i], C.len[i], &C.hslot[i], &C.hprev[32 * i], &C.hgen[i], &C.hnonce[32 * i]))
            ok = false;
      });
      ev_add(ev_parse, k, "parse", t0, n);
      std::lock_guard<std::mutex> g(mu);
      C.host_ok = ok;
      C.parsed = true;
      if (C.decoded) C.chunks.clear();
      cv.notify_all();
    }
  });
  // ---- reader (this thread): build batch k into slot k % T (member k % m) and read the chain's
  // inputs of its headers on the host
  if (pl.on) Placement::pin_self(pl.reader());
  uint64_t next_index = 0, built = 0;
  for (uint64_t k = 0;; k++) {
    Slot& C = S[k % T];
    {
      std::unique_lock<std::mutex> g(mu);
      cv.wait(g, [&] { return stop || C.state == 0; });
      if (stop) break;
    }
    auto t0 = std::chrono::steady_clock::now();
    C.spans.clear();
    C.chunks.clear();
    C.off.clear();
    C.len.clear();
    C.hptr.clear();
    const uint8_t* p;
    uint32_t l;
    uint64_t s, e_prev = 0;
    uint32_t nep = 0;
    size_t arena = 0;
    const Chunk* span_chunk = nullptr;
    // the first batches ramp up to batch_max (rp_ramp_cap): the nonce chain (the replay's
    // sequential part) starts as soon as possible, and each next batch is read and decoded by
    // the time the chain has been over the one before
    const size_t cap = rp_ramp_cap(ramp, k, batch_max);
    bool no_view = false;
    while (C.off.size() < cap && rd.peek(&p, &l, &s)) {
      const uint64_t e = epoch_of(s);
      if (C.off.empty() || e != e_prev) {
        if (nep == 256) break;
        const int w = view_of(e);
        if (w < 0) { no_view = true; break; }
        if (C.off.empty()) C.view = w;
        else if (w != C.view) break;          // a batch never spans two ledger views
        nep++;
        e_prev = e;
      }
      if (C.chunks.empty() || C.chunks.back() != rd.cur) C.chunks.push_back(rd.cur);
      praos_span* last = C.spans.empty() ? nullptr : &C.spans.back();
      if (last && span_chunk == rd.cur.get() && p >= last->p + last->len && p - (last->p + last->len) <= SPAN_GAP) {
        const size_t ext = (size_t)(p + l - (last->p + last->len));
        C.off.push_back(arena + (size_t)(p - (last->p + last->len)));
        last->len += ext;
        arena += ext;
      } else {
        C.spans.push_back({p, l});
        span_chunk = rd.cur.get();
        C.off.push_back(arena);
        arena += l;
      }
      C.len.push_back(l);
      C.hptr.push_back(p);
      rd.pop();
    }
    t_io += ms_since(t0);
    ev_add(ev_reader, k, "read", t0, C.off.size());
    if (!rd.err.empty()) { praos_set_error_(ctx, rd.err); fail(PRAOS_E_ARG); break; }
    if (no_view && C.off.empty()) {
      praos_set_error_(ctx, "replay: no ledger view for epoch " + std::to_string(epoch_of(s)));
      fail(PRAOS_E_ARG);
      break;
    }
    if (C.off.empty()) break;
    t0 = std::chrono::steady_clock::now();
    const size_t n = C.n = C.off.size();
    C.index0 = next_index;
    next_index += n;
    praos_ctx* const mc = member(k);
    if (!rp_batch_fits(C.b, n, arena)) {
      if (C.b) rp_batch_destroy(mc, C.b);
      C.b = rp_batch_take(mc, member_slot(k), n, arena, tpraos);
      if (!C.b) { fail(PRAOS_E_OOM); break; }
    }
    rp_batch_results(C.b, &C.bits, &C.pidx);          // pinned, kept with the batch
    std::lock_guard<std::mutex> g(mu);
    C.state = 1;
    C.batch = k;
    built = k + 1;
    cv.notify_all();
  }
  {
    std::lock_guard<std::mutex> g(mu);
    nbatches = built;                         // the chain and the fold finish what was handed on
    cv.notify_all();
  }
  chain.join();
  launcher.join();
  folder.join();
  uploader.join();
  parser.join();
  parse.reset();
  const auto t_join = std::chrono::steady_clock::now();
  if (pl.on) {                                // the caller's thread and the copy threads as they were
    if (pl.reader_saved) (void)pthread_setaffinity_np(pthread_self(), sizeof pl.reader_was, &pl.reader_was);
    for (int q = 0; q < m; q++) rp_copy_pin(mem[q], {});
  }
  for (int k = 0; k < T; k++) {
    Slot& C = S[k];
    // a replay that stopped early may have queued the crypto of up to two later batches:
    // they finish before the batch goes back to the context (the next call's upload
    // overwrites its buffers; rp_upload_decode also orders itself after run_ev)
    if (C.b) rp_batch_quiesce(C.b);
    if (C.b) rp_batch_keep(member(k), member_slot(k), C.b);
  }
  // every batch has finished: the members get their own tables back, the views' go
  for (int q = 0; q < m; q++) {
    rp_tables_set(mem[q], own[q]);
    for (rp_view* t : dev_views[q]) rp_view_free(mem[q], t);
  }
  ev_add(ev_fold, nbatches, "teardown", t_join, 0);
  if (trace_path) {
    if (FILE* f = std::fopen(trace_path, "a")) {
      for (const auto* v : {&ev_reader, &ev_parse, &ev_up, &ev_chain, &ev_launch, &ev_fold})
        for (const Ev& e : *v) std::fprintf(f, "%llu %s %.3f %.3f %zu\n", (unsigned long long)e.k, e.what, e.t0, e.t1, e.n);
      std::fprintf(f, "end - 0 %.3f 0\n", ms_since(t_base));
      std::fclose(f);
    }
  }
  stats->ms_io = t_io;
  stats->ms_device = t_dev + t_wait;
  stats->ms_nonce = t_nonce;
  stats->ms_fold = t_fold;
  stats->epochs = (uint32_t)epochs_seen;
  stats->batches = (uint32_t)batches;
  stats->chunks = (uint32_t)rd.chunk;
  stats->validated = validated;
  if (first_rc != PRAOS_OK) return first_rc;
  if (stopped) {
    stats->stop_index = stop_index;
    stats->stop_verdict = stop_verdict;
    stats->headers = headers_done;
  } else {
    stats->headers = next_index;
    stats->stop_index = next_index;
  }
  return PRAOS_OK;
}

extern "C" int praos_replay_immutable(praos_ctx* ctx, const char* dir, const praos_pool* pools, uint32_t npools,
                                      const praos_params* params, const praos_epoch_info* ei, praos_envelope* env,
                                      praos_chain_state* st, size_t batch_max, uint8_t* verdicts,
                                      size_t verdicts_cap, praos_replay_stats* stats) {
  praos_replay_scope_(ctx, true);
  const int r = rp_replay(&ctx, 1, dir, pools, npools, params, ei, env, st, batch_max, verdicts, nullptr, verdicts_cap,
                          stats, false, nullptr);
  praos_replay_scope_(ctx, false);
  return r;
}

extern "C" int praos_replay_immutable_tpraos(praos_ctx* ctx, const char* dir, const praos_pool* pools,
                                             uint32_t npools, const praos_params* params, const praos_epoch_info* ei,
                                             const praos_nonce* extra_entropy, praos_envelope* env,
                                             praos_chain_state* st, size_t batch_max, uint8_t* verdicts,
                                             uint16_t* failures, size_t verdicts_cap, praos_replay_stats* stats) {
  praos_replay_scope_(ctx, true);
  const int r = rp_replay(&ctx, 1, dir, pools, npools, params, ei, env, st, batch_max, verdicts, failures,
                          verdicts_cap, stats, true, extra_entropy);
  praos_replay_scope_(ctx, false);
  return r;
}

extern "C" int praos_replay_immutable_views(praos_ctx* ctx, const char* dir, const praos_ledger_view* views,
                                            uint32_t nviews, const praos_params* params, const praos_epoch_info* ei,
                                            praos_envelope* env, praos_chain_state* st, size_t batch_max,
                                            uint8_t* verdicts, size_t verdicts_cap, praos_replay_stats* stats) {
  if (!views || nviews == 0) return PRAOS_E_ARG;
  praos_replay_scope_(ctx, true);
  const int r = rp_replay(&ctx, 1, dir, nullptr, 0, params, ei, env, st, batch_max, verdicts, nullptr, verdicts_cap,
                          stats, false, nullptr, views, nviews);
  praos_replay_scope_(ctx, false);
  return r;
}
