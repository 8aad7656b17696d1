// praos_replay.hip -- db-analyser-style chain replay over an ImmutableDB directory
// (SURVEY.md sec. 8 row N3): host C++ on top of the library's own C ABI.
//
// Mirrors the reference's streaming loop (DBAnalyser/Analysis.hs:815-847,
// processAllImmutableDB: ImmutableDB.streamAll, one iteratorNext per block) and its
// header-validation pass (benchmarkLedgerOps, :479-607: tick, then validateHeader),
// in batches: headers are read through the secondary index into batches of up to
// batch_max headers (any number of epochs, up to 256), decoded on the device
// (praos_batch_decode), given their epoch nonces -- the nonce tickChainDepState
// (Praos.hs:407-431) reaches at each header, computed on the host from the certified
// VRF outputs as if every header were valid -- crypto-checked under those nonces
// (praos_batch_set_nonces + praos_batch_run) and folded on the host with
// praos_validate_headers_nonces (envelope, then updateChainDepState), which accepts a
// header only if the nonce its crypto ran with is the one the real fold ticks to.  One
// ledger view (pools, parameters) for the whole replay.  Like the reference, the
// replay ends at the first invalid header.
//
// On-disk format (ImmutableDB, Storage/ImmutableDB/Impl): NNNNN.chunk holds the
// stored blocks back to back; NNNNN.secondary one 56-byte Entry per block
// (Impl/Index/Secondary.hs:93-128): blockOffset u64 BE, headerOffset u16 BE,
// headerSize u16 BE, checksum u32 BE, headerHash 32 bytes, blockOrEBB (slot) u64 BE.
// The primary index maps relative slots to entries and is not needed for a full
// sequential replay.  Chunks are read from 00000 upwards until one is missing.
#include "praos_hip.h"
#include "host_util.hpp"

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

void praos_set_error_(praos_ctx* c, const std::string& m);   // praos_api.hip

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

// Streams (header bytes, slot) out of the chunk files, one chunk in memory at a time.
struct ChunkReader {
  std::string dir, err;
  int chunk = 0;
  bool done = false;
  std::vector<uint8_t> data, sec;
  size_t entry = 0, nentries = 0;
  void load_next() {
    char name[32];
    std::snprintf(name, sizeof name, "/%05d.chunk", chunk);
    if (!read_file(dir + name, data)) { done = true; return; }
    std::snprintf(name, sizeof name, "/%05d.secondary", chunk);
    if (!read_file(dir + name, sec) || sec.size() % 56 != 0) {
      err = std::string("missing or malformed secondary index ") + (name + 1);
      done = true;
      return;
    }
    chunk++;
    entry = 0;
    nentries = sec.size() / 56;
  }
  // the next entry, without consuming it; false at the end of the database
  bool peek(const uint8_t** hdr, uint32_t* len, uint64_t* slot, const uint8_t** hash = nullptr) {
    while (!done && entry >= nentries) load_next();
    if (done) return false;
    const uint8_t* e = sec.data() + 56 * entry;
    const uint64_t boff = be(e, 8), hoff = be(e + 8, 2), hsz = be(e + 10, 2);
    if (boff > data.size() || hoff + hsz > data.size() - boff) {
      err = "secondary index entry outside its chunk (chunk " + std::to_string(chunk - 1) + ", entry " +
            std::to_string(entry) + ")";
      done = true;
      return false;
    }
    *hdr = data.data() + boff + hoff;
    *len = (uint32_t)hsz;
    *slot = be(e + 48, 8);
    if (hash) *hash = e + 16;
    return true;
  }
  void pop() { entry++; }
};

}  // namespace

// TPraos mode (eras Shelley..Alonzo, HFEras.hs:43-49; TPraos.hs:361-387): stored BHeaders
// (praos_batch_upload_tpraos_bytes), the TPraos nonce rules -- the header's nonce is
// mkNonceFromOutputVRF of its eta certificate (Blake2b-256 of the output, no range
// extension) and TICKN adds the extra entropy (eta0 := eta_c ⭒ eta_h ⭒ extraEntropy) --
// and the TPraos fold (PRTCL predicate-failure sets into failures[]).
static int replay_impl(praos_ctx* ctx, const char* dir, const praos_pool* pools, uint32_t npools,
                       const praos_params* params, const praos_epoch_info* ei, praos_envelope* env,
                       praos_chain_state* st, size_t batch_max, uint8_t* verdicts, uint16_t* failures,
                       size_t verdicts_cap, praos_replay_stats* stats, bool tpraos,
                       const praos_nonce* extra_entropy) {
  if (!ctx || !dir || !params || (npools && !pools) || !ei || !env || !st || !stats || batch_max == 0 ||
      ei->epoch_length == 0 || (verdicts_cap && !verdicts))
    return PRAOS_E_ARG;
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
  // The ledger view (pools, parameters) is installed once; the epoch nonces travel
  // with each batch (praos_batch_set_nonces), so a batch may span many epochs and stay
  // large enough to fill the device even when epochs are short.
  {
    praos_nonce eta0{};
    uint32_t l;
    uint64_t s0 = 0;
    const uint8_t* p;
    if (rd.peek(&p, &l, &s0) && praos_ticked_epoch_nonce(st, ei, s0, &eta0) != PRAOS_OK) {
      praos_set_error_(ctx, "replay: first slot before the epoch base");
      return PRAOS_E_ARG;
    }
    // (the installed nonce only seeds praos_set_epoch: every batch carries its own nonces)
    if (!rd.err.empty()) { praos_set_error_(ctx, rd.err); return PRAOS_E_ARG; }
    const int r = praos_set_epoch(ctx, eta0.neutral ? nullptr : eta0.hash, pools, npools, params);
    if (r != PRAOS_OK) return r;
  }
  // Two batches in flight: while the host folds batch k, the device verifies batch k+1
  // (its nonces come from the speculative nonce chain, which runs ahead of the fold).
  struct Stage {
    praos_batch* b = nullptr;
    size_t n = 0;
    uint64_t index0 = 0;
    std::vector<uint8_t> arena;
    std::vector<uint64_t> off, slot, block_no, ocn;
    std::vector<uint32_t> len, bsize;
    std::vector<uint8_t> prev, gen, cold, hh, nonce, v, vout, eidx;
    std::vector<uint16_t> dstat, bits, fails;
    std::vector<int32_t> pidx;
    std::vector<praos_nonce> etas;
  };
  Stage stage[2];
  // the speculative nonce state (tick + reupdate as if every header were valid)
  struct Spec {
    int32_t origin;
    uint64_t last;
    praos_nonce evolving, candidate, epoch_nonce, lab, leb;
    bool dead;
  } sp{st->last_slot_origin, st->last_slot, st->evolving, st->candidate, st->epoch_nonce, st->lab,
       st->last_epoch_block, false};
  praos_nonce last_eta{};
  bool have_last = false;
  uint64_t next_index = 0;
  const unsigned nthreads = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  // read, upload and decode the next batch, derive its nonces; false at the end
  auto prepare = [&](Stage& S, int& rc) -> bool {
    rc = PRAOS_OK;
    auto t_io = std::chrono::steady_clock::now();
    S.arena.clear();
    S.off.clear();
    S.len.clear();
    const uint8_t* p;
    uint32_t l;
    uint64_t s, e_prev = 0;
    uint32_t nep = 0;
    while (S.off.size() < batch_max && rd.peek(&p, &l, &s)) {
      const uint64_t e = epoch_of(s);
      if (S.off.empty() || e != e_prev) {
        if (nep == 256) break;
        nep++;
        e_prev = e;
      }
      if (S.arena.capacity() < S.arena.size() + l) S.arena.reserve(2 * S.arena.size() + (size_t(1) << 20));
      S.off.push_back(S.arena.size());
      S.len.push_back(l);
      S.arena.insert(S.arena.end(), p, p + l);
      rd.pop();
    }
    stats->ms_io += ms_since(t_io);
    if (!rd.err.empty()) { praos_set_error_(ctx, rd.err); rc = PRAOS_E_ARG; return false; }
    if (S.off.empty()) return false;
    const size_t n = S.n = S.off.size();
    S.index0 = next_index;
    next_index += n;
    auto t_dev = std::chrono::steady_clock::now();
    praos_header_bytes hb{n, S.arena.data(), S.arena.size(), S.off.data(), S.len.data()};
    S.b = tpraos ? praos_batch_upload_tpraos_bytes(ctx, &hb) : praos_batch_upload_bytes(ctx, &hb);
    if (!S.b) { rc = PRAOS_E_OOM; return false; }
    S.dstat.resize(n); S.block_no.resize(n); S.slot.resize(n); S.ocn.resize(n); S.bsize.resize(n);
    S.prev.resize(32 * n); S.gen.resize(n); S.cold.resize(32 * n); S.hh.resize(32 * n); S.vout.resize(64 * n);
    S.bits.resize(n); S.pidx.resize(n); S.nonce.resize(32 * n); S.v.resize(n); S.eidx.resize(n); S.fails.resize(n);
    praos_decoded dec{};
    dec.status = S.dstat.data(); dec.block_no = S.block_no.data(); dec.slot = S.slot.data();
    dec.prev_hash = S.prev.data(); dec.prev_is_genesis = S.gen.data(); dec.cold_vk = S.cold.data();
    dec.body_size = S.bsize.data(); dec.ocert_n = S.ocn.data(); dec.header_hash = S.hh.data();
    dec.vrf_out = S.vout.data();
    rc = praos_batch_decode(ctx, S.b);
    if (rc == PRAOS_OK) rc = praos_batch_download_decoded(ctx, S.b, &dec);
    if (rc != PRAOS_OK) return false;
    stats->ms_device += ms_since(t_dev);
    // vrfNonceValue of every CERTIFIED output (Praos/VRF.hs:88-131), in parallel; then the
    // nonce chain in order (tick at epoch changes, evolving ⭒ eta, candidate freeze)
    auto t_nonce = std::chrono::steady_clock::now();
    std::vector<praos_nonce> eta_of(n);
    {
      std::vector<std::thread> th;
      for (unsigned t = 0; t < nthreads; t++)
        th.emplace_back([&, t] {
          for (size_t i = n * t / nthreads; i < n * (t + 1) / nthreads; i++) {
            if (tpraos) {        // mkNonceFromOutputVRF (the eta certificate's output)
              praos_host::blake2b(eta_of[i].hash, 32, S.vout.data() + 64 * i, 64);
            } else {
              uint8_t m[65], h1[32];
              m[0] = 'N';
              std::memcpy(m + 1, S.vout.data() + 64 * i, 64);
              praos_host::blake2b(h1, 32, m, 65);
              praos_host::blake2b(eta_of[i].hash, 32, h1, 32);
            }
            eta_of[i].neutral = 0;
          }
        });
      for (auto& t : th) t.join();
    }
    S.etas.clear();
    for (size_t i = 0; i < n; i++) {
      const uint64_t e_new = epoch_of(S.slot[i]);
      if (!sp.dead && e_new > (sp.origin ? 0 : epoch_of(sp.last))) {
        sp.epoch_nonce = praos_host::nonce_combine(sp.candidate, sp.leb);
        if (tpraos && extra_entropy) sp.epoch_nonce = praos_host::nonce_combine(sp.epoch_nonce, *extra_entropy);
        sp.leb = sp.lab;
      }
      if (S.etas.empty() || !praos_host::nonce_eq(S.etas.back(), sp.epoch_nonce)) S.etas.push_back(sp.epoch_nonce);
      S.eidx[i] = (uint8_t)(S.etas.size() - 1);
      if (sp.dead || (S.dstat[i] & PRAOS_DEC_FAILED)) { sp.dead = true; continue; }   // the chain stops here
      sp.origin = 0;
      sp.last = S.slot[i];
      sp.lab.neutral = S.gen[i] ? 1 : 0;
      std::memset(sp.lab.hash, 0, 32);
      if (!S.gen[i]) std::memcpy(sp.lab.hash, S.prev.data() + 32 * i, 32);
      sp.evolving = praos_host::nonce_combine(sp.evolving, eta_of[i]);
      const uint64_t first_next = ei->epoch_base_slot + (e_new - ei->epoch_base_no + 1) * ei->epoch_length;
      if (S.slot[i] + ei->stability_window < first_next) sp.candidate = sp.evolving;
    }
    if (S.etas.size() > 256) { praos_set_error_(ctx, "replay: > 256 epochs in a batch"); rc = PRAOS_E_STATE; return false; }
    for (const praos_nonce& e : S.etas)
      if (!have_last || !praos_host::nonce_eq(e, last_eta)) { stats->epochs++; last_eta = e; have_last = true; }
    stats->ms_nonce += ms_since(t_nonce);
    rc = praos_batch_set_nonces(ctx, S.b, S.etas.data(), (uint32_t)S.etas.size(), S.eidx.data());
    return rc == PRAOS_OK;
  };
  auto launch = [&](Stage& S) {
    auto t = std::chrono::steady_clock::now();
    const int r = praos_batch_run(ctx, S.b);   // async on the ctx stream
    stats->ms_device += ms_since(t);
    stats->batches++;
    return r;
  };
  auto download = [&](Stage& S) {
    auto t = std::chrono::steady_clock::now();
    praos_out out{S.bits.data(), S.pidx.data(), nullptr, nullptr, S.nonce.data()};
    const int r = praos_batch_download(ctx, S.b, &out);
    stats->ms_device += ms_since(t);
    return r;
  };
  // envelope + updateChainDepState over a verified batch; true when the chain stops
  auto fold = [&](Stage& S, int& rc) -> bool {
    auto t_fold = std::chrono::steady_clock::now();
    const size_t n = S.n;
    praos_out out{S.bits.data(), S.pidx.data(), nullptr, nullptr, S.nonce.data()};
    praos_headers h{};
    h.n = n;
    h.slot = S.slot.data();
    h.cold_vk = S.cold.data();
    h.ocert_n = S.ocn.data();
    env->block_no = S.block_no.data();
    env->header_hash = S.hh.data();
    env->header_size = S.len.data();
    env->body_size = S.bsize.data();
    size_t stop = 0, done = 0;
    if (tpraos) {
      praos_tpraos_headers th{};
      th.h = h;
      praos_tpraos_out to{S.bits.data(), S.pidx.data(), nullptr, nullptr, S.nonce.data()};
      rc = praos_tpraos_validate_headers_nonces(ctx, &th, S.prev.data(), S.gen.data(), &to, env, ei, extra_entropy,
                                                st, S.etas.data(), (uint32_t)S.etas.size(), S.eidx.data(),
                                                S.v.data(), S.fails.data(), &stop, &done);
    } else {
      rc = praos_validate_headers_nonces(ctx, &h, S.prev.data(), S.gen.data(), &out, env, ei, st, S.etas.data(),
                                         (uint32_t)S.etas.size(), S.eidx.data(), S.v.data(), &stop, &done);
    }
    env->block_no = nullptr;
    env->header_hash = nullptr;
    env->header_size = nullptr;
    env->body_size = nullptr;
    stats->ms_fold += ms_since(t_fold);
    if (rc != PRAOS_OK) return true;
    for (size_t k = 0; k < done && S.index0 + k < verdicts_cap; k++) {
      verdicts[S.index0 + k] = S.v[k];
      if (failures) failures[S.index0 + k] = tpraos ? S.fails[k] : 0;
    }
    if (stop < done) {          // the chain stops at the first invalid header
      stats->validated += stop;
      stats->stop_index = S.index0 + stop;
      stats->stop_verdict = S.v[stop];
      stats->headers = S.index0 + stop + 1;
      return true;
    }
    if (done < n) {             // every header valid so far, yet a nonce the fold disagrees with
      praos_set_error_(ctx, "replay: epoch nonce of header " + std::to_string(S.index0 + done) + " diverged");
      rc = PRAOS_E_STATE;
      return true;
    }
    stats->validated += n;
    stats->headers = S.index0 + n;
    return false;
  };
  auto release = [&](Stage& S) {
    if (S.b) praos_batch_free(ctx, S.b);
    S.b = nullptr;
  };
  bool stopped = false;
  int rc = PRAOS_OK;
  int cur = 0;
  bool have_cur = prepare(stage[cur], rc);
  if (rc == PRAOS_OK && have_cur) rc = launch(stage[cur]);
  while (rc == PRAOS_OK && have_cur) {
    Stage& C = stage[cur];
    Stage& N = stage[cur ^ 1];
    // the next batch is read and decoded while C's crypto runs; its decode queues behind it
    const bool have_next = !sp.dead && prepare(N, rc);
    if (rc != PRAOS_OK) break;
    rc = download(C);
    if (rc != PRAOS_OK) break;
    if (have_next) {
      rc = launch(N);           // N's crypto overlaps C's fold
      if (rc != PRAOS_OK) break;
    }
    stopped = fold(C, rc);
    release(C);
    if (stopped || rc != PRAOS_OK) break;
    have_cur = have_next;
    cur ^= 1;
  }
  release(stage[0]);
  release(stage[1]);
  if (rc != PRAOS_OK) return rc;
  const uint64_t index0 = stopped ? stats->headers : next_index;
  if (!stopped) stats->stop_index = index0;
  stats->chunks = (uint32_t)rd.chunk;
  return PRAOS_OK;
}

extern "C" int praos_replay_immutable(praos_ctx* ctx, const char* dir, const praos_pool* pools, uint32_t npools,
                                      const praos_params* params, const praos_epoch_info* ei, praos_envelope* env,
                                      praos_chain_state* st, size_t batch_max, uint8_t* verdicts,
                                      size_t verdicts_cap, praos_replay_stats* stats) {
  return replay_impl(ctx, dir, pools, npools, params, ei, env, st, batch_max, verdicts, nullptr, verdicts_cap, stats,
                     false, nullptr);
}

extern "C" int praos_replay_immutable_tpraos(praos_ctx* ctx, const char* dir, const praos_pool* pools,
                                             uint32_t npools, const praos_params* params, const praos_epoch_info* ei,
                                             const praos_nonce* extra_entropy, praos_envelope* env,
                                             praos_chain_state* st, size_t batch_max, uint8_t* verdicts,
                                             uint16_t* failures, size_t verdicts_cap, praos_replay_stats* stats) {
  return replay_impl(ctx, dir, pools, npools, params, ei, env, st, batch_max, verdicts, failures, verdicts_cap, stats,
                     true, extra_entropy);
}
