// praos_replay.hip -- db-analyser-style chain replay over an ImmutableDB directory
// (SURVEY.md sec. 8 row N3): host C++ on top of the library's own C ABI.
//
// Mirrors the reference's streaming loop (DBAnalyser/Analysis.hs:815-847,
// processAllImmutableDB: ImmutableDB.streamAll, one iteratorNext per block) and its
// header-validation pass (benchmarkLedgerOps, :479-607: tick, then validateHeader),
// in batches: headers are read through the secondary index, cut into batches that
// never cross an epoch boundary, decoded and crypto-checked on the device in one pass
// (praos_batch_upload_bytes / praos_batch_run), then folded on the host with
// praos_validate_headers (envelope, then updateChainDepState).  Before each epoch the
// epoch nonce the state ticks to (tickChainDepState, Praos.hs:407-431) is installed
// with praos_set_epoch (same pools and parameters: one ledger view for the replay).
// Like the reference, the replay ends at the first invalid header.
//
// On-disk format (ImmutableDB, Storage/ImmutableDB/Impl): NNNNN.chunk holds the
// stored blocks back to back; NNNNN.secondary one 56-byte Entry per block
// (Impl/Index/Secondary.hs:93-128): blockOffset u64 BE, headerOffset u16 BE,
// headerSize u16 BE, checksum u32 BE, headerHash 32 bytes, blockOrEBB (slot) u64 BE.
// The primary index maps relative slots to entries and is not needed for a full
// sequential replay.  Chunks are read from 00000 upwards until one is missing.
#include "praos_kernels.h"
#include "host_util.hpp"

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <string>
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

extern "C" int praos_replay_immutable(praos_ctx* ctx, const char* dir, const praos_pool* pools, uint32_t npools,
                                      const praos_params* params, const praos_epoch_info* ei, praos_envelope* env,
                                      praos_chain_state* st, size_t batch_max, uint8_t* verdicts,
                                      size_t verdicts_cap, praos_replay_stats* stats) {
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
  praos_nonce cur{};
  bool have_eta = false;
  std::vector<uint8_t> arena;
  std::vector<uint64_t> off, slot, block_no, ocn;
  std::vector<uint32_t> len, bsize;
  std::vector<uint8_t> prev, gen, cold, hh, nonce, v;
  std::vector<uint16_t> dstat, bits;
  std::vector<int32_t> pidx;
  uint64_t index0 = 0;          // global index of the batch's first header
  bool stopped = false;
  while (!stopped) {
    // ---- one batch: at most batch_max headers, all in the first header's epoch
    auto t_io = std::chrono::steady_clock::now();
    arena.clear();
    off.clear();
    len.clear();
    uint64_t first_slot = 0;
    const uint8_t* p;
    uint32_t l;
    uint64_t s;
    while (off.size() < batch_max && rd.peek(&p, &l, &s)) {
      if (off.empty()) first_slot = s;
      else if (epoch_of(s) != epoch_of(first_slot)) break;
      off.push_back(arena.size());
      len.push_back(l);
      arena.insert(arena.end(), p, p + l);
      rd.pop();
    }
    stats->ms_io += ms_since(t_io);
    if (!rd.err.empty()) { praos_set_error_(ctx, rd.err); return PRAOS_E_ARG; }
    if (off.empty()) break;
    size_t first = 0;           // first header of the batch not yet folded
    uint64_t eta_slot = first_slot;
    int idle = 0;               // folds in a row that made no progress
    while (first < off.size()) {
      const size_t n = off.size() - first;
      praos_nonce eta{};
      if (praos_ticked_epoch_nonce(st, ei, eta_slot, &eta) != PRAOS_OK) {
        praos_set_error_(ctx, "replay: slot " + std::to_string(eta_slot) + " before the epoch base");
        return PRAOS_E_ARG;
      }
      if (!have_eta || !praos_host::nonce_eq(eta, cur)) {
        const int r = praos_set_epoch(ctx, eta.neutral ? nullptr : eta.hash, pools, npools, params);
        if (r != PRAOS_OK) return r;
        cur = eta;
        have_eta = true;
        stats->epochs++;
      }
      auto t_dev = std::chrono::steady_clock::now();
      praos_header_bytes hb{n, arena.data(), arena.size(), off.data() + first, len.data() + first};
      praos_batch* b = praos_batch_upload_bytes(ctx, &hb);
      if (!b) return PRAOS_E_OOM;
      dstat.resize(n); block_no.resize(n); slot.resize(n); ocn.resize(n); bsize.resize(n);
      prev.resize(32 * n); gen.resize(n); cold.resize(32 * n); hh.resize(32 * n);
      bits.resize(n); pidx.resize(n); nonce.resize(32 * n); v.resize(n);
      praos_decoded dec{};
      dec.status = dstat.data(); dec.block_no = block_no.data(); dec.slot = slot.data();
      dec.prev_hash = prev.data(); dec.prev_is_genesis = gen.data(); dec.cold_vk = cold.data();
      dec.body_size = bsize.data(); dec.ocert_n = ocn.data(); dec.header_hash = hh.data();
      praos_out out{bits.data(), pidx.data(), nullptr, nullptr, nonce.data()};
      int r = praos_batch_run(ctx, b);
      if (r == PRAOS_OK) r = praos_batch_download(ctx, b, &out);
      if (r == PRAOS_OK) r = praos_batch_download_decoded(ctx, b, &dec);
      praos_batch_free(ctx, b);
      if (r != PRAOS_OK) return r;
      stats->ms_device += ms_since(t_dev);
      stats->batches++;
      // ---- validateHeader over the batch: envelope, then updateChainDepState
      auto t_fold = std::chrono::steady_clock::now();
      praos_headers h{};
      h.n = n;
      h.slot = slot.data();
      h.cold_vk = cold.data();
      h.ocert_n = ocn.data();
      env->block_no = block_no.data();
      env->header_hash = hh.data();
      env->header_size = len.data() + first;
      env->body_size = bsize.data();
      size_t stop = 0, done = 0;
      r = praos_validate_headers(ctx, &h, prev.data(), gen.data(), &out, env, ei, st, v.data(), &stop, &done);
      env->block_no = nullptr;
      env->header_hash = nullptr;
      env->header_size = nullptr;
      env->body_size = nullptr;
      stats->ms_fold += ms_since(t_fold);
      if (r != PRAOS_OK) return r;
      const uint64_t g0 = index0 + first;
      for (size_t k = 0; k < done && g0 + k < verdicts_cap; k++) verdicts[g0 + k] = v[k];
      if (stop < done) {        // the chain stops at the first invalid header
        stats->validated += stop;
        stats->stop_index = g0 + stop;
        stats->stop_verdict = v[stop];
        stats->headers = g0 + stop + 1;
        stopped = true;
        break;
      }
      stats->validated += done;
      first += done;
      if (first < off.size()) {
        // the fold met a header whose ticked nonce is not the installed one: only a
        // secondary-index slot that disagrees with the header's own slot does that
        // (batches never cross an epoch); re-tick from the decoded slot
        eta_slot = slot[done];
        if (done == 0 && ++idle > 1) {
          praos_set_error_(ctx, "replay: the epoch nonce of header " + std::to_string(g0) + " cannot be reached");
          return PRAOS_E_STATE;
        }
        if (done) idle = 0;
      }
    }
    index0 += off.size();
    if (!stopped) stats->headers = index0;
  }
  if (!stopped) stats->stop_index = index0;
  stats->chunks = (uint32_t)rd.chunk;
  return PRAOS_OK;
}
