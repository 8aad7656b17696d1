// praos_group.hip -- one process driving several GPUs (in-library
// multi-device): a group holds one praos_ctx per member device and splits every batch
// into contiguous shards, one per member, each run by its own host thread on its own
// context (HIP device and stream), outputs written in place in the caller's arrays.
// Headers of one epoch are independent (Praos.hs:441-459 checks one header against
// the epoch's ledger view only), so the shards need no exchange; the sequential fold
// (praos_validate_headers / praos_update_chain_dep_state) runs afterwards over the
// gathered outputs in slot order on any member context.
//
// A device may appear several times (several contexts on one GPU: the multi-threaded
// use the C ABI allows, one context per host thread).
#include <hip/hip_runtime.h>

#include "praos_hip.h"
#include "replay_internal.hpp"

#include <algorithm>
#include <string>
#include <thread>
#include <vector>

struct praos_group {
  std::vector<praos_ctx*> ctx;
  std::string err;
  std::vector<void*> registered;          // praos_group_host_register ranges
};

void praos_replay_scope_(praos_ctx* c, bool on);   // praos_api.hip
int praos_ctx_note_registered_(praos_ctx* c, void* p, size_t len, bool add);   // praos_api.hip
int praos_ctx_device_(praos_ctx* c);                                            // praos_api.hip

namespace {

// [i0, i1) of member k when n items are split over m members
inline void shard(size_t n, size_t m, size_t k, size_t* i0, size_t* i1) {
  *i0 = n * k / m;
  *i1 = n * (k + 1) / m;
}

template <typename T>
inline T* at(T* p, size_t i, size_t per) { return p ? p + i * per : nullptr; }

praos_out out_at(const praos_out* o, size_t i) {
  return {at(o->bits, i, 1), at(o->pool_idx, i, 1), at(o->beta, i, 64), at(o->leader, i, 32), at(o->nonce, i, 32)};
}

praos_tpraos_out tp_out_at(const praos_tpraos_out* o, size_t i) {
  return {at(o->bits, i, 1), at(o->pool_idx, i, 1), at(o->beta_eta, i, 64), at(o->beta_leader, i, 64),
          at(o->nonce, i, 32)};
}

// the shard [i0, i1) of a SoA header batch (body_off stays absolute into the shared body_bytes)
praos_headers headers_at(const praos_headers* h, size_t i0, size_t i1) {
  praos_headers s = *h;
  s.n = i1 - i0;
  s.slot = at(h->slot, i0, 1);
  s.cold_vk = at(h->cold_vk, i0, 32);
  s.vrf_vk = at(h->vrf_vk, i0, 32);
  s.vrf_out = at(h->vrf_out, i0, 64);
  s.vrf_proof = at(h->vrf_proof, i0, 80);
  s.hot_vk = at(h->hot_vk, i0, 32);
  s.ocert_n = at(h->ocert_n, i0, 1);
  s.ocert_c0 = at(h->ocert_c0, i0, 1);
  s.ocert_sig = at(h->ocert_sig, i0, 64);
  s.kes_sig = at(h->kes_sig, i0, 448);
  s.body_off = at(h->body_off, i0, 1);
  s.body_len = at(h->body_len, i0, 1);
  return s;
}

// only the shard's window of the arena travels to the member's device: offsets rebased
// into `off`, the window returned
praos_header_bytes bytes_at(const praos_header_bytes* in, size_t i0, size_t i1, std::vector<uint64_t>& off) {
  uint64_t lo = UINT64_MAX, hi = 0;
  for (size_t i = i0; i < i1; i++) {
    lo = std::min<uint64_t>(lo, in->off[i]);
    hi = std::max<uint64_t>(hi, in->off[i] + in->len[i]);
  }
  if (hi > in->bytes_len) { lo = 0; hi = in->bytes_len; }   // out-of-range entries: the decoder flags them
  lo = std::min<uint64_t>(lo, hi);
  off.assign(in->off + i0, in->off + i1);
  for (auto& o : off) o -= std::min<uint64_t>(o, lo);
  return {i1 - i0, in->bytes + lo, (size_t)(hi - lo), off.data(), in->len + i0};
}

praos_decoded dec_at(const praos_decoded* d, size_t i, size_t signed_stride = PRAOS_SIGNED_STRIDE) {
  praos_decoded r;
  r.status = at(d->status, i, 1);
  r.block_no = at(d->block_no, i, 1);
  r.slot = at(d->slot, i, 1);
  r.prev_hash = at(d->prev_hash, i, 32);
  r.prev_is_genesis = at(d->prev_is_genesis, i, 1);
  r.cold_vk = at(d->cold_vk, i, 32);
  r.vrf_vk = at(d->vrf_vk, i, 32);
  r.vrf_out = at(d->vrf_out, i, 64);
  r.vrf_proof = at(d->vrf_proof, i, 80);
  r.body_size = at(d->body_size, i, 1);
  r.body_hash = at(d->body_hash, i, 32);
  r.hot_vk = at(d->hot_vk, i, 32);
  r.ocert_n = at(d->ocert_n, i, 1);
  r.ocert_c0 = at(d->ocert_c0, i, 1);
  r.ocert_sig = at(d->ocert_sig, i, 64);
  r.prot_major = at(d->prot_major, i, 1);
  r.prot_minor = at(d->prot_minor, i, 1);
  r.kes_sig = at(d->kes_sig, i, 448);
  r.signed_len = at(d->signed_len, i, 1);
  r.signed_body = at(d->signed_body, i, signed_stride);
  r.header_hash = at(d->header_hash, i, 32);
  return r;
}

// run f(k) for every member on its own thread; the first failing member's code wins
template <typename F>
int fan_out(praos_group* g, F f) {
  const size_t m = g->ctx.size();
  std::vector<int> rc(m, PRAOS_OK);
  std::vector<std::thread> th;
  th.reserve(m);
  for (size_t k = 0; k < m; k++) th.emplace_back([&, k] { rc[k] = f(k); });
  for (auto& t : th) t.join();
  for (size_t k = 0; k < m; k++)
    if (rc[k] != PRAOS_OK) {
      g->err = "member " + std::to_string(k) + ": " + praos_last_error(g->ctx[k]);
      return rc[k];
    }
  return PRAOS_OK;
}

}  // namespace

extern "C" {

praos_group* praos_group_open(const int* devices, int ndev) {
  if (!devices || ndev <= 0) return nullptr;
  praos_group* g = new praos_group();
  for (int k = 0; k < ndev; k++) {
    praos_ctx* c = praos_open(devices[k]);
    if (!c || devices[k] < 0) {
      if (c) praos_close(c);
      for (praos_ctx* o : g->ctx) praos_close(o);
      delete g;
      return nullptr;
    }
    g->ctx.push_back(c);
  }
  return g;
}

void praos_group_close(praos_group* g) {
  if (!g) return;
  // ranges the caller left registered are unpinned here (after the members' work has drained)
  std::vector<void*> left;
  left.swap(g->registered);
  const int dev0 = g->ctx.empty() ? -1 : praos_ctx_device_(g->ctx[0]);
  for (praos_ctx* c : g->ctx) praos_close(c);
  if (dev0 >= 0 && !left.empty()) {
    (void)hipSetDevice(dev0);
    for (void* p : left) (void)hipHostUnregister(p);
  }
  delete g;
}

int praos_group_size(praos_group* g) { return g ? (int)g->ctx.size() : 0; }

praos_ctx* praos_group_ctx(praos_group* g, int k) {
  return g && k >= 0 && k < (int)g->ctx.size() ? g->ctx[k] : nullptr;
}

const char* praos_group_last_error(praos_group* g) { return g ? g->err.c_str() : "no group"; }

int praos_group_set_option(praos_group* g, int opt, int value) {
  if (!g) return PRAOS_E_ARG;
  for (praos_ctx* c : g->ctx) {
    const int r = praos_set_option(c, opt, value);
    if (r != PRAOS_OK) return r;
  }
  return PRAOS_OK;
}

int praos_group_set_epoch(praos_group* g, const uint8_t eta0[32], const praos_pool* pools, uint32_t npools,
                          const praos_params* params) {
  if (!g) return PRAOS_E_ARG;
  return fan_out(g, [&](size_t k) { return praos_set_epoch(g->ctx[k], eta0, pools, npools, params); });
}

int praos_group_set_overlay(praos_group* g, const praos_overlay* ov) {
  if (!g) return PRAOS_E_ARG;
  return fan_out(g, [&](size_t k) { return praos_set_overlay(g->ctx[k], ov); });
}

int praos_group_verify_headers(praos_group* g, const praos_headers* h, praos_out* out) {
  if (!g || !h || !out || !out->bits) return PRAOS_E_ARG;
  const size_t m = g->ctx.size();
  return fan_out(g, [&](size_t k) {
    size_t i0, i1;
    shard(h->n, m, k, &i0, &i1);
    if (i1 == i0) return (int)PRAOS_OK;
    praos_headers s = headers_at(h, i0, i1);
    praos_out o = out_at(out, i0);
    return praos_verify_headers(g->ctx[k], &s, &o);
  });
}

int praos_group_verify_header_bytes(praos_group* g, const praos_header_bytes* in, praos_out* out,
                                    praos_decoded* dec) {
  if (!g || !in || !out || !out->bits || (in->n && (!in->off || !in->len))) return PRAOS_E_ARG;
  const size_t m = g->ctx.size();
  return fan_out(g, [&](size_t k) {
    size_t i0, i1;
    shard(in->n, m, k, &i0, &i1);
    if (i1 == i0) return (int)PRAOS_OK;
    std::vector<uint64_t> off;
    praos_header_bytes s = bytes_at(in, i0, i1, off);
    praos_out o = out_at(out, i0);
    if (!dec) return praos_verify_header_bytes(g->ctx[k], &s, &o, nullptr);
    praos_decoded d = dec_at(dec, i0);
    return praos_verify_header_bytes(g->ctx[k], &s, &o, &d);
  });
}

// TPraos (Shelley..Alonzo) batches over the group: the same contiguous shards of
// praos_verify_tpraos_headers / praos_verify_tpraos_header_bytes (TPraos.hs:378-387; one
// header is checked against the epoch's ledger view only, so the shards need no exchange).
int praos_group_verify_tpraos_headers(praos_group* g, const praos_tpraos_headers* h, praos_tpraos_out* out) {
  if (!g || !h || !out || !out->bits || (h->h.n && (!h->leader_out || !h->leader_proof))) return PRAOS_E_ARG;
  const size_t m = g->ctx.size();
  return fan_out(g, [&](size_t k) {
    size_t i0, i1;
    shard(h->h.n, m, k, &i0, &i1);
    if (i1 == i0) return (int)PRAOS_OK;
    praos_tpraos_headers s{headers_at(&h->h, i0, i1), at(h->leader_out, i0, 64), at(h->leader_proof, i0, 80)};
    praos_tpraos_out o = tp_out_at(out, i0);
    return praos_verify_tpraos_headers(g->ctx[k], &s, &o);
  });
}

int praos_group_verify_tpraos_header_bytes(praos_group* g, const praos_header_bytes* in, praos_tpraos_out* out,
                                           praos_decoded* dec, uint8_t* leader_out, uint8_t* leader_proof) {
  if (!g || !in || !out || !out->bits || (in->n && (!in->off || !in->len))) return PRAOS_E_ARG;
  const size_t m = g->ctx.size();
  return fan_out(g, [&](size_t k) {
    size_t i0, i1;
    shard(in->n, m, k, &i0, &i1);
    if (i1 == i0) return (int)PRAOS_OK;
    std::vector<uint64_t> off;
    praos_header_bytes s = bytes_at(in, i0, i1, off);
    praos_tpraos_out o = tp_out_at(out, i0);
    praos_decoded d;
    if (dec) d = dec_at(dec, i0, PRAOS_TP_SIGNED_STRIDE);
    return praos_verify_tpraos_header_bytes(g->ctx[k], &s, &o, dec ? &d : nullptr, at(leader_out, i0, 64),
                                            at(leader_proof, i0, 80));
  });
}

// ImmutableDB chunk validation over the group (ABI 14): verifyBlockIntegrity of each block
// (Shelley/Ledger/Integrity.hs:14-20), blocks independent, contiguous shards on the members.
int praos_group_verify_block_integrity(praos_group* g, const praos_header_bytes* blocks, uint64_t slots_per_kes_period,
                                       uint8_t* result, uint8_t* body_hash) {
  if (!g || !blocks || !result || (blocks->n && (!blocks->off || !blocks->len))) return PRAOS_E_ARG;
  const size_t m = g->ctx.size();
  return fan_out(g, [&](size_t k) {
    size_t i0, i1;
    shard(blocks->n, m, k, &i0, &i1);
    if (i1 == i0) return (int)PRAOS_OK;
    std::vector<uint64_t> off;
    praos_header_bytes s = bytes_at(blocks, i0, i1, off);
    return praos_verify_block_integrity(g->ctx[k], &s, slots_per_kes_period, result + i0, at(body_hash, i0, 32));
  });
}

// Page-locks a caller buffer once for every member (hipHostRegisterPortable: one pinning the
// member devices all read by DMA), so each member's upload of its shard is a direct copy.
int praos_group_host_register(praos_group* g, void* p, size_t len) {
  if (!g || !p || len == 0 || g->ctx.empty()) return PRAOS_E_ARG;
  if (hipSetDevice(praos_ctx_device_(g->ctx[0])) != hipSuccess ||
      hipHostRegister(p, len, hipHostRegisterPortable) != hipSuccess) {
    g->err = "hipHostRegister failed";
    return PRAOS_E_HIP;
  }
  for (praos_ctx* c : g->ctx) praos_ctx_note_registered_(c, p, len, true);
  g->registered.push_back(p);
  return PRAOS_OK;
}

int praos_group_host_unregister(praos_group* g, void* p) {
  if (!g || !p) return PRAOS_E_ARG;
  auto it = std::find(g->registered.begin(), g->registered.end(), p);
  if (it == g->registered.end()) { g->err = "range not registered with the group"; return PRAOS_E_ARG; }
  g->registered.erase(it);
  for (praos_ctx* c : g->ctx) praos_ctx_note_registered_(c, p, 0, false);
  (void)hipSetDevice(praos_ctx_device_(g->ctx[0]));
  if (hipHostUnregister(p) != hipSuccess) { g->err = "hipHostUnregister failed"; return PRAOS_E_HIP; }
  return PRAOS_OK;
}

// The ImmutableDB replay over the group (db-analyser's processAllImmutableDB, Analysis.hs:815-847):
// consecutive batches dealt to the members in turn, one nonce chain and one fold in chain order
// (rp_replay, praos_replay.hip); outputs as praos_replay_immutable's on one context.
static int group_replay(praos_group* g, const char* dir, const praos_pool* pools, uint32_t npools,
                        const praos_params* params, const praos_epoch_info* ei, praos_envelope* env,
                        praos_chain_state* st, size_t batch_max, uint8_t* verdicts, uint16_t* failures,
                        size_t verdicts_cap, praos_replay_stats* stats, bool tpraos,
                        const praos_nonce* extra_entropy, const praos_ledger_view* views = nullptr,
                        uint32_t nviews = 0) {
  if (!g || g->ctx.empty()) return PRAOS_E_ARG;
  for (praos_ctx* c : g->ctx) praos_replay_scope_(c, true);
  const int r = rp_replay(g->ctx.data(), (int)g->ctx.size(), dir, pools, npools, params, ei, env, st, batch_max,
                          verdicts, failures, verdicts_cap, stats, tpraos, extra_entropy, views, nviews);
  for (praos_ctx* c : g->ctx) praos_replay_scope_(c, false);
  if (r != PRAOS_OK) g->err = praos_last_error(g->ctx[0]);
  return r;
}

int praos_group_replay_immutable(praos_group* g, const char* dir, const praos_pool* pools, uint32_t npools,
                                 const praos_params* params, const praos_epoch_info* ei, praos_envelope* env,
                                 praos_chain_state* st, size_t batch_max, uint8_t* verdicts, size_t verdicts_cap,
                                 praos_replay_stats* stats) {
  return group_replay(g, dir, pools, npools, params, ei, env, st, batch_max, verdicts, nullptr, verdicts_cap, stats,
                      false, nullptr);
}

int praos_group_replay_immutable_tpraos(praos_group* g, const char* dir, const praos_pool* pools, uint32_t npools,
                                        const praos_params* params, const praos_epoch_info* ei,
                                        const praos_nonce* extra_entropy, praos_envelope* env, praos_chain_state* st,
                                        size_t batch_max, uint8_t* verdicts, uint16_t* failures, size_t verdicts_cap,
                                        praos_replay_stats* stats) {
  return group_replay(g, dir, pools, npools, params, ei, env, st, batch_max, verdicts, failures, verdicts_cap, stats,
                      true, extra_entropy);
}

int praos_group_replay_immutable_views(praos_group* g, const char* dir, const praos_ledger_view* views,
                                       uint32_t nviews, const praos_params* params, const praos_epoch_info* ei,
                                       praos_envelope* env, praos_chain_state* st, size_t batch_max,
                                       uint8_t* verdicts, size_t verdicts_cap, praos_replay_stats* stats) {
  if (!views || nviews == 0) return PRAOS_E_ARG;
  return group_replay(g, dir, nullptr, 0, params, ei, env, st, batch_max, verdicts, nullptr, verdicts_cap, stats,
                      false, nullptr, views, nviews);
}

}  // extern "C"
