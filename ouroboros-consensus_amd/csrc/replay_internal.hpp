#pragma once
// replay_internal.hpp -- entry points of libpraos_hip used by the replay driver
// (praos_replay.hip) for its threaded pipeline; C++ linkage, not part of the C ABI.
#include "praos_hip.h"
#include <cstddef>
#include <cstdint>

struct praos_span {           // a run of stored bytes in host memory (e.g. an mmapped chunk file)
  const uint8_t* p;
  size_t len;
};

// A persistent from-bytes batch with room for n_cap headers over bytes_cap stored bytes, its
// own events and pinned host buffers for the nonce table.
praos_batch* rp_batch_alloc(praos_ctx* c, size_t n_cap, size_t bytes_cap, bool tpraos);
void rp_batch_destroy(praos_ctx* c, praos_batch* b);
bool rp_batch_fits(const praos_batch* b, size_t n, size_t bytes);
// The context keeps the replay's batches between calls (RP_SLOTS of them, freed by praos_close):
// rp_batch_take returns slot k's batch when it fits n headers over `bytes` (else a new one),
// rp_batch_keep hands it back.
constexpr int RP_SLOTS = 4;
praos_batch* rp_batch_take(praos_ctx* c, int k, size_t n, size_t bytes, bool tpraos);
void rp_batch_keep(praos_ctx* c, int k, praos_batch* b);
// the batch's pinned result buffers (bits, pool index: its header capacity each)
void rp_batch_results(praos_batch* b, uint16_t** bits, int32_t** pidx);
// Waits for the batch's last decode and crypto run (a stopped replay leaves queued runs).
void rp_batch_quiesce(praos_batch* b);
// Copy stream: the spans' concatenation (the arena) and the per-header (offset, length) go
// H2D through the pinned staging buffers, then decode and the nonce value of each header's
// certified VRF output (k_vrf_nonce).  Returns once the host side is queued.
int rp_upload_decode(praos_ctx* c, praos_batch* b, size_t n, const praos_span* spans, size_t nspans,
                     const uint64_t* hoff, const uint32_t* hlen);
// D2H of the decoded fields the nonce chain and the fold read, and the nonce values, into the
// batch's pinned area (copy stream; returns when they are in host memory).  d's pointers and
// *nonce stay valid until the batch's next download.
constexpr size_t DEC_H_BYTES = 3 * 8 + 4 * 32 + 4 + 2 + 1;
int rp_download_decoded(praos_ctx* c, praos_batch* b, praos_decoded* d, uint8_t** nonce);
// The crypto run under per-header epoch nonces (etas[eta_idx[i]]), queued after the decode;
// the host arrays are copied before return.
int rp_run(praos_ctx* c, praos_batch* b, const praos_nonce* etas, uint32_t k, const uint8_t* eta_idx);
// Waits for the run and copies its bits and pool indices out (download stream).
int rp_download_results(praos_ctx* c, praos_batch* b, uint16_t* bits, int32_t* pool_idx);
// The pool part of one ledger view (praos_api.hip): host map (hash28 -> caller index) and, when
// built for a device, the tables the VRF join and the leader test read.
struct rp_view;
rp_view* rp_view_make(praos_ctx* c, const praos_pool* pools, uint32_t npools, const praos_params* params,
                      bool device);
void rp_view_free(praos_ctx* c, rp_view* v);
// The device pool tables a context's launches read (praos_set_epoch's, or a view's swapped in by
// the launcher thread: kernels already queued keep the pointers they were launched with).
struct rp_tables {
  uint32_t npools;
  uint32_t *hash, *vrf, *x;
  int32_t* map;
};
rp_tables rp_tables_get(const praos_ctx* c);
void rp_tables_set(praos_ctx* c, const rp_tables& t);
rp_tables rp_view_tables(const rp_view* v);
// praos_validate_headers_nonces / praos_tpraos_validate_headers_nonces with the evolving nonce
// after each header precomputed by the caller's nonce chain (used until the first invalid header);
// view (may be NULL: the context's praos_set_epoch pools) is the ledger view the batch was verified
// under.
int rp_fold(praos_ctx* c, const praos_headers* h, const uint8_t* prev_hash, const uint8_t* prev_is_genesis,
            const praos_out* crypto, praos_envelope* env, const praos_epoch_info* ei, praos_chain_state* st,
            const praos_nonce* etas, uint32_t k, const uint8_t* eta_idx, const praos_nonce* evolving_after,
            bool tpraos, const praos_nonce* extra_entropy, uint8_t* verdict, uint16_t* failures, size_t* chain_stop,
            size_t* processed, const rp_view* view);
// The replay of praos_replay_immutable[_tpraos|_views] over m contexts (praos_replay.hip): batch k
// is uploaded, decoded and verified on mem[k % m]; the nonce chain and the fold run once, in chain
// order, the fold and the error text on mem[0].  m = 1 is the single-context replay.  views
// (nviews > 0, Praos only): a ledger view per epoch instead of pools / env's limits.
int rp_replay(praos_ctx* const* mem, int m, const char* dir, const praos_pool* pools, uint32_t npools,
              const praos_params* params, const praos_epoch_info* ei, praos_envelope* env, praos_chain_state* st,
              size_t batch_max, uint8_t* verdicts, uint16_t* failures, size_t verdicts_cap,
              praos_replay_stats* stats, bool tpraos, const praos_nonce* extra_entropy,
              const praos_ledger_view* views = nullptr, uint32_t nviews = 0);
