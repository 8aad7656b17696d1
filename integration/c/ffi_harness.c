/* ffi_harness.c -- replays, from C, the foreign-call sequence of the Haskell binding
 * (integration/haskell/Ouroboros/Consensus/Protocol/Praos/Batch.hs) against
 * libpraos_hip.so, plus the multi-threaded uses the ABI allows.  Driven by
 * tests/test_gpu_ffi.py, which builds the ImmutableDB and the epoch file and compares
 * the JSON this prints with its own results.
 *
 *   ffi_harness <immutable dir> <epoch file> <threads>
 *   ffi_harness --chunk <immutable dir> <chunk no> <slots per KES period> <members>
 *
 * --chunk: ImmutableDB chunk validation as Batch.hs verifyChunkIntegrity runs it (the batched
 *   checkIntegrity of parseChunkFile, ImmutableDB/Impl/Parser.hs:118-141, Validation.hs:379-384):
 *   the chunk's blocks cut at the secondary index's block offsets, each block's CRC32 against
 *   the entry's checksum, and the blocks whose CRC does not match through
 *   praos_verify_block_integrity (phase "chunk") and praos_group_verify_block_integrity over
 *   <members> contexts on device 0 (phase "chunk_group").  Prints per block -1 (CRC matched, not
 *   checked) or the PRAOS_BLK_* bits, the first corrupt block and the offset parseChunkFile
 *   truncates the chunk file at.
 *
 * epoch file (text, one record per line):
 *   eta0 <64 hex>                      genesis epoch nonce
 *   params <spkp> <maxevo> <f_is_one> <vrf_check_output> <c_raw 32 hex, LE>
 *   epoch <base_slot> <base_no> <length> <stability_window>
 *   env <max_major_pv> <lv_prot_major> <max_header_size> <max_body_size>
 *   pool <hash28 56 hex> <vrf_hash32 64 hex> <sigma_fp 32 hex, LE>
 *   view <first_epoch> <lv_prot_major> <max_header_size> <max_body_size>   (optional, Praos) from
 *                                      this epoch on, the ledger view is the pool lines that follow
 *                                      (until the next view line) and these limits: the LedgerView
 *                                      db-analyser forecasts per epoch (ledgerViewForecastAt,
 *                                      Analysis.hs:564-572).  Pool lines before the first view line
 *                                      form view 0 (from epoch 0, the env line's limits).
 *   tpraos <extra entropy 64 hex | neutral>   (optional) a TPraos (Shelley..Alonzo) database:
 *                                      the binding's TPraos sequence (praos_tpraos_ticked_epoch_nonce
 *                                      -> praos_set_epoch -> praos_verify_tpraos_header_bytes ->
 *                                      praos_tpraos_update_chain_dep_state) and
 *                                      praos_replay_immutable_tpraos; no "threads" phase
 *
 * Output: one JSON object per phase.
 *   "binding":  praosReplayEpochs as the Haskell module runs it (stream the chunk files,
 *               cut at epoch boundaries, praos_ticked_epoch_nonce -> praos_set_epoch ->
 *               praos_verify_header_bytes -> praos_validate_headers, stop at the first
 *               invalid header) and the PraosState CBOR (praos_state_encode) it ends in;
 *   "typed":    the sequence of Batch/Validate.hs validateEpochHeaders (praosValidateHeaderSpans):
 *               per epoch praos_ticked_epoch_nonce -> praos_set_epoch -> praos_host_register of
 *               the arena (the binding does it from 64 MiB on; always here, so the path runs) ->
 *               praos_verify_header_bytes with the decoded fields in one 157-byte-per-header
 *               allocation -> praos_host_unregister -> praos_validate_headers ->
 *               praos_state_encode; also prints the stopping header's verdict and bits, what
 *               Batch.Errors rebuilds the typed HeaderError from (must agree);
 *   "typed_group": the same sequence over a praos_group of <threads> members on device 0, as
 *               validateEpochHeaders runs it on a group context (Batch.hs withPraosBatchDevices):
 *               praos_group_set_epoch -> praos_group_host_register -> praos_group_verify_header_bytes
 *               -> praos_group_host_unregister -> praos_validate_headers on member 0 (must agree);
 *   "binding_group" (TPraos): the TPraos sequence with praos_group_verify_tpraos_header_bytes;
 *   "replay":   praos_replay_immutable over the same directory (must agree);
 *   "replay_group": praos_group_replay_immutable[_tpraos] over <threads> members (must agree);
 *   "analysis": the db-analyser analysis (integration/haskell/.../BenchmarkHeaderBatch.hs): the
 *               ImmutableDB streamed epoch by epoch into a reused, once-registered arena; at each
 *               epoch boundary the next epoch's ledger view is "forecast" (looked up here; the
 *               Haskell side forecasts it from the ledger state it advances) while the previous
 *               epoch validates on a worker thread -- forecast -> praos_ticked_epoch_nonce ->
 *               praos_set_epoch (that epoch's PoolDistr) -> praos_verify_header_bytes ->
 *               praos_validate_headers (that epoch's envelope limits) -> praos_state_encode;
 *               "analysis_group" the same on a group (must agree);
 *   "replay_views" / "replay_views_group": praos_[group_]replay_immutable_views with every view of
 *               the file in one call (must agree with "analysis"); with several views "binding",
 *               "typed" and "replay" use view 0 throughout (a single ledger view for the whole
 *               database, which the test expects to diverge once the PoolDistr changes);
 *   TPraos phases also print the stopping header's PRTCL failure set and the
 *   SL.ChainTransitionError constructors Batch/Errors.hs tpraosChainTransitionError builds from
 *   it (the table below mirrors the Haskell one; tests/test_abi.py checks the two agree);
 *   "threads":  the first epoch's headers split over <threads> POSIX threads, each with
 *               its own praos_ctx on device 0, and the same through praos_group_open
 *               with <threads> members: bits / pool_idx / nonce equal to one context's.
 */
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "praos_hip.h"

#define DIE(...) do { fprintf(stderr, __VA_ARGS__); fputc('\n', stderr); exit(2); } while (0)
#define CK(ctx, x) do { int rc_ = (x); if (rc_ != PRAOS_OK) DIE("%s -> %d: %s", #x, rc_, praos_last_error(ctx)); } while (0)

static void hex_in(const char* s, uint8_t* out, size_t n) {
  if (strlen(s) != 2 * n) DIE("hex field of %zu bytes expected: %s", n, s);
  for (size_t i = 0; i < n; i++) {
    unsigned v;
    if (sscanf(s + 2 * i, "%2x", &v) != 1) DIE("bad hex %s", s);
    out[i] = (uint8_t)v;
  }
}

static void hex_out(const uint8_t* p, size_t n) {
  for (size_t i = 0; i < n; i++) printf("%02x", p[i]);
}

static uint64_t be(const uint8_t* p, int n) {
  uint64_t v = 0;
  for (int k = 0; k < n; k++) v = (v << 8) | p[k];
  return v;
}

static uint8_t* slurp(const char* path, size_t* len) {
  FILE* f = fopen(path, "rb");
  if (!f) return NULL;
  fseek(f, 0, SEEK_END);
  long sz = ftell(f);
  fseek(f, 0, SEEK_SET);
  uint8_t* p = malloc(sz > 0 ? (size_t)sz : 1);
  if (sz > 0 && fread(p, 1, (size_t)sz, f) != (size_t)sz) DIE("read %s", path);
  fclose(f);
  *len = (size_t)(sz > 0 ? sz : 0);
  return p;
}

/* ---- inputs ---- */
static uint8_t g_eta0[32];
static praos_params g_params;
static praos_epoch_info g_ei;
static praos_envelope g_env0;
static praos_pool* g_pools;
static uint32_t g_npools;
static int g_tpraos;
static praos_nonce g_extra;              /* TICKN's extra entropy (TPraos) */
/* ledger views per epoch ("view" lines); view 0 = the pools before the first view line */
enum { MAXV = 256 };
static praos_ledger_view g_views[MAXV];
static uint32_t g_nviews;
static praos_pool* g_vpools[MAXV];
static uint32_t g_vcap[MAXV];

static void read_epoch_file(const char* path) {
  FILE* f = fopen(path, "r");
  if (!f) DIE("open %s", path);
  char line[512], a[128], b[128], c[128];
  uint32_t cap = 0;
  int cur = 0;                               /* the view pool lines go to (0: g_pools) */
  while (fgets(line, sizeof line, f)) {
    unsigned long long x, y, z, w;
    if (sscanf(line, "view %llu %llu %llu %llu", &x, &y, &z, &w) == 4) {
      if (g_nviews == 0) g_nviews = 1;       /* view 0 = g_pools (filled in below) */
      if (g_nviews == MAXV) DIE("too many views");
      cur = (int)g_nviews++;
      memset(&g_views[cur], 0, sizeof g_views[cur]);
      g_views[cur].first_epoch = x;
      g_views[cur].lv_prot_major = y; g_views[cur].max_header_size = z; g_views[cur].max_body_size = w;
    } else if (cur > 0 && sscanf(line, "pool %127s %127s %127s", a, b, c) == 3) {
      praos_ledger_view* v = &g_views[cur];
      if (v->npools == g_vcap[cur]) {
        g_vcap[cur] = g_vcap[cur] ? 2 * g_vcap[cur] : 64;
        g_vpools[cur] = realloc(g_vpools[cur], g_vcap[cur] * sizeof *g_vpools[cur]);
      }
      praos_pool* pp = &g_vpools[cur][v->npools++];
      hex_in(a, pp->hash28, 28);
      hex_in(b, pp->vrf_hash32, 32);
      hex_in(c, pp->sigma_fp, 16);
      v->pools = g_vpools[cur];
    } else if (sscanf(line, "eta0 %127s", a) == 1) {
      hex_in(a, g_eta0, 32);
    } else if (sscanf(line, "params %llu %llu %llu %llu %127s", &x, &y, &z, &w, a) == 5) {
      g_params.slots_per_kes_period = x;
      g_params.max_kes_evo = y;
      g_params.f_is_one = (int32_t)z;
      g_params.vrf_check_output = (int32_t)w;
      hex_in(a, g_params.c_raw, 16);
    } else if (sscanf(line, "epoch %llu %llu %llu %llu", &x, &y, &z, &w) == 4) {
      g_ei.epoch_base_slot = x; g_ei.epoch_base_no = y; g_ei.epoch_length = z; g_ei.stability_window = w;
    } else if (sscanf(line, "env %llu %llu %llu %llu", &x, &y, &z, &w) == 4) {
      g_env0.max_major_pv = x; g_env0.lv_prot_major = y; g_env0.max_header_size = z; g_env0.max_body_size = w;
    } else if (sscanf(line, "tpraos %127s", a) == 1) {
      g_tpraos = 1;
      if (strcmp(a, "neutral") == 0) g_extra.neutral = 1;
      else hex_in(a, g_extra.hash, 32);
    } else if (sscanf(line, "pool %127s %127s %127s", a, b, c) == 3) {
      if (g_npools == cap) {
        cap = cap ? 2 * cap : 64;
        g_pools = realloc(g_pools, cap * sizeof *g_pools);
      }
      hex_in(a, g_pools[g_npools].hash28, 28);
      hex_in(b, g_pools[g_npools].vrf_hash32, 32);
      hex_in(c, g_pools[g_npools].sigma_fp, 16);
      g_npools++;
    }
  }
  fclose(f);
  g_env0.tip_is_origin = 1;
  if (g_nviews == 0) g_nviews = 1;
  g_views[0].first_epoch = 0;
  g_views[0].pools = g_pools;
  g_views[0].npools = g_npools;
  g_views[0].lv_prot_major = g_env0.lv_prot_major;
  g_views[0].max_header_size = g_env0.max_header_size;
  g_views[0].max_body_size = g_env0.max_body_size;
  for (uint32_t k = 1; k < g_nviews; k++)
    if (g_views[k].first_epoch <= g_views[k - 1].first_epoch) DIE("view lines: first_epoch must increase");
}

/* the "forecast": the ledger view of epoch e (the last view line with first_epoch <= e) */
static const praos_ledger_view* view_for(uint64_t e) {
  const praos_ledger_view* v = &g_views[0];
  for (uint32_t k = 1; k < g_nviews; k++)
    if (g_views[k].first_epoch <= e) v = &g_views[k];
  return v;
}

/* the stored headers, in chain order, through the secondary indexes */
typedef struct {
  uint8_t* bytes;   /* all headers back to back */
  size_t len, n, cap;
  uint64_t* off;
  uint32_t* hlen;
  uint64_t* slot;
} chain_t;

static void read_chain(const char* dir, chain_t* ch) {
  memset(ch, 0, sizeof *ch);
  for (int c = 0;; c++) {
    char p[4096];
    size_t dl, sl;
    snprintf(p, sizeof p, "%s/%05d.chunk", dir, c);
    uint8_t* data = slurp(p, &dl);
    if (!data) break;
    snprintf(p, sizeof p, "%s/%05d.secondary", dir, c);
    uint8_t* sec = slurp(p, &sl);
    if (!sec || sl % 56) DIE("secondary %d", c);
    for (size_t e = 0; e < sl / 56; e++) {
      const uint8_t* r = sec + 56 * e;
      const uint64_t boff = be(r, 8), hoff = be(r + 8, 2), hsz = be(r + 10, 2);
      if (boff + hoff + hsz > dl) DIE("entry outside chunk");
      if (ch->n == ch->cap) {
        ch->cap = ch->cap ? 2 * ch->cap : 1024;
        ch->off = realloc(ch->off, ch->cap * 8);
        ch->hlen = realloc(ch->hlen, ch->cap * 4);
        ch->slot = realloc(ch->slot, ch->cap * 8);
      }
      ch->bytes = realloc(ch->bytes, ch->len + hsz);
      memcpy(ch->bytes + ch->len, data + boff + hoff, hsz);
      ch->off[ch->n] = ch->len;
      ch->hlen[ch->n] = (uint32_t)hsz;
      ch->slot[ch->n] = be(r + 48, 8);
      ch->len += hsz;
      ch->n++;
    }
    free(data);
    free(sec);
  }
}

/* ---- chain state storage ---- */
enum { CAP = 1 << 16 };
typedef struct {
  praos_chain_state st;
  uint8_t hk[28 * CAP];
  uint64_t ctr[CAP];
} state_buf;

static void genesis_state(state_buf* s) {
  memset(s, 0, sizeof *s);
  s->st.last_slot_origin = 1;
  s->st.counter_hash28 = s->hk;
  s->st.counter = s->ctr;
  s->st.cap = CAP;
  memcpy(s->st.evolving.hash, g_eta0, 32);
  memcpy(s->st.candidate.hash, g_eta0, 32);
  memcpy(s->st.epoch_nonce.hash, g_eta0, 32);
  s->st.lab.neutral = 1;
  s->st.last_epoch_block.neutral = 1;
}

/* stop_bits < 0: not reported */
static void print_state(const char* phase, const state_buf* s, const praos_envelope* env, uint64_t validated,
                        uint64_t stop, int stop_verdict, uint64_t epochs, long stop_bits) {
  size_t len = 0;
  static uint8_t buf[64 + 48 * CAP];
  if (praos_state_encode(&s->st, buf, sizeof buf, &len) != PRAOS_OK) DIE("state_encode");
  if (stop_bits >= 0) printf("{\"stop_bits\": %ld, ", stop_bits);
  else printf("{");
  printf("\"phase\": \"%s\", \"validated\": %llu, \"stop_index\": %llu, \"stop_verdict\": %d, \"epochs\": %llu, "
         "\"tip_slot\": %llu, \"tip_block_no\": %llu, \"tip_hash\": \"", phase, (unsigned long long)validated,
         (unsigned long long)stop, stop_verdict, (unsigned long long)epochs, (unsigned long long)env->tip_slot,
         (unsigned long long)env->tip_block_no);
  hex_out(env->tip_hash, 32);
  printf("\", \"state_cbor\": \"");
  hex_out(buf, len);
  printf("\"}\n");
  fflush(stdout);
}

/* PRAOS_TPF_* -> the PRTCL predicate failure Batch/Errors.hs tpraosChainTransitionError builds,
 * in the order ValidateAll collects them: OVERLAY's own (NotActiveSlot, or WrongGenesisColdKey
 * then the first failure of the VRF checks), then those of the OCERT sub-rule in the order
 * ocertTransition checks them.  (mirrored by the Haskell table;
 * tests/test_abi.py::test_tpraos_error_table_matches_haskell) */
static const struct { unsigned bit; const char* name; } TPF_NAMES[] = {
  {PRAOS_TPF_NOT_ACTIVE, "NotActiveSlotOVERLAY"},
  {PRAOS_TPF_GEN_COLD, "WrongGenesisColdKeyOVERLAY"},
  {PRAOS_TPF_VRF_KEY_UNKNOWN, "VRFKeyUnknown"},
  {PRAOS_TPF_VRF_KEY_WRONG, "VRFKeyWrongVRFKey"},
  {PRAOS_TPF_GEN_VRF, "WrongGenesisVRFKeyOVERLAY"},
  {PRAOS_TPF_BAD_NONCE, "VRFKeyBadNonce"},
  {PRAOS_TPF_BAD_LEADER, "VRFKeyBadLeaderValue"},
  {PRAOS_TPF_LEADER_TOO_BIG, "VRFLeaderValueTooBig"},
  {PRAOS_TPF_KES_BEFORE_START, "OcertFailure KESBeforeStartOCERT"},
  {PRAOS_TPF_KES_AFTER_END, "OcertFailure KESAfterEndOCERT"},
  {PRAOS_TPF_OCERT_SIG, "OcertFailure InvalidSignatureOCERT"},
  {PRAOS_TPF_KES_SIG, "OcertFailure InvalidKesSignatureOCERT"},
  {PRAOS_TPF_COUNTER_MISSING, "OcertFailure NoCounterForKeyHashOCERT"},
  {PRAOS_TPF_COUNTER_TOO_SMALL, "OcertFailure CounterTooSmallOCERT"},
  {PRAOS_TPF_COUNTER_OVER_INC, "OcertFailure CounterOverIncrementedOCERT"},
};

/* the stopping TPraos header's failure set and the ChainTransitionError it stands for */
static void print_tpraos_stop(unsigned fails) {
  printf("{\"phase\": \"tpraos_stop\", \"failures\": %u, \"errors\": [", fails);
  int first = 1;
  for (size_t k = 0; k < sizeof TPF_NAMES / sizeof TPF_NAMES[0]; k++)
    if (fails & TPF_NAMES[k].bit) {
      printf("%s\"OverlayFailure (%s)\"", first ? "" : ", ", TPF_NAMES[k].name);
      first = 0;
    }
  printf("]}\n");
  fflush(stdout);
}

/* ---- phase 1: the Haskell binding's call sequence (Batch.hs praosReplayEpochs) ---- */
static void phase_binding(const chain_t* ch, int members) {
  praos_group* g = NULL;
  praos_ctx* ctx;
  if (members > 0) {
    int devs[64] = {0};
    g = praos_group_open(devs, members);
    if (!g) DIE("praos_group_open");
    ctx = praos_group_ctx(g, 0);
  } else {
    ctx = praos_open(0);
  }
  if (!ctx) DIE("praos_open(0)");
  unsigned stop_fails = 0;
  static state_buf S;
  genesis_state(&S);
  praos_envelope env = g_env0;
  uint64_t validated = 0, stop_index = ch->n, epochs = 0;
  int stop_verdict = 0;
  size_t i = 0;
  while (i < ch->n) {
    /* one epoch's headers */
    const uint64_t e = (ch->slot[i] - g_ei.epoch_base_slot) / g_ei.epoch_length;
    size_t j = i;
    while (j < ch->n && (ch->slot[j] - g_ei.epoch_base_slot) / g_ei.epoch_length == e) j++;
    const size_t n = j - i;
    praos_nonce eta;
    if (g_tpraos) CK(ctx, praos_tpraos_ticked_epoch_nonce(&S.st, &g_ei, ch->slot[i], &g_extra, &eta));
    else CK(ctx, praos_ticked_epoch_nonce(&S.st, &g_ei, ch->slot[i], &eta));
    if (g) {
      if (praos_group_set_epoch(g, eta.neutral ? NULL : eta.hash, g_pools, g_npools, &g_params) != PRAOS_OK)
        DIE("%s", praos_group_last_error(g));
    } else {
      CK(ctx, praos_set_epoch(ctx, eta.neutral ? NULL : eta.hash, g_pools, g_npools, &g_params));
    }
    epochs++;
    uint64_t* off = malloc(8 * n);
    for (size_t k = 0; k < n; k++) off[k] = ch->off[i + k];
    praos_header_bytes hb = {n, ch->bytes, ch->len, off, ch->hlen + i};
    uint16_t* bits = calloc(n, 2);
    int32_t* pidx = calloc(n, 4);
    uint8_t* nonce = calloc(n, 32);
    praos_out out = {bits, pidx, NULL, NULL, nonce};
    praos_decoded dec;
    memset(&dec, 0, sizeof dec);
    uint64_t *slot = calloc(n, 8), *bno = calloc(n, 8), *ocn = calloc(n, 8);
    uint8_t *prev = calloc(n, 32), *gen = calloc(n, 1), *cold = calloc(n, 32), *hh = calloc(n, 32);
    uint32_t* bsz = calloc(n, 4);
    dec.slot = slot; dec.block_no = bno; dec.ocert_n = ocn; dec.prev_hash = prev; dec.prev_is_genesis = gen;
    dec.cold_vk = cold; dec.header_hash = hh; dec.body_size = bsz;
    praos_headers h;
    memset(&h, 0, sizeof h);
    h.n = n; h.slot = slot; h.cold_vk = cold; h.ocert_n = ocn;
    env.block_no = bno; env.header_hash = hh; env.header_size = ch->hlen + i; env.body_size = bsz;
    uint8_t* verdict = calloc(n, 1);
    size_t stop = 0, done = 0;
    if (g_tpraos) {
      uint16_t* fails = calloc(n, 2);
      praos_tpraos_out tout = {bits, pidx, NULL, NULL, nonce};
      if (g) {
        if (praos_group_verify_tpraos_header_bytes(g, &hb, &tout, &dec, NULL, NULL) != PRAOS_OK)
          DIE("%s", praos_group_last_error(g));
      } else {
        CK(ctx, praos_verify_tpraos_header_bytes(ctx, &hb, &tout, &dec, NULL, NULL));
      }
      praos_tpraos_headers th;
      memset(&th, 0, sizeof th);
      th.h = h;
      CK(ctx, praos_tpraos_update_chain_dep_state(ctx, &th, prev, gen, &tout, &env, &g_ei, &g_extra, &S.st, verdict,
                                                  fails, &stop, &done));
      if (stop < n) stop_fails = fails[stop];
      free(fails);
    } else if (g) {
      if (praos_group_verify_header_bytes(g, &hb, &out, &dec) != PRAOS_OK) DIE("%s", praos_group_last_error(g));
      CK(ctx, praos_validate_headers(ctx, &h, prev, gen, &out, &env, &g_ei, &S.st, verdict, &stop, &done));
    } else {
      CK(ctx, praos_verify_header_bytes(ctx, &hb, &out, &dec));
      CK(ctx, praos_validate_headers(ctx, &h, prev, gen, &out, &env, &g_ei, &S.st, verdict, &stop, &done));
    }
    if (done != n) DIE("an epoch batch did not fold through (%zu of %zu)", done, n);
    const int stopped = stop < n;
    if (stopped) { stop_index = i + stop; stop_verdict = verdict[stop]; validated += stop; }
    else validated += n;
    free(off); free(bits); free(pidx); free(nonce); free(slot); free(bno); free(ocn); free(prev); free(gen);
    free(cold); free(hh); free(bsz); free(verdict);
    if (stopped) break;
    i = j;
  }
  print_state(g ? "binding_group" : "binding", &S, &env, validated, stop_index, stop_verdict, epochs, -1);
  if (g_tpraos && !g && stop_index < ch->n) print_tpraos_stop(stop_fails);
  if (g) praos_group_close(g);
  else praos_close(ctx);
}

/* ---- phase 1b: Batch/Validate.hs validateEpochHeaders (Storable vectors, registered arena) ----
 * sub > 0 (one context): each epoch's headers as `sub` consecutive batches through the streaming
 * form (Batch.hs praosSubmitHeaderBytes / praosDrainHeaderBytes: praos_verify_header_bytes_submit
 * with the chunked pipeline forced on, then praos_verify_drain), folded in order afterwards. */
typedef struct {
  size_t i0, n, alen;
  uint8_t *arena, *verdict, *decbuf;
  uint64_t* off;
  uint16_t* bits;
  int32_t* pidx;
  praos_header_bytes hb;
  praos_out out;
  praos_decoded dec;
} part_t;

static void part_init(part_t* p, const chain_t* ch, size_t i0, size_t n) {
  memset(p, 0, sizeof *p);
  p->i0 = i0;
  p->n = n;
  for (size_t k = 0; k < n; k++) p->alen += ch->hlen[i0 + k];
  p->arena = malloc(p->alen ? p->alen : 1);
  p->off = malloc(8 * (n ? n : 1));
  for (size_t k = 0, o = 0; k < n; o += ch->hlen[i0 + k], k++) {   /* the spans back to back */
    memcpy(p->arena + o, ch->bytes + ch->off[i0 + k], ch->hlen[i0 + k]);
    p->off[k] = o;
  }
  p->verdict = calloc(n ? n : 1, 1);
  p->bits = calloc(n ? n : 1, 2);
  p->pidx = calloc(n ? n : 1, 4);
  p->decbuf = calloc(n ? n : 1, 157);  /* slot, block no, ocert n | prev, cold, hash | body size | gen | nonce */
  praos_header_bytes hb = {n, p->arena, p->alen, p->off, ch->hlen + i0};
  p->hb = hb;
  praos_out out = {p->bits, p->pidx, NULL, NULL, p->decbuf + 125 * n};   /* nonce values: the fold evolves them */
  p->out = out;
  p->dec.slot = (uint64_t*)p->decbuf;
  p->dec.block_no = (uint64_t*)(p->decbuf + 8 * n);
  p->dec.ocert_n = (uint64_t*)(p->decbuf + 16 * n);
  p->dec.prev_hash = p->decbuf + 24 * n;
  p->dec.cold_vk = p->decbuf + 56 * n;
  p->dec.header_hash = p->decbuf + 88 * n;
  p->dec.body_size = (uint32_t*)(p->decbuf + 120 * n);
  p->dec.prev_is_genesis = p->decbuf + 124 * n;
}

static void part_free(part_t* p) {
  free(p->arena); free(p->off); free(p->verdict); free(p->bits); free(p->pidx); free(p->decbuf);
}

static void phase_typed(const chain_t* ch, int members, int sub) {
  praos_group* g = NULL;
  praos_ctx* ctx;
  if (members > 0) {
    int devs[64] = {0};
    g = praos_group_open(devs, members);
    if (!g) DIE("praos_group_open");
    ctx = praos_group_ctx(g, 0);
  } else {
    ctx = praos_open(0);
  }
  if (!ctx) DIE("praos_open(0)");
  if (sub > 0) CK(ctx, praos_set_option(ctx, PRAOS_OPT_PIPELINE, 2));
  static state_buf S;
  genesis_state(&S);
  praos_envelope env = g_env0;
  uint64_t validated = 0, stop_index = ch->n, epochs = 0;
  int stop_verdict = 0;
  unsigned stop_bits = 0;
  size_t i = 0;
  int stopped = 0;
  while (i < ch->n && !stopped) {
    const uint64_t e = (ch->slot[i] - g_ei.epoch_base_slot) / g_ei.epoch_length;
    size_t j = i;
    while (j < ch->n && (ch->slot[j] - g_ei.epoch_base_slot) / g_ei.epoch_length == e) j++;
    praos_nonce eta;
    CK(ctx, praos_ticked_epoch_nonce(&S.st, &g_ei, ch->slot[i], &eta));
    if (g) {
      if (praos_group_set_epoch(g, eta.neutral ? NULL : eta.hash, g_pools, g_npools, &g_params) != PRAOS_OK)
        DIE("%s", praos_group_last_error(g));
    } else {
      CK(ctx, praos_set_epoch(ctx, eta.neutral ? NULL : eta.hash, g_pools, g_npools, &g_params));
    }
    epochs++;
    const int np = sub > 0 ? sub : 1;
    part_t parts[8];
    for (int q = 0; q < np; q++) {
      const size_t a = i + (j - i) * (size_t)q / (size_t)np, b = i + (j - i) * (size_t)(q + 1) / (size_t)np;
      part_init(&parts[q], ch, a, b - a);
    }
    for (int q = 0; q < np; q++) {
      part_t* p = &parts[q];
      if (g) {
        if (praos_group_host_register(g, p->arena, p->alen ? p->alen : 1) != PRAOS_OK ||
            praos_group_verify_header_bytes(g, &p->hb, &p->out, &p->dec) != PRAOS_OK ||
            praos_group_host_unregister(g, p->arena) != PRAOS_OK)
          DIE("%s", praos_group_last_error(g));
      } else if (sub > 0) {
        CK(ctx, praos_host_register(ctx, p->arena, p->alen ? p->alen : 1));
        CK(ctx, praos_verify_header_bytes_submit(ctx, &p->hb, &p->out, &p->dec));
      } else {
        CK(ctx, praos_host_register(ctx, p->arena, p->alen ? p->alen : 1));
        CK(ctx, praos_verify_header_bytes(ctx, &p->hb, &p->out, &p->dec));
        CK(ctx, praos_host_unregister(ctx, p->arena));
      }
    }
    if (sub > 0) {
      CK(ctx, praos_verify_drain(ctx));
      for (int q = 0; q < np; q++) CK(ctx, praos_host_unregister(ctx, parts[q].arena));
    }
    for (int q = 0; q < np && !stopped; q++) {
      part_t* p = &parts[q];
      const size_t n = p->n;
      praos_headers h;
      memset(&h, 0, sizeof h);
      h.n = n; h.slot = p->dec.slot; h.cold_vk = p->dec.cold_vk; h.ocert_n = p->dec.ocert_n;
      env.block_no = p->dec.block_no; env.header_hash = p->dec.header_hash; env.header_size = ch->hlen + p->i0;
      env.body_size = p->dec.body_size;
      size_t stop = 0, done = 0;
      CK(ctx, praos_validate_headers(ctx, &h, p->dec.prev_hash, p->dec.prev_is_genesis, &p->out, &env, &g_ei, &S.st,
                                     p->verdict, &stop, &done));
      if (done != n) DIE("an epoch batch did not fold through (%zu of %zu)", done, n);
      if (stop < n) {
        stopped = 1;
        stop_index = p->i0 + stop; stop_verdict = p->verdict[stop]; stop_bits = p->bits[stop]; validated += stop;
      } else {
        validated += n;
      }
    }
    for (int q = 0; q < np; q++) part_free(&parts[q]);
    i = j;
  }
  print_state(g ? "typed_group" : sub > 0 ? "typed_stream" : "typed", &S, &env, validated, stop_index, stop_verdict,
              epochs, (long)stop_bits);
  if (g) praos_group_close(g);
  else praos_close(ctx);
}

/* ---- phase 2: the library's own driver ---- */
static void phase_replay(const char* dir, int members) {
  static state_buf S;
  genesis_state(&S);
  praos_envelope env = g_env0;
  praos_replay_stats rs;
  if (members > 0) {
    int devs[64] = {0};
    praos_group* g = praos_group_open(devs, members);
    if (!g) DIE("praos_group_open");
    const int rc = g_tpraos
        ? praos_group_replay_immutable_tpraos(g, dir, g_pools, g_npools, &g_params, &g_ei, &g_extra, &env, &S.st, 97,
                                              NULL, NULL, 0, &rs)
        : praos_group_replay_immutable(g, dir, g_pools, g_npools, &g_params, &g_ei, &env, &S.st, 97, NULL, 0, &rs);
    if (rc != PRAOS_OK) DIE("group replay -> %d: %s", rc, praos_group_last_error(g));
    print_state("replay_group", &S, &env, rs.validated, rs.stop_index, (int)rs.stop_verdict, rs.epochs, -1);
    praos_group_close(g);
    return;
  }
  praos_ctx* ctx = praos_open(0);
  if (!ctx) DIE("praos_open(0)");
  if (g_tpraos)
    CK(ctx, praos_replay_immutable_tpraos(ctx, dir, g_pools, g_npools, &g_params, &g_ei, &g_extra, &env, &S.st,
                                          1 << 16, NULL, NULL, 0, &rs));
  else
    CK(ctx, praos_replay_immutable(ctx, dir, g_pools, g_npools, &g_params, &g_ei, &env, &S.st, 1 << 16, NULL, 0,
                                   &rs));
  print_state("replay", &S, &env, rs.validated, rs.stop_index, (int)rs.stop_verdict, rs.epochs, -1);
  praos_close(ctx);
}

/* ---- phase 2b: the db-analyser analysis (BenchmarkHeaderBatch.hs), epoch e on a worker thread
 *      while the stream / ledger of epoch e+1 goes on ---- */
typedef struct {                 /* one epoch's arena as the analysis fills it (reused, registered once) */
  uint8_t* bytes;
  size_t cap, len;
  uint64_t* off;
  uint32_t* hlen;
  size_t n, ncap;
  uint64_t first_slot, epoch;
  int registered;
} arena_t;

typedef struct {
  praos_ctx* ctx;
  praos_group* g;
  arena_t* a;
  const praos_ledger_view* view;
  state_buf* S;
  praos_envelope* env;
  /* out */
  size_t stop;
  int verdict;
  int rc;
  char err[256];
} epoch_job;

static void arena_push(arena_t* a, const uint8_t* hdr, uint32_t len, uint64_t slot, uint64_t epoch,
                       praos_ctx* ctx, praos_group* g) {
  if (a->n == 0) { a->first_slot = slot; a->epoch = epoch; a->len = 0; }
  if (a->len + len > a->cap) {              /* grow: unregister, reallocate, register once more */
    if (a->registered) {
      if (g) praos_group_host_unregister(g, a->bytes);
      else praos_host_unregister(ctx, a->bytes);
    }
    a->cap = 2 * (a->len + len);
    a->bytes = realloc(a->bytes, a->cap);
    const int rc = g ? praos_group_host_register(g, a->bytes, a->cap) : praos_host_register(ctx, a->bytes, a->cap);
    if (rc != PRAOS_OK) DIE("host_register -> %d", rc);
    a->registered = 1;
  }
  if (a->n == a->ncap) {
    a->ncap = a->ncap ? 2 * a->ncap : 4096;
    a->off = realloc(a->off, 8 * a->ncap);
    a->hlen = realloc(a->hlen, 4 * a->ncap);
  }
  memcpy(a->bytes + a->len, hdr, len);
  a->off[a->n] = a->len;
  a->hlen[a->n] = len;
  a->len += len;
  a->n++;
}

/* validateEpochHeaders (Batch/Validate.hs) of one epoch under its forecast ledger view */
static void* epoch_worker(void* arg) {
  epoch_job* j = arg;
  arena_t* a = j->a;
  const size_t n = a->n;
  j->rc = PRAOS_OK;
  j->stop = n;
  praos_nonce eta;
  int rc = praos_ticked_epoch_nonce(&j->S->st, &g_ei, a->first_slot, &eta);
  if (rc == PRAOS_OK)
    rc = j->g ? praos_group_set_epoch(j->g, eta.neutral ? NULL : eta.hash, j->view->pools, j->view->npools, &g_params)
              : praos_set_epoch(j->ctx, eta.neutral ? NULL : eta.hash, j->view->pools, j->view->npools, &g_params);
  uint8_t* verdict = calloc(n, 1);
  uint16_t* bits = calloc(n, 2);
  int32_t* pidx = calloc(n, 4);
  uint8_t* decbuf = calloc(n, 157);
  uint64_t *slot = (uint64_t*)decbuf, *bno = (uint64_t*)(decbuf + 8 * n), *ocn = (uint64_t*)(decbuf + 16 * n);
  uint8_t *prev = decbuf + 24 * n, *cold = decbuf + 56 * n, *hh = decbuf + 88 * n, *gen = decbuf + 124 * n;
  uint32_t* bsz = (uint32_t*)(decbuf + 120 * n);
  uint8_t* nonce = decbuf + 125 * n;
  praos_header_bytes hb = {n, a->bytes, a->len, a->off, a->hlen};
  praos_out out = {bits, pidx, NULL, NULL, nonce};
  praos_decoded dec;
  memset(&dec, 0, sizeof dec);
  dec.slot = slot; dec.block_no = bno; dec.ocert_n = ocn; dec.prev_hash = prev; dec.prev_is_genesis = gen;
  dec.cold_vk = cold; dec.header_hash = hh; dec.body_size = bsz;
  if (rc == PRAOS_OK)
    rc = j->g ? praos_group_verify_header_bytes(j->g, &hb, &out, &dec) : praos_verify_header_bytes(j->ctx, &hb, &out, &dec);
  if (rc == PRAOS_OK) {
    praos_headers h;
    memset(&h, 0, sizeof h);
    h.n = n; h.slot = slot; h.cold_vk = cold; h.ocert_n = ocn;
    praos_envelope* env = j->env;
    env->lv_prot_major = j->view->lv_prot_major;        /* the forecast view's envelope limits */
    env->max_header_size = j->view->max_header_size;
    env->max_body_size = j->view->max_body_size;
    env->block_no = bno; env->header_hash = hh; env->header_size = a->hlen; env->body_size = bsz;
    size_t stop = 0, done = 0;
    praos_ctx* c0 = j->g ? praos_group_ctx(j->g, 0) : j->ctx;
    rc = praos_validate_headers(c0, &h, prev, gen, &out, env, &g_ei, &j->S->st, verdict, &stop, &done);
    env->block_no = NULL; env->header_hash = NULL; env->header_size = NULL; env->body_size = NULL;
    if (rc == PRAOS_OK && done != n) { rc = -100; snprintf(j->err, sizeof j->err, "epoch did not fold through"); }
    j->stop = stop;
    if (stop < n) j->verdict = verdict[stop];
  }
  if (rc != PRAOS_OK && !j->err[0])
    snprintf(j->err, sizeof j->err, "%s", j->g ? praos_group_last_error(j->g) : praos_last_error(j->ctx));
  j->rc = rc;
  free(verdict); free(bits); free(pidx); free(decbuf);
  return NULL;
}

static void phase_analysis(const chain_t* ch, int members) {
  praos_group* g = NULL;
  praos_ctx* ctx = NULL;
  if (members > 0) {
    int devs[64] = {0};
    if (members > 64) DIE("members: 1..64");
    g = praos_group_open(devs, members);
    if (!g) DIE("praos_group_open");
  } else {
    ctx = praos_open(0);
    if (!ctx) DIE("praos_open(0)");
  }
  static state_buf S;
  genesis_state(&S);
  praos_envelope env = g_env0;
  arena_t ar[2];
  memset(ar, 0, sizeof ar);
  uint64_t validated = 0, stop_index = ch->n, epochs = 0, first_index[2] = {0, 0};
  int stop_verdict = 0, cur = 0, running = 0, stopped = 0;
  pthread_t th;
  epoch_job job;
  /* waits for the epoch on the worker; 1 if the chain goes on */
  #define JOIN_WORKER()                                                                   \
    do {                                                                                  \
      if (running) {                                                                      \
        pthread_join(th, NULL);                                                           \
        running = 0;                                                                      \
        if (job.rc != PRAOS_OK) DIE("analysis epoch: %d %s", job.rc, job.err);            \
        const int w = 1 - cur;                                                            \
        if (job.stop < ar[w].n) {                                                         \
          stop_index = first_index[w] + job.stop; stop_verdict = job.verdict;             \
          validated += job.stop; stopped = 1;                                             \
        } else {                                                                          \
          validated += ar[w].n;                                                           \
        }                                                                                 \
      }                                                                                   \
    } while (0)
  for (size_t i = 0; i <= ch->n && !stopped; i++) {
    const uint64_t e = i < ch->n ? (ch->slot[i] - g_ei.epoch_base_slot) / g_ei.epoch_length : UINT64_MAX;
    if (ar[cur].n && (i == ch->n || e != ar[cur].epoch)) {
      /* epoch ar[cur] complete: its view was forecast from the ledger state before its first
       * block; the previous epoch's validation must finish first (its state is this one's input) */
      JOIN_WORKER();
      if (stopped) break;
      memset(&job, 0, sizeof job);
      job.ctx = ctx; job.g = g; job.a = &ar[cur]; job.view = view_for(ar[cur].epoch); job.S = &S; job.env = &env;
      epochs++;
      if (pthread_create(&th, NULL, epoch_worker, &job) != 0) DIE("pthread_create");
      running = 1;
      cur = 1 - cur;                          /* the stream goes on into the other arena */
      ar[cur].n = 0;
    }
    if (i == ch->n) break;
    if (ar[cur].n == 0) first_index[cur] = i;
    arena_push(&ar[cur], ch->bytes + ch->off[i], ch->hlen[i], ch->slot[i], e, ctx, g);
  }
  JOIN_WORKER();
  #undef JOIN_WORKER
  print_state(g ? "analysis_group" : "analysis", &S, &env, validated, stop_index, stop_verdict, epochs, -1);
  for (int k = 0; k < 2; k++) {
    if (ar[k].registered) {
      if (g) praos_group_host_unregister(g, ar[k].bytes);
      else praos_host_unregister(ctx, ar[k].bytes);
    }
    free(ar[k].bytes); free(ar[k].off); free(ar[k].hlen);
  }
  if (g) praos_group_close(g);
  else praos_close(ctx);
}

/* ---- phase 2c: every ledger view in one replay call ---- */
static void phase_replay_views(const char* dir, int members) {
  static state_buf S;
  genesis_state(&S);
  praos_envelope env = g_env0;
  praos_replay_stats rs;
  if (members > 0) {
    int devs[64] = {0};
    if (members > 64) DIE("members: 1..64");
    praos_group* g = praos_group_open(devs, members);
    if (!g) DIE("praos_group_open");
    const int rc = praos_group_replay_immutable_views(g, dir, g_views, g_nviews, &g_params, &g_ei, &env, &S.st, 97,
                                                      NULL, 0, &rs);
    if (rc != PRAOS_OK) DIE("group views replay -> %d: %s", rc, praos_group_last_error(g));
    print_state("replay_views_group", &S, &env, rs.validated, rs.stop_index, (int)rs.stop_verdict, rs.epochs, -1);
    praos_group_close(g);
    return;
  }
  praos_ctx* ctx = praos_open(0);
  if (!ctx) DIE("praos_open(0)");
  CK(ctx, praos_replay_immutable_views(ctx, dir, g_views, g_nviews, &g_params, &g_ei, &env, &S.st, 1 << 16, NULL, 0,
                                       &rs));
  print_state("replay_views", &S, &env, rs.validated, rs.stop_index, (int)rs.stop_verdict, rs.epochs, -1);
  praos_close(ctx);
}

/* ---- phase 3: several threads, one context each; and a group ---- */
typedef struct {
  const chain_t* ch;
  size_t i0, i1;
  uint16_t* bits;
  int32_t* pidx;
  uint8_t* nonce;
  int rc;
} job_t;

static void* worker(void* arg) {
  job_t* j = arg;
  praos_ctx* ctx = praos_open(0);
  if (!ctx) { j->rc = -100; return NULL; }
  j->rc = praos_set_epoch(ctx, g_eta0, g_pools, g_npools, &g_params);
  const size_t n = j->i1 - j->i0;
  if (j->rc == PRAOS_OK && n) {
    praos_header_bytes hb = {n, j->ch->bytes, j->ch->len, j->ch->off + j->i0, j->ch->hlen + j->i0};
    praos_out out = {j->bits + j->i0, j->pidx + j->i0, NULL, NULL, j->nonce + 32 * j->i0};
    for (int rep = 0; rep < 3 && j->rc == PRAOS_OK; rep++)   /* repeated: contexts interleave on the device */
      j->rc = praos_verify_header_bytes(ctx, &hb, &out, NULL);
  }
  praos_close(ctx);
  return NULL;
}

static void phase_threads(const chain_t* ch, int T) {
  size_t n = 0;   /* the first epoch: eta0 is the genesis nonce */
  while (n < ch->n && (ch->slot[n] - g_ei.epoch_base_slot) / g_ei.epoch_length == 0) n++;
  uint16_t *b1 = calloc(n, 2), *bt = calloc(n, 2), *bg = calloc(n, 2);
  int32_t *p1 = calloc(n, 4), *pt = calloc(n, 4), *pg = calloc(n, 4);
  uint8_t *n1 = calloc(n, 32), *nt = calloc(n, 32), *ng = calloc(n, 32);
  /* one context */
  praos_ctx* ctx = praos_open(0);
  if (!ctx) DIE("praos_open(0)");
  CK(ctx, praos_set_epoch(ctx, g_eta0, g_pools, g_npools, &g_params));
  praos_header_bytes hb = {n, ch->bytes, ch->len, ch->off, ch->hlen};
  praos_out o1 = {b1, p1, NULL, NULL, n1};
  CK(ctx, praos_verify_header_bytes(ctx, &hb, &o1, NULL));
  praos_close(ctx);
  /* T threads x own context */
  pthread_t* th = calloc((size_t)T, sizeof *th);
  job_t* jobs = calloc((size_t)T, sizeof *jobs);
  for (int k = 0; k < T; k++) {
    jobs[k] = (job_t){ch, n * k / T, n * (k + 1) / T, bt, pt, nt, 0};
    pthread_create(&th[k], NULL, worker, &jobs[k]);
  }
  int trc = 0;
  for (int k = 0; k < T; k++) {
    pthread_join(th[k], NULL);
    if (jobs[k].rc) trc = jobs[k].rc;
  }
  /* a group of T members on device 0 */
  int* devs = calloc((size_t)T, sizeof *devs);
  praos_group* g = praos_group_open(devs, T);
  if (!g) DIE("praos_group_open");
  if (praos_group_set_epoch(g, g_eta0, g_pools, g_npools, &g_params) != PRAOS_OK) DIE("%s", praos_group_last_error(g));
  praos_out og = {bg, pg, NULL, NULL, ng};
  if (praos_group_verify_header_bytes(g, &hb, &og, NULL) != PRAOS_OK) DIE("%s", praos_group_last_error(g));
  const int gsize = praos_group_size(g);
  praos_group_close(g);
  size_t valid = 0;
  for (size_t i = 0; i < n; i++) valid += b1[i] == 0;
  const int same_t = !trc && !memcmp(b1, bt, 2 * n) && !memcmp(p1, pt, 4 * n) && !memcmp(n1, nt, 32 * n);
  const int same_g = !memcmp(b1, bg, 2 * n) && !memcmp(p1, pg, 4 * n) && !memcmp(n1, ng, 32 * n);
  printf("{\"phase\": \"threads\", \"threads\": %d, \"group_size\": %d, \"headers\": %zu, \"valid\": %zu, "
         "\"thread_rc\": %d, \"threads_equal\": %s, \"group_equal\": %s}\n", T, gsize, n, valid, trc,
         same_t ? "true" : "false", same_g ? "true" : "false");
  fflush(stdout);
}

/* ---- chunk validation (Batch.hs verifyChunkIntegrity) ---- */
static uint32_t crc32_ieee(const uint8_t* p, size_t n) {   /* System.FS.CRC (zlib's CRC-32) */
  static uint32_t tab[256];
  static int init;
  if (!init) {
    for (uint32_t i = 0; i < 256; i++) {
      uint32_t c = i;
      for (int k = 0; k < 8; k++) c = c & 1 ? 0xEDB88320u ^ (c >> 1) : c >> 1;
      tab[i] = c;
    }
    init = 1;
  }
  uint32_t c = 0xFFFFFFFFu;
  for (size_t i = 0; i < n; i++) c = tab[(c ^ p[i]) & 0xFF] ^ (c >> 8);
  return c ^ 0xFFFFFFFFu;
}

static int chunk_main(const char* dir, int chunk, uint64_t spkp, int members) {
  char p[4096];
  size_t dl, sl;
  snprintf(p, sizeof p, "%s/%05d.chunk", dir, chunk);
  uint8_t* data = slurp(p, &dl);
  snprintf(p, sizeof p, "%s/%05d.secondary", dir, chunk);
  uint8_t* sec = slurp(p, &sl);
  if (!data || !sec || sl % 56) DIE("chunk %d: missing file or malformed secondary index", chunk);
  const size_t n = sl / 56;
  /* block i = [blockOffset_i, blockOffset_i+1), the last to the end of the chunk (Secondary.hs) */
  uint64_t* boff = calloc(n + 1, 8);
  for (size_t i = 0; i < n; i++) boff[i] = be(sec + 56 * i, 8);
  boff[n] = dl;
  size_t nchk = 0;
  uint64_t* off = calloc(n + 1, 8);
  uint32_t* len = calloc(n + 1, 4);
  size_t* which = calloc(n + 1, sizeof *which);
  for (size_t i = 0; i < n; i++) {
    if (boff[i] > boff[i + 1] || boff[i + 1] > dl) DIE("entry %zu outside its chunk", i);
    const uint32_t want = (uint32_t)be(sec + 56 * i + 12, 4);
    if (crc32_ieee(data + boff[i], boff[i + 1] - boff[i]) == want) continue;   /* checksum matches: trusted */
    off[nchk] = boff[i];
    len[nchk] = (uint32_t)(boff[i + 1] - boff[i]);
    which[nchk++] = i;
  }
  praos_header_bytes hb = {nchk, data, dl, off, len};
  uint8_t* res = calloc(nchk + 1, 1);
  for (int pass = 0; pass < 2; pass++) {
    memset(res, 0xEE, nchk + 1);
    if (pass == 0) {
      praos_ctx* ctx = praos_open(0);
      if (!ctx) DIE("praos_open(0)");
      CK(ctx, praos_verify_block_integrity(ctx, &hb, spkp, res, NULL));
      praos_close(ctx);
    } else {
      int devs[64] = {0};
      if (members < 1 || members > 64) DIE("members: 1..64");
      praos_group* g = praos_group_open(devs, members);
      if (!g) DIE("praos_group_open");
      if (praos_group_verify_block_integrity(g, &hb, spkp, res, NULL) != PRAOS_OK)
        DIE("%s", praos_group_last_error(g));
      praos_group_close(g);
    }
    /* parseChunkFile stops at the first corrupt block and truncates the file at its offset */
    size_t first = n;
    for (size_t j = 0; j < nchk; j++)
      if (res[j]) { first = which[j]; break; }
    printf("{\"phase\": \"%s\", \"blocks\": %zu, \"checked\": %zu, \"first_corrupt\": %zu, "
           "\"truncate_at\": %llu, \"results\": [", pass ? "chunk_group" : "chunk", n, nchk, first,
           (unsigned long long)(first < n ? boff[first] : dl));
    for (size_t i = 0, j = 0; i < n; i++) {
      int r = -1;
      if (j < nchk && which[j] == i) r = res[j++];
      printf("%s%d", i ? ", " : "", r);
    }
    printf("]}\n");
    fflush(stdout);
  }
  free(boff); free(off); free(len); free(which); free(res); free(data); free(sec);
  return 0;
}

int main(int argc, char** argv) {
  if (praos_abi_version() != PRAOS_ABI_VERSION) DIE("ABI version %d, header %d", praos_abi_version(), PRAOS_ABI_VERSION);
  if (argc == 6 && strcmp(argv[1], "--chunk") == 0)
    return chunk_main(argv[2], atoi(argv[3]), strtoull(argv[4], NULL, 10), atoi(argv[5]));
  if (argc != 4) DIE("usage: %s <immutable dir> <epoch file> <threads> | --chunk <dir> <chunk> <spkp> <members>",
                     argv[0]);
  read_epoch_file(argv[2]);
  chain_t ch;
  read_chain(argv[1], &ch);
  const int T = atoi(argv[3]);
  if (T < 1 || T > 64) DIE("threads: 1..64");
  phase_binding(&ch, 0);
  if (g_tpraos) phase_binding(&ch, T);
  if (!g_tpraos) phase_typed(&ch, 0, 0);
  if (!g_tpraos) phase_typed(&ch, T, 0);
  if (!g_tpraos) phase_typed(&ch, 0, 3);
  phase_replay(argv[1], 0);
  phase_replay(argv[1], T);
  if (!g_tpraos) {
    phase_analysis(&ch, 0);
    phase_analysis(&ch, T);
    phase_replay_views(argv[1], 0);
    phase_replay_views(argv[1], T);
  }
  if (!g_tpraos) phase_threads(&ch, T);
  return 0;
}
