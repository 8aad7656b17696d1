/*
 * praos_hip.h -- C ABI of libpraos_hip.so, the MI355X (gfx950) batch validator
 * for Ouroboros Praos block-header crypto.
 *
 * Drop-in boundary: the reference validates one header at a
 * time in Haskell, calling C crypto per signature through cardano-crypto-class
 * FFI (`foreign import ccall` into libsodium; result CInt 0 = ok / -1 = fail).
 * This ABI replaces, for a contiguous batch of headers of one epoch:
 *
 *   praos_verify_headers  <- Praos.validateKESSignature  (Praos.hs:558-606)
 *                            + Praos.validateVRFSignature (Praos.hs:528-556)
 *                            as composed by updateChainDepState (Praos.hs:441-459)
 *   praos_verify_ocert    <- DSIGN.verifySignedDSIGN vkcold (ocertToSignable oc) tau
 *                            (Praos.hs:580; Ed25519DSIGN -> libsodium verify_detached)
 *   praos_verify_kes      <- KES.verifySignedKES vk_hot t hvSigned hvSignature
 *                            (Praos.hs:582; Shelley/Protocol/Praos.hs:85 for integrity)
 *   praos_verify_vrf      <- VRF.verifyCertified vrfK (mkInputVRF slot eta0) vrfCert
 *                            (Praos.hs:543; PraosVRF -> crypto_vrf_ietfdraft03_verify)
 *   praos_check_leader    <- checkLeaderNatValue (vrfLeaderValue cert) sigma f
 *                            (Praos.hs:549)
 *   praos_decode_headers  <- DecCBOR (Annotator (Header c)) + HeaderBody decoding, the
 *                            signable re-serialisation and headerHash
 *                            (Praos/Header.hs:90-94, :147-151, :187-231) over stored
 *                            header bytes (ImmutableDB chunk + secondary index)
 *   praos_verify_header_bytes <- decode + praos_verify_headers in one device pass
 *   praos_apply_batch     <- the first-error-wins order of updateChainDepState plus
 *                            the OCert counter rule (Praos.hs:584-606) and the
 *                            reupdateChainDepState counter/nonce update (Praos.hs:468-502)
 *
 * Conventions (mirroring the reference FFI): plain pointers + sizes, caller-owned
 * host buffers, nothing retained after return.  Return value 0 = ok, < 0 = system
 * error (PRAOS_E_*).  Cryptographic failures are DATA (bits in the outputs),
 * never return codes.  One context per host thread; calls block.
 */
#ifndef PRAOS_HIP_H
#define PRAOS_HIP_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PRAOS_ABI_VERSION 15

/* ---- return codes ---- */
#define PRAOS_OK 0
#define PRAOS_E_HIP (-1)     /* HIP runtime error (see praos_last_error) */
#define PRAOS_E_ARG (-2)     /* bad argument / inconsistent sizes */
#define PRAOS_E_OOM (-3)     /* device allocation failed */
#define PRAOS_E_STATE (-4)   /* praos_set_epoch not called */

/* ---- per-header check bits (uint16), one per reference error constructor ---- */
#define PRAOS_BIT_KES_BEFORE_START   0x0001u /* KESBeforeStartOCERT c0 kp */
#define PRAOS_BIT_KES_AFTER_END      0x0002u /* KESAfterEndOCERT kp c0 maxKESEvo */
#define PRAOS_BIT_OCERT_SIG          0x0004u /* InvalidSignatureOCERT n c0 "Verification failed" */
#define PRAOS_BIT_KES_MERKLE         0x0008u /* InvalidKesSignatureOCERT kp c0 t "Reject" */
#define PRAOS_BIT_KES_LEAF           0x0010u /* InvalidKesSignatureOCERT kp c0 t (Ed25519 leaf) */
#define PRAOS_BIT_COUNTER_MISSING    0x0020u /* NoCounterForKeyHashOCERT (praos_apply_batch) */
#define PRAOS_BIT_COUNTER_TOO_SMALL  0x0040u /* CounterTooSmallOCERT (praos_apply_batch) */
#define PRAOS_BIT_COUNTER_OVER_INC   0x0080u /* CounterOverIncrementedOCERT (praos_apply_batch) */
#define PRAOS_BIT_VRF_KEY_UNKNOWN    0x0100u /* VRFKeyUnknown */
#define PRAOS_BIT_VRF_KEY_WRONG      0x0200u /* VRFKeyWrongVRFKey */
#define PRAOS_BIT_VRF_PROOF          0x0400u /* VRFKeyBadProof: draft-03 proof rejected */
#define PRAOS_BIT_VRF_OUTPUT         0x0800u /* VRFKeyBadProof: certified output != proof_to_hash */
#define PRAOS_BIT_LEADER             0x1000u /* VRFLeaderValueTooBig */
#define PRAOS_BIT_INPUT              0x8000u /* malformed batch entry (e.g. body out of range) */
/* TPraos (praos_verify_tpraos_headers) reuses bits 0-4, 8, 9, 12 and replaces 10/11: */
#define PRAOS_BIT_TP_VRF_NONCE       0x0400u /* VRFKeyBadNonce (eta cert: proof or output) */
#define PRAOS_BIT_TP_VRF_LEADER      0x0800u /* VRFKeyBadLeaderValue (leader cert) */
/* ... and, with an overlay schedule (praos_set_overlay, d > 0): */
#define PRAOS_BIT_TP_OVERLAY         0x2000u /* informational: an ACTIVE overlay slot (genesis delegate's
                                                slot); bits 8/9 then mean the two bits below and no
                                                pool lookup or leader test applies */
#define PRAOS_BIT_TP_GEN_COLD        0x0100u /* (with TP_OVERLAY) WrongGenesisColdKeyOVERLAY */
#define PRAOS_BIT_TP_GEN_VRF         0x0200u /* (with TP_OVERLAY) WrongGenesisVRFKeyOVERLAY */
#define PRAOS_BIT_TP_NOT_ACTIVE      0x4000u /* NotActiveSlotOVERLAY (an overlay slot nobody may fill;
                                                no VRF check is made) */

/* ---- verdict codes of praos_apply_batch (first failing check, Praos.hs order) ---- */
enum praos_verdict {
  PRAOS_V_OK = 0,
  PRAOS_V_KES_BEFORE_START = 1,
  PRAOS_V_KES_AFTER_END = 2,
  PRAOS_V_OCERT_SIG = 3,
  PRAOS_V_KES_SIG = 4,            /* detail: bit KES_MERKLE or KES_LEAF */
  PRAOS_V_COUNTER_MISSING = 5,
  PRAOS_V_COUNTER_TOO_SMALL = 6,
  PRAOS_V_COUNTER_OVER_INC = 7,
  PRAOS_V_VRF_KEY_UNKNOWN = 8,
  PRAOS_V_VRF_KEY_WRONG = 9,
  PRAOS_V_VRF_BAD_PROOF = 10,
  PRAOS_V_LEADER_TOO_BIG = 11,
  PRAOS_V_INPUT = 12,
  /* envelope (praos_validate_headers only): HeaderEnvelopeError, then PraosEnvelopeError */
  PRAOS_V_ENV_BLOCK_NO = 13,      /* UnexpectedBlockNo expected actual */
  PRAOS_V_ENV_SLOT_NO = 14,       /* UnexpectedSlotNo expected actual */
  PRAOS_V_ENV_PREV_HASH = 15,     /* UnexpectedPrevHash oldTip actual */
  PRAOS_V_ENV_OBSOLETE_NODE = 16, /* ObsoleteNode lvProtVerMajor maxMajorPV */
  PRAOS_V_ENV_HEADER_SIZE = 17,   /* HeaderSizeTooLarge size max */
  PRAOS_V_ENV_BLOCK_SIZE = 18     /* BlockSizeTooLarge size max */
};

typedef struct praos_ctx praos_ctx;
typedef struct praos_batch praos_batch;

/* PraosParams fields used by header validation (Praos.hs:184-210) and the
 * active slot coefficient in the form checkLeaderNatValue consumes. */
typedef struct {
  uint64_t slots_per_kes_period;  /* praosSlotsPerKESPeriod (must be > 0) */
  uint64_t max_kes_evo;           /* praosMaxKESEvo */
  int32_t f_is_one;               /* activeSlotVal f == maxBound -> leader check always true */
  int32_t vrf_check_output;       /* 1: verifyCertified also requires certified output == beta
                                     (cardano-crypto-class >= 2.1 semantics); 0: proof only */
  uint8_t c_raw[16];              /* activeSlotLog f: Fixed E34 raw value, int128 LE two's complement, <= 0 */
} praos_params;

/* One entry of the stake distribution (PoolDistr, Views.hs:41-51). */
typedef struct {
  uint8_t hash28[28];             /* KeyHash 'StakePool = Blake2b-224(cold vk) */
  uint8_t vrf_hash32[32];         /* individualPoolStakeVrf = Blake2b-256(vrf vk) */
  uint8_t sigma_fp[16];           /* fromRational individualPoolStake: Fixed E34 raw, uint128 LE */
} praos_pool;

/* Headers of one batch, struct-of-arrays over caller memory (HeaderView,
 * Views.hs:22-39).  Fixed-width fields are n records each. */
typedef struct {
  size_t n;
  const uint64_t* slot;           /* hvSlotNo */
  const uint8_t* cold_vk;         /* hvVK, n*32 */
  const uint8_t* vrf_vk;          /* hvVrfVK, n*32 */
  const uint8_t* vrf_out;         /* certifiedOutput of hvVrfRes, n*64 */
  const uint8_t* vrf_proof;       /* certifiedProof, n*80 */
  const uint8_t* hot_vk;          /* OCert ocertVkHot, n*32 */
  const uint64_t* ocert_n;        /* ocertN */
  const uint64_t* ocert_c0;       /* ocertKESPeriod */
  const uint8_t* ocert_sig;       /* ocertSigma, n*64 */
  const uint8_t* kes_sig;         /* hvSignature (Sum6KES raw), n*448 */
  const uint64_t* body_off;       /* hvSigned: offset of the signed body bytes in body_bytes */
  const uint32_t* body_len;       /* hvSigned length */
  const uint8_t* body_bytes;
  size_t body_bytes_len;
} praos_headers;

/* A Nonce (Praos.hs): 32-byte hash, or NeutralNonce. */
typedef struct {
  uint8_t hash[32];
  int32_t neutral;                /* 1 = NeutralNonce */
} praos_nonce;

/* Outputs (any pointer may be NULL except bits). */
typedef struct {
  uint16_t* bits;                 /* n: PRAOS_BIT_* (crypto + range checks) */
  int32_t* pool_idx;              /* n: index into the praos_set_epoch pool array, -1 unknown */
  uint8_t* beta;                  /* n*64: proof_to_hash (zeros if Gamma undecodable) */
  uint8_t* leader;                /* n*32: vrfLeaderValue, big-endian natural */
  uint8_t* nonce;                 /* n*32: vrfNonceValue */
} praos_out;

/* ---- context ---- */
/* device >= 0: a HIP device.  PRAOS_HOST_ONLY: a context without a device that
 * supports only the host-side sequential part (praos_set_epoch, praos_apply_batch,
 * praos_update_chain_dep_state); every GPU entry point then returns PRAOS_E_STATE.
 * There is no CPU crypto path. */
#define PRAOS_HOST_ONLY (-1)
praos_ctx* praos_open(int device);               /* NULL on failure */
void praos_close(praos_ctx* ctx);
const char* praos_last_error(praos_ctx* ctx);
int praos_abi_version(void);

/* Epoch-constant inputs: eta0 (NULL = NeutralNonce), pool distribution, params. */
int praos_set_epoch(praos_ctx* ctx, const uint8_t eta0[32], const praos_pool* pools, uint32_t npools,
                    const praos_params* params);

/* Blocking: H2D, all checks on the GPU, D2H. */
int praos_verify_headers(praos_ctx* ctx, const praos_headers* h, praos_out* out);

/* Device-resident pipeline (bench / streaming): upload once, run many times. */
praos_batch* praos_batch_upload(praos_ctx* ctx, const praos_headers* h);
int praos_batch_run(praos_ctx* ctx, praos_batch* b);          /* async on the ctx stream */
int praos_batch_sync(praos_ctx* ctx);
int praos_batch_download(praos_ctx* ctx, praos_batch* b, praos_out* out);
void praos_batch_free(praos_ctx* ctx, praos_batch* b);
/* Options.  PRAOS_OPT_CONCURRENT (default 1): run the OCert, KES and VRF
 * kernels on three streams so their tail waves overlap. */
#define PRAOS_OPT_CONCURRENT 1
/* PRAOS_OPT_KERNELS: bit mask of the crypto kernels praos_batch_run launches
 * (1 = OCert + KES-period checks, 2 = Sum6KES, 4 = VRF + leader; default 7).
 * Used by the single-primitive benchmark configs; skipped checks report 0 bits. */
#define PRAOS_OPT_KERNELS 2
/* PRAOS_OPT_KEYCACHE (default 2): a public key (cold key, VRF key) used by at
 * least this many headers of a batch is decoded once per run and expanded into
 * multi-power tables, so those headers' OCert / VRF-U scalar chains are 16
 * windows long instead of 64 (k_keys.hip).  0 disables the cache.  Verdicts
 * are identical either way (keys are matched byte for byte). */
#define PRAOS_OPT_KEYCACHE 3
/* PRAOS_OPT_DEDUP (default 1): the OCert signature check (Praos.hs:580) depends only
 * on the 144 bytes (cold vk, hot vk, n, c0, sigma); a pool forges every header of an
 * epoch under one operational certificate, so each distinct tuple of a batch is
 * verified once (tuples compared byte for byte on the device) and its verdict is
 * copied to every header carrying the same bytes; the KES-period checks stay per
 * header.  Verdicts are identical either way. */
#define PRAOS_OPT_DEDUP 4
/* PRAOS_OPT_PIPELINE (default 0 = auto): praos_verify_header_bytes uploads a batch in
 * this many chunks (1 = no pipeline, up to 8): the stored bytes of chunk k+1 move host ->
 * device on a copy stream while chunk k is decoded and its VRF stage V runs; the rest of
 * the batch runs once after the last chunk, and the VRF outputs move back while the KES
 * checks finish; auto = up to 8 chunks of at least 49,152 headers, the first a quarter of the
 * others' size (nothing runs until it has landed). */
#define PRAOS_OPT_PIPELINE 5
/* PRAOS_OPT_KES_PAIR (default -1 = automatic): the cached Sum6KES leaf verifies take two
 * headers per lane from this many cache hits on, encoding both R' with one field inversion
 * (0 = never).  Automatic: from 196,608 hits when the KES pass runs alone (PRAOS_OPT_KERNELS
 * == 2); beside the OCert / VRF passes the longer waves cost more than they save.  Verdicts
 * are identical either way. */
#define PRAOS_OPT_KES_PAIR 6
/* PRAOS_OPT_POOL_KEYS (default -1 = on inside praos_replay_immutable*, off otherwise): the
 * cold-key and VRF-key cache entries (decoded key, validity flags, multi-power tables) are
 * kept across runs of the context in a store of 16,384 entries per kind, so a key seen by an
 * earlier batch is a cache hit without being decoded and expanded again; new keys are cached
 * from their first use (they recur in the batches that follow).  Keys are matched byte for
 * byte; verdicts are identical either way.  1 = on, 0 = off, 2 = on and emptied before the
 * next run.  A store more than 3/4 full is emptied before a run. */
#define PRAOS_OPT_POOL_KEYS 7
/* PRAOS_OPT_KES_NOCACHE (default 58000): batches of fewer headers than this check every Sum6KES
 * leaf signature uncached (no leaf-key cache: the per-lane chains run beside the VRF's stage V,
 * and the key chain -- lists, precompute, tables -- is not on the step's critical path; the
 * 1/8-epoch shard of a strong-scaling run is below it).  0 = the cache at every size.  Verdicts
 * are identical either way. */
#define PRAOS_OPT_KES_NOCACHE 8
int praos_set_option(praos_ctx* ctx, int opt, int value);
/* Key-cache statistics of the last praos_batch_run (after praos_batch_sync):
 * out[0..2] = cold keys cached, OCert items on cached keys, OCert items
 * uncached; out[3..5] = the same for VRF keys; out[6..8] for the KES leaf keys
 * (the Ed25519 key each Sum6KES signature ends on).  With the pool-key store on
 * (PRAOS_OPT_POOL_KEYS) out[0] / out[3] count the store's entries after the run.  Returns 0. */
int praos_batch_stats(praos_ctx* ctx, praos_batch* b, uint32_t out[9]);
/* OCert dedup of the last praos_batch_run: out[0] = distinct OCert tuples verified,
 * out[1] = headers (out[0] = 0 when the dedup did not run).  Returns 0. */
int praos_batch_dedup_stats(praos_ctx* ctx, praos_batch* b, uint32_t out[2]);
/* Per-kernel time of the last praos_batch_run (ms, HIP events on the ctx stream).
 * which: 0 = ocert, 1 = kes, 2 = vrf, 3 = leader, 4 = whole run, 5 = header
 * decode (batches from praos_batch_upload_bytes; 0 otherwise), 6 = the VRF stage-V
 * kernel k_vrf_v alone (events around its launch on its own stream), 7 = the cached
 * Sum6KES kernel k_kes_ck alone (events around its launch on the KES stream).  With concurrent
 * streams, 0-2 are measured from the common start to each kernel's end. */
float praos_batch_kernel_ms(praos_ctx* ctx, int which);

/* Page-locks [p, p + len) of caller memory (hipHostRegister) for the context's device, e.g.
 * a replay reader's chunk buffer or a Haskell pinned ByteString that lives across many calls;
 * uploads whose source lies inside a registered range move by direct DMA instead of through
 * the library's pinned staging buffers and host copy threads.  Returns 0, or PRAOS_E_HIP.
 * Unregister before freeing the memory. */
int praos_host_register(praos_ctx* ctx, void* p, size_t len);
int praos_host_unregister(praos_ctx* ctx, void* p);

/* ---- stored headers: decode on the GPU ----
 * Input: a byte arena (e.g. an ImmutableDB chunk file as read) and per header
 * the (offset, length) of its CBOR item -- blockOffset + headerOffset and
 * headerSize from the secondary index (ImmutableDB/Impl/Index/Secondary.hs:93-128).
 * The header is HeaderRaw = [body, kesSig] (Praos/Header.hs:201-231) with the
 * 10-field HeaderBody (:160-199).  The KES message is the canonical
 * re-serialisation of the decoded body (`serialize' hb`, :90-94): equal to the
 * stored slice when that is canonical, re-encoded on the GPU otherwise.
 * header_hash = Blake2b-256 of the stored header bytes (headerHash, :147-151). */
typedef struct {
  size_t n;
  const uint8_t* bytes;           /* arena */
  size_t bytes_len;
  const uint64_t* off;            /* n: header i = bytes[off[i], off[i] + len[i]) */
  const uint32_t* len;            /* n */
} praos_header_bytes;

/* decode status (uint16 per header): the first failure, or 0 / NONCANONICAL */
#define PRAOS_DEC_RANGE        0x01u /* slice outside the arena */
#define PRAOS_DEC_SYNTAX       0x02u /* truncated / wrong major type / wrong array length */
#define PRAOS_DEC_SIZE         0x04u /* fixed-size byte string of the wrong length */
#define PRAOS_DEC_UNSUPPORTED  0x08u /* indefinite-length item or tag (never emitted by the reference) */
#define PRAOS_DEC_TRAILING     0x10u /* bytes after the header item within len */
#define PRAOS_DEC_NONCANONICAL 0x20u /* informational: stored body not canonical; signed bytes re-encoded */
#define PRAOS_DEC_OVERFLOW     0x40u /* integer out of range (bodySize > Word32, ProtVer major > maxVersion) */
#define PRAOS_MAX_PROT_MAJOR   9     /* cardano-ledger-binary maxVersion at the reference's CHaP index-state */
#define PRAOS_DEC_FAILED       0x5Fu /* mask of the failure bits */
#define PRAOS_SIGNED_STRIDE    448   /* bytes per header in praos_decoded.signed_body */

/* Decoded fields (caller buffers; every pointer may be NULL = not returned).
 * A header that fails to decode has all fields zero and signed_len 0xffffffff. */
typedef struct {
  uint16_t* status;               /* n: PRAOS_DEC_* */
  uint64_t* block_no;             /* hbBlockNo */
  uint64_t* slot;                 /* hbSlotNo */
  uint8_t* prev_hash;             /* n*32 hbPrev (zeros when GenesisHash) */
  uint8_t* prev_is_genesis;       /* n */
  uint8_t* cold_vk;               /* n*32 hbVk */
  uint8_t* vrf_vk;                /* n*32 hbVrfVk */
  uint8_t* vrf_out;               /* n*64 */
  uint8_t* vrf_proof;             /* n*80 */
  uint32_t* body_size;            /* hbBodySize */
  uint8_t* body_hash;             /* n*32 hbBodyHash */
  uint8_t* hot_vk;                /* n*32 ocertVkHot */
  uint64_t* ocert_n;
  uint64_t* ocert_c0;
  uint8_t* ocert_sig;             /* n*64 */
  uint64_t* prot_major;
  uint64_t* prot_minor;
  uint8_t* kes_sig;               /* n*448 */
  uint32_t* signed_len;           /* n: length of the KES message */
  uint8_t* signed_body;           /* n*stride, the KES message (serialize' hb): stride PRAOS_SIGNED_STRIDE,
                                     PRAOS_TP_SIGNED_STRIDE for praos_verify_tpraos_header_bytes */
  uint8_t* header_hash;           /* n*32 */
} praos_decoded;

int praos_decode_headers(praos_ctx* ctx, const praos_header_bytes* in, praos_decoded* out);
/* Decode + full header validation on the device.  bits gets PRAOS_BIT_INPUT for
 * a header that does not decode; dec may be NULL. */
int praos_verify_header_bytes(praos_ctx* ctx, const praos_header_bytes* in, praos_out* out, praos_decoded* dec);
/* ABI 15: the streaming form (a node or db-analyser validating batch after batch).  The call is
 * queued and returns at once; a context keeps three calls in flight, so the next submits' uploads,
 * decodes and stage V run under this call's key chains.  Its outputs (out, dec) are written by
 * the third submit after it, which waits for it, or by praos_verify_drain; in, the bytes it
 * points to, out and dec must stay valid and unchanged until then.  Outputs equal the blocking
 * call's.  Batches too small for the chunked pipeline (PRAOS_OPT_PIPELINE) run the blocking call
 * after the calls in flight.  praos_verify_header_bytes and praos_close drain first. */
int praos_verify_header_bytes_submit(praos_ctx* ctx, const praos_header_bytes* in, praos_out* out,
                                     praos_decoded* dec);
int praos_verify_drain(praos_ctx* ctx);
/* Device-resident form: the batch keeps the arena; praos_batch_run decodes and
 * then validates (bench / streaming replay).  praos_batch_download_decoded
 * copies the decoded fields of the last run. */
praos_batch* praos_batch_upload_bytes(praos_ctx* ctx, const praos_header_bytes* in);
int praos_batch_download_decoded(praos_ctx* ctx, praos_batch* b, praos_decoded* dec);
/* Decode a from-bytes batch now (async on the ctx stream; praos_batch_run then skips
 * the decode): lets the caller read the decoded fields -- e.g. slots and the certified
 * VRF outputs that drive the epoch nonces -- before the crypto runs. */
int praos_batch_decode(praos_ctx* ctx, praos_batch* b);
/* Several epochs in one batch (same ledger view, consecutive epoch nonces): header i
 * is verified under etas[eta_idx[i]] (k <= 256 entries) instead of the praos_set_epoch
 * nonce, from the next praos_batch_run on.  mkInputVRF (Praos/VRF.hs:55-69) is the only
 * nonce-dependent input.  Fold such outputs with praos_validate_headers_nonces. */
int praos_batch_set_nonces(praos_ctx* ctx, praos_batch* b, const praos_nonce* etas, uint32_t k,
                           const uint8_t* eta_idx);

/* ---- ImmutableDB block-integrity batch ----
 * Replaces verifyBlockIntegrity spkp blk (Shelley/Ledger/Integrity.hs:14-20), the
 * check ImmutableDB validation runs per stored block (--validate-all-blocks):
 *   verifyHeaderIntegrity (Shelley/Protocol/Praos.hs:84-101): Sum6KES verify of the
 *     header at t = kp - c0 if kp >= c0 else 0 (no OCert / VRF / maxKESEvo checks);
 *   blockMatchesHeader (Shelley/Ledger/Block.hs:150-158): hashTxSeq of the stored
 *     segments (Blake2b-256 over the segments' Blake2b-256 hashes) == hbBodyHash.
 * Input: praos_header_bytes whose (off, len) describe whole stored blocks: the
 * HardForkBlock wrapper [eraTag 6|7, [header, s1..s4]] or a bare [header, s1..s3|s4].
 * result[i] = 0 (verifyBlockIntegrity True) or PRAOS_BLK_* bits; body_hash (may be
 * NULL) gets the computed hashTxSeq (zeros when the block does not decode). */
#define PRAOS_BLK_DECODE    0x01u /* block envelope, a segment or the header does not decode */
#define PRAOS_BLK_KES       0x02u /* verifyHeaderIntegrity False */
#define PRAOS_BLK_BODY_HASH 0x04u /* blockMatchesHeader False */
int praos_verify_block_integrity(praos_ctx* ctx, const praos_header_bytes* blocks, uint64_t slots_per_kes_period,
                                 uint8_t* result, uint8_t* body_hash);
/* Device-resident form (bench / streaming ImmutableDB validation): upload once,
 * run any number of times, download the last run's results. */
praos_batch* praos_block_batch_upload(praos_ctx* ctx, const praos_header_bytes* blocks);
int praos_block_batch_run(praos_ctx* ctx, praos_batch* b, uint64_t slots_per_kes_period);
int praos_block_batch_download(praos_ctx* ctx, praos_batch* b, uint8_t* result, uint8_t* body_hash);

/* ---- TPraos (Shelley..Alonzo), the d = 0 path of cardano-protocol-tpraos ----
 * Replaces SL.updateChainDepState's crypto (TPraos.hs:378-387): OVERLAY
 * praosVrfChecks (pool, VRF key, eta cert with mkSeed seedEta, leader cert with
 * mkSeed seedL, checkLeaderValue on the 64-byte leader output, bound 2^512) and
 * the OCERT rule (same predicates as Praos a2).  Overlay slots (d > 0, genesis
 * delegates) are not handled. */
typedef struct {
  praos_headers h;                /* vrf_out / vrf_proof = bheaderEta; body = the signed BHBody bytes */
  const uint8_t* leader_out;      /* bheaderL certified output, n*64 */
  const uint8_t* leader_proof;    /* n*80 */
} praos_tpraos_headers;
typedef struct {
  uint16_t* bits;                 /* n: PRAOS_BIT_* / PRAOS_BIT_TP_* */
  int32_t* pool_idx;              /* n */
  uint8_t* beta_eta;              /* n*64 */
  uint8_t* beta_leader;           /* n*64 */
  uint8_t* nonce;                 /* n*32: mkNonceFromOutputVRF (Blake2b-256 of the eta output) */
} praos_tpraos_out;
int praos_verify_tpraos_headers(praos_ctx* ctx, const praos_tpraos_headers* h, praos_tpraos_out* out);

/* TPraos headers from stored bytes (ImmutableDB chunk spans of Shelley..Alonzo blocks):
 * BHeader = [BHBody, kesSig] decoded on the device (cardano-protocol-tpraos
 * DecCBOR BHeader / BHBody: 15 fields, the eta and leader certificates as two
 * [output, proof] pairs, OCert and ProtVer inlined; the KES message is the canonical
 * re-encoding `serialize' bhb`, the stored slice when canonical), then the crypto of
 * praos_verify_tpraos_headers.  A header that does not decode gets PRAOS_BIT_INPUT.
 * dec (may be NULL) receives the decoded fields, signed_body with a
 * PRAOS_TP_SIGNED_STRIDE stride; leader_out / leader_proof (may be NULL, n*64 / n*80)
 * the leader certificate.  Replaces, per epoch, the header crypto of
 * TPraos.updateChainDepState (TPraos.hs:378-387) for eras Shelley..Alonzo
 * (HFEras.hs:43-49); the fold is praos_tpraos_update_chain_dep_state. */
#define PRAOS_TP_SIGNED_STRIDE 640
int praos_verify_tpraos_header_bytes(praos_ctx* ctx, const praos_header_bytes* in, praos_tpraos_out* out,
                                     praos_decoded* dec, uint8_t* leader_out, uint8_t* leader_proof);
/* Device-resident form (the TPraos replay): praos_batch_run on such a batch decodes and
 * runs the TPraos kernels (under per-header nonces after praos_batch_set_nonces);
 * praos_batch_download_decoded / praos_batch_download_tpraos copy the results. */
praos_batch* praos_batch_upload_tpraos_bytes(praos_ctx* ctx, const praos_header_bytes* in);
int praos_batch_download_tpraos(praos_ctx* ctx, praos_batch* b, praos_tpraos_out* out);

/* ---- TPraos decentralisation overlay (d > 0; Shelley..Alonzo before d reached 0) ----
 * cardano-protocol-tpraos OVERLAY (lookupInOverlaySchedule, the same call
 * TPraos.checkIsLeader makes at TPraos.hs:304-337): with s = slot - first slot of its
 * epoch, the slot is in the overlay schedule iff ceiling(s d) < ceiling((s + 1) d);
 * then position = ceiling(s d) is active iff position mod ascInv == 0 (ascInv =
 * floor(1 / f)), and its genesis key is the (position div ascInv) mod |genDelegs|-th
 * of the genesis key hashes in ascending byte order.  An active overlay slot must be
 * forged by that key's delegate (WrongGenesisColdKeyOVERLAY) with the delegate's VRF
 * key (WrongGenesisVRFKeyOVERLAY), both certificates verify (VRFKeyBadNonce /
 * VRFKeyBadLeaderValue), and no leader-value test applies; a non-active overlay slot
 * fails NotActiveSlotOVERLAY.  Other slots take the Praos checks (pool, VRF key,
 * certificates, leader value).  The OCERT rule runs for every header; genesis
 * delegates count as known issuers (currentIssueNo). */
typedef struct {
  uint8_t genesis_hash28[28];     /* KeyHash 'Genesis: a key of lvGenDelegs */
  uint8_t delegate_hash28[28];    /* genDelegKeyHash: the delegate's cold-key hash */
  uint8_t vrf_hash32[32];         /* genDelegVrfHash */
} praos_gen_deleg;
typedef struct {
  uint64_t d_num, d_den;          /* lvD, a UnitInterval: d = d_num / d_den (d_den > 0, d_num <= d_den) */
  uint64_t asc_num, asc_den;      /* activeSlotVal f = asc_num / asc_den (0 < f <= 1) */
  uint64_t epoch_base_slot;       /* fixed-size epochs (first slot of the slot's epoch = epochInfoFirst) */
  uint64_t epoch_length;
  const praos_gen_deleg* gen_delegs;  /* any order (sorted by genesis hash inside) */
  uint32_t n_gen_delegs;          /* > 0 when d > 0 */
} praos_overlay;
/* ov == NULL or d_num == 0: no overlay (the d = 0 behaviour).  Kept until replaced. */
int praos_set_overlay(praos_ctx* ctx, const praos_overlay* ov);
/* The schedule itself (host-side; host-only contexts too): cls[i] = -1 (not an overlay
 * slot), -2 (NonActiveSlot) or k >= 0 (ActiveSlot of the k-th genesis key in ascending
 * hash order). */
int praos_overlay_classify(praos_ctx* ctx, size_t n, const uint64_t* slots, int32_t* cls);


/* ---- single-primitive batches (configs C2-C4); outputs 1 = valid, 0 = invalid ---- */
/* Ed25519 over the OCert signable hot_vk || BE64(n) || BE64(c0). */
int praos_verify_ocert(praos_ctx* ctx, size_t n, const uint8_t* cold_vk, const uint8_t* hot_vk,
                       const uint64_t* ocert_n, const uint64_t* ocert_c0, const uint8_t* sig, uint8_t* ok);
/* Sum6KES: result 0 = ok, 1 = Merkle "Reject", 2 = leaf Ed25519 failure. */
int praos_verify_kes(praos_ctx* ctx, size_t n, const uint8_t* vk, const uint32_t* period, const uint8_t* sig,
                     const uint64_t* msg_off, const uint32_t* msg_len, const uint8_t* msg_bytes,
                     size_t msg_bytes_len, uint8_t* result);
/* ECVRF-ED25519-SHA512-Elligator2 draft-03 verify; alpha is 32 bytes per item. */
int praos_verify_vrf(praos_ctx* ctx, size_t n, const uint8_t* vk, const uint8_t* proof, const uint8_t* alpha,
                     uint8_t* ok, uint8_t* beta);
/* checkLeaderNatValue; leader = 32-byte big-endian naturals, sigma_fp per item. */
int praos_check_leader(praos_ctx* ctx, size_t n, const uint8_t* leader, const uint8_t* sigma_fp,
                       const praos_params* params, uint8_t* is_leader);

/* ---- host-side sequential part (Praos.hs:441-502 order and state) ----
 * Counter map: the OCert issue numbers of praosStateOCertCounters, keyed by
 * issuer hash (Blake2b-224 of cold vk).  Walks the batch in order: verdict =
 * first failing check, then (as the reference does after a valid header)
 * counters[hk] := n.  `assume_valid_prefix` semantics: every header is judged
 * against the state left by all earlier headers of the batch as if valid.
 * chain_stop receives the index of the first non-OK header (n if none). */
typedef struct {
  const uint8_t* hash28;          /* m*28, any order */
  uint64_t* counter;              /* m: in = current counters; updated in place for existing keys */
  size_t m;
} praos_counters;

int praos_apply_batch(praos_ctx* ctx, const praos_headers* h, const praos_out* crypto,
                      praos_counters* counters, uint8_t* verdict, size_t* chain_stop);

/* ---- full chain-dependent state fold (tickChainDepState + updateChainDepState +
 *      reupdateChainDepState, Praos.hs:407-502) over a batch ----
 * Nonce = NeutralNonce | Nonce (32-byte hash); a ⭒ b = Blake2b-256(a || b), Neutral is
 * the identity.  Epochs: fixed size from a base (epoch of slot s =
 * base_no + (s - base_slot) / length); stability_window = computeStabilityWindow k f
 * (Praos.hs:497-498; ceiling(3k/f), computed by the caller).
 * Per header i, in order: tick (isNewEpoch last_slot slot_i, Ledger/Util.hs:20-40:
 * epoch_nonce := candidate ⭒ last_epoch_block, last_epoch_block := lab); the ticked
 * epoch nonce must equal the ctx's eta0 (the nonce the crypto outputs were computed
 * with), else the fold stops there (*processed = i) so the caller can set_epoch and
 * verify the rest; verdict as praos_apply_batch; on OK the ticked state is kept and
 * reupdated: last_slot := slot, lab := prevHashToNonce prev_hash, evolving :=
 * evolving ⭒ vrfNonceValue, candidate := evolving' if slot + stability_window <
 * firstSlotNextEpoch, counters[hk] := n (new keys appended; PRAOS_E_ARG past cap). */

typedef struct {
  int32_t last_slot_origin;       /* praosStateLastSlot = Origin */
  uint64_t last_slot;
  uint8_t* counter_hash28;        /* praosStateOCertCounters: cap*28 */
  uint64_t* counter;              /* cap */
  size_t m;                       /* entries in use (in/out) */
  size_t cap;
  praos_nonce evolving;           /* praosStateEvolvingNonce */
  praos_nonce candidate;          /* praosStateCandidateNonce */
  praos_nonce epoch_nonce;        /* praosStateEpochNonce */
  praos_nonce lab;                /* praosStateLabNonce */
  praos_nonce last_epoch_block;   /* praosStateLastEpochBlockNonce */
} praos_chain_state;

typedef struct {
  uint64_t epoch_base_slot;
  uint64_t epoch_base_no;
  uint64_t epoch_length;          /* > 0 */
  uint64_t stability_window;
} praos_epoch_info;

/* prev_hash: n*32 (hvPrevHash); prev_is_genesis: n flags (GenesisHash), may be NULL. */
int praos_update_chain_dep_state(praos_ctx* ctx, const praos_headers* h, const uint8_t* prev_hash,
                                 const uint8_t* prev_is_genesis, const praos_out* crypto,
                                 const praos_epoch_info* ei, praos_chain_state* st, uint8_t* verdict,
                                 size_t* chain_stop, size_t* processed);

/* ---- PraosState CBOR (checkpoint / resume of a replay) ----
 * Serialise (PraosState c), Praos.hs:274-310: [0, [lastSlot, ocertCounters, evolving,
 * candidate, epoch, lab, lastEpochBlock]].  encode: *len gets the size; PRAOS_E_ARG
 * if cap is too small (call with cap 0 to size).  decode: counters into the caller's
 * arrays (st->cap entries). */
int praos_state_encode(const praos_chain_state* st, uint8_t* out, size_t cap, size_t* len);
int praos_state_decode(const uint8_t* in, size_t len, praos_chain_state* st);

/* ---- validateHeader over a batch (HeaderValidation.hs:413-432) ----
 * The envelope first -- validateEnvelope (:297-344: block number = tip + 1 (0 after
 * Origin), slot >= tip slot + 1 (>= 0 after Origin), prev hash = tip hash (GenesisHash
 * after Origin)) and the Praos additionalEnvelopeChecks (Shelley/Protocol/Praos.hs:66-80:
 * ObsoleteNode, HeaderSizeTooLarge, BlockSizeTooLarge) -- then updateChainDepState as
 * praos_update_chain_dep_state does.  The tip advances with every valid header; on
 * return env's tip (like st) is the one at chain_stop.  Per-header inputs come from
 * the decoder (praos_decoded: block_no, header_hash, body_size; header_size = the
 * stored header length). */
typedef struct {
  const uint64_t* block_no;       /* n: hbBlockNo */
  const uint8_t* header_hash;     /* n*32: headerHash (Blake2b-256 of the header bytes) */
  const uint32_t* header_size;    /* n: bhviewHSize, bytes of the serialised header */
  const uint32_t* body_size;      /* n: bhviewBSize = hbBodySize */
  int32_t tip_is_origin;          /* HeaderState tip before the batch (in / out) */
  uint64_t tip_slot;
  uint64_t tip_block_no;
  uint8_t tip_hash[32];
  uint64_t max_major_pv;          /* praosMaxMajorPV */
  uint64_t lv_prot_major;         /* pvMajor (lvProtocolVersion lv) */
  uint64_t max_header_size;       /* lvMaxHeaderSize */
  uint64_t max_body_size;         /* lvMaxBodySize */
} praos_envelope;

/* The epoch nonce tickChainDepState (Praos.hs:407-431) gives the state at `slot`:
 * candidate ⭒ lastEpochBlock when the slot is in a later epoch than the state's last
 * slot (isNewEpoch), else the current epoch nonce.  What praos_set_epoch needs before
 * validating headers of that slot's epoch.  Pure: st is not changed. */
int praos_ticked_epoch_nonce(const praos_chain_state* st, const praos_epoch_info* ei, uint64_t slot,
                             praos_nonce* out);
/* The TPraos tick (cardano-protocol-tpraos TICKN, TPraos.hs:361-376): candidate ⭒
 * lastEpochBlock ⭒ extra_entropy (NULL = NeutralNonce) on a new epoch. */
int praos_tpraos_ticked_epoch_nonce(const praos_chain_state* st, const praos_epoch_info* ei, uint64_t slot,
                                    const praos_nonce* extra_entropy, praos_nonce* out);

int praos_validate_headers(praos_ctx* ctx, const praos_headers* h, const uint8_t* prev_hash,
                           const uint8_t* prev_is_genesis, const praos_out* crypto, praos_envelope* env,
                           const praos_epoch_info* ei, praos_chain_state* st, uint8_t* verdict, size_t* chain_stop,
                           size_t* processed);

/* praos_validate_headers (env != NULL) / praos_update_chain_dep_state (env == NULL) over
 * outputs verified under per-header nonces (praos_batch_set_nonces): the fold goes on
 * while the nonce the state ticks to at header i equals etas[eta_idx[i]]. */
int praos_validate_headers_nonces(praos_ctx* ctx, const praos_headers* h, const uint8_t* prev_hash,
                                  const uint8_t* prev_is_genesis, const praos_out* crypto, praos_envelope* env,
                                  const praos_epoch_info* ei, praos_chain_state* st, const praos_nonce* etas,
                                  uint32_t k, const uint8_t* eta_idx, uint8_t* verdict, size_t* chain_stop,
                                  size_t* processed);

/* ---- TPraos chain-dependent state: SL.tickChainDepState + SL.updateChainDepState
 *      (TPraos.hs:361-387; cardano-protocol-tpraos TICKN, PRTCL = UPDN + OVERLAY + OCERT)
 * The state has the Praos shape (praos_chain_state: counters = csProtocol's OCert map,
 * evolving / candidate = eta_v / eta_c, epoch_nonce / last_epoch_block = TicknState eta_0 /
 * eta_h, lab = csLabNonce).  Per header: tick on a new epoch: epoch_nonce := candidate ⭒
 * last_epoch_block ⭒ extra_entropy, last_epoch_block := lab; the envelope (env != NULL;
 * chainChecks are the Praos envelope checks); then the predicate failures of PRTCL,
 * collected as the ledger's STS rules collect them (ValidateAll): OVERLAY's
 * Either-chains (first failure within praosVrfChecks / pbftVrfChecks) plus every OCERT
 * predicate, into failures[i] (PRAOS_TPF_*); verdict[i] = PRAOS_V_OK, PRAOS_V_ENV_*,
 * PRAOS_V_INPUT or PRAOS_V_TPRAOS (failures[i] != 0).  On a valid header: eta_v :=
 * eta_v ⭒ mkNonceFromOutputVRF(eta cert), eta_c := eta_v' if slot + window <
 * firstSlotNextEpoch (ei->stability_window: the caller's UPDN window), lab :=
 * prevHashToNonce prev, counters[hk] := n.  chain_stop / processed / state at the stop
 * as praos_update_chain_dep_state. */
#define PRAOS_V_TPRAOS 19
#define PRAOS_TPF_KES_BEFORE_START  0x0001u /* KESBeforeStartOCERT */
#define PRAOS_TPF_KES_AFTER_END     0x0002u /* KESAfterEndOCERT */
#define PRAOS_TPF_OCERT_SIG         0x0004u /* InvalidSignatureOCERT */
#define PRAOS_TPF_KES_SIG           0x0008u /* InvalidKesSignatureOCERT */
#define PRAOS_TPF_COUNTER_MISSING   0x0010u /* NoCounterForKeyHashOCERT */
#define PRAOS_TPF_COUNTER_TOO_SMALL 0x0020u /* CounterTooSmallOCERT */
#define PRAOS_TPF_COUNTER_OVER_INC  0x0040u /* CounterOverIncrementedOCERT */
#define PRAOS_TPF_VRF_KEY_UNKNOWN   0x0100u /* VRFKeyUnknown */
#define PRAOS_TPF_VRF_KEY_WRONG     0x0200u /* VRFKeyWrongVRFKey */
#define PRAOS_TPF_BAD_NONCE         0x0400u /* VRFKeyBadNonce */
#define PRAOS_TPF_BAD_LEADER        0x0800u /* VRFKeyBadLeaderValue */
#define PRAOS_TPF_LEADER_TOO_BIG    0x1000u /* VRFLeaderValueTooBig */
#define PRAOS_TPF_NOT_ACTIVE        0x2000u /* NotActiveSlotOVERLAY */
#define PRAOS_TPF_GEN_COLD          0x4000u /* WrongGenesisColdKeyOVERLAY */
#define PRAOS_TPF_GEN_VRF           0x8000u /* WrongGenesisVRFKeyOVERLAY */
int praos_tpraos_update_chain_dep_state(praos_ctx* ctx, const praos_tpraos_headers* h, const uint8_t* prev_hash,
                                        const uint8_t* prev_is_genesis, const praos_tpraos_out* crypto,
                                        praos_envelope* env, const praos_epoch_info* ei,
                                        const praos_nonce* extra_entropy, praos_chain_state* st, uint8_t* verdict,
                                        uint16_t* failures, size_t* chain_stop, size_t* processed);
/* The same fold over outputs verified under per-header nonces (praos_batch_set_nonces): it
 * goes on while the nonce the state ticks to at header i equals etas[eta_idx[i]]
 * (praos_validate_headers_nonces for TPraos). */
int praos_tpraos_validate_headers_nonces(praos_ctx* ctx, const praos_tpraos_headers* h, const uint8_t* prev_hash,
                                         const uint8_t* prev_is_genesis, const praos_tpraos_out* crypto,
                                         praos_envelope* env, const praos_epoch_info* ei,
                                         const praos_nonce* extra_entropy, praos_chain_state* st,
                                         const praos_nonce* etas, uint32_t k, const uint8_t* eta_idx,
                                         uint8_t* verdict, uint16_t* failures, size_t* chain_stop,
                                         size_t* processed);

/* ---- chain replay from an ImmutableDB directory (db-analyser) ----
 * Replaces the per-block loop of DBAnalyser/Analysis.hs:815-847 (processAllImmutableDB
 * driving benchmarkLedgerOps / validateHeader, :479-607) for the header-validation
 * pass.  Reads dir/NNNNN.chunk + dir/NNNNN.secondary (56-byte Entry per block,
 * Storage/ImmutableDB/Impl/Index/Secondary.hs:93-128) from chunk 0 up in batches of at
 * most batch_max headers (spanning up to 256 epochs).  Each batch is decoded on the
 * device, given per-header epoch nonces (tickChainDepState, Praos.hs:407-431, run ahead
 * over the certified VRF outputs), verified under them (praos_batch_set_nonces) and
 * folded with praos_validate_headers_nonces, which re-derives every nonce it relies on;
 * the fold of batch k overlaps the device work of batch k+1.  One ledger view (pools,
 * params) for the whole replay.  Ends at the first invalid header (stop_index,
 * stop_verdict) or at the end of the database (stop_index = headers).  *st and env's
 * tip are the state and tip after the last valid header; verdicts[i] (i < verdicts_cap,
 * may be NULL with cap 0) for every header up to and including the stop.  Resume: when
 * env's tip is not Origin (a checkpointed state, praos_state_decode), the blocks up to
 * and including the tip (matched by slot and header hash in the secondary index) are
 * skipped; indices count from the first block after it. */
typedef struct {
  uint64_t skipped;               /* blocks up to the resume tip, not replayed */
  uint64_t headers;               /* headers read and judged (through the stop) */
  uint64_t validated;             /* valid headers folded into *st */
  uint64_t stop_index;            /* first invalid header, or headers when none */
  uint32_t stop_verdict;          /* its PRAOS_V_* (0 when none) */
  uint32_t epochs;                /* distinct epoch nonces the headers were verified under */
  uint32_t batches;               /* device passes */
  uint32_t chunks;                /* chunk files read */
  double ms_io;                   /* reading chunks + secondary indexes, building batches */
  double ms_device;               /* upload + decode + crypto + download */
  double ms_fold;                 /* envelope + updateChainDepState on the host */
  double ms_nonce;                /* epoch nonces ahead of the crypto (host) */
} praos_replay_stats;

int praos_replay_immutable(praos_ctx* ctx, const char* dir, const praos_pool* pools, uint32_t npools,
                           const praos_params* params, const praos_epoch_info* ei, praos_envelope* env,
                           praos_chain_state* st, size_t batch_max, uint8_t* verdicts, size_t verdicts_cap,
                           praos_replay_stats* stats);
/* ABI 14.  The ledger view per epoch, as db-analyser sources it: the reference forecasts each
 * header's LedgerView from the ledger state it advances block by block (Analysis.hs:564-572,
 * ledgerViewForecastAt over applyTheBlock; Shelley/Ledger/SupportsProtocol.hs:100-125: lvPoolDistr
 * = nesPd, lvMaxHeaderSize / lvMaxBodySize / lvProtocolVersion from the epoch's protocol
 * parameters).  All of them change only at an epoch boundary (the NEWEPOCH rule), so one view
 * per epoch is the reference's per-header forecast.  views[] is sorted by first_epoch; epoch e
 * uses the last entry with first_epoch <= e (a view holds until the next entry's epoch). */
typedef struct {
  uint64_t first_epoch;
  const praos_pool* pools;        /* lvPoolDistr: hash28, VRF key hash, sigma (Fixed E34) */
  uint32_t npools;
  uint32_t reserved;              /* 0 */
  uint64_t lv_prot_major;         /* pvMajor (lvProtocolVersion) */
  uint64_t max_header_size;       /* lvMaxHeaderSize */
  uint64_t max_body_size;         /* lvMaxBodySize */
} praos_ledger_view;

/* praos_replay_immutable with a ledger view per epoch instead of one for the whole replay: a
 * batch never spans two views; each member's device gets a view's pool tables (hash, VRF key
 * hash, leader threshold x = -(sigma * c)) before the first batch that needs them, and the fold
 * of a batch uses that batch's view (PoolDistr membership for the OCert counters, the envelope
 * limits; env's limit fields are ignored).  Everything else -- pipeline, stop, resume, outputs --
 * as praos_replay_immutable.  PRAOS_E_ARG when no view covers a replayed epoch. */
int praos_replay_immutable_views(praos_ctx* ctx, const char* dir, const praos_ledger_view* views, uint32_t nviews,
                                 const praos_params* params, const praos_epoch_info* ei, praos_envelope* env,
                                 praos_chain_state* st, size_t batch_max, uint8_t* verdicts, size_t verdicts_cap,
                                 praos_replay_stats* stats);
/* The same replay over a TPraos (Shelley..Alonzo) ImmutableDB: stored BHeaders, the TPraos
 * nonce rules (mkNonceFromOutputVRF of the eta certificate; TICKN with extra_entropy, NULL
 * = NeutralNonce) and the TPraos fold; failures (may be NULL, verdicts_cap entries) gets
 * each header's PRAOS_TPF_* set.  Replaces db-analyser's header revalidation over the
 * TPraos eras (TPraos.hs:361-387 per block). */
int praos_replay_immutable_tpraos(praos_ctx* ctx, const char* dir, const praos_pool* pools, uint32_t npools,
                                  const praos_params* params, const praos_epoch_info* ei,
                                  const praos_nonce* extra_entropy, praos_envelope* env, praos_chain_state* st,
                                  size_t batch_max, uint8_t* verdicts, uint16_t* failures, size_t verdicts_cap,
                                  praos_replay_stats* stats);

/* ---- several GPUs from one process ----
 * A group = one context per entry of devices[] (a device may repeat: several
 * contexts on one GPU), each driven by its own host thread.  Batch calls split the
 * n headers into contiguous shards (member k: [n*k/m, n*(k+1)/m)), run them
 * concurrently and write every output in place, so the caller's arrays look exactly
 * as after the single-context call.  The fold (praos_validate_headers) then runs
 * over the gathered outputs on praos_group_ctx(g, 0).  No exchange between devices
 * (headers of one epoch are independent, Praos.hs:441-459). */
typedef struct praos_group praos_group;
praos_group* praos_group_open(const int* devices, int ndev);     /* NULL on failure */
void praos_group_close(praos_group* g);
int praos_group_size(praos_group* g);
praos_ctx* praos_group_ctx(praos_group* g, int k);               /* member k's context */
const char* praos_group_last_error(praos_group* g);
int praos_group_set_option(praos_group* g, int opt, int value);
int praos_group_set_epoch(praos_group* g, const uint8_t eta0[32], const praos_pool* pools, uint32_t npools,
                          const praos_params* params);
int praos_group_verify_headers(praos_group* g, const praos_headers* h, praos_out* out);
int praos_group_verify_header_bytes(praos_group* g, const praos_header_bytes* in, praos_out* out,
                                    praos_decoded* dec);
/* TPraos batches over the group (ABI 12): praos_verify_tpraos_headers /
 * praos_verify_tpraos_header_bytes per shard (TPraos.hs:378-387), outputs in place; dec's
 * signed_body has the PRAOS_TP_SIGNED_STRIDE stride, leader_out / leader_proof may be NULL. */
int praos_group_verify_tpraos_headers(praos_group* g, const praos_tpraos_headers* h, praos_tpraos_out* out);
int praos_group_verify_tpraos_header_bytes(praos_group* g, const praos_header_bytes* in, praos_tpraos_out* out,
                                           praos_decoded* dec, uint8_t* leader_out, uint8_t* leader_proof);
/* ABI 13.  A caller buffer page-locked once for every member (the Haskell arena of an epoch:
 * each member's shard uploads by direct DMA), and the ImmutableDB replay over the group
 * (db-analyser's processAllImmutableDB, DBAnalyser/Analysis.hs:815-847, on several GPUs):
 * consecutive batches are dealt to the members in turn, the nonce chain and the fold
 * (envelope + updateChainDepState) run once in chain order on member 0; arguments, outputs,
 * stop and resume exactly as praos_replay_immutable[_tpraos] on one context. */
int praos_group_set_overlay(praos_group* g, const praos_overlay* ov);   /* praos_set_overlay on every member */
int praos_group_host_register(praos_group* g, void* p, size_t len);
int praos_group_host_unregister(praos_group* g, void* p);
int praos_group_replay_immutable(praos_group* g, const char* dir, const praos_pool* pools, uint32_t npools,
                                 const praos_params* params, const praos_epoch_info* ei, praos_envelope* env,
                                 praos_chain_state* st, size_t batch_max, uint8_t* verdicts, size_t verdicts_cap,
                                 praos_replay_stats* stats);
int praos_group_replay_immutable_tpraos(praos_group* g, const char* dir, const praos_pool* pools, uint32_t npools,
                                        const praos_params* params, const praos_epoch_info* ei,
                                        const praos_nonce* extra_entropy, praos_envelope* env, praos_chain_state* st,
                                        size_t batch_max, uint8_t* verdicts, uint16_t* failures, size_t verdicts_cap,
                                        praos_replay_stats* stats);
/* ABI 14: praos_verify_block_integrity over the group (ImmutableDB chunk validation on several
 * GPUs: contiguous shards of the blocks, results in place). */
int praos_group_verify_block_integrity(praos_group* g, const praos_header_bytes* blocks,
                                       uint64_t slots_per_kes_period, uint8_t* result, uint8_t* body_hash);
/* ABI 14: praos_replay_immutable_views over the group. */
int praos_group_replay_immutable_views(praos_group* g, const char* dir, const praos_ledger_view* views,
                                       uint32_t nviews, const praos_params* params, const praos_epoch_info* ei,
                                       praos_envelope* env, praos_chain_state* st, size_t batch_max,
                                       uint8_t* verdicts, size_t verdicts_cap, praos_replay_stats* stats);

/* ---- synthetic chain generator (db-synthesizer analogue, for benches) ----
 * Signs on the GPU: OCert (Ed25519), Sum6KES (Blake2b-256 tree + Ed25519 leaf),
 * VRF draft-03 proofs for alpha = mkInputVRF(slot, eta0).  Keys derive from
 * 32-byte seeds: cold/VRF/KES seed of pool i = Blake2b-256(tag || seed || i). */
typedef struct {
  uint64_t n;                     /* headers */
  uint32_t npools;
  uint64_t first_slot;
  uint64_t slot_stride;           /* slot of header i = first_slot + i * slot_stride */
  uint32_t body_len;              /* > 0: pseudo-random signed bodies of this length;
                                     0: the genuine canonical HeaderBody CBOR of each header
                                     (PRAOS_SIGNED_STRIDE bytes per header; praos_synthesize_tpraos:
                                     the 15-field BHBody, PRAOS_TP_SIGNED_STRIDE bytes) */
  uint32_t corrupt_per_10000;     /* seeded corruptions (Corruption.hs model: +1 at a byte) */
  uint32_t nkes;                  /* distinct Sum6KES keys (0 = one per pool); header of pool p uses key p mod nkes */
  uint8_t seed[32];
  const uint8_t* body_hash;       /* n*32 hbBodyHash of each CBOR body (e.g. hashTxSeq of the block's
                                     segments, for stored-block corpora); NULL = pseudo-random */
  /* Leader schedule (from praos_leader_schedule): header i is forged in slot
   * sched_slot[i] by pool sched_pool[i], blockNo = block_no0 + i.  NULL: slot of
   * header i = first_slot + i * slot_stride and pools assigned by hash -- such a
   * chain is NOT leader-valid (most headers fail VRFLeaderValueTooBig). */
  const uint64_t* sched_slot;
  const uint32_t* sched_pool;
  uint64_t block_no0;
  /* Chain linking (CBOR bodies, Praos or TPraos): link_prev = 1 makes hbPrev of header i the
   * headerHash of header i-1 -- header 0 gets prev0, or GenesisHash when prev0 is NULL --
   * re-signing each KES signature in order (sequential on the device: ~0.1 ms per
   * header).  header_hash (optional, n*32) receives the header hashes (before any
   * seeded corruption). */
  int32_t link_prev;
  const uint8_t* prev0;
  uint8_t* header_hash;
  /* Fields the seeded corruptions may hit (PRAOS_CORRUPT_* bits; 0 = all five: OCert
   * signature, KES signature, VRF proof, VRF output, signed body), so a single-primitive
   * batch corrupts only what its check reads (configs[1..3]: 1 % means 1 %). */
  uint32_t corrupt_fields;
} praos_synth_params;

#define PRAOS_CORRUPT_OCERT     0x01u  /* +1 at a byte of cold vk || hot vk || BE64 n || BE64 c0 || sigma
                                          (the 144 bytes of an OCert verify; signature only for CBOR bodies) */
#define PRAOS_CORRUPT_KES_SIG   0x02u
#define PRAOS_CORRUPT_VRF_PROOF 0x04u
#define PRAOS_CORRUPT_VRF_OUT   0x08u
#define PRAOS_CORRUPT_BODY      0x10u

/* Fills caller buffers (same layout as praos_headers; body_off/body_len/body_bytes
 * sized n, n, n*stride+8 with stride = round_up(body_len, 8), or PRAOS_SIGNED_STRIDE
 * when body_len = 0).  Also returns the pool table
 * (npools entries, sigma_fp left for the caller to set). */
int praos_synthesize(praos_ctx* ctx, const praos_synth_params* sp, const praos_params* params,
                     const uint8_t eta0[32], praos_pool* pools_out, uint64_t* slot, uint8_t* cold_vk,
                     uint8_t* vrf_vk, uint8_t* vrf_out, uint8_t* vrf_proof, uint8_t* hot_vk, uint64_t* ocert_n,
                     uint64_t* ocert_c0, uint8_t* ocert_sig, uint8_t* kes_sig, uint64_t* body_off,
                     uint32_t* body_len, uint8_t* body_bytes, uint8_t* corrupted);

/* Leader schedule of the generator's pools (db-synthesizer, Forging.hs:139-148):
 * the pools derived from `seed` (as praos_synthesize derives them, npools of them,
 * stake sigma_fp[p], Fixed E34 raw uint128 LE) are the forgers, tried in index
 * order.  For every slot s in [first_slot, first_slot + nslots): leader[s -
 * first_slot] = the first pool p for which checkIsLeader holds (Praos.hs:375-397:
 * meetsLeaderThreshold, :505-526, on evalCertified (mkInputVRF s eta0) under p's
 * VRF key), or -1 (no block in that slot).  tpraos = 1: the TPraos leader cert
 * (mkSeed seedL, 64-byte output, bound 2^512).  Cost: one VRF evaluation per
 * (slot, pool) pair up to the slot's leader, i.e. ~npools per empty slot. */
int praos_leader_schedule(praos_ctx* ctx, const uint8_t seed[32], uint32_t npools, const uint8_t* sigma_fp,
                          const praos_params* params, const uint8_t eta0[32], uint64_t first_slot, uint64_t nslots,
                          int tpraos, int32_t* leader);

/* TPraos variant of the generator: the VRF cert pair uses mkSeed alphas;
 * leader_out/leader_proof receive the leader cert (n*64, n*80). */
int praos_synthesize_tpraos(praos_ctx* ctx, const praos_synth_params* sp, const praos_params* params,
                            const uint8_t eta0[32], praos_pool* pools_out, uint64_t* slot, uint8_t* cold_vk,
                            uint8_t* vrf_vk, uint8_t* vrf_out, uint8_t* vrf_proof, uint8_t* hot_vk, uint64_t* ocert_n,
                            uint64_t* ocert_c0, uint8_t* ocert_sig, uint8_t* kes_sig, uint64_t* body_off,
                            uint32_t* body_len, uint8_t* body_bytes, uint8_t* leader_out, uint8_t* leader_proof,
                            uint8_t* corrupted);

/* ---- self-test entry points (unit tests of the device arithmetic) ---- */
/* op: 0 mul, 1 sq, 2 add, 3 sub, 4 invert (the build's: binary GCD unless PRAOS_INV_GCD=0), 5 pow22523,
   6 canon, 7 invert by Fermat's z^(p-2), 8 invert by the binary GCD; inputs/outputs n*32 bytes LE */
int praos_debug_fe(praos_ctx* ctx, int op, size_t n, const uint8_t* a, const uint8_t* b, uint8_t* r);
/* SHA-512 of (64-byte prefix || msg) per item; out n*64 */
int praos_debug_sha512(praos_ctx* ctx, size_t n, const uint8_t* prefix, const uint64_t* msg_off,
                       const uint32_t* msg_len, const uint8_t* msg_bytes, size_t msg_bytes_len, uint8_t* out);
/* BLAKE2b-256 of 64-byte inputs; out n*32 */
int praos_debug_blake2b(praos_ctx* ctx, size_t n, const uint8_t* in64, uint8_t* out);
/* x mod L for 64-byte inputs; out n*32 */
int praos_debug_sc_reduce(praos_ctx* ctx, size_t n, const uint8_t* in64, uint8_t* out);
/* decode point (1 = ok) and re-encode; out n*32, ok n */
int praos_debug_decode(praos_ctx* ctx, size_t n, const uint8_t* in32, uint8_t* out, uint8_t* ok);
/* [s]B for 32-byte scalars (< 2^255); out n*32 */
int praos_debug_scalarmult_base(praos_ctx* ctx, size_t n, const uint8_t* s, uint8_t* out);
/* leader check with explicit x_raw per item (4 words LE); is_leader, iters out */
int praos_debug_leader(praos_ctx* ctx, size_t n, const uint8_t* leader, const uint8_t* x_raw16, uint8_t* is_leader,
                       int32_t* iters);
/* the same for the TPraos form: 64-byte big-endian leader values, bound 2^512 */
int praos_debug_leader512(praos_ctx* ctx, size_t n, const uint8_t* leader64, const uint8_t* x_raw16,
                          uint8_t* is_leader, int32_t* iters);
/* Elligator2 hash-to-curve of the VRF suite: h(pk, alpha); out n*32 */
int praos_debug_hash_to_curve(praos_ctx* ctx, size_t n, const uint8_t* pk, const uint8_t* alpha, uint8_t* out);

#ifdef __cplusplus
}
#endif
#endif
