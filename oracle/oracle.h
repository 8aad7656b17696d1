/*
 * oracle.h -- CPU restatement of the Praos header-crypto path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (libpraos_hip) links,
 * loads or calls this code; only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py use it, and only as the checker / the timed
 * CPU port.  Representation is deliberately different from the GPU kernels
 * (radix-2^51 field limbs, plain double-and-add, bit-serial bignum division)
 * so that a shared bug is unlikely.
 *
 * What it restates (the reference is Haskell calling third-party C; see
 * SURVEY.md sec. 2b / App. C):
 *   - Ed25519 verify, libsodium 1.0.18 `crypto_sign_ed25519_verify_detached`
 *     as bound by cardano-crypto-class `Ed25519DSIGN`
 *     (call sites: Praos.hs:580 OCert, KES leaf under Praos.hs:582)
 *   - Sum6KES verify (cardano-crypto-class `KES.Sum`, Blake2b_256 vk hashes)
 *     (Praos.hs:582; Shelley/Protocol/Praos.hs:85)
 *   - ECVRF-ED25519-SHA512-Elligator2 draft-03 verify + proof_to_hash
 *     (IOG libsodium fork `crypto_vrf_ietfdraft03_*`, bound by
 *     cardano-crypto-praos `Cardano.Crypto.VRF.Praos`; call site Praos.hs:543)
 *   - mkInputVRF / vrfLeaderValue / vrfNonceValue (Praos/VRF.hs:55-131)
 *   - checkLeaderNatValue + taylorExpCmp in Fixed E34 (cardano-protocol-tpraos
 *     BHeader / cardano-ledger-core NonIntegral; call site Praos.hs:549)
 *   - validateKESSignature / validateVRFSignature check order
 *     (Praos.hs:558-606, Praos.hs:528-556)
 */
#ifndef PRAOS_ORACLE_H
#define PRAOS_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- hashes ---- */
void orc_sha512(uint8_t out[64], const uint8_t *m, size_t n);
void orc_blake2b(uint8_t *out, size_t outlen, const uint8_t *m, size_t n);

/* ---- Ed25519 (libsodium 1.0.18 rules) ---- */
/* 0 = valid, -1 = "Verification failed" */
int orc_ed25519_verify(const uint8_t sig[64], const uint8_t *m, size_t n, const uint8_t pk[32]);
void orc_ed25519_pk_from_seed(uint8_t pk[32], const uint8_t seed[32]);
void orc_ed25519_sign(uint8_t sig[64], const uint8_t *m, size_t n, const uint8_t seed[32]);

/* ---- ECVRF draft-03 ---- */
/* 0 = proof valid (beta written), -1 = invalid */
int orc_vrf_verify(uint8_t beta[64], const uint8_t pk[32], const uint8_t proof[80],
                   const uint8_t *alpha, size_t alphalen);
int orc_vrf_proof_to_hash(uint8_t beta[64], const uint8_t proof[80]);
void orc_vrf_pk_from_seed(uint8_t pk[32], const uint8_t seed[32]);
int orc_vrf_prove(uint8_t proof[80], const uint8_t seed[32], const uint8_t *alpha, size_t alphalen);

/* ---- Sum6KES (Blake2b-256, Ed25519 leaves) ---- */
#define ORC_KES_DEPTH 6
#define ORC_KES_SIG_BYTES (64 + 64 * ORC_KES_DEPTH)
/* 0 = ok, 1 = "Reject" (Merkle hash mismatch), 2 = leaf "Verification failed" */
int orc_kes_verify(const uint8_t vk[32], uint32_t t, const uint8_t *m, size_t n,
                   const uint8_t sig[ORC_KES_SIG_BYTES]);
/* key derivation by expandSeed recursion; vk = Merkle root */
void orc_kes_vk_from_seed(uint8_t vk[32], const uint8_t seed[32]);
int orc_kes_sign(uint8_t sig[ORC_KES_SIG_BYTES], const uint8_t seed[32], uint32_t t,
                 const uint8_t *m, size_t n);

/* ---- Leader check (Fixed E34) ---- */
/* c_raw: raw FixedPoint of activeSlotLog f (negative), as signed 128-bit
 * two's complement little-endian (16 bytes).  sigma_fp: raw FixedPoint of
 * sigma (fromRational sigma), unsigned 128-bit LE.  leader: 32-byte big-endian
 * natural (Blake2b-256("L"||out)).  Returns 1 = leader (BELOW), 0 = not.
 * iters (optional) receives the Taylor iterations used. */
int orc_check_leader(const uint8_t leader_be[32], const uint8_t sigma_fp[16],
                     const uint8_t c_raw[16], int f_is_one, int *iters);

/* ---- Praos header (per-check bits), mirrors Praos.hs:441-606 ---- */
enum {
  ORC_BIT_KES_BEFORE_START = 1u << 0,  /* KESBeforeStartOCERT */
  ORC_BIT_KES_AFTER_END    = 1u << 1,  /* KESAfterEndOCERT */
  ORC_BIT_OCERT_SIG        = 1u << 2,  /* InvalidSignatureOCERT */
  ORC_BIT_KES_MERKLE       = 1u << 3,  /* InvalidKesSignatureOCERT "Reject" */
  ORC_BIT_KES_LEAF         = 1u << 4,  /* InvalidKesSignatureOCERT leaf */
  ORC_BIT_VRF_KEY_UNKNOWN  = 1u << 8,  /* VRFKeyUnknown */
  ORC_BIT_VRF_KEY_WRONG    = 1u << 9,  /* VRFKeyWrongVRFKey */
  ORC_BIT_VRF_PROOF        = 1u << 10, /* VRFKeyBadProof (proof) */
  ORC_BIT_VRF_OUTPUT       = 1u << 11, /* VRFKeyBadProof (claimed output != beta) */
  ORC_BIT_LEADER           = 1u << 12, /* VRFLeaderValueTooBig */
};

typedef struct {
  uint8_t hash28[28];
  uint8_t vrf_hash32[32];
  uint8_t sigma_fp[16];   /* raw Fixed E34 of sigma, unsigned LE */
} orc_pool;

typedef struct {
  uint64_t slot;
  uint8_t cold_vk[32];
  uint8_t vrf_vk[32];
  uint8_t vrf_out[64];
  uint8_t vrf_proof[80];
  uint8_t hot_vk[32];
  uint64_t ocert_n;
  uint64_t ocert_c0;
  uint8_t ocert_sig[64];
  uint8_t kes_sig[ORC_KES_SIG_BYTES];
  const uint8_t *body;
  size_t body_len;
} orc_header;

typedef struct {
  uint8_t eta0[32];
  int eta0_neutral;
  uint64_t slots_per_kes_period;
  uint64_t max_kes_evo;
  int f_is_one;
  uint8_t c_raw[16];
  const orc_pool *pools;     /* sorted by hash28 (memcmp order) */
  uint32_t npools;
} orc_epoch;

typedef struct {
  uint32_t bits;
  int32_t pool_idx;       /* -1 if issuer not in pool distribution */
  uint8_t beta[64];       /* proof_to_hash (zero if Gamma undecodable) */
  uint8_t leader[32];     /* Blake2b256("L"||claimed out), big-endian natural */
  uint8_t nonce[32];      /* Blake2b256(Blake2b256("N"||claimed out)) */
  uint8_t issuer_hash[28];
} orc_result;

void orc_praos_header(const orc_epoch *ep, const orc_header *h, orc_result *r);

/* ---- TPraos header (Shelley..Alonzo), d = 0 path ----
 * cardano-protocol-tpraos (>= 1.0.1 < 1.1, ouroboros-consensus-cardano.cabal:132):
 * OVERLAY praosVrfChecks then OCERT (TPraos.hs:378-398 calls SL.updateChainDepState).
 *   seed alpha = Blake2b256(BE64 slot || eta0) XOR Blake2b256(BE64 k), k = 0 (eta), 1 (leader)
 *   leader value = certified leader output (64 B) as a big-endian natural < 2^512
 *   nonce        = Blake2b256(certified eta output)                                   */
enum {
  ORC_BIT_TP_VRF_NONCE   = 1u << 10,  /* VRFKeyBadNonce (proof rejected or output mismatch) */
  ORC_BIT_TP_VRF_LEADER  = 1u << 11,  /* VRFKeyBadLeaderValue */
};
typedef struct {
  orc_header h;             /* vrf_out / vrf_proof = the eta certificate */
  uint8_t leader_out[64];
  uint8_t leader_proof[80];
} orc_tp_header;
typedef struct {
  uint32_t bits;
  int32_t pool_idx;
  uint8_t beta_eta[64];
  uint8_t beta_leader[64];
  uint8_t nonce[32];
} orc_tp_result;
void orc_tpraos_seed(uint8_t out[32], uint64_t slot, const uint8_t eta0[32], int eta0_neutral, uint64_t k);
void orc_tpraos_header(const orc_epoch *ep, const orc_tp_header *h, orc_tp_result *r);
/* leader check against a 512-bit big-endian value (TPraos checkLeaderValue) */
int orc_check_leader512(const uint8_t leader_be[64], const uint8_t sigma_fp[16], const uint8_t c_raw[16],
                        int f_is_one, int *iters);

#ifdef __cplusplus
}
#endif
#endif
