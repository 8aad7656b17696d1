// k_synth.hip -- synthetic chain generator kernels (db-synthesizer analogue).
#include "kcommon.hpp"
#include "arena.hpp"

// ------------------------------------------------------------------ synthetic chain generator
// seeds: Blake2b-256(tag || master seed(32) || BE32(i))
__device__ __forceinline__ void derive_seed(uint32_t out[8], uint32_t tag, const uint32_t master[8], uint32_t i) {
  uint64_t m[16];
  // bytes: tag(1) master(32) i(4) = 37
  uint8_t bytes[40];
  bytes[0] = (uint8_t)tag;
#pragma unroll
  for (int k = 0; k < 32; k++) bytes[1 + k] = (uint8_t)(master[k / 4] >> (8 * (k % 4)));
  bytes[33] = (uint8_t)(i >> 24); bytes[34] = (uint8_t)(i >> 16); bytes[35] = (uint8_t)(i >> 8); bytes[36] = (uint8_t)i;
  bytes[37] = bytes[38] = bytes[39] = 0;
#pragma unroll
  for (int w = 0; w < 5; w++) {
    uint64_t v = 0;
#pragma unroll
    for (int k = 7; k >= 0; k--) v = (v << 8) | bytes[8 * w + k];
    m[w] = v;
  }
#pragma unroll
  for (int w = 5; w < 16; w++) m[w] = 0;
  uint64_t h[4];
  blake2b_1block(h, m, 37, 32);
#pragma unroll
  for (int k = 0; k < 4; k++) { out[2 * k] = (uint32_t)h[k]; out[2 * k + 1] = (uint32_t)(h[k] >> 32); }
}

// KES expandSeed: r_b = Blake2b-256(b || s), b in {1, 2}
__device__ __forceinline__ void kes_expand(uint32_t out[8], uint32_t b, const uint32_t s[8]) {
  uint64_t m[16];
  uint64_t prev = b & 0xff;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const uint64_t w = ((uint64_t)s[2 * k + 1] << 32) | s[2 * k];
    m[k] = prev | (w << 8);
    prev = w >> 56;
  }
  m[4] = prev;
#pragma unroll
  for (int k = 5; k < 16; k++) m[k] = 0;
  uint64_t h[4];
  blake2b_1block(h, m, 33, 32);
#pragma unroll
  for (int k = 0; k < 4; k++) { out[2 * k] = (uint32_t)h[k]; out[2 * k + 1] = (uint32_t)(h[k] >> 32); }
}

// per pool: cold/vrf/kes seeds, cold pk, vrf pk, pool hash, vrf hash
__global__ void __launch_bounds__(NT) k_synth_pools(uint32_t npools, const ge_niels* gbtab, const uint32_t* master,
                                                    uint32_t* cold_seed, uint32_t* cold_pk, uint32_t* vrf_seed,
                                                    uint32_t* vrf_pk, uint32_t* kes_seed, uint8_t* pool_hash28,
                                                    uint8_t* pool_vrf32) {
  __shared__ ge_niels sbtab[2 * BTAB_N];
  const ge_niels* btab = stage_btab<5>(gbtab, sbtab);
  const uint32_t p = blockIdx.x * NT + threadIdx.x;
  if (p >= npools) return;
  uint32_t ms[8], cs[8], vs[8], ks[8], az[16], cpk[8], vpk[8], h[8];
#pragma unroll
  for (int k = 0; k < 8; k++) ms[k] = master[k];
  derive_seed(cs, 1, ms, p);
  derive_seed(vs, 2, ms, p);
  derive_seed(ks, 3, ms, p);
  ed25519_expand(az, cs);
  ed25519_pk_from_az(cpk, az, btab);
  ed25519_expand(az, vs);
  ed25519_pk_from_az(vpk, az, btab);
#pragma unroll
  for (int k = 0; k < 8; k++) {
    cold_seed[8 * p + k] = cs[k]; cold_pk[8 * p + k] = cpk[k];
    vrf_seed[8 * p + k] = vs[k]; vrf_pk[8 * p + k] = vpk[k]; kes_seed[8 * p + k] = ks[k];
  }
  blake2b_32(h, cpk, 28);
  for (int k = 0; k < 28; k++) pool_hash28[28 * p + k] = (uint8_t)(h[k / 4] >> (8 * (k % 4)));
  blake2b_32(h, vpk, 32);
  for (int k = 0; k < 32; k++) pool_vrf32[32 * p + k] = (uint8_t)(h[k / 4] >> (8 * (k % 4)));
}

// per (pool, leaf): leaf seed by expandSeed down the path, leaf Ed25519 pk.
// tree layout per pool: node[1..127] (heap order, root = 1), 8 words each;
// leaves are nodes 64..127 (leaf j = node 64 + j).
__global__ void __launch_bounds__(NT) k_synth_kes_leaves(uint32_t npools, const ge_niels* gbtab,
                                                         const uint32_t* kes_seed, uint32_t* leaf_seed,
                                                         uint32_t* tree) {
  __shared__ ge_niels sbtab[2 * BTAB_N];
  const ge_niels* btab = stage_btab<5>(gbtab, sbtab);
  const uint32_t g = blockIdx.x * NT + threadIdx.x;
  if (g >= npools * 64u) return;
  const uint32_t p = g / 64, j = g % 64;
  uint32_t s[8], r[8], az[16], pk[8];
#pragma unroll
  for (int k = 0; k < 8; k++) s[k] = kes_seed[8 * p + k];
  for (int d = 5; d >= 0; d--) {                 // top level first: bit 5 of j
    kes_expand(r, ((j >> d) & 1) ? 2u : 1u, s);
#pragma unroll
    for (int k = 0; k < 8; k++) s[k] = r[k];
  }
  ed25519_expand(az, s);
  ed25519_pk_from_az(pk, az, btab);
#pragma unroll
  for (int k = 0; k < 8; k++) {
    leaf_seed[8 * g + k] = s[k];
    tree[(size_t)p * 128 * 8 + (64 + j) * 8 + k] = pk[k];
  }
}

// per pool: internal nodes bottom-up, node v = Blake2b-256(node 2v || node 2v+1)
__global__ void k_synth_kes_tree(uint32_t npools, uint32_t* tree) {
  const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= npools) return;
  uint32_t* t = tree + (size_t)p * 128 * 8;
  for (int v = 63; v >= 1; v--) {
    uint32_t in[16], h[8];
    for (int k = 0; k < 8; k++) { in[k] = t[(2 * v) * 8 + k]; in[8 + k] = t[(2 * v + 1) * 8 + k]; }
    blake2b256_64(h, in);
    for (int k = 0; k < 8; k++) t[v * 8 + k] = h[k];
  }
}

// ------------------------------------------------------------------ leader schedule
// VRF secret scalar x = (clamped SHA-512(seed))[0..32) mod L per pool (the scalar
// vrf_prove_core uses), so Gamma = x H and beta = proof_to_hash exactly as the proof.
__global__ void k_synth_vrf_scalar(uint32_t npools, const uint32_t* __restrict__ vrf_seed, uint32_t* __restrict__ vrf_x) {
  const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= npools) return;
  uint32_t seed[8], az[16], x[8];
#pragma unroll
  for (int k = 0; k < 8; k++) seed[k] = vrf_seed[8 * p + k];
  ed25519_expand(az, seed);
  sc_reduce256(x, az);
#pragma unroll
  for (int k = 0; k < 8; k++) vrf_x[8 * p + k] = x[k];
}

// db-synthesizer slot loop (Forging.hs:139-148): per slot, the forgers are tried in
// order and the first whose checkShouldForge says ShouldForge forges.  Here one
// lane = one (slot, pool) of the pools [p0, p0 + pn): checkIsLeader (Praos.hs:375-397)
// = meetsLeaderThreshold (:505-526) on evalCertified (mkInputVRF slot eta0); the
// minimum leading pool index per slot is kept with a vector atomicMin (first
// leader wins).  Pools are processed in increasing chunks, so a lane whose slot
// already has a leader from an earlier chunk returns at once.
// TPraos (tpraos = 1): the leader cert of the pair, mkSeed seedL, and the raw
// 64-byte output as the natural (bound 2^512, cardano-protocol-tpraos checkLeaderValue).
__global__ void __launch_bounds__(NT) k_synth_leader_search(uint64_t first_slot, uint64_t nslots, uint32_t p0,
                                                            uint32_t pn, const uint32_t* __restrict__ vrf_x,
                                                            const uint32_t* __restrict__ vrf_pk,
                                                            const uint32_t* __restrict__ pool_thr,
                                                            const uint32_t* __restrict__ eta0, int eta0_neutral,
                                                            int f_is_one, int tpraos, int32_t* __restrict__ leader) {
  const uint64_t g = (uint64_t)blockIdx.x * NT + threadIdx.x;
  const uint64_t si = g / pn;
  const uint32_t p = p0 + (uint32_t)(g % pn);
  if (si >= nslots) return;
  if (leader[si] < (int32_t)p) return;                 // an earlier forger already leads this slot
  const uint64_t s = first_slot + si;
  uint32_t e0[8], alpha[8], ys[8], x[8], thr[4];
#pragma unroll
  for (int k = 0; k < 8; k++) { e0[k] = eta0[k]; ys[k] = vrf_pk[8 * p + k]; x[k] = vrf_x[8 * p + k]; }
#pragma unroll
  for (int k = 0; k < 4; k++) thr[k] = pool_thr[4 * p + k];
  if (tpraos) tpraos_seed(alpha, s, e0, eta0_neutral != 0, 1ull);
  else mk_input_vrf(alpha, s, e0, eta0_neutral != 0);
  ge_p3 H, G, G2, G4, G8;
  vrf_hash_to_curve(H, ys, alpha);
  ge_scalarmult_var(G, x, H);
  ge_p3_dbl_to_p3(G2, G);
  ge_p3_dbl_to_p3(G4, G2);
  ge_p3_dbl_to_p3(G8, G4);
  uint32_t g8s[8], beta[16];
  ge_tobytes(g8s, G8.X, G8.Y, G8.Z);
  vrf_beta(beta, g8s);
  bool lead = true;
  if (!f_is_one) {
    if (tpraos) {
      uint32_t l[16];
#pragma unroll
      for (int k = 0; k < 16; k++) l[k] = __builtin_bswap32(beta[15 - k]);
      lead = leader_check_t<16>(l, thr, nullptr);
    } else {
      uint32_t lv[8], l[8];
      blake2b256_tag64(lv, 'L', beta);                   // vrfLeaderValue, Praos/VRF.hs:103-112
#pragma unroll
      for (int k = 0; k < 8; k++) l[k] = __builtin_bswap32(lv[7 - k]);
      lead = leader_check(l, thr, nullptr);
    }
  }
  if (lead) atomicMin(&leader[si], (int32_t)p);
}

__device__ __forceinline__ uint64_t mix64(uint64_t x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdULL; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ULL; x ^= x >> 33;
  return x;
}

// byte writer of the canonical CBOR body (generator only)
struct SynthWr {
  uint8_t* o;
  uint32_t n;
};
__device__ __forceinline__ void sw_byte(SynthWr& w, uint32_t b) { w.o[w.n++] = (uint8_t)b; }
__device__ void sw_head(SynthWr& w, uint32_t mt, uint64_t v) {
  if (v < 24) { sw_byte(w, (mt << 5) | (uint32_t)v); return; }
  const int nb = v < 256 ? 1 : v < 65536 ? 2 : v < (1ull << 32) ? 4 : 8;
  sw_byte(w, (mt << 5) | (nb == 1 ? 24u : nb == 2 ? 25u : nb == 4 ? 26u : 27u));
  for (int k = nb - 1; k >= 0; k--) sw_byte(w, (uint32_t)(v >> (8 * k)));
}
__device__ void sw_bytes(SynthWr& w, const uint8_t* src, uint32_t n) {
  sw_head(w, 2, n);
  for (uint32_t k = 0; k < n; k++) sw_byte(w, src[k]);
}

// per header: body bytes, OCert signature, KES signature, VRF proof/output.
__global__ void __launch_bounds__(NT) k_synth_headers(
    size_t n, const ge_niels* gbtab, uint32_t npools, uint32_t nkes, uint64_t first_slot, uint64_t slot_stride,
    uint64_t slots_per_kes_period, uint32_t blen, uint64_t salt, const uint32_t* eta0, int eta0_neutral,
    const uint32_t* cold_seed, const uint32_t* cold_pk, const uint32_t* vrf_seed, const uint32_t* vrf_pk,
    const uint32_t* leaf_seed, const uint32_t* tree, uint8_t* msg_scratch, uint64_t* slot, uint8_t* cold_vk,
    uint8_t* vrf_vk, uint8_t* vrf_out, uint8_t* vrf_proof, uint8_t* hot_vk, uint64_t* ocert_n, uint64_t* ocert_c0,
    uint8_t* ocert_sig, uint8_t* kes_sig, uint64_t* body_off, uint32_t* body_len, uint8_t* body_bytes, int tpraos,
    uint8_t* l_out, uint8_t* l_proof, const uint8_t* __restrict__ body_hash_in,
    const uint64_t* __restrict__ sched_slot, const uint32_t* __restrict__ sched_pool, uint64_t block_no0,
    uint32_t* __restrict__ leaf_of) {
  __shared__ ge_niels sbtab[2 * BTAB_N];
  const ge_niels* btab = stage_btab<5>(gbtab, sbtab);
  const size_t i = (size_t)blockIdx.x * NT + threadIdx.x;
  if (i >= n) return;
  // a leader schedule (praos_leader_schedule) gives slot and forging pool per
  // header; without one, slots are evenly spaced and pools hashed (not leader-valid)
  // (npools >= n without a schedule: header i gets pool i, so every key is distinct)
  const uint32_t p = sched_pool ? sched_pool[i] : npools >= n ? (uint32_t)i : (uint32_t)(mix64(i ^ salt) % npools);
  const uint64_t s = sched_slot ? sched_slot[i] : first_slot + i * slot_stride;
  const uint64_t kp = s / slots_per_kes_period;
  const uint64_t c0 = kp - (kp % 60u);          // OCert issued at a period boundary <= kp
  const uint64_t t = kp - c0;                   // < 60 <= maxKESEvo (62)
  const uint64_t nn = c0 / 60u;                 // issue number grows with each new OCert
  slot[i] = s; ocert_n[i] = nn; ocert_c0[i] = c0;
  const uint32_t kk = p % nkes;                 // KES key of this pool
  const uint32_t* T = tree + (size_t)kk * 128 * 8;
  uint32_t hv[8], cpk[8], vpk[8];
#pragma unroll
  for (int k = 0; k < 8; k++) { hv[k] = T[8 + k]; cpk[k] = cold_pk[8 * p + k]; vpk[k] = vrf_pk[8 * p + k]; }
  store_words(hot_vk + 32 * i, hv, 8);
  store_words(cold_vk + 32 * i, cpk, 8);
  store_words(vrf_vk + 32 * i, vpk, 8);
  // OCert signature over hot_vk || BE64(n) || BE64(c0)
  uint8_t* msg = msg_scratch + 48 * i;
  store_words(msg, hv, 8);
  for (int k = 0; k < 8; k++) { msg[32 + k] = (uint8_t)(nn >> (56 - 8 * k)); msg[40 + k] = (uint8_t)(c0 >> (56 - 8 * k)); }
  uint32_t seed[8], az[16], sig[16];
#pragma unroll
  for (int k = 0; k < 8; k++) seed[k] = cold_seed[8 * p + k];
  ed25519_expand(az, seed);
  ed25519_sign_core(sig, az, cpk, msg, 48, btab);
  store_words(ocert_sig + 64 * i, sig, 16);
  // VRF proof(s): Praos alpha = mkInputVRF(slot, eta0); TPraos: the eta cert
  // with mkSeed seedEta and the leader cert with mkSeed seedL.  output = beta.
  uint32_t e0[8], alpha[8], proof[20];
#pragma unroll
  for (int k = 0; k < 8; k++) { e0[k] = eta0[k]; seed[k] = vrf_seed[8 * p + k]; }
  ed25519_expand(az, seed);
  for (int cert = 0; cert < (tpraos ? 2 : 1); cert++) {
    if (tpraos) tpraos_seed(alpha, s, e0, eta0_neutral != 0, (uint64_t)cert);
    else mk_input_vrf(alpha, s, e0, eta0_neutral != 0);
    vrf_prove_core(proof, az, vpk, alpha, btab);
    store_words((cert ? l_proof : vrf_proof) + 80 * i, proof, 20);
    ge_p3 G, G2, G4, G8;
    ge_frombytes(G, proof, false);
    ge_p3_dbl_to_p3(G2, G);
    ge_p3_dbl_to_p3(G4, G2);
    ge_p3_dbl_to_p3(G8, G4);
    uint32_t g8s[8], beta[16];
    ge_tobytes(g8s, G8.X, G8.Y, G8.Z);
    vrf_beta(beta, g8s);
    store_words((cert ? l_out : vrf_out) + 64 * i, beta, 16);
  }
  // body: blen > 0: deterministic pseudo-random bytes (a signed-message stand-in);
  // blen == 0: the genuine canonical HeaderBody CBOR (Praos/Header.hs:160-185) of
  // this header, 448-byte stride, so the header bytes can be decoded and the KES
  // message is exactly `serialize' hb`; with tpraos the 15-field BHBody of
  // cardano-protocol-tpraos (encodeBHBody: both certificates, OCert and ProtVer
  // inlined), 640-byte stride.
  const uint64_t bstride = blen ? (((uint64_t)blen + 7) & ~7ull) : (tpraos ? 640ull : 448ull);
  const uint64_t boff = (uint64_t)i * bstride;
  uint32_t bl = blen;
  uint64_t st = mix64(i * 0x9e3779b97f4a7c15ULL ^ salt ^ 0xb0d1);
  if (blen) {
    for (uint32_t k = 0; k < blen; k += 8) {
      st = mix64(st + k);
      *(uint64_t*)(body_bytes + boff + k) = st;
    }
    for (uint32_t k = blen; k < ((blen + 7) & ~7u); k++) body_bytes[boff + k] = 0;
  } else {
    SynthWr w{body_bytes + boff, 0};
    sw_head(w, 4, tpraos ? 15 : 10);
    sw_head(w, 0, sched_slot ? block_no0 + i : first_slot / slot_stride + i);   // blockNo
    sw_head(w, 0, s);                                           // slotNo
    sw_head(w, 2, 32);                                          // prevHash (pseudo-random)
    for (int k = 0; k < 4; k++) { st = mix64(st + k); for (int b = 0; b < 8; b++) sw_byte(w, (uint32_t)(st >> (8 * b))); }
    sw_bytes(w, cold_vk + 32 * i, 32);
    sw_bytes(w, vrf_vk + 32 * i, 32);
    sw_head(w, 4, 2);
    sw_bytes(w, vrf_out + 64 * i, 64);
    sw_bytes(w, vrf_proof + 80 * i, 80);
    if (tpraos) {                                               // bheaderL
      sw_head(w, 4, 2);
      sw_bytes(w, l_out + 64 * i, 64);
      sw_bytes(w, l_proof + 80 * i, 80);
    }
    st = mix64(st + 17);
    sw_head(w, 0, st & 0xffffu);                                // bodySize
    sw_head(w, 2, 32);                                          // bodyHash (caller's, else pseudo-random)
    for (int k = 0; k < 4; k++) {
      st = mix64(st + k);
      for (int b = 0; b < 8; b++)
        sw_byte(w, body_hash_in ? (uint32_t)body_hash_in[32 * i + 8 * k + b] : (uint32_t)(st >> (8 * b)));
    }
    if (!tpraos) sw_head(w, 4, 4);
    sw_bytes(w, hot_vk + 32 * i, 32);
    sw_head(w, 0, nn);
    sw_head(w, 0, c0);
    sw_bytes(w, ocert_sig + 64 * i, 64);
    if (!tpraos) sw_head(w, 4, 2);
    sw_head(w, 0, tpraos ? 6 : 8);                              // protocol version 8.0 (Babbage) / 6.0 (Alonzo)
    sw_head(w, 0, 0);
    bl = w.n;
    for (uint32_t k = bl; k < ((bl + 7) & ~7u); k++) body_bytes[boff + k] = 0;
  }
  body_off[i] = boff;
  body_len[i] = bl;
  // KES: leaf t signs the body; path pairs from the tree (leaf level first)
  const uint32_t leaf = (uint32_t)t;
  if (leaf_of) leaf_of[i] = kk * 64u + leaf;      // for k_synth_link
  uint32_t lpk[8];
#pragma unroll
  for (int k = 0; k < 8; k++) { seed[k] = leaf_seed[(8 * (size_t)kk * 64) + 8 * leaf + k]; lpk[k] = T[(64 + leaf) * 8 + k]; }
  ed25519_expand(az, seed);
  ed25519_sign_core(sig, az, lpk, body_bytes + boff, bl, btab);
  uint8_t* ks = kes_sig + 448 * i;
  store_words(ks, sig, 16);
  uint32_t node = 64 + leaf;
  for (int d = 1; d <= 6; d++) {                // level d pair = children of the ancestor at height d
    const uint32_t parent = node >> 1;
    store_words(ks + 64 * d, T + (2 * parent) * 8, 8);
    store_words(ks + 64 * d + 32, T + (2 * parent + 1) * 8, 8);
    node = parent;
  }
}

// Per KES leaf key, for the linker: the clamped scalar a, a fixed signing nonce r =
// SHA-512(prefix) mod L (the RFC 8032 nonce of the empty message) and R = [r]B.  Any r gives
// a valid Ed25519 signature (verification never sees how r was chosen), so the sequential
// re-signing of a linked chain needs no scalar multiplication per block.
__global__ void __launch_bounds__(NT) k_synth_link_keys(uint32_t nleaves, const ge_niels* __restrict__ gbtab,
                                                        const uint32_t* __restrict__ leaf_seed,
                                                        uint32_t* __restrict__ keys) {
  __shared__ ge_niels sbtab[2 * BTAB_N];
  const ge_niels* btab = stage_btab<5>(gbtab, sbtab);
  const uint32_t li = blockIdx.x * NT + threadIdx.x;
  if (li >= nleaves) return;
  uint32_t seed[8], az[16];
#pragma unroll
  for (int k = 0; k < 8; k++) seed[k] = leaf_seed[8 * (size_t)li + k];
  ed25519_expand(az, seed);
  uint32_t S[9], d[16], r[8];
#pragma unroll
  for (int k = 0; k < 8; k++) S[k] = az[8 + k];
  S[8] = 0x80u;
  sha512_regs<9, 32>(d, S);
  sc_reduce512(r, d);
  ge_p3 R;
  ge_scalarmult_base(R, r, btab);
  uint32_t rs[8];
  ge_tobytes(rs, R.X, R.Y, R.Z);
  uint32_t* o = keys + 24 * (size_t)li;
#pragma unroll
  for (int k = 0; k < 8; k++) { o[k] = az[k]; o[8 + k] = r[k]; o[16 + k] = rs[k]; }
}

// Chain linking (sequential): prevHash of header i := headerHash of header i-1
// (HeaderValidation.hs:308-309 checks exactly that), so every KES signature has to be
// redone in order -- the body, and with it the header hash, changes.  Header 0 gets
// prev0, or GenesisHash (CBOR null, the body shrinks by 33 bytes) when prev0 is null.
// headerHash = Blake2b-256 of the stored header [body, kesSig] (Praos/Header.hs:147-151).
// One wave: lane 0 signs and hashes from an LDS copy of the header that the wave builds
// (byte loops over global memory in one lane cost ~1 ms per block); the leaf keys' a, r, R
// come from k_synth_link_keys.
__global__ void __launch_bounds__(64) k_synth_link(size_t n, const uint8_t* __restrict__ prev0,
                                                   const uint32_t* __restrict__ lkeys,
                                                   const uint32_t* __restrict__ tree, const uint32_t* __restrict__ leaf_of,
                                                   uint8_t* __restrict__ body_bytes, const uint64_t* __restrict__ body_off,
                                                   uint32_t* __restrict__ body_len, uint8_t* __restrict__ kes_sig,
                                                   uint8_t* __restrict__ header_hash, uint32_t stride) {
  __shared__ __attribute__((aligned(16))) uint8_t body_s[640];  // the signed body (8-aligned for SHA-512)
  __shared__ __attribute__((aligned(16))) uint8_t hdr[1152];    // 0x82 | body | 59 01 c0 | kesSig 448 | pad
  __shared__ uint32_t prev_s[8];
  __shared__ uint32_t bl_s;
  const unsigned lane = threadIdx.x;
  bool genesis = prev0 == nullptr;
  if (lane == 0 && !genesis) load_words(prev_s, prev0, 8);
  auto ulen = [](uint32_t ib) -> uint32_t {
    const uint32_t ai = ib & 31u;
    return ai < 24 ? 1u : ai == 24 ? 2u : ai == 25 ? 3u : ai == 26 ? 5u : 9u;
  };
  for (size_t i = 0; i < n; i++) {
    uint8_t* b = body_bytes + body_off[i];
    uint32_t bl = body_len[i];
    for (uint32_t k = lane; k < 640; k += 64) body_s[k] = k < bl && k < stride ? b[k] : 0;
    __syncthreads();
    if (lane == 0) {
      uint32_t q = 1;
      q += ulen(body_s[q]);                       // blockNo
      q += ulen(body_s[q]);                       // slotNo; body_s[q] = 0x58 (bytes(32)) or 0xf6 (null)
      bool ok = true;
      if (genesis) {
        if (body_s[q] == 0x58) {                  // bytes(32) -> null: shift the tail left by 33
          for (uint32_t k = q + 1; k + 33 < bl; k++) body_s[k] = body_s[k + 33];
          body_s[q] = 0xf6;
          bl -= 33;
          for (uint32_t k = bl; k < 640; k++) body_s[k] = 0;
          body_len[i] = bl;
        }
      } else if (body_s[q] != 0x58) {
        ok = false;                               // not produced by k_synth_headers
      } else {
        for (int k = 0; k < 32; k++) body_s[q + 2 + k] = (uint8_t)(prev_s[k / 4] >> (8 * (k % 4)));
      }
      bl_s = ok ? bl : 0xffffffffu;
      if (ok) {
        // KES leaf signature over the new body with the leaf's fixed nonce; the Merkle path
        // of the signature is unchanged
        const uint32_t li = leaf_of[i];
        const uint32_t* T = tree + (size_t)(li / 64u) * 128 * 8;
        const uint32_t* lk = lkeys + 24 * (size_t)li;
        uint32_t pre[16], d[16], h[8], a[8], r[8], S[8];
#pragma unroll
        for (int k = 0; k < 8; k++) {
          pre[k] = lk[16 + k];                    // R
          pre[8 + k] = T[(64 + li % 64u) * 8 + k];  // A (the leaf's public key)
          a[k] = lk[k];
          r[k] = lk[8 + k];
        }
        sha512_stream(d, pre, 64, body_s, bl);
        sc_reduce512(h, d);
        sc_muladd(S, h, a, r);
        uint32_t sig[16];
#pragma unroll
        for (int k = 0; k < 8; k++) { sig[k] = pre[k]; sig[8 + k] = S[k]; }
        store_words(kes_sig + 448 * i, sig, 16);
        hdr[0] = 0x82;
        hdr[1 + bl] = 0x59; hdr[2 + bl] = 0x01; hdr[3 + bl] = 0xc0;
        for (int k = 0; k < 64; k++) hdr[4 + bl + k] = (uint8_t)(sig[k / 4] >> (8 * (k % 4)));
      }
    }
    __syncthreads();
    if (bl_s == 0xffffffffu) return;
    bl = bl_s;
    // header bytes in LDS: body, the Merkle path (unchanged) after the new leaf signature,
    // zero pad; the new body back to global memory
    for (uint32_t k = lane; k < bl; k += 64) hdr[1 + k] = body_s[k];
    for (uint32_t k = 64 + lane; k < 448; k += 64) hdr[4 + bl + k] = kes_sig[448 * i + k];
    for (uint32_t k = 4 + bl + 448 + lane; k < 1152; k += 64) hdr[k] = 0;
    for (uint32_t k = lane; k < ((bl + 7) & ~7u) + 8 && k < stride; k += 64) b[k] = body_s[k];
    __syncthreads();
    if (lane == 0) {
      uint32_t hh[8];
      b2b256_range(hh, hdr, 0, 4 + bl + 448);
      if (header_hash) store_words(header_hash + 32 * i, hh, 8);
#pragma unroll
      for (int k = 0; k < 8; k++) prev_s[k] = hh[k];
    }
    genesis = false;
    __syncthreads();
  }
}

// Corruption model (consensus-testlib Test/Util/Corruption.hs:29-35): increment
// the byte at offset k mod len of one chosen field; the field is drawn from the set
// `fields` (PRAOS_CORRUPT_* bits, praos_hip.h).
__device__ __forceinline__ void bump_be64(uint64_t* v, uint32_t byte) {   // +1 (mod 256) at byte of BE64(v)
  const uint32_t sh = 8u * (7u - (byte & 7u));
  const uint64_t b = ((*v >> sh) + 1u) & 0xffu;
  *v = (*v & ~(0xffull << sh)) | (b << sh);
}
__global__ void k_synth_corrupt(size_t n, uint32_t per10000, uint64_t salt, uint8_t* ocert_sig, uint8_t* kes_sig,
                                uint8_t* vrf_proof, uint8_t* vrf_out, uint8_t* body_bytes, const uint64_t* body_off,
                                const uint32_t* body_len, uint8_t* corrupted, uint8_t* l_proof, int cbor_body,
                                uint32_t fields, uint8_t* cold_vk, uint8_t* hot_vk, uint64_t* ocert_n,
                                uint64_t* ocert_c0) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  // CBOR bodies carry copies of the OCert signature and the VRF cert: a corruption
  // of those fields is applied to the copy as well, so the stored header bytes
  // (praos_hip/chunk.py) hold exactly the corrupted header.
  int32_t at_vrf_out = -1, at_vrf_proof = -1, at_ocert_sig = -1, at_l_proof = -1;
  if (cbor_body) {                         // 1: Praos HeaderBody, 2: TPraos BHBody
    const uint8_t* b = body_bytes + body_off[i];
    auto ulen = [](uint32_t ib) -> int32_t {
      const uint32_t ai = ib & 31u;
      return ai < 24 ? 1 : ai == 24 ? 2 : ai == 25 ? 3 : ai == 26 ? 5 : 9;
    };
    int32_t q = 1;
    q += ulen(b[q]);                       // blockNo
    q += ulen(b[q]);                       // slotNo
    q += (b[q] == 0xf6 ? 1 : 34) + 34 + 34 + 1;   // prevHash (or GenesisHash null), vk, vrfVk, [ of the cert
    at_vrf_out = q + 2;
    q += 66;
    at_vrf_proof = q + 2;
    q += 82;
    if (cbor_body == 2) {                  // [ leader out, leader proof ]
      at_l_proof = q + 1 + 66 + 2;
      q += 1 + 66 + 82;
    }
    q += ulen(b[q]);                       // bodySize
    q += cbor_body == 2 ? 34 + 34 : 34 + 1 + 34;   // bodyHash, ([ of the OCert,) hotVk
    q += ulen(b[q]);                       // n
    q += ulen(b[q]);                       // c0
    at_ocert_sig = q + 2;
  }
  const uint64_t r = mix64(i ^ salt ^ 0xc0ffee);
  const bool c = (r % 10000u) < per10000;
  corrupted[i] = c ? 1 : 0;
  if (!c) return;
  // the (r >> 20) % popcount(fields)-th set bit of fields picks the field
  const uint32_t nf = (uint32_t)__popc(fields & 0x1fu);
  uint32_t pick = (uint32_t)((r >> 20) % (nf ? nf : 1u)), which = 0;
  for (uint32_t f = 0; f < 5; f++)
    if (fields & (1u << f)) {
      if (pick == 0) { which = f; break; }
      pick--;
    }
  const uint32_t k = (uint32_t)(r >> 32);
  switch (which) {
    case 0:
      if (fields != 0x1fu && !cbor_body) {       // the OCert verify's 144 input bytes
        const uint32_t o = k % 144u;
        if (o < 32) cold_vk[32 * i + o] += 1;
        else if (o < 64) hot_vk[32 * i + o - 32] += 1;
        else if (o < 72) bump_be64(ocert_n + i, o - 64);
        else if (o < 80) bump_be64(ocert_c0 + i, o - 72);
        else ocert_sig[64 * i + o - 80] += 1;
        corrupted[i] = 1;
        break;
      }
      ocert_sig[64 * i + k % 64] += 1; corrupted[i] = 1;
      if (at_ocert_sig >= 0) body_bytes[body_off[i] + at_ocert_sig + k % 64] += 1;
      break;
    case 1: kes_sig[448 * i + k % 448] += 1; corrupted[i] = 2; break;
    case 2:
      if (l_proof && (k & 0x10000)) {
        l_proof[80 * i + k % 80] += 1; corrupted[i] = 6;
        if (at_l_proof >= 0) body_bytes[body_off[i] + at_l_proof + k % 80] += 1;
        break;
      }
      vrf_proof[80 * i + k % 80] += 1; corrupted[i] = 3;
      if (at_vrf_proof >= 0) body_bytes[body_off[i] + at_vrf_proof + k % 80] += 1;
      break;
    case 3:
      vrf_out[64 * i + k % 64] += 1; corrupted[i] = 4;
      if (at_vrf_out >= 0) body_bytes[body_off[i] + at_vrf_out + k % 64] += 1;
      break;
    default:
      if (body_len[i] == 0) { ocert_sig[64 * i + k % 64] += 1; corrupted[i] = 1; break; }
      body_bytes[body_off[i] + k % body_len[i]] += 1; corrupted[i] = 5; break;
  }
}

// ---- host launchers (kernels are only launchable from their own module)
void launch_synth_pools(dim3 grid, dim3 block, hipStream_t stream, uint32_t npools, const ge_niels* gbtab, const uint32_t* master, uint32_t* cold_seed, uint32_t* cold_pk, uint32_t* vrf_seed, uint32_t* vrf_pk, uint32_t* kes_seed, uint8_t* pool_hash28, uint8_t* pool_vrf32) {
  hipLaunchKernelGGL(k_synth_pools, grid, block, 0, stream, npools, gbtab, master, cold_seed, cold_pk, vrf_seed, vrf_pk, kes_seed, pool_hash28, pool_vrf32);
}

void launch_synth_kes_leaves(dim3 grid, dim3 block, hipStream_t stream, uint32_t npools, const ge_niels* gbtab, const uint32_t* kes_seed, uint32_t* leaf_seed, uint32_t* tree) {
  hipLaunchKernelGGL(k_synth_kes_leaves, grid, block, 0, stream, npools, gbtab, kes_seed, leaf_seed, tree);
}

void launch_synth_kes_tree(dim3 grid, dim3 block, hipStream_t stream, uint32_t npools, uint32_t* tree) {
  hipLaunchKernelGGL(k_synth_kes_tree, grid, block, 0, stream, npools, tree);
}


void launch_synth_headers(dim3 grid, dim3 block, hipStream_t stream, size_t n, const ge_niels* gbtab, uint32_t npools,
                          uint32_t nkes, uint64_t first_slot, uint64_t slot_stride, uint64_t slots_per_kes_period,
                          uint32_t blen, uint64_t salt, const uint32_t* eta0, int eta0_neutral,
                          const uint32_t* cold_seed, const uint32_t* cold_pk, const uint32_t* vrf_seed,
                          const uint32_t* vrf_pk, const uint32_t* leaf_seed, const uint32_t* tree,
                          uint8_t* msg_scratch, uint64_t* slot, uint8_t* cold_vk, uint8_t* vrf_vk, uint8_t* vrf_out,
                          uint8_t* vrf_proof, uint8_t* hot_vk, uint64_t* ocert_n, uint64_t* ocert_c0,
                          uint8_t* ocert_sig, uint8_t* kes_sig, uint64_t* body_off, uint32_t* body_len,
                          uint8_t* body_bytes, int tpraos, uint8_t* l_out, uint8_t* l_proof,
                          const uint8_t* body_hash_in, const uint64_t* sched_slot, const uint32_t* sched_pool,
                          uint64_t block_no0, uint32_t* leaf_of) {
  hipLaunchKernelGGL(k_synth_headers, grid, block, 0, stream, n, gbtab, npools, nkes, first_slot, slot_stride,
                     slots_per_kes_period, blen, salt, eta0, eta0_neutral, cold_seed, cold_pk, vrf_seed, vrf_pk,
                     leaf_seed, tree, msg_scratch, slot, cold_vk, vrf_vk, vrf_out, vrf_proof, hot_vk, ocert_n,
                     ocert_c0, ocert_sig, kes_sig, body_off, body_len, body_bytes, tpraos, l_out, l_proof,
                     body_hash_in, sched_slot, sched_pool, block_no0, leaf_of);
}
void launch_synth_link(hipStream_t stream, size_t n, const ge_niels* gbtab, const uint8_t* prev0,
                       const uint32_t* leaf_seed, uint32_t nleaves, uint32_t* lkeys, const uint32_t* tree,
                       const uint32_t* leaf_of, uint8_t* body_bytes, const uint64_t* body_off, uint32_t* body_len,
                       uint8_t* kes_sig, uint8_t* header_hash, uint32_t stride) {
  hipLaunchKernelGGL(k_synth_link_keys, dim3((nleaves + NT - 1) / NT), dim3(NT), 0, stream, nleaves, gbtab, leaf_seed,
                     lkeys);
  hipLaunchKernelGGL(k_synth_link, dim3(1), dim3(64), 0, stream, n, prev0, lkeys, tree, leaf_of, body_bytes, body_off,
                     body_len, kes_sig, header_hash, stride);
}
void launch_synth_vrf_scalar(dim3 grid, dim3 block, hipStream_t stream, uint32_t npools, const uint32_t* vrf_seed,
                             uint32_t* vrf_x) {
  hipLaunchKernelGGL(k_synth_vrf_scalar, grid, block, 0, stream, npools, vrf_seed, vrf_x);
}
void launch_synth_leader_search(dim3 grid, dim3 block, hipStream_t stream, uint64_t first_slot, uint64_t nslots,
                                uint32_t p0, uint32_t pn, const uint32_t* vrf_x, const uint32_t* vrf_pk,
                                const uint32_t* pool_thr, const uint32_t* eta0, int eta0_neutral, int f_is_one,
                                int tpraos, int32_t* leader) {
  hipLaunchKernelGGL(k_synth_leader_search, grid, block, 0, stream, first_slot, nslots, p0, pn, vrf_x, vrf_pk,
                     pool_thr, eta0, eta0_neutral, f_is_one, tpraos, leader);
}
void launch_synth_corrupt(dim3 grid, dim3 block, hipStream_t stream, size_t n, uint32_t per10000, uint64_t salt,
                          uint8_t* ocert_sig, uint8_t* kes_sig, uint8_t* vrf_proof, uint8_t* vrf_out,
                          uint8_t* body_bytes, const uint64_t* body_off, const uint32_t* body_len,
                          uint8_t* corrupted, uint8_t* l_proof, int cbor_body, uint32_t fields, uint8_t* cold_vk,
                          uint8_t* hot_vk, uint64_t* ocert_n, uint64_t* ocert_c0) {
  hipLaunchKernelGGL(k_synth_corrupt, grid, block, 0, stream, n, per10000, salt, ocert_sig, kes_sig, vrf_proof,
                     vrf_out, body_bytes, body_off, body_len, corrupted, l_proof, cbor_body, fields, cold_vk, hot_vk,
                     ocert_n, ocert_c0);
}
