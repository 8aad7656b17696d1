// k_ed25519.hpp -- the OCert and Sum6KES per-header inputs and checks around the Ed25519
// verify, shared by k_ed25519.hip and its ILP-4 build for small batches (k_miss4.hip).
#pragma once
#include "kcommon.hpp"

// ------------------------------------------------------------------ OCert + KES period checks
// bits |= KES_BEFORE_START / KES_AFTER_END / OCERT_SIG.  If ok_out != null the
// kernel is the plain praos_verify_ocert batch (ok_out[i] = 1 when valid).
// Items: i in [0, n), or list[0 .. *count) when list != null (key-cache
// partition, k_keys.hip): k_ocert takes the misses, k_ocert_ck the hits.
struct OcertIn {
  const uint8_t* __restrict__ cold_vk;
  const uint8_t* __restrict__ hot_vk;
  const uint64_t* __restrict__ ocert_n;
  const uint64_t* __restrict__ ocert_c0;
  const uint8_t* __restrict__ sig;
  const uint64_t* __restrict__ slot;
  uint64_t slots_per_kes_period, max_kes_evo;
  uint16_t* __restrict__ bits;
  uint8_t* __restrict__ ok_out;
  ge_cached* __restrict__ tabs;          // per-lane tables (LT_ED entries per item)
  int wave_prio;                         // cached verifies: waves at s_setprio <wave_prio> (0 = off)
};

__device__ __forceinline__ void ocert_store(const OcertIn& a, size_t i, bool ok) {
  if (a.ok_out) {
    a.ok_out[i] = ok ? 1 : 0;
    return;
  }
  uint16_t b = ok ? 0 : PRAOS_BIT_OCERT_SIG;
  const uint64_t c0 = a.ocert_c0[i];
  const uint64_t kp = a.slot[i] / a.slots_per_kes_period;     // Praos.hs:596-599
  if (!(c0 <= kp)) b |= PRAOS_BIT_KES_BEFORE_START;            // Praos.hs:567
  if (!(kp < c0 + a.max_kes_evo)) b |= PRAOS_BIT_KES_AFTER_END; // Praos.hs:568
  a.bits[i] = b;
}

__device__ __forceinline__ void ocert_load(const OcertIn& a, size_t i, uint32_t sg[16], uint32_t hram[16],
                                           uint32_t pk[8]) {
  uint32_t hot[8];
  load_words(pk, a.cold_vk + 32 * i, 8);
  load_words(hot, a.hot_vk + 32 * i, 8);
  load_words(sg, a.sig + 64 * i, 16);
  ocert_hram(hram, sg, pk, hot, a.ocert_n[i], a.ocert_c0[i]);
}

// ------------------------------------------------------------------ KES
// Header mode: t = kp >= c0 ? kp - c0 : 0 (Praos.hs:570), result to bits.
// Plain mode (result != null): t = period[i], result 0 ok / 1 Reject / 2 leaf.
// Items: i in [0, n), or list[0 .. *count) (leaf-key cache partition): k_kes takes
// the misses, k_kes_ck the hits.
struct KesIn {
  const uint8_t* __restrict__ hot_vk;
  const uint8_t* __restrict__ kes_sig;
  const uint64_t* __restrict__ body_off;
  const uint32_t* __restrict__ body_len;
  const uint8_t* __restrict__ body;
  size_t body_bytes_len;
  const uint64_t* __restrict__ slot;
  const uint64_t* __restrict__ ocert_c0;
  uint64_t slots_per_kes_period;
  const uint32_t* __restrict__ period;
  uint16_t* __restrict__ bits;
  uint8_t* __restrict__ result;
  ge_cached* __restrict__ tabs;
  int wave_prio;                         // cached verifies: waves at s_setprio <wave_prio> (0 = off)
};

__device__ __forceinline__ uint64_t kes_t(const KesIn& a, size_t i) {
  if (a.period) return a.period[i];
  const uint64_t kp = a.slot[i] / a.slots_per_kes_period, c0 = a.ocert_c0[i];
  return kp >= c0 ? kp - c0 : 0;
}

// Merkle walk + SHA-512(R || leaf || M); returns merkle_ok, in_range, the leaf
// key and the signature words.
__device__ __forceinline__ void kes_prepare(const KesIn& a, size_t i, uint32_t sg[16], uint32_t leaf[8],
                                            uint32_t hram[16], bool& merkle_ok, bool& in_range) {
  const uint8_t* sig = a.kes_sig + 448 * i;
  uint32_t vk[8];
  load_words(vk, a.hot_vk + 32 * i, 8);
  merkle_ok = kes_merkle(leaf, vk, kes_t(a, i), sig);
  load_words(sg, sig, 16);
  uint64_t off = a.body_off[i];
  uint32_t len = a.body_len[i];
  in_range = (off & 7) == 0 && off <= a.body_bytes_len && len <= a.body_bytes_len - off;
  if (!in_range) { off = 0; len = 0; }
  uint32_t pre[16];
#pragma unroll
  for (int k = 0; k < 8; k++) { pre[k] = sg[k]; pre[8 + k] = leaf[k]; }
  sha512_stream(hram, pre, 64, a.body + off, len);
}

// Merkle walk shared per leaf-key cache entry (KES path dedup): the walk reads hot_vk, t and
// the six vk pairs sig[64 .. 448); an item whose bytes equal its entry representative's gets
// the representative's verdict (k_kes_merkle_reps) and selects its leaf as the walk would.
__device__ __forceinline__ bool kes_path_same(const KesIn& a, size_t i, size_t r, uint64_t ti) {
  if (i == r) return true;
  if (kes_t(a, r) != ti) return false;
  const uint4* p = (const uint4*)(a.kes_sig + 448 * i + 64);
  const uint4* q = (const uint4*)(a.kes_sig + 448 * r + 64);
  bool same = true;
#pragma unroll
  for (int k = 0; k < 24; k++) {
    const uint4 x = p[k], y = q[k];
    same &= x.x == y.x && x.y == y.y && x.z == y.z && x.w == y.w;
  }
  const uint4* hp = (const uint4*)(a.hot_vk + 32 * i);
  const uint4* hq = (const uint4*)(a.hot_vk + 32 * r);
#pragma unroll
  for (int k = 0; k < 2; k++) {
    const uint4 x = hp[k], y = hq[k];
    same &= x.x == y.x && x.y == y.y && x.z == y.z && x.w == y.w;
  }
  return same;
}

// the depth-1 entry kes_merkle ends on (as k_kes_leafkeys)
__device__ __forceinline__ void kes_leaf_select(uint32_t leaf[8], uint64_t t, const uint8_t* __restrict__ sig) {
#pragma unroll
  for (int d = 6; d >= 2; d--) {
    const uint64_t T = 1ull << (d - 1);
    t = t >= T ? t - T : t;
  }
  load_words(leaf, sig + 64 + (t >= 1 ? 32 : 0), 8);
}

// kes_prepare with the path dedup: rep / rep_ok = the item's cache entry's representative and
// its walk verdict (rep_ok null: every item walks)
__device__ __forceinline__ void kes_prepare_dd(const KesIn& a, size_t i, size_t rep, const uint8_t* rep_ok,
                                               uint32_t sg[16], uint32_t leaf[8], uint32_t hram[16],
                                               bool& merkle_ok, bool& in_range) {
  const uint8_t* sig = a.kes_sig + 448 * i;
  const uint64_t t = kes_t(a, i);
  if (rep_ok && kes_path_same(a, i, rep, t)) {
    merkle_ok = *rep_ok != 0;
    kes_leaf_select(leaf, t, sig);
  } else {
    uint32_t vk[8];
    load_words(vk, a.hot_vk + 32 * i, 8);
    merkle_ok = kes_merkle(leaf, vk, t, sig);
  }
  load_words(sg, sig, 16);
  uint64_t off = a.body_off[i];
  uint32_t len = a.body_len[i];
  in_range = (off & 7) == 0 && off <= a.body_bytes_len && len <= a.body_bytes_len - off;
  if (!in_range) { off = 0; len = 0; }
  uint32_t pre[16];
#pragma unroll
  for (int k = 0; k < 8; k++) { pre[k] = sg[k]; pre[8 + k] = leaf[k]; }
  sha512_stream(hram, pre, 64, a.body + off, len);
}

__device__ __forceinline__ void kes_store(const KesIn& a, size_t i, bool merkle_ok, bool leaf_ok, bool in_range) {
  if (a.result) {
    a.result[i] = !in_range ? 3 : (!merkle_ok ? 1 : (leaf_ok ? 0 : 2));
    return;
  }
  uint16_t b = 0;
  if (!merkle_ok) b |= PRAOS_BIT_KES_MERKLE;
  else if (!leaf_ok) b |= PRAOS_BIT_KES_LEAF;
  if (!in_range) b |= PRAOS_BIT_INPUT;
  a.bits[i] = b;
}
