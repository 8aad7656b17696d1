// k_keys.hpp -- the key-cache precompute of one entry (k_keys.hip), shared with its ILP-4
// build for small batches (k_keys4.hip).
#pragma once
#include "kcommon.hpp"

// kind 0 (cold key, Ed25519): flag = ge_is_canonical && !ge_has_small_order &&
//        decodes; tables of -A (ge25519_frombytes_negate_vartime), 16 chunks.
// kind 1 (VRF key): flag = !ge_has_small_order && decodes (vrf_validate_key);
//        kinfo[1..8] = canonical encoding of Y; tables of -Y, 9 chunks.
// chunk tables per key: Ed25519 scalars are < 2^256 (16 chunks); the VRF challenge c
// is < 2^128 (8 chunks + the top digit's table)
__device__ __forceinline__ int key_chunks(int kind) { return kind == 0 ? KT_CHUNKS : 9; }

// decode + checks of entry e's key: P (the point the tables expand), kinfo[9e ..] (when write)
FE_INLINE void key_decode_entry(int kind, uint32_t e, const uint32_t* __restrict__ entry_rep,
                                const uint8_t* __restrict__ keys, uint32_t* __restrict__ kinfo, ge_p3& P, bool write) {
  uint32_t pk[8];
  load_words(pk, keys + 32 * (size_t)entry_rep[e], 8);
  bool ok;
  uint32_t* info = kinfo + 9 * (size_t)e;
  if (kind == 0) {
    ok = ge_is_canonical(pk) && !ge_has_small_order(pk);
    ok = ge_frombytes(P, pk, /*negate=*/true) && ok;
  } else {
    ok = !ge_has_small_order(pk);
    ge_p3 Y;
    ok = ge_frombytes(Y, pk, false) && ok;
    uint32_t ys[8];
    ge_enc_affine(ys, Y);
    if (write) {
#pragma unroll
      for (int q = 0; q < 8; q++) info[1 + q] = ys[q];
    }
    P = Y;
    fe_neg(P.X, Y.X);
    fe_neg(P.T, Y.T);
  }
  if (write) info[0] = ok ? 1u : 0u;
}

FE_INLINE void key_precompute_entry(int kind, uint32_t e, const uint32_t* __restrict__ entry_rep,
                                    const uint8_t* __restrict__ keys, ge_cached* __restrict__ ktab,
                                    uint32_t* __restrict__ kinfo) {
  ge_p3 P;
  key_decode_entry(kind, e, entry_rep, keys, kinfo, P, true);
  key_chunk_bases(ktab + (size_t)e * KT_STRIDE, P, key_chunks(kind));
}
