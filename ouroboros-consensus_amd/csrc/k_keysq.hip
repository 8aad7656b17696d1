// k_keysq.hip -- the key-cache precompute (k_keys.hip) with four lanes per key, for batches
// whose precompute is a short list of long chains on the cached verifies' critical path (a
// 54k-header shard of an epoch: 3000 VRF keys = 47 waves of one 128-doubling chain each).
//
// The four lanes of a quad hold the same point and decode the same key (the same instruction
// stream: no cost in latency).  The chunk-base chain (key_chunk_bases: Q_{k+1} = 2^16 Q_k)
// splits each doubling over the quad instead of interleaving it in one lane:
//   squarings   lane 0: X^2, lane 1: Y^2, lane 2: Z^2, lane 3: (X+Y)^2     (one fe_sq stream)
//   -> the four squares to every lane of the quad (DPP quad_perm broadcasts)
//   p1p1        X' = AA - (YY + XX), Y' = YY + XX, Z' = YY - XX, T' = 2 ZZ - Z'  (every lane)
//   products    lane 0: X'T', lane 1: Y'Z', lane 2: Z'T', lane 3: X'Y'     (one fe_mul stream)
//   -> the four products to every lane: (X : Y : Z) for the next doubling, T at a chunk base
// so one doubling issues one squaring and one multiply instead of four squarings and three
// multiplies (ge_p2_dbl + ge_p1p1_to_p2), plus 64 DPP moves and the selects.  Lane q writes
// coordinate q of each chunk base.  Same formulas, same field arithmetic, same tables as
// k_key_precompute (the A/B and the cached-vs-uncached verdict tests compare them).
#include "k_keys.hpp"

namespace {

// value of lane L of this lane's quad (v_mov_b32 with DPP quad_perm [L, L, L, L])
template <int L>
FE_INLINE uint32_t quad_lane(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, L * 0x55, 0xf, 0xf, false);
}
template <int L>
FE_INLINE void fe_quad(fe& r, const fe& a) {
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = quad_lane<L>(a.v[i]);
}
// lane masks of the quad position (all ones where q == i), made once: a select written as
// nested conditionals compiled to divergent branches, four exec-masked paths per limb
struct QMask { uint32_t m[4]; };
FE_INLINE QMask quad_masks(uint32_t q) {
  QMask k;
#pragma unroll
  for (int i = 0; i < 4; i++) k.m[i] = 0u - (uint32_t)(q == (uint32_t)i);
  return k;
}
FE_INLINE void fe_sel4(fe& r, const QMask& k, const fe& a0, const fe& a1, const fe& a2, const fe& a3) {
#pragma unroll
  for (int i = 0; i < 8; i++)
    r.v[i] = (a0.v[i] & k.m[0]) | (a1.v[i] & k.m[1]) | (a2.v[i] & k.m[2]) | (a3.v[i] & k.m[3]);
}

// (X : Y : Z) <- 2 (X : Y : Z) as p2; with T: the p3 coordinate T of the result too
FE_INLINE void quad_dbl(fe& X, fe& Y, fe& Z, fe* T, const QMask& q) {
  fe s, xy;
  fe_add(xy, X, Y);
  fe_sel4(s, q, X, Y, Z, xy);
  fe_sq(s, s);
  fe XX, YY, ZZ, AA;
  fe_quad<0>(XX, s);
  fe_quad<1>(YY, s);
  fe_quad<2>(ZZ, s);
  fe_quad<3>(AA, s);
  fe Xp, Yp, Zp, Tp;
  fe_add(Tp, ZZ, ZZ);
  fe_add(Yp, YY, XX);
  fe_sub(Zp, YY, XX);
  fe_sub(Xp, AA, Yp);
  fe_sub(Tp, Tp, Zp);
  fe a, b;
  fe_sel4(a, q, Xp, Yp, Zp, Xp);
  fe_sel4(b, q, Tp, Zp, Tp, Yp);
  fe_mul(a, a, b);
  fe_quad<0>(X, a);
  fe_quad<1>(Y, a);
  fe_quad<2>(Z, a);
  if (T) fe_quad<3>(*T, a);
}

// key_chunk_bases over a quad: Q_0 = P, Q_{k+1} = 2^16 Q_k, lane q stores coordinate q of Q_k
// (a ge_p3 in the 128 bytes of ktab[8k], as pass 2 reads it)
FE_INLINE void quad_chunk_bases(ge_cached* __restrict__ ktab, const ge_p3& P, int nchunks, uint32_t q, bool write) {
  const QMask m = quad_masks(q);
  fe X = P.X, Y = P.Y, Z = P.Z, T = P.T;
#pragma clang loop unroll(disable)
  for (int k = 0; k < nchunks; k++) {
    if (write) {
      fe w;
      fe_sel4(w, m, X, Y, Z, T);
      store_words((uint8_t*)(ktab + 8 * k) + 32 * q, w.v, 8);
    }
    if (k + 1 < nchunks) {
#pragma clang loop unroll(disable)
      for (int d = 0; d < 15; d++) quad_dbl(X, Y, Z, nullptr, m);
      quad_dbl(X, Y, Z, &T, m);
    }
  }
}

}  // namespace

__global__ void __launch_bounds__(64) k_key_precomputeq(int kind, const uint32_t* __restrict__ counters,
                                                         uint32_t max_entries, const uint32_t* __restrict__ entry_rep,
                                                         const uint8_t* __restrict__ keys, ge_cached* __restrict__ ktab,
                                                         uint32_t* __restrict__ kinfo, int wave_prio,
                                                         const uint32_t* __restrict__ base) {
  if (wave_prio) __builtin_amdgcn_s_setprio(3);
  const uint32_t ne = min(counters[0], max_entries);
  const uint32_t q = threadIdx.x & 3u;
  const uint32_t e0 = base ? *base : 0u;
  // quad-uniform loop: the four lanes of a key leave it together (the DPP moves read the quad)
  for (uint32_t e = e0 + ((blockIdx.x * blockDim.x + threadIdx.x) >> 2); e < ne; e += (gridDim.x * blockDim.x) >> 2) {
    ge_p3 P;
    key_decode_entry(kind, e, entry_rep, keys, kinfo, P, q == 0);
    quad_chunk_bases(ktab + (size_t)e * KT_STRIDE, P, key_chunks(kind), q, true);
  }
}

void launch_key_precomputeq(int kind, hipStream_t stream, const uint32_t* counters, uint32_t max_entries,
                            const uint32_t* entry_rep, const uint8_t* keys, ge_cached* ktab, uint32_t* kinfo,
                            int wave_prio, const uint32_t* base, uint32_t span) {
  hipLaunchKernelGGL(k_key_precomputeq, dim3((unsigned)(((size_t)span * 4 + 63) / 64)), dim3(64), 0, stream, kind,
                     counters, max_entries, entry_rep, keys, ktab, kinfo, wave_prio, base);
}
