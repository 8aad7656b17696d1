// scalarmult.hpp -- per-lane multi-scalar multiplication for gfx950.
//
// Every scalar multiplication on the Praos path is one Straus/Horner chain
// over 4-bit windows (4 doublings between windows, shared by all terms):
//   * per-lane variable bases P, Q: signed radix-16 digits in [-8, 7], 8-entry
//     cached tables {1..8}P in private memory (indexed by a per-lane digit);
//   * the fixed base B (and B' = 2^128 B): signed radix-256 digits in
//     [-128, 127] with 128-entry affine-niels tables {1..128}B, {1..128}B'
//     staged in LDS per block (k_init_btab builds them once per context).
//     A fixed-base digit is added every other window (one byte = 2 windows),
//     which halves the fixed-base additions of a radix-16 schedule.
//
// Digits are produced on the fly from the scalar kept in registers, recoded
// once as w = s + 0x88..88 (radix 16) or s + 0x80..80 (radix 256): the
// signed digit j is then nibble/byte j of w minus 8/128 (exact for s < 2^253,
// which holds for every scalar here: values reduced mod L, or < 2^128).  The
// register is shifted left by one window per step, so no digit array exists.
//
// Window schedules are uniform across the wave (no divergence): digits may be
// zero (identity added), exactly as in a constant-time schedule.  Results are
// exact group elements, so verdicts depend only on the encodings, as in
// libsodium (which uses a different, sliding-window schedule).
#pragma once
#include "ge25519.hpp"

#define BTAB_N 128                     // entries per fixed-base table
#define BTAB_WORDS (BTAB_N * 24)       // u32 words per table (niels = 3 fe)

// w = s + 0x8888...88 (radix-16 signed recoding); requires s < 2^253
FE_INLINE void sc_recode16(uint32_t w[8], const uint32_t s[8]) {
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) w[i] = addc(s[i], 0x88888888u, c, &c);
}
// w = s + 0x8080...80 (radix-256 signed recoding); requires s < 2^253
FE_INLINE void sc_recode256(uint32_t w[8], const uint32_t s[8]) {
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) w[i] = addc(s[i], 0x80808080u, c, &c);
}

template <int NW, int SH>
FE_INLINE void shl_small(uint32_t w[NW]) {          // w <<= SH, 0 < SH < 32
#pragma unroll
  for (int i = NW - 1; i > 0; i--) w[i] = __builtin_amdgcn_alignbit(w[i], w[i - 1], 32 - SH);
  w[0] <<= SH;
}
template <int NW, int BITS>
FE_INLINE void shl_const(uint32_t w[NW]) {          // w <<= BITS (compile-time)
  constexpr int WS = BITS / 32, B = BITS % 32;
  if constexpr (WS > 0) {
#pragma unroll
    for (int i = NW - 1; i >= 0; i--) w[i] = i >= WS ? w[i - WS] : 0u;
  }
  if constexpr (B > 0) shl_small<NW, B>(w);
}

// table[k] = (k+1) * P in cached form
FE_INLINE void build_cached_table(ge_cached* __restrict__ tab, const ge_p3& P) {
  ge_p3 acc, P2;
  ge_p1p1 t;
  ge_p3_to_cached(tab[0], P);
  ge_p3_dbl_to_p3(P2, P);
  ge_p3_to_cached(tab[1], P2);
  acc = P2;
#pragma clang loop unroll(disable)
  for (int k = 2; k < 8; k++) {
    ge_add(t, acc, tab[0]);
    ge_p1p1_to_p3(acc, t);
    ge_p3_to_cached(tab[k], acc);
  }
}

// Table selects are branch-free: the gather of entry max(|d|, 1) is issued
// unconditionally and the identity / negation applied after it arrives.  (An
// `if (d == 0)` around the load compiles to an exec-masked branch whose join waits
// for the load at once; straight-line code lets the caller's independent work --
// the p1p1 -> p3 conversion of the accumulator -- run under the load's latency.)
FE_INLINE void cached_fix(ge_cached& c, bool zero, bool neg) {
#pragma unroll
  for (int i = 0; i < 8; i++) {
    c.YpX.v[i] = zero ? (i == 0 ? 1u : 0u) : c.YpX.v[i];
    c.YmX.v[i] = zero ? (i == 0 ? 1u : 0u) : c.YmX.v[i];
    c.Z.v[i] = zero ? (i == 0 ? 1u : 0u) : c.Z.v[i];
    c.T2d.v[i] = zero ? 0u : c.T2d.v[i];
  }
  ge_cached_cneg(c, neg);
}
FE_INLINE void niels_fix(ge_niels& c, bool zero, bool neg) {
#pragma unroll
  for (int i = 0; i < 8; i++) {
    c.ypx.v[i] = zero ? (i == 0 ? 1u : 0u) : c.ypx.v[i];
    c.ymx.v[i] = zero ? (i == 0 ? 1u : 0u) : c.ymx.v[i];
    c.xy2d.v[i] = zero ? 0u : c.xy2d.v[i];
  }
  ge_niels_cneg(c, neg);
}
FE_INLINE void select_cached(ge_cached& c, const ge_cached tab[8], int d) {
  const int a = d < 0 ? -d : d;
  c = tab[a == 0 ? 0 : a - 1];
  cached_fix(c, a == 0, d < 0);
}
FE_INLINE void select_niels(ge_niels& c, const ge_niels* __restrict__ tab, int d) {
  const int a = d < 0 ? -d : d;
  c = tab[a == 0 ? 0 : a - 1];
  niels_fix(c, a == 0, d < 0);
}

// x (p1p1) <- 4 doublings of acc (p2); the last one is left unconverted
FE_INLINE void dbl4_p1p1(ge_p1p1& x, const ge_p2& acc) {
  ge_p2 q = acc;
  ge_p2_dbl(x, q); ge_p1p1_to_p2(q, x);
  ge_p2_dbl(x, q); ge_p1p1_to_p2(q, x);
  ge_p2_dbl(x, q); ge_p1p1_to_p2(q, x);
  ge_p2_dbl(x, q);
}

FE_INLINE void ge_p1p1_identity(ge_p1p1& x) { fe_set(x.X, 0); fe_set(x.Y, 1); fe_set(x.Z, 1); fe_set(x.T, 1); }

// out = sum over terms, as p1p1 (caller converts to p2 or p3):
//   [p] P  with p's radix-16 recoding pw, digits j < NP      (tp: table of P)
//   [q] Q  with q's radix-16 recoding qw, digits j < NQ      (tq: table of Q)
//   [b] B  with b's radix-256 recoding fw:
//          NB = 32:             all 32 bytes on B            (btab[0..128))
//          NB = 16 and TWO_B:   bytes 0..15 on B, bytes 16..31 on B' = 2^128 B
//                               (btab[128..256)), i.e. a 128-window-bit chain
// over nibble windows j = NWIN-1 .. 0 (fixed-base bytes k at windows 2k).
template <int NWIN, int NP, int NQ, int NB, bool TWO_B>
FE_INLINE void straus(ge_p1p1& out, const ge_cached* tp, uint32_t pw[8], const ge_cached* tq, uint32_t qw[8],
                      const ge_niels* __restrict__ btab, uint32_t fw[8]) {
  static_assert(NWIN >= 1 && NWIN <= 64 && NP <= NWIN && NQ <= NWIN, "window counts");
  static_assert(NB == 0 || (NB == 32 && !TWO_B) || (NB == 16 && TWO_B), "fixed-base layout");
  static_assert(NB == 0 || 2 * (NB - 1) <= NWIN - 1, "fixed-base bytes beyond the chain");
  static_assert(NB == 0 || NWIN - 1 <= 2 * NB, "chain starts above the top fixed-base byte");
  // align nibble NWIN-1 to the top of pw / qw
  if constexpr (NP > 0) shl_const<8, 4 * (64 - NWIN)>(pw);
  if constexpr (NQ > 0) shl_const<8, 4 * (64 - NWIN)>(qw);
  ge_p2 acc;
  ge_p1p1 x;
  ge_p3 a3;
#pragma clang loop unroll(disable)
  for (int j = NWIN - 1; j >= 0; j--) {
    if (j == NWIN - 1) ge_p1p1_identity(x);
    else dbl4_p1p1(x, acc);
    if constexpr (NP > 0) {
      if (j < NP) {
        ge_cached c;
        select_cached(c, tp, (int)(pw[7] >> 28) - 8);
        ge_p1p1_to_p3(a3, x);
        ge_add(x, a3, c);
      }
      shl_small<8, 4>(pw);
    }
    if constexpr (NQ > 0) {
      if (j < NQ) {
        ge_cached c;
        select_cached(c, tq, (int)(qw[7] >> 28) - 8);
        ge_p1p1_to_p3(a3, x);
        ge_add(x, a3, c);
      }
      shl_small<8, 4>(qw);
    }
    if constexpr (NB > 0) {
      if ((j & 1) == 0 && (j >> 1) < NB) {
        ge_niels nb;
        if constexpr (TWO_B) {
          select_niels(nb, btab, (int)(fw[3] >> 24) - 128);
          ge_p1p1_to_p3(a3, x);
          ge_madd(x, a3, nb);
          select_niels(nb, btab + BTAB_N, (int)(fw[7] >> 24) - 128);
          ge_p1p1_to_p3(a3, x);
          ge_madd(x, a3, nb);
          shl_small<4, 8>(fw);
          shl_small<4, 8>(fw + 4);
        } else {
          select_niels(nb, btab, (int)(fw[7] >> 24) - 128);
          ge_p1p1_to_p3(a3, x);
          ge_madd(x, a3, nb);
          shl_small<8, 8>(fw);
        }
      }
    }
    if (j > 0) ge_p1p1_to_p2(acc, x);
  }
  out = x;
}

// ---------------------------------------------------------------- rolled chains
// The same schedules with every group operation emitted ONCE per chain: the 4
// doublings of a window are a runtime loop, and so are the per-lane-table
// terms and the fixed-base terms of a window (their digits and tables picked
// by the uniform loop index).  A fully unrolled window of the V chain is ~60 KB
// of code -- the size of the instruction cache two CUs share -- and the
// OCert / KES / VRF kernels run concurrently, so waves stalled on instruction
// fetch (SQ_WAIT_INST_ANY ~19 % of k_vrf_ck's wave cycles).  Rolled, a chain's
// working set is one doubling + one addition + one mixed addition (~25 KB).
// Operation counts and results are identical to straus / straus_chunked.
#ifndef PRAOS_ROLLED
#define PRAOS_ROLLED 1
#endif

// x <- 16 x (4 doublings; p1p1 in and out)
FE_INLINE void dbl4_rolled(ge_p1p1& x) {
#pragma clang loop unroll(disable)
  for (int k = 0; k < 4; k++) {
    ge_p2 q;
    ge_p1p1_to_p2(q, x);
    ge_p2_dbl(x, q);
  }
}
// x += signed-digit multiple from a table: the entry's gather is issued first and
// the accumulator's p1p1 -> p3 conversion (independent of it) runs under its latency
FE_INLINE void add_cached_sel(ge_p1p1& x, const ge_cached* __restrict__ tab, int d) {
  const int a = d < 0 ? -d : d;
  ge_cached c = tab[a == 0 ? 0 : a - 1];
  ge_p3 a3;
  ge_p1p1_to_p3(a3, x);
  cached_fix(c, a == 0, d < 0);
  ge_add(x, a3, c);
}
FE_INLINE void add_niels_sel(ge_p1p1& x, const ge_niels* __restrict__ tab, int d) {
  const int a = d < 0 ? -d : d;
  ge_niels c = tab[a == 0 ? 0 : a - 1];
  ge_p3 a3;
  ge_p1p1_to_p3(a3, x);
  niels_fix(c, a == 0, d < 0);
  ge_madd(x, a3, c);
}

template <int NWIN, int NP, int NQ, int NB, bool TWO_B>
FE_INLINE void straus_rolled(ge_p1p1& out, const ge_cached* tp, uint32_t pw[8], const ge_cached* tq,
                             uint32_t qw[8], const ge_niels* __restrict__ btab, uint32_t fw[8]) {
  static_assert(NWIN >= 1 && NWIN <= 64 && NP <= NWIN && NQ <= NP, "window counts (terms ordered NQ <= NP)");
  static_assert(NB == 0 || (NB == 32 && !TWO_B) || (NB == 16 && TWO_B), "fixed-base layout");
  static_assert(NB == 0 || 2 * (NB - 1) <= NWIN - 1, "fixed-base bytes beyond the chain");
  static_assert(NB == 0 || NWIN - 1 <= 2 * NB, "chain starts above the top fixed-base byte");
  if constexpr (NP > 0) shl_const<8, 4 * (64 - NWIN)>(pw);
  if constexpr (NQ > 0) shl_const<8, 4 * (64 - NWIN)>(qw);
  ge_p1p1 x;
  ge_p1p1_identity(x);
#pragma clang loop unroll(disable)
  for (int j = NWIN - 1; j >= 0; j--) {
    if (j != NWIN - 1) dbl4_rolled(x);
    if constexpr (NP > 0) {
      const int nt = (NQ > 0 && j < NQ) ? 2 : (j < NP ? 1 : 0);
#pragma clang loop unroll(disable)
      for (int t = 0; t < nt; t++) {
        uint32_t top = pw[7];
        if constexpr (NQ > 0) top = t == 0 ? pw[7] : qw[7];
        add_cached_sel(x, (NQ > 0 && t != 0) ? tq : tp, (int)(top >> 28) - 8);
      }
      shl_small<8, 4>(pw);
      if constexpr (NQ > 0) shl_small<8, 4>(qw);
    }
    if constexpr (NB > 0) {
      if ((j & 1) == 0 && (j >> 1) < NB) {
        constexpr int NT2 = TWO_B ? 2 : 1;
#pragma clang loop unroll(disable)
        for (int t = 0; t < NT2; t++) {
          const uint32_t top = TWO_B ? (t == 0 ? fw[3] : fw[7]) : fw[7];
          add_niels_sel(x, btab + BTAB_N * t, (int)(top >> 24) - 128);
        }
        if constexpr (TWO_B) {
          shl_small<4, 8>(fw);
          shl_small<4, 8>(fw + 4);
        } else {
          shl_small<8, 8>(fw);
        }
      }
    }
  }
  out = x;
}

// R = [s]B (fixed base only), s < 2^253 (reduce mod L first)
FE_INLINE void ge_scalarmult_base(ge_p3& R, const uint32_t s[8], const ge_niels* __restrict__ btab) {
  uint32_t fw[8];
  sc_recode256(fw, s);
  ge_p1p1 x;
  straus<31, 0, 0, 16, true>(x, nullptr, nullptr, nullptr, nullptr, btab, fw);
  ge_p1p1_to_p3(R, x);
}

// R = [s]P (single per-lane base), s < 2^253
FE_INLINE void ge_scalarmult_var(ge_p3& R, const uint32_t s[8], const ge_p3& P) {
  ge_cached tab[8];
  build_cached_table(tab, P);
  uint32_t pw[8];
  sc_recode16(pw, s);
  ge_p1p1 x;
  straus<64, 64, 0, 0, false>(x, tab, pw, nullptr, nullptr, nullptr, nullptr);
  ge_p1p1_to_p3(R, x);
}

// ---------------------------------------------------------------- cached keys
// A public key that recurs in a batch (pool cold keys, VRF keys, KES leaf keys)
// is decoded once and expanded into KT_CHUNKS tables {1..8} (2^(16k) P) in global
// memory (k_keys.hip).  A scalar below 2^256 is then 16 chunks of 16 bits sharing
// one 4-window chain (12 doublings) instead of a 64-window one (252 doublings).
// The fixed-base term needs no doublings at all: byte j of its radix-256 recoding
// is added after the chain: 16-bit digit j from the comb table j = {1..32768} 65536^j B
// (C16_T tables in global memory, 48 MB: resident in the MALL), 16 mixed additions.
#define KT_CHUNKS 16
#define KT_STRIDE (KT_CHUNKS * 8)      // ge_cached entries per cached key
#define BCOMB_T 32                     // comb tables: 256^j B, j < 32
#define C16_T 16                       // radix-2^16 comb (cached-key chains): 65536^j B, j < 16,
#define C16_N 32768                    //   entries {1..32768}: 48 MB of affine niels (MALL-resident)

// w = s + 0x8000 8000 ... 8000 (radix-65536 signed recoding); requires s < 2^253
FE_INLINE void sc_recode65536(uint32_t w[8], const uint32_t s[8]) {
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) w[i] = addc(s[i], 0x80008000u, c, &c);
}

// w[k] for a uniform runtime k < N (a select chain; no dynamic register index)
template <int N>
FE_INLINE uint32_t word_sel(const uint32_t w[8], int k) {
  uint32_t r = w[0];
#pragma unroll
  for (int i = 1; i < N; i++) r = k == i ? w[i] : r;
  return r;
}

// out = [p] P + [b] B (as p1p1) with P cached (ktab: KT_CHUNKS tables of P):
//   p: radix-16 recoding pw; chunk k < NPC (nibbles 4k .. 4k+3) adds its nibble
//      4k + m at window m from table k; P_TOP: nibble 4 NPC (in {0, 1} for
//      p < 2^(16 NPC)) comes from table NPC at m = 0;
//   b: radix-65536 recoding fw (sc_recode65536, b < 2^253); 16-bit digit j from the
//      comb table j = {1..32768} 65536^j B (C16_T tables) after the chain.
// Each group operation is emitted once (runtime loops, see straus_rolled).
template <int NPC, bool P_TOP>
FE_INLINE void straus_comb(ge_p1p1& out, const ge_cached* __restrict__ ktab, const uint32_t pw[8],
                           const ge_niels* __restrict__ comb, const uint32_t fw[8]) {
  static_assert(NPC >= 1 && NPC + (P_TOP ? 1 : 0) <= KT_CHUNKS, "chunk count");
  ge_p1p1 x;
  ge_p1p1_identity(x);
#pragma clang loop unroll(disable)
  for (int m = 3; m >= 0; m--) {
    if (m != 3) dbl4_rolled(x);
    const int nt = NPC + ((P_TOP && m == 0) ? 1 : 0);
#pragma clang loop unroll(disable)
    for (int k = 0; k < nt; k++) {
      const uint32_t w = word_sel<(NPC + 2) / 2>(pw, k >> 1);       // nibble 4k + m
      add_cached_sel(x, ktab + 8 * k, (int)((w >> (16 * (k & 1) + 4 * m)) & 15u) - 8);
    }
  }
#pragma clang loop unroll(disable)
  for (int j = 0; j < C16_T; j++) {
    const uint32_t w = word_sel<8>(fw, j >> 1);                     // 16-bit digit j
    add_niels_sel(x, comb + (size_t)C16_N * j, (int)((w >> (16 * (j & 1))) & 0xffffu) - 32768);
  }
  out = x;
}

// Key tables in two passes (k_keys.hip), so no lane runs the whole precompute: pass 1
// (one lane per key) writes the chunk bases Q_k = 2^(16k) P as p3 into entry 0 of
// each chunk table (a p3 and a cached point are both 4 field elements); pass 2 (one
// lane per key and chunk) expands Q_k into ktab[8k + j] = (j+1) Q_k.
FE_INLINE void key_chunk_bases(ge_cached* __restrict__ ktab, const ge_p3& P, int nchunks) {
  ge_p3 Q = P;
#pragma clang loop unroll(disable)
  for (int k = 0; k < nchunks; k++) {
    *(ge_p3*)(ktab + 8 * k) = Q;
    if (k + 1 < nchunks) {
      ge_p2 q;
      ge_p1p1 t;
      ge_p3_to_p2(q, Q);
#pragma clang loop unroll(disable)
      for (int d = 0; d < 15; d++) { ge_p2_dbl(t, q); ge_p1p1_to_p2(q, t); }
      ge_p2_dbl(t, q);
      ge_p1p1_to_p3(Q, t);
    }
  }
}
FE_INLINE void key_chunk_table(ge_cached* __restrict__ tab8) {   // entries stored as they are made
  const ge_p3 Q = *(const ge_p3*)tab8;
  ge_cached c1, ck;
  ge_p3_to_cached(c1, Q);
  tab8[0] = c1;
  ge_p3 acc;
  ge_p3_dbl_to_p3(acc, Q);
  ge_p3_to_cached(ck, acc);
  tab8[1] = ck;
#pragma clang loop unroll(disable)
  for (int k = 2; k < 8; k++) {
    ge_p1p1 t;
    ge_add(t, acc, c1);
    ge_p1p1_to_p3(acc, t);
    ge_p3_to_cached(ck, acc);
    tab8[k] = ck;
  }
}

#if PRAOS_ROLLED
#define STRAUS straus_rolled
#else
#define STRAUS straus
#endif
