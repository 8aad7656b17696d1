// scalarmult.hpp -- per-lane multi-scalar multiplication for gfx950.
//
// All scalar multiplications on the Praos path are Straus/Shamir sums over
// 64 signed radix-16 windows (Horner: 4 doublings per window):
//   * fixed base B: 8-entry affine-niels table {1..8}B shared by the block in
//     LDS (computed once per context by k_init_basetab);
//   * per-lane variable bases: 8-entry cached tables {1..8}P in private
//     memory (scratch: indexed by a per-lane digit, so not register-resident).
// Digits are recoded once into LDS (int8, lane-interleaved: conflict-free).
// Results are mathematically exact group elements, so verdicts depend only on
// the encodings, exactly as in libsodium (which uses a different schedule).
#pragma once
#include "ge25519.hpp"

// LDS layout helpers: digit j of lane t in plane k: dig[(j * NPLANE + k) * nthreads + t]
struct DigitPlanes {
  int8_t* base;
  int nthreads;
  int nplane;
  FE_INLINE int8_t get(int j, int k, int t) const { return base[(j * nplane + k) * nthreads + t]; }
  FE_INLINE void put(int j, int k, int t, int8_t v) { base[(j * nplane + k) * nthreads + t] = v; }
};

FE_INLINE void store_digits(DigitPlanes& dp, int plane, int t, const uint32_t s[8]) {
  int8_t e[64];
  sc_signed_radix16(e, s);
#pragma unroll
  for (int j = 0; j < 64; j++) dp.put(j, plane, t, e[j]);
}

// table[k] = (k+1) * P in cached form
FE_INLINE void build_cached_table(ge_cached tab[8], const ge_p3& P) {
  ge_p3 acc = P, P2;
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

FE_INLINE void select_cached(ge_cached& c, const ge_cached tab[8], int d) {
  const int a = d < 0 ? -d : d;
  if (a == 0) {
    ge_cached_identity(c);
  } else {
    c = tab[a - 1];
  }
  ge_cached_cneg(c, d < 0);
}
FE_INLINE void select_niels(ge_niels& c, const ge_niels* __restrict__ tab, int d) {
  const int a = d < 0 ? -d : d;
  if (a == 0) {
    ge_niels_identity(c);
  } else {
    c = tab[a - 1];
  }
  ge_niels_cneg(c, d < 0);
}

// 4 doublings: p2 -> p3
FE_INLINE void dbl4(ge_p3& r, const ge_p2& p) {
  ge_p1p1 t;
  ge_p2 q = p;
  ge_p2_dbl(t, q); ge_p1p1_to_p2(q, t);
  ge_p2_dbl(t, q); ge_p1p1_to_p2(q, t);
  ge_p2_dbl(t, q); ge_p1p1_to_p2(q, t);
  ge_p2_dbl(t, q); ge_p1p1_to_p3(r, t);
}

// R = [s]B + [a]P   (digit planes: plane_a for a, plane_s for s)
// nwin_a: windows (from 0) in which a may have non-zero digits (<= 64).
FE_INLINE void ge_double_scalarmult_base(ge_p2& R, const DigitPlanes& dp, int plane_a, int plane_s, int t,
                                         const ge_p3& P, int nwin_a, const ge_niels* __restrict__ btab) {
  ge_cached tab[8];
  build_cached_table(tab, P);
  ge_p2 acc;
  ge_p2_identity(acc);
  ge_p1p1 x;
  ge_p3 a3;
#pragma clang loop unroll(disable)
  for (int j = 63; j >= 0; j--) {
    dbl4(a3, acc);
    if (j < nwin_a) {
      ge_cached c;
      select_cached(c, tab, dp.get(j, plane_a, t));
      ge_add(x, a3, c);
      ge_p1p1_to_p3(a3, x);
    }
    ge_niels nb;
    select_niels(nb, btab, dp.get(j, plane_s, t));
    ge_madd(x, a3, nb);
    ge_p1p1_to_p2(acc, x);
  }
  R = acc;
}

// R = [a]P + [b]Q   (two per-lane bases; b may be short: nwin_b windows)
FE_INLINE void ge_double_scalarmult_var(ge_p2& R, const DigitPlanes& dp, int plane_a, int plane_b, int t,
                                        const ge_p3& P, const ge_p3& Q, int nwin_b) {
  ge_cached tp[8], tq[8];
  build_cached_table(tp, P);
  build_cached_table(tq, Q);
  ge_p2 acc;
  ge_p2_identity(acc);
  ge_p1p1 x;
  ge_p3 a3;
#pragma clang loop unroll(disable)
  for (int j = 63; j >= 0; j--) {
    dbl4(a3, acc);
    ge_cached c;
    if (j < nwin_b) {
      select_cached(c, tq, dp.get(j, plane_b, t));
      ge_add(x, a3, c);
      ge_p1p1_to_p3(a3, x);
    }
    select_cached(c, tp, dp.get(j, plane_a, t));
    ge_add(x, a3, c);
    ge_p1p1_to_p2(acc, x);
  }
  R = acc;
}

// R = [s]B (fixed base only), s < 2^255
FE_INLINE void ge_scalarmult_base(ge_p3& R, const DigitPlanes& dp, int plane_s, int t,
                                  const ge_niels* __restrict__ btab) {
  ge_p2 acc;
  ge_p2_identity(acc);
  ge_p1p1 x;
  ge_p3 a3;
#pragma clang loop unroll(disable)
  for (int j = 63; j >= 0; j--) {
    dbl4(a3, acc);
    ge_niels nb;
    select_niels(nb, btab, dp.get(j, plane_s, t));
    ge_madd(x, a3, nb);
    if (j == 0) ge_p1p1_to_p3(R, x);
    else ge_p1p1_to_p2(acc, x);
  }
}

// R = [s]P (single per-lane base)
FE_INLINE void ge_scalarmult_var(ge_p3& R, const DigitPlanes& dp, int plane_s, int t, const ge_p3& P) {
  ge_cached tab[8];
  build_cached_table(tab, P);
  ge_p2 acc;
  ge_p2_identity(acc);
  ge_p1p1 x;
  ge_p3 a3;
#pragma clang loop unroll(disable)
  for (int j = 63; j >= 0; j--) {
    dbl4(a3, acc);
    ge_cached c;
    select_cached(c, tab, dp.get(j, plane_s, t));
    ge_add(x, a3, c);
    if (j == 0) ge_p1p1_to_p3(R, x);
    else ge_p1p1_to_p2(acc, x);
  }
}
