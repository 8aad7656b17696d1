// fe_inv_gcd.hpp -- 1/y mod p (p = 2^255 - 19) by a binary GCD on approximated operands,
// for the encodings' inversions (ge_tobytes and the batched ones of the VRF join and the paired
// Ed25519 verifies) in place of Fermat's z^(p-2).
//
// The algorithm is T. Pornin's "optimized binary GCD" (IACR ePrint 2020/972, Algorithm 2):
// a = y, b = p; each outer iteration takes a 62-bit approximation of a and b (their low 30 bits
// exact, their top 32 bits), runs 30 binary-GCD steps on the approximations alone, recording
// the 2x2 update matrix [[f0 g0] [f1 g1]] (|f| + |g| <= 2^30 per row), then applies the matrix
// to the full a and b ((a f0 + b g0) / 2^30, exact) and to the Bezout pair u, v.  The bound is
// 2 len(p) - 1 = 509 steps, so 17 outer iterations of 30 steps (510) always reach a = 0, b = 1;
// random inputs get there in 13 or 14, and the loop leaves once every lane of the wave has.
// u and v are not divided by 2^30 per iteration: u' = u f0 + v g0 mod p, so after k iterations
// v is y^-1 2^(30 k) and one multiplication by 2^(-30 k) ends it.  y = 0 gives v = 0, as
// 0^(p-2) does.
//
// Cost per inversion, counted in the gfx950 ISA (tools/microbench/inv_gcd.hip prints both):
// ~13-14 x (30 x ~24 + ~560) VALU instructions, mostly VOP2 selects and subtractions, against
// Fermat's 254 squarings + 11 products (~32k VALU instructions, most of them 64-bit MACs).
// The result is the same field element as Fermat's (the caller canonicalises for encoding);
// the library checks the GCD ended (a = 0, b = 1 or y = 0) and otherwise takes the Fermat chain,
// a branch no input has been seen to take (tests/test_inv_gcd.py runs the same code on the host
// over random and structured inputs and asserts it never does).
//
// Plain integer C++ only, so that the same text compiles for the host test (FEG_HOST).
#pragma once
#include <stdint.h>

#ifndef FEG_INLINE
#define FEG_INLINE __device__ __forceinline__
#endif

#ifndef FEG_ITERS
#define FEG_ITERS 17   // 17 x 30 = 510 >= 2 len(p) - 1 (fewer only for the host test of the margin)
#endif

// p = 2^255 - 19
#define FEG_P0 0xffffffedu
#define FEG_PM 0xffffffffu
#define FEG_P7 0x7fffffffu

// 2^(-30 k) mod p for k = 0 .. 17, little-endian words: the correction after k iterations
#define FEG_CTAB { \
    {0x00000001u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u}, \
    {0xfffffff4u, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0x50d79435u}, \
    {0xfffffff8u, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0x435e50d7u, 0x35e50d79u}, \
    {0xffffffeeu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0x0d79435fu, 0xd79435e5u, 0x79435e50u}, \
    {0xfffffff4u, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0x35e50d7fu, 0x5e50d794u, 0xe50d7943u, 0x50d79435u}, \
    {0xfffffff8u, 0xffffffffu, 0xffffffffu, 0xd79435ffu, 0x79435e50u, 0x9435e50du, 0x435e50d7u, 0x35e50d79u}, \
    {0xffffffeeu, 0xffffffffu, 0x5e50d7ffu, 0xe50d7943u, 0x50d79435u, 0x0d79435eu, 0xd79435e5u, 0x79435e50u}, \
    {0xfffffff4u, 0x79435fffu, 0x9435e50du, 0x435e50d7u, 0x35e50d79u, 0x5e50d794u, 0xe50d7943u, 0x50d79435u}, \
    {0xe50d7ff8u, 0x50d79435u, 0x0d79435eu, 0xd79435e5u, 0x79435e50u, 0x9435e50du, 0x435e50d7u, 0x35e50d79u}, \
    {0x435e50d4u, 0x35e50d79u, 0x5e50d794u, 0xe50d7943u, 0x50d79435u, 0x0d79435eu, 0xd79435e5u, 0x181c5e50u}, \
    {0xd79435d7u, 0x79435e50u, 0x9435e50du, 0x435e50d7u, 0x35e50d79u, 0x5e50d794u, 0x60717943u, 0x5eab9cb8u}, \
    {0xe50d7941u, 0x50d79435u, 0x0d79435eu, 0xd79435e5u, 0x79435e50u, 0x81c5e50du, 0x7aae72e1u, 0x0ff4a75bu}, \
    {0x435e50ceu, 0x35e50d79u, 0x5e50d794u, 0xe50d7943u, 0x07179435u, 0xeab9cb86u, 0x3fd29d6du, 0x408827b6u}, \
    {0xd79435d3u, 0x79435e50u, 0x9435e50du, 0x1c5e50d7u, 0xaae72e18u, 0xff4a75b7u, 0x02209ed8u, 0x799e2375u}, \
    {0xe50d7938u, 0x50d79435u, 0x7179435eu, 0xab9cb860u, 0xfd29d6deu, 0x08827b63u, 0xe6788dd4u, 0x4c965683u}, \
    {0x435e50c8u, 0xc5e50d79u, 0xae72e181u, 0xf4a75b7au, 0x2209ed8fu, 0x99e23750u, 0x32595a0fu, 0x68f3f1d1u}, \
    {0x179435e2u, 0xb9cb8607u, 0xd29d6deau, 0x8827b63fu, 0x6788dd40u, 0xc965683eu, 0xa3cfc744u, 0x1490aa31u}, \
    {0xe72e181bu, 0x4a75b7aau, 0x209ed8ffu, 0x9e237502u, 0x2595a0f9u, 0x8f3f1d13u, 0x5242a8c6u, 0x093805acu}, \
}

// FEG_ALL(x): x holds on every active lane of the wave (the early exit must be wave-uniform:
// the lanes of a wave then share one correction constant); on the host, this element alone
#ifndef FEG_ALL
#define FEG_ALL(x) __all(x)
#endif
// iterations before the first exit test: random inputs end within 13 (99.9 %) or 14
// (tests/test_inv_gcd.py measures it), the bound is 17
// FEG_INNER32=1: the inner steps on 32-bit halves (A/B against the 64-bit compare and shift);
// FEG_INNER_MASK=1: the conditions as VGPR masks (A/B against compares into SGPR masks)
#ifndef FEG_INNER32
#define FEG_INNER32 0
#endif
#ifndef FEG_INNER_MASK
#define FEG_INNER_MASK 0
#endif
#ifndef FEG_EXIT_FROM
#define FEG_EXIT_FROM 12
#endif

// the 64-bit window x >> s of an 8-limb value (s in [30, 223])
FEG_INLINE uint64_t feg_window(const uint32_t x[8], uint32_t s) {
  const uint32_t j = s >> 5, r = s & 31u;
  uint32_t x0 = 0, x1 = 0, x2 = 0;
#pragma unroll
  for (uint32_t k = 0; k < 8; k++) {
    x0 = k == j ? x[k] : x0;
    x1 = k == j + 1 ? x[k] : x1;
    x2 = k == j + 2 ? x[k] : x2;
  }
  const uint64_t lo = (((uint64_t)x1 << 32) | x0) >> r;
  const uint64_t hi = r ? (uint64_t)x2 << (64u - r) : 0;
  return lo | hi;
}

// r = (x f + y g) / 2^30 for x, y in [0, 2^256), |f| + |g| <= 2^30 (the division is exact);
// r as 256-bit two's complement (|r| < 2^255 here); returns r < 0
FEG_INLINE bool feg_lin_shift(uint32_t r[8], const uint32_t x[8], const uint32_t y[8], int32_t f, int32_t g) {
  const uint32_t mf = f < 0 ? 0xffffffffu : 0u, mg = g < 0 ? 0xffffffffu : 0u;
  const uint32_t fa = (uint32_t)((f ^ (int32_t)mf) - (int32_t)mf);
  const uint32_t ga = (uint32_t)((g ^ (int32_t)mg) - (int32_t)mg);
  // (x ^ m) - m is -x for m = -1: with the 9th limb the sign extension; mod 2^288
  uint32_t t[9];
  uint64_t acc = 0;
  uint32_t bx = mf & 1u, by = mg & 1u;   // the +1 of the two's complement, carried limb by limb
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint64_t xs = (uint64_t)(x[i] ^ mf) + bx;
    const uint64_t ys = (uint64_t)(y[i] ^ mg) + by;
    bx = (uint32_t)(xs >> 32);
    by = (uint32_t)(ys >> 32);
    acc += (uint64_t)(uint32_t)xs * fa;
    acc += (uint64_t)(uint32_t)ys * ga;
    t[i] = (uint32_t)acc;
    acc >>= 32;
  }
  t[8] = (uint32_t)acc + (mf + bx) * fa + (mg + by) * ga;   // mod 2^32
#pragma unroll
  for (int i = 0; i < 8; i++) r[i] = (t[i] >> 30) | (t[i + 1] << 2);
  return (int32_t)t[8] < 0;
}

// r = -r (256-bit two's complement)
FEG_INLINE void feg_neg256(uint32_t r[8]) {
  uint32_t c = 1;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint64_t s = (uint64_t)(~r[i]) + c;
    r[i] = (uint32_t)s;
    c = (uint32_t)(s >> 32);
  }
}

// r = (x f + y g) mod p, weakly reduced to [0, 2^256), for x, y in [0, 2^256), |f| + |g| <= 2^30.
// For f < 0: ~x = 2^256 - 1 - x = 37 - x (mod p), so x f = (~x) |f| - 37 |f|; the products are
// then all nonnegative, and the -37 terms join the top fold (2^256 = 38) as one signed addend.
FEG_INLINE void feg_lin_mod(uint32_t r[8], const uint32_t x[8], const uint32_t y[8], int32_t f, int32_t g) {
  const uint32_t mf = f < 0 ? 0xffffffffu : 0u, mg = g < 0 ? 0xffffffffu : 0u;
  const uint32_t fa = (uint32_t)((f ^ (int32_t)mf) - (int32_t)mf);
  const uint32_t ga = (uint32_t)((g ^ (int32_t)mg) - (int32_t)mg);
  uint32_t t[8];
  uint64_t acc = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    acc += (uint64_t)(x[i] ^ mf) * fa;
    acc += (uint64_t)(y[i] ^ mg) * ga;
    t[i] = (uint32_t)acc;
    acc >>= 32;
  }
  // value = t + 38 acc - 37 (|f| [f < 0] + |g| [g < 0])  (acc < 2^31: the addend is in (-2^37, 2^37))
  int64_t s = (int64_t)t[0] + (int64_t)(38ull * acc) - 37ll * ((int64_t)(mf & fa) + (int64_t)(mg & ga));
  r[0] = (uint32_t)s;
  int64_t c = s >> 32;
#pragma unroll
  for (int i = 1; i < 8; i++) {
    s = (int64_t)t[i] + c;
    r[i] = (uint32_t)s;
    c = s >> 32;
  }
  // carry-out c in {-1, 0, 1}: 2^256 c = 38 c (mod p); a second round only after a wrap
  while (c != 0) {
    s = (int64_t)r[0] + 38 * c;
    r[0] = (uint32_t)s;
    c = s >> 32;
#pragma unroll
    for (int i = 1; i < 8; i++) {
      s = (int64_t)r[i] + c;
      r[i] = (uint32_t)s;
      c = s >> 32;
    }
  }
}

// v = y^-1 2^(30 k) mod p (weakly reduced) for canonical y in [0, p), k = *iters, the outer
// iterations run (<= 17: the loop leaves once a = 0 on every lane of the wave; an ended lane's
// further iterations only double v 30 times each, which k accounts for); returns whether the
// GCD ended (a = 0 and b = 1, or y = 0)
FEG_INLINE bool feg_core(uint32_t vout[8], const uint32_t y[8], int* iters) {
  uint32_t a[8], b[8], u[8], v[8];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    a[i] = y[i];
    b[i] = i == 0 ? FEG_P0 : (i == 7 ? FEG_P7 : FEG_PM);
    u[i] = i == 0 ? 1u : 0u;
    v[i] = 0;
  }
  int it = 0;
#pragma nounroll
  while (it < FEG_ITERS) {
    // n = max(len(a), len(b), 62); the approximations: the top 32 bits [n - 32, n) above the
    // low 30 bits (exact once n = 62)
    uint32_t n = 0;
#pragma unroll
    for (int k = 1; k < 8; k++) {
      const uint32_t m = a[k] | b[k];
      n = m ? 32u * k + 32u - (uint32_t)__builtin_clz(m) : n;
    }
    n = n < 62u ? 62u : n;
    const uint32_t s = n - 32u;
    uint64_t ah = (feg_window(a, s) << 30) | (a[0] & 0x3fffffffu);
    uint64_t bh = (feg_window(b, s) << 30) | (b[0] & 0x3fffffffu);
    int32_t f0 = 1, g0 = 0, f1 = 0, g1 = 1;
#if FEG_INNER32
    // the same steps on 32-bit halves: d = a - b gives a < b as its borrow, and the new a is
    // |d| / 2 (odd) or a / 2; no 64-bit compare or shift
    uint32_t al = (uint32_t)ah, ahi = (uint32_t)(ah >> 32), bl = (uint32_t)bh, bhi = (uint32_t)(bh >> 32);
#pragma unroll
    for (int j = 0; j < 30; j++) {
      const bool odd = (al & 1u) != 0;
      const uint64_t dl = (uint64_t)al - bl;
      const uint32_t br0 = (uint32_t)(dl >> 63);
      const uint64_t dh = (uint64_t)ahi - bhi - br0;
      const bool lt = (dh >> 63) != 0;
      const bool sw = odd && lt;
      uint32_t xl = (uint32_t)dl, xh = (uint32_t)dh;
      const uint64_t nl = 0ull - xl;
      const uint32_t nh = 0u - xh - (uint32_t)(nl >> 63);
      xl = lt ? (uint32_t)nl : xl;
      xh = lt ? nh : xh;
      xl = odd ? xl : al;
      xh = odd ? xh : ahi;
      bl = sw ? al : bl;
      bhi = sw ? ahi : bhi;
      al = (xl >> 1) | (xh << 31);
      ahi = xh >> 1;
      const int32_t nf0 = sw ? f1 : f0, ng0 = sw ? g1 : g0, nf1 = sw ? f0 : f1, ng1 = sw ? g0 : g1;
      f0 = odd ? nf0 - nf1 : nf0;
      g0 = odd ? ng0 - ng1 : ng0;
      f1 = nf1 * 2;
      g1 = ng1 * 2;
    }
#elif FEG_INNER_MASK
    // the same steps with the conditions as all-ones VGPR masks and bit selects: no compare into
    // an SGPR mask and no scalar AND between the vector instructions of a step (ah, bh < 2^62, so
    // the sign of ah - bh is ah < bh)
#pragma unroll
    for (int j = 0; j < 30; j++) {
      const uint64_t d = ah - bh;
      const uint32_t oddm = 0u - ((uint32_t)ah & 1u);
      const uint32_t ltm = (uint32_t)((int64_t)d >> 63);
      const uint32_t swm = oddm & ltm;
      const uint64_t sw64 = ((uint64_t)swm << 32) | swm, odd64 = ((uint64_t)oddm << 32) | oddm;
      const uint64_t lt64 = ((uint64_t)ltm << 32) | ltm;
      const uint64_t ad = (d ^ lt64) - lt64;                   // |ah - bh|
      bh = (ah & sw64) | (bh & ~sw64);
      ah = ((ad & odd64) | (ah & ~odd64)) >> 1;
      const int32_t sf = (int32_t)swm, so = (int32_t)oddm;
      const int32_t nf0 = (f1 & sf) | (f0 & ~sf), ng0 = (g1 & sf) | (g0 & ~sf);
      const int32_t nf1 = (f0 & sf) | (f1 & ~sf), ng1 = (g0 & sf) | (g1 & ~sf);
      f0 = nf0 - (nf1 & so);
      g0 = ng0 - (ng1 & so);
      f1 = nf1 * 2;
      g1 = ng1 * 2;
    }
#else
#pragma unroll
    for (int j = 0; j < 30; j++) {
      const bool odd = (ah & 1u) != 0;
      const bool sw = odd && ah < bh;
      const uint64_t na = sw ? bh : ah, nb = sw ? ah : bh;
      const int32_t nf0 = sw ? f1 : f0, ng0 = sw ? g1 : g0, nf1 = sw ? f0 : f1, ng1 = sw ? g0 : g1;
      ah = (odd ? na - nb : na) >> 1;
      bh = nb;
      f0 = odd ? nf0 - nf1 : nf0;
      g0 = odd ? ng0 - ng1 : ng0;
      f1 = nf1 * 2;
      g1 = ng1 * 2;
    }
#endif
    uint32_t na[8], nb[8];
    if (feg_lin_shift(na, a, b, f0, g0)) {
      feg_neg256(na);
      f0 = -f0;
      g0 = -g0;
    }
    if (feg_lin_shift(nb, a, b, f1, g1)) {
      feg_neg256(nb);
      f1 = -f1;
      g1 = -g1;
    }
    uint32_t nu[8], nv[8];
    feg_lin_mod(nu, u, v, f0, g0);
    feg_lin_mod(nv, u, v, f1, g1);
    uint32_t az = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
      a[i] = na[i];
      b[i] = nb[i];
      u[i] = nu[i];
      v[i] = nv[i];
      az |= na[i];
    }
    it++;
    if (it >= FEG_EXIT_FROM && FEG_ALL(az == 0)) break;
  }
  *iters = it;
  uint32_t az = 0, bo = b[0] ^ 1u, yz = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    az |= a[i];
    if (i) bo |= b[i];
    yz |= y[i];
    vout[i] = v[i];
  }
  return az == 0 && (bo == 0 || yz == 0);
}
