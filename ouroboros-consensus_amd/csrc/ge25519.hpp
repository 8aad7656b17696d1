// ge25519.hpp -- edwards25519 group arithmetic for gfx950 (one point per lane).
//
// Coordinates follow the extended twisted-Edwards model (Hisil et al.):
//   p2 = (X:Y:Z), p3 = (X:Y:Z:T), p1p1 = ((X:Z),(Y:T)),
//   cached = (Y+X, Y-X, Z, 2dT), niels = affine (y+x, y-x, 2dxy).
// Decoding follows libsodium 1.0.18 `ge25519_frombytes` exactly (the reference
// binds libsodium through cardano-crypto-class): y is read
// from the low 255 bits and reduced mod p, a non-square gives failure, and the
// sign bit selects x (x = 0 with sign 1 decodes to x = 0).
#pragma once
#include "fe25519.hpp"

struct ge_p2 { fe X, Y, Z; };
struct ge_p3 { fe X, Y, Z, T; };
struct ge_p1p1 { fe X, Y, Z, T; };
struct ge_cached { fe YpX, YmX, Z, T2d; };
struct ge_niels { fe ypx, ymx, xy2d; };

FE_INLINE void ge_p3_identity(ge_p3& p) { fe_set(p.X, 0); fe_set(p.Y, 1); fe_set(p.Z, 1); fe_set(p.T, 0); }
FE_INLINE void ge_p2_identity(ge_p2& p) { fe_set(p.X, 0); fe_set(p.Y, 1); fe_set(p.Z, 1); }
FE_INLINE void ge_cached_identity(ge_cached& c) { fe_set(c.YpX, 1); fe_set(c.YmX, 1); fe_set(c.Z, 1); fe_set(c.T2d, 0); }
FE_INLINE void ge_niels_identity(ge_niels& c) { fe_set(c.ypx, 1); fe_set(c.ymx, 1); fe_set(c.xy2d, 0); }

// PRAOS_ILP4 (a module built for latency-bound small batches, fewer waves per SIMD): the
// independent products of each formula -- 3 or 4 of them -- interleaved in one pass
// (fe_mul3 / fe_mul4 / fe_sq4); otherwise in pairs (fe_mul2 / fe_sq2), which keeps the
// register footprint of the 3-waves-per-SIMD kernels.  Same operations, same results.
#ifndef PRAOS_ILP4
#define PRAOS_ILP4 0
#endif

// (r and p are distinct objects at every call site; the paired products read p only)
FE_INLINE void ge_p1p1_to_p2(ge_p2& r, const ge_p1p1& p) {
#if PRAOS_ILP4
  fe_mul3(r.X, p.X, p.T, r.Y, p.Y, p.Z, r.Z, p.Z, p.T);
#else
  fe_mul2(r.X, p.X, p.T, r.Y, p.Y, p.Z);
  fe_mul(r.Z, p.Z, p.T);
#endif
}
FE_INLINE void ge_p1p1_to_p3(ge_p3& r, const ge_p1p1& p) {
#if PRAOS_ILP4
  fe_mul4(r.X, p.X, p.T, r.Y, p.Y, p.Z, r.Z, p.Z, p.T, r.T, p.X, p.Y);
#else
  fe_mul2(r.X, p.X, p.T, r.Y, p.Y, p.Z);
  fe_mul2(r.Z, p.Z, p.T, r.T, p.X, p.Y);
#endif
}
FE_INLINE void ge_p3_to_p2(ge_p2& r, const ge_p3& p) { r.X = p.X; r.Y = p.Y; r.Z = p.Z; }

FE_INLINE void ge_p3_to_cached(ge_cached& c, const ge_p3& p) {
  fe d2;
  fe_const(d2, FE_D2);
  fe_add(c.YpX, p.Y, p.X);
  fe_sub(c.YmX, p.Y, p.X);
  c.Z = p.Z;
  fe_mul(c.T2d, p.T, d2);
}

// r = 2p  (dbl-2008-hwcd with a = -1)
FE_INLINE void ge_p2_dbl(ge_p1p1& r, const ge_p2& p) {
  fe t0;
  fe_add(r.Y, p.X, p.Y);
#if PRAOS_ILP4
  fe_sq4(r.X, p.X, r.Z, p.Y, r.T, p.Z, t0, r.Y);
#else
  fe_sq2(r.X, p.X, r.Z, p.Y);
  fe_sq2(r.T, p.Z, t0, r.Y);
#endif
  fe_add(r.T, r.T, r.T);
  fe_add(r.Y, r.Z, r.X);
  fe_sub(r.Z, r.Z, r.X);
  fe_sub(r.X, t0, r.Y);
  fe_sub(r.T, r.T, r.Z);
}

// r = p + q
FE_INLINE void ge_add(ge_p1p1& r, const ge_p3& p, const ge_cached& q) {
  fe t0;
  fe_add(r.X, p.Y, p.X);
  fe_sub(r.Y, p.Y, p.X);
#if PRAOS_ILP4
  fe_mul4(r.Z, r.X, q.YpX, r.Y, r.Y, q.YmX, r.T, q.T2d, p.T, r.X, p.Z, q.Z);
#else
  fe_mul2(r.Z, r.X, q.YpX, r.Y, r.Y, q.YmX);
  fe_mul2(r.T, q.T2d, p.T, r.X, p.Z, q.Z);
#endif
  fe_add(t0, r.X, r.X);
  fe_sub(r.X, r.Z, r.Y);
  fe_add(r.Y, r.Z, r.Y);
  fe_add(r.Z, t0, r.T);
  fe_sub(r.T, t0, r.T);
}

// r = p + q, q affine niels
FE_INLINE void ge_madd(ge_p1p1& r, const ge_p3& p, const ge_niels& q) {
  fe t0;
  fe_add(r.X, p.Y, p.X);
  fe_sub(r.Y, p.Y, p.X);
#if PRAOS_ILP4
  fe_mul3(r.Z, r.X, q.ypx, r.Y, r.Y, q.ymx, r.T, q.xy2d, p.T);
#else
  fe_mul2(r.Z, r.X, q.ypx, r.Y, r.Y, q.ymx);
  fe_mul(r.T, q.xy2d, p.T);
#endif
  fe_add(t0, p.Z, p.Z);
  fe_sub(r.X, r.Z, r.Y);
  fe_add(r.Y, r.Z, r.Y);
  fe_add(r.Z, t0, r.T);
  fe_sub(r.T, t0, r.T);
}

FE_INLINE void ge_cached_cneg(ge_cached& c, bool neg) {
  fe t = c.YpX;
  fe_cmov(c.YpX, c.YmX, neg);
  fe_cmov(c.YmX, t, neg);
  fe n;
  fe_neg(n, c.T2d);
  fe_cmov(c.T2d, n, neg);
}
FE_INLINE void ge_niels_cneg(ge_niels& c, bool neg) {
  fe t = c.ypx;
  fe_cmov(c.ypx, c.ymx, neg);
  fe_cmov(c.ymx, t, neg);
  fe n;
  fe_neg(n, c.xy2d);
  fe_cmov(c.xy2d, n, neg);
}

FE_INLINE void ge_p3_dbl_to_p3(ge_p3& r, const ge_p3& p) {
  ge_p1p1 t;
  ge_p2 q;
  ge_p3_to_p2(q, p);
  ge_p2_dbl(t, q);
  ge_p1p1_to_p3(r, t);
}

// little-endian encoding words of an arbitrary projective point
FE_INLINE void ge_tobytes(uint32_t s[8], const fe& X, const fe& Y, const fe& Z) {
  fe zi, x, y;
  fe_invert(zi, Z);
  fe_mul(x, X, zi);
  fe_mul(y, Y, zi);
  fe_tobytes32(s, y);
  s[7] ^= (uint32_t)fe_isnegative(x) << 31;
}
// encoding when the inverse of Z is already known (batched inversions)
FE_INLINE void ge_tobytes_zi(uint32_t s[8], const fe& X, const fe& Y, const fe& zi) {
  fe x, y;
  fe_mul(x, X, zi);
  fe_mul(y, Y, zi);
  fe_tobytes32(s, y);
  s[7] ^= (uint32_t)fe_isnegative(x) << 31;
}

// x = sqrt(u / v) exactly as libsodium ge25519_frombytes computes it:
// x = u v^3 (u v^7)^((p-5)/8), multiplied by sqrt(-1) when v x^2 != u.
// Returns false when u / v is not a square (neither v x^2 == u nor == -u).
FE_INLINE bool fe_sqrt_ratio(fe& x, const fe& u, const fe& v) {
  fe v3, vxx, chk;
  fe_sq(v3, v);
  fe_mul(v3, v3, v);                 // v^3
  fe_sq(x, v3);
  fe_mul(x, x, v);
  fe_mul(x, x, u);                   // u v^7
  fe_pow22523(x, x);
  fe_mul(x, x, v3);
  fe_mul(x, x, u);                   // u v^3 (u v^7)^((p-5)/8)
  fe_sq(vxx, x);
  fe_mul(vxx, vxx, v);
  fe_sub(chk, vxx, u);
  const bool has_m_root = fe_iszero(chk);
  fe_add(chk, vxx, u);
  const bool has_p_root = fe_iszero(chk);
  fe xs, sq;
  fe_const(sq, FE_SQRTM1);
  fe_mul(xs, x, sq);
  fe_cmov(x, xs, !has_m_root);
  return has_m_root || has_p_root;
}

// libsodium ge25519_frombytes; negate=true gives ge25519_frombytes_negate_vartime.
// Returns false when the encoding is not on the curve.
FE_INLINE bool ge_frombytes(ge_p3& h, const uint32_t s[8], bool negate) {
  fe u, v, one, d;
  fe_set(one, 1);
  fe_const(d, FE_D);
  fe_frombytes32(h.Y, s);
  fe_set(h.Z, 1);
  fe_sq(u, h.Y);
  fe_mul(v, u, d);
  fe_sub(u, u, one);                 // u = y^2 - 1
  fe_add(v, v, one);                 // v = d y^2 + 1
  const bool ok = fe_sqrt_ratio(h.X, u, v);
  const bool sign = (s[7] >> 31) != 0;
  const bool flip = negate ? (fe_isnegative(h.X) == sign) : (fe_isnegative(h.X) != sign);
  fe nx;
  fe_neg(nx, h.X);
  fe_cmov(h.X, nx, flip);
  fe_mul(h.T, h.X, h.Y);
  return ok;
}

// ---- small-order blacklist and canonicity (libsodium ed25519_ref10.c)
FE_INLINE bool ge_has_small_order(const uint32_t s[8]) {
  // y in {0, 1, p-1, p, p+1, y8a, y8b}, sign bit ignored
  const uint32_t top = s[7] & 0x7fffffffu;
  uint32_t mid_or = s[1] | s[2] | s[3] | s[4] | s[5] | s[6];
  uint32_t mid_and = s[1] & s[2] & s[3] & s[4] & s[5] & s[6];
  bool r = false;
  r |= (mid_or == 0 && top == 0 && (s[0] == 0 || s[0] == 1));
  r |= (mid_and == 0xffffffffu && top == 0x7fffffffu &&
        (s[0] == 0xffffffecu || s[0] == 0xffffffedu || s[0] == 0xffffffeeu));
  const uint32_t a[8] = {0x8f95e826u, 0xb027b2c2u, 0x89f4c345u, 0xf098eff2u,
                         0x05acdfd5u, 0x3933c6d3u, 0x880238b1u, 0x05fc536du};
  const uint32_t b[8] = {0x706a17c7u, 0x4fd84d3du, 0x760b3cbau, 0x0f67100du,
                         0xfa53202au, 0xc6cc392cu, 0x77fdc74eu, 0x7a03ac92u};
  bool ea = true, eb = true;
#pragma unroll
  for (int i = 0; i < 7; i++) { ea &= s[i] == a[i]; eb &= s[i] == b[i]; }
  ea &= top == a[7];
  eb &= top == b[7];
  return r || ea || eb;
}
FE_INLINE bool ge_is_canonical(const uint32_t s[8]) {   // 255-bit y < p
  const uint32_t top = s[7] & 0x7fffffffu;
  const bool all1 = (s[1] & s[2] & s[3] & s[4] & s[5] & s[6]) == 0xffffffffu && top == 0x7fffffffu;
  return !(all1 && s[0] >= 0xffffffedu);
}
