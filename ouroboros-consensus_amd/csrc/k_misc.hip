// k_misc.hip -- base-point table init, Fixed E34 leader check, self-test kernels.
#include "kcommon.hpp"

// ------------------------------------------------------------------ init
// btab[BTAB_N t + k] = (k+1) 256^t B (t < BCOMB_T, k < BTAB_N) as affine niels
// (y+x, y-x, 2dxy); one lane per entry (runs once per context).
__global__ void k_init_btab(ge_niels* btab) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= BCOMB_T * BTAB_N) return;
  const int k = e % BTAB_N, tb = e / BTAB_N;
  const uint32_t benc[8] = {0x66666658u, 0x66666666u, 0x66666666u, 0x66666666u,
                            0x66666666u, 0x66666666u, 0x66666666u, 0x66666666u};
  ge_p3 B, acc;
  ge_frombytes(B, benc, false);
  if (tb > 0) {
    for (int i = 0; i < 8 * tb; i++) {
      ge_p3_dbl_to_p3(acc, B);
      B = acc;
    }
  }
  acc = B;
  ge_cached bc;
  ge_p3_to_cached(bc, B);
  for (int i = 0; i < k; i++) {
    ge_p1p1 t;
    ge_add(t, acc, bc);
    ge_p1p1_to_p3(acc, t);
  }
  fe zi, x, y, xy, d2;
  fe_invert(zi, acc.Z);
  fe_mul(x, acc.X, zi);
  fe_mul(y, acc.Y, zi);
  fe_canon(x, x);
  fe_canon(y, y);
  ge_niels n;
  fe_add(n.ypx, y, x);
  fe_sub(n.ymx, y, x);
  fe_mul(xy, x, y);
  fe_const(d2, FE_D2);
  fe_mul(n.xy2d, xy, d2);
  btab[e] = n;
}

// bcomb16[C16_N j + k] = (k+1) 65536^j B (j < C16_T, k < C16_N) as affine niels: one
// lane per entry, a fixed-base multiplication by (k+1) 2^(16 j) mod L over the LDS
// tables of the radix-256 comb, then the affine conversion (runs once per context).
__global__ void __launch_bounds__(NT) k_init_bcomb16(const ge_niels* gbtab, ge_niels* bcomb16) {
  __shared__ ge_niels sbtab[2 * BTAB_N];
  const ge_niels* btab = stage_btab<5>(gbtab, sbtab);
  const uint32_t e = blockIdx.x * NT + threadIdx.x;
  if (e >= C16_T * C16_N) return;
  const uint32_t j = e / C16_N, k = e % C16_N + 1;
  uint32_t w[8], r[8];
#pragma unroll
  for (int q = 0; q < 8; q++) w[q] = 0;
  const int bit = 16 * (int)j;                     // k << 16 j, 1 <= k <= 2^15
  w[bit >> 5] = k << (bit & 31);
  sc_reduce256(r, w);
  ge_p3 P;
  ge_scalarmult_base(P, r, btab);
  fe zi, x, y, xy, d2;
  fe_invert(zi, P.Z);
  fe_mul(x, P.X, zi);
  fe_mul(y, P.Y, zi);
  fe_canon(x, x);
  fe_canon(y, y);
  ge_niels n;
  fe_add(n.ypx, y, x);
  fe_sub(n.ymx, y, x);
  fe_mul(xy, x, y);
  fe_const(d2, FE_D2);
  fe_mul(n.xy2d, xy, d2);
  bcomb16[e] = n;
}

// ------------------------------------------------------------------ leader
// Header mode: leader bytes from leader_in (big-endian natural), x from the
// pool table (sorted index), bit LEADER.  Plain mode (x_item != null): x per
// item, is_leader out.
__global__ void __launch_bounds__(NT) k_leader(size_t n, const uint8_t* __restrict__ leader_in,
                                               const int32_t* __restrict__ pool_sorted_idx,
                                               const uint32_t* __restrict__ pool_x, const uint32_t* __restrict__ x_item,
                                               int f_is_one, int leader_words, const uint16_t* __restrict__ b_ocert,
                                               const uint16_t* __restrict__ b_kes, const uint16_t* __restrict__ b_vrf,
                                               uint16_t* __restrict__ bits, uint8_t* __restrict__ is_leader,
                                               int32_t* __restrict__ iters, const uint16_t* __restrict__ dec_status) {
  const size_t i = (size_t)blockIdx.x * NT + threadIdx.x;
  if (i >= n) return;
  uint32_t x[4];
  bool skip = false;
  uint16_t b = 0;
  if (x_item) {
#pragma unroll
    for (int k = 0; k < 4; k++) x[k] = x_item[4 * i + k];
  } else {
    b = b_ocert[i] | b_kes[i] | b_vrf[i];      // the three crypto kernels' bits
    // a stored header that did not decode is malformed input whatever kernels ran
    if (dec_status && (dec_status[i] & PRAOS_DEC_FAILED)) b |= PRAOS_BIT_INPUT;
    const int32_t s = pool_sorted_idx[i];
    skip = s < 0;                              // VRFKeyUnknown precedes the leader check
#pragma unroll
    for (int k = 0; k < 4; k++) x[k] = skip ? 0u : pool_x[4 * s + k];
  }
  bool lead = true;
  int it = 0;
  if (!skip && !f_is_one) {
    if (leader_words == 16) {                  // TPraos: raw 64-byte output, bound 2^512
      uint32_t raw[16], l[16];
      load_words(raw, leader_in + 64 * i, 16);
#pragma unroll
      for (int k = 0; k < 16; k++) l[k] = __builtin_bswap32(raw[15 - k]);
      lead = leader_check_t<16>(l, x, &it);
    } else {                                   // Praos: Blake2b-256 range extension, bound 2^256
      uint32_t raw[8], l[8];
      load_words(raw, leader_in + 32 * i, 8);
#pragma unroll
      for (int k = 0; k < 8; k++) l[k] = __builtin_bswap32(raw[7 - k]);  // big-endian bytes -> LE words
      lead = leader_check(l, x, &it);
    }
  }
  if (iters) iters[i] = it;
  if (is_leader) { is_leader[i] = lead ? 1 : 0; return; }
  bits[i] = b | (lead ? 0 : PRAOS_BIT_LEADER);
}

// ------------------------------------------------------------------ debug / self-test kernels
// The header's nonce contribution from its CERTIFIED VRF output, before any verification
// (the replay's nonce chain runs ahead of the crypto): Praos vrfNonceValue =
// Blake2b-256(Blake2b-256("N" || output)) (Praos/VRF.hs:88-131), TPraos mkNonceFromOutputVRF =
// Blake2b-256(output of the eta certificate).  The VRF join later writes the same values.
__global__ void __launch_bounds__(NT) k_vrf_nonce(size_t n, const uint8_t* __restrict__ vrf_out, int tpraos,
                                                   uint8_t* __restrict__ nonce_out) {
  const size_t i = (size_t)blockIdx.x * NT + threadIdx.x;
  if (i >= n) return;
  uint32_t out[16], nn[8];
  const uint4* q = (const uint4*)(vrf_out + 64 * i);
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const uint4 v = q[k];
    out[4 * k] = v.x; out[4 * k + 1] = v.y; out[4 * k + 2] = v.z; out[4 * k + 3] = v.w;
  }
  if (tpraos) {
    blake2b256_of64(nn, out);
  } else {
    uint32_t nv[8];
    blake2b256_tag64(nv, 'N', out);
    blake2b_32(nn, nv, 32);
  }
  uint4* d = (uint4*)(nonce_out + 32 * i);
  d[0] = make_uint4(nn[0], nn[1], nn[2], nn[3]);
  d[1] = make_uint4(nn[4], nn[5], nn[6], nn[7]);
}

__global__ void k_debug_fe(int op, size_t n, const uint8_t* a, const uint8_t* b, uint8_t* r) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  fe x, y, z;
  load_words(x.v, a + 32 * i, 8);
  load_words(y.v, b + 32 * i, 8);
  switch (op) {
    case 0: fe_mul(z, x, y); break;
    case 1: fe_sq(z, x); break;
    case 2: fe_add(z, x, y); break;
    case 3: fe_sub(z, x, y); break;
    case 4: fe_invert(z, x); break;
    case 5: fe_pow22523(z, x); break;
    case 7: z = fe_invert_v(x); break;         // Fermat's chain (the PRAOS_INV_GCD=0 inversion)
    case 8: z = fe_invert_gcd_v(x); break;     // the binary GCD (fe_inv_gcd.hpp)
    default: fe_canon(z, x); break;
  }
  store_words(r + 32 * i, z.v, 8);
}

__global__ void k_debug_sha512(size_t n, const uint8_t* prefix, const uint64_t* off, const uint32_t* len,
                               const uint8_t* msg, uint8_t* out) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t pre[16], d[16];
  load_words(pre, prefix + 64 * i, 16);
  sha512_stream(d, pre, 64, msg + off[i], len[i]);
  store_words(out + 64 * i, d, 16);
}

__global__ void k_debug_blake2b(size_t n, const uint8_t* in, uint8_t* out) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t w[16], h[8];
  load_words(w, in + 64 * i, 16);
  blake2b256_64(h, w);
  store_words(out + 32 * i, h, 8);
}

__global__ void k_debug_sc_reduce(size_t n, const uint8_t* in, uint8_t* out) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t w[16], r[8];
  load_words(w, in + 64 * i, 16);
  sc_reduce512(r, w);
  store_words(out + 32 * i, r, 8);
}

__global__ void k_debug_decode(size_t n, const uint8_t* in, uint8_t* out, uint8_t* ok) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t w[8], e[8];
  load_words(w, in + 32 * i, 8);
  ge_p3 P;
  ok[i] = ge_frombytes(P, w, false) ? 1 : 0;
  ge_tobytes(e, P.X, P.Y, P.Z);
  store_words(out + 32 * i, e, 8);
}

// [s mod L] B (B has order L, so this is [s]B for any 256-bit s)
__global__ void __launch_bounds__(NT) k_debug_smul_base(size_t n, const ge_niels* gbtab, const uint8_t* s,
                                                        uint8_t* out) {
  __shared__ ge_niels sbtab[2 * BTAB_N];
  const ge_niels* btab = stage_btab<5>(gbtab, sbtab);
  const size_t i = (size_t)blockIdx.x * NT + threadIdx.x;
  if (i >= n) return;
  uint32_t w[8], r[8], e[8];
  load_words(w, s + 32 * i, 8);
  sc_reduce256(r, w);
  ge_p3 R;
  ge_scalarmult_base(R, r, btab);
  ge_tobytes(e, R.X, R.Y, R.Z);
  store_words(out + 32 * i, e, 8);
}

__global__ void k_debug_h2c(size_t n, const uint8_t* pk, const uint8_t* alpha, uint8_t* out) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t w[8], a[8], hs[8], ys[8];
  load_words(w, pk + 32 * i, 8);
  load_words(a, alpha + 32 * i, 8);
  ge_p3 Y, H;
  ge_frombytes(Y, w, false);
  ge_enc_affine(ys, Y);
  vrf_hash_to_curve(H, ys, a);
  ge_tobytes(hs, H.X, H.Y, H.Z);
  store_words(out + 32 * i, hs, 8);
}


// ---- host launchers (kernels are only launchable from their own module)
void launch_init_bcomb16(hipStream_t stream, const ge_niels* btab, ge_niels* bcomb16) {
  hipLaunchKernelGGL(k_init_bcomb16, dim3((C16_T * C16_N + NT - 1) / NT), dim3(NT), 0, stream, btab, bcomb16);
}
void launch_init_btab(dim3 grid, dim3 block, hipStream_t stream, ge_niels* btab) {
  hipLaunchKernelGGL(k_init_btab, grid, block, 0, stream, btab);
}


void launch_debug_fe(dim3 grid, dim3 block, hipStream_t stream, int op, size_t n, const uint8_t* a, const uint8_t* b, uint8_t* r) {
  hipLaunchKernelGGL(k_debug_fe, grid, block, 0, stream, op, n, a, b, r);
}

void launch_debug_sha512(dim3 grid, dim3 block, hipStream_t stream, size_t n, const uint8_t* prefix, const uint64_t* off, const uint32_t* len, const uint8_t* msg, uint8_t* out) {
  hipLaunchKernelGGL(k_debug_sha512, grid, block, 0, stream, n, prefix, off, len, msg, out);
}

void launch_debug_blake2b(dim3 grid, dim3 block, hipStream_t stream, size_t n, const uint8_t* in, uint8_t* out) {
  hipLaunchKernelGGL(k_debug_blake2b, grid, block, 0, stream, n, in, out);
}

void launch_debug_sc_reduce(dim3 grid, dim3 block, hipStream_t stream, size_t n, const uint8_t* in, uint8_t* out) {
  hipLaunchKernelGGL(k_debug_sc_reduce, grid, block, 0, stream, n, in, out);
}

void launch_debug_decode(dim3 grid, dim3 block, hipStream_t stream, size_t n, const uint8_t* in, uint8_t* out, uint8_t* ok) {
  hipLaunchKernelGGL(k_debug_decode, grid, block, 0, stream, n, in, out, ok);
}

void launch_debug_smul_base(dim3 grid, dim3 block, hipStream_t stream, size_t n, const ge_niels* gbtab, const uint8_t* s, uint8_t* out) {
  hipLaunchKernelGGL(k_debug_smul_base, grid, block, 0, stream, n, gbtab, s, out);
}

void launch_debug_h2c(dim3 grid, dim3 block, hipStream_t stream, size_t n, const uint8_t* pk, const uint8_t* alpha, uint8_t* out) {
  hipLaunchKernelGGL(k_debug_h2c, grid, block, 0, stream, n, pk, alpha, out);
}
void launch_leader(dim3 grid, dim3 block, hipStream_t stream, size_t n, const uint8_t* leader_in,
                   const int32_t* pool_sorted_idx, const uint32_t* pool_x, const uint32_t* x_item, int f_is_one,
                   int leader_words, const uint16_t* b_ocert, const uint16_t* b_kes, const uint16_t* b_vrf, uint16_t* bits,
                   uint8_t* is_leader, int32_t* iters, const uint16_t* dec_status) {
  hipLaunchKernelGGL(k_leader, grid, block, 0, stream, n, leader_in, pool_sorted_idx, pool_x, x_item, f_is_one,
                     leader_words, b_ocert,
                     b_kes, b_vrf, bits, is_leader, iters, dec_status);
}
void launch_vrf_nonce(hipStream_t stream, size_t n, const uint8_t* vrf_out, int tpraos, uint8_t* nonce_out) {
  if (n) hipLaunchKernelGGL(k_vrf_nonce, dim3((unsigned)((n + NT - 1) / NT)), dim3(NT), 0, stream, n, vrf_out, tpraos,
                            nonce_out);
}
