// k_decode.hip -- stored Praos header bytes -> HeaderView struct of arrays
// (SURVEY.md section 8f row 2), one header per lane.
//
// Input: a byte arena (e.g. an ImmutableDB chunk file as read from disk) and
// per header the (offset, length) pair the secondary index gives
// (blockOffset + headerOffset, headerSize; Secondary.hs:93-128).  Output: the
// SoA the crypto kernels read, plus the remaining HeaderBody fields, the
// header hash and the signed body bytes.  Restates (Praos/Header.hs):
//   * DecCBOR (Annotator (Header c)) :228-231, HeaderRaw = [body, kesSig] :201-210;
//   * DecCBOR HeaderBody :187-199 (10-field record, CertifiedVRF pair, OCert
//     group, ProtVer pair); decodeWord32 for bodySize;
//   * SignableRepresentation :90-94: the KES message is `serialize' hb`, the
//     canonical re-encoding.  For a canonical stored body (the normal case)
//     that is the stored slice, copied; otherwise it is re-encoded here.
//   * headerHash :147-151: Blake2b-256 of the stored header bytes.
// The CPU restatement is oracle/cbor_header.py (same status semantics: the
// first failure wins; NONCANONICAL is informational).
//
// Block batches (k_block.hip) also accept TPraos headers (allow_tp): BHeader =
// [BHBody, kesSig] with the 15-field BHBody of cardano-protocol-tpraos
// (encodeBHBody: the eta and leader certificates as two [out, proof] pairs, OCert and
// ProtVer inlined), the integrity check of Shelley/Protocol/TPraos.hs:59-76.  The eta
// certificate goes to vrf_out/vrf_proof; the leader certificate is only needed to
// re-encode a non-canonical body and is then read back from the arena.  Signed
// bodies of block batches use a 640-byte stride (max canonical BHBody 598 bytes).
//
// Memory: every field load goes through ld64u (two aligned 8-byte loads and a
// funnel shift), so a lane walks its ~850-byte header with 8-byte accesses;
// the arena is padded by 16 bytes so the second load never leaves it.  The
// SoA stores are aligned records (16-byte stores), the signed bodies go to a
// fixed 448-byte stride (8-aligned, what the SHA-512 feeder of k_kes reads).
#include "kcommon.hpp"
#include "arena.hpp"

namespace {


struct Rd {
  const uint8_t* __restrict__ p;
  uint64_t pos, end;
  uint32_t st;      // first failure (PRAOS_DEC_*), 0 while ok
  bool canon;       // all heads so far shortest-form
};

__device__ __forceinline__ uint32_t rd_byte(Rd& r) {
  if (r.st) return 0;
  if (r.pos >= r.end) { r.st = PRAOS_DEC_SYNTAX; return 0; }
  return r.p[r.pos++];
}

// head of one item: major type (or -1 after a failure) and argument
__device__ __noinline__ int rd_head(Rd& r, uint64_t& arg) {
  arg = 0;
  const uint32_t ib = rd_byte(r);
  if (r.st) return -1;
  const int mt = (int)(ib >> 5);
  const uint32_t ai = ib & 31u;
  if (ai < 24) { arg = ai; return mt; }
  if (ai <= 27) {
    const int nb = 1 << (ai - 24);
    if (r.pos + (uint64_t)nb > r.end) { r.st = PRAOS_DEC_SYNTAX; return -1; }
    const uint64_t w = __builtin_bswap64(ld64u(r.p, r.pos));   // big-endian argument bytes
    const uint64_t v = nb == 8 ? w : (w >> (64 - 8 * nb));
    r.pos += (uint64_t)nb;
    const uint64_t lo = ai == 24 ? 24u : ai == 25 ? 256u : ai == 26 ? 65536u : (1ull << 32);
    if (v < lo) r.canon = false;
    arg = v;
    return mt;
  }
  r.st = ai == 31 ? PRAOS_DEC_UNSUPPORTED : PRAOS_DEC_SYNTAX;
  return -1;
}

__device__ __forceinline__ uint64_t rd_expect(Rd& r, int want) {
  uint64_t v;
  const int mt = rd_head(r, v);
  if (r.st) return 0;
  if (mt == 6) { r.st = PRAOS_DEC_UNSUPPORTED; return 0; }
  if (mt != want) { r.st = PRAOS_DEC_SYNTAX; return 0; }
  return v;
}

__device__ __forceinline__ void rd_array(Rd& r, uint64_t n) {
  const uint64_t v = rd_expect(r, 4);
  if (!r.st && v != n) r.st = PRAOS_DEC_SYNTAX;
}

__device__ __forceinline__ uint64_t rd_uint(Rd& r, uint64_t limit) {
  const uint64_t v = rd_expect(r, 0);
  if (!r.st && v > limit) { r.st = PRAOS_DEC_OVERFLOW; return 0; }
  return v;
}

// fixed-length byte string -> aligned destination record (N multiple of 16)
// fixed-length byte string that is only skipped; returns the payload offset
template <int N>
__device__ __forceinline__ uint64_t rd_skip(Rd& r) {
  const uint64_t ln = rd_expect(r, 2);
  if (!r.st && ln != (uint64_t)N) r.st = PRAOS_DEC_SIZE;
  if (!r.st && r.pos + N > r.end) r.st = PRAOS_DEC_SYNTAX;
  if (r.st) return 0;
  const uint64_t at = r.pos;
  r.pos += N;
  return at;
}

template <int N>
__device__ __forceinline__ void rd_bytes(Rd& r, uint8_t* __restrict__ dst) {
  const uint64_t ln = rd_expect(r, 2);
  if (!r.st && ln != (uint64_t)N) r.st = PRAOS_DEC_SIZE;
  if (!r.st && r.pos + N > r.end) r.st = PRAOS_DEC_SYNTAX;
  if (r.st) return;
  uint64_t* d = (uint64_t*)dst;
#pragma unroll 4
  for (int k = 0; k < N / 8; k++) d[k] = ld64u(r.p, r.pos + 8 * k);
  r.pos += N;
}

// ---- canonical encoder (slow path: non-canonical stored bodies) ----
struct Wr {
  uint8_t* __restrict__ o;
  uint32_t n;
};
__device__ __forceinline__ void wr_byte(Wr& w, uint32_t b) { w.o[w.n++] = (uint8_t)b; }
__device__ void wr_head(Wr& w, uint32_t mt, uint64_t v) {
  const uint32_t m = mt << 5;
  if (v < 24) { wr_byte(w, m | (uint32_t)v); return; }
  const int nb = v < 256 ? 1 : v < 65536 ? 2 : v < (1ull << 32) ? 4 : 8;
  wr_byte(w, m | (nb == 1 ? 24u : nb == 2 ? 25u : nb == 4 ? 26u : 27u));
  for (int k = nb - 1; k >= 0; k--) wr_byte(w, (uint32_t)(v >> (8 * k)));
}
__device__ void wr_bytes(Wr& w, const uint8_t* __restrict__ src, uint32_t n) {
  wr_head(w, 2, n);
  for (uint32_t k = 0; k < n; k++) wr_byte(w, src[k]);
}

}  // namespace

struct DecOut {
  // SoA consumed by the crypto kernels
  uint64_t* slot;
  uint8_t *cold_vk, *vrf_vk, *vrf_out, *vrf_proof, *hot_vk, *ocert_sig, *kes_sig;
  uint64_t *ocert_n, *ocert_c0;
  uint64_t* body_off;            // = i * 448 into `signed_body`
  uint32_t* body_len;            // signed length; 0xffffffff on failure (k_kes flags PRAOS_BIT_INPUT)
  uint8_t* signed_body;
  // remaining HeaderBody fields
  uint64_t* block_no;
  uint8_t *prev_hash, *prev_genesis;
  uint32_t* body_size;
  uint8_t* body_hash;
  uint64_t *prot_major, *prot_minor;
  uint8_t* header_hash;
  uint16_t* status;
  // TPraos leader certificate (header batches of praos_verify_tpraos_header_bytes; NULL otherwise)
  uint8_t *lead_out, *lead_proof;
};

__global__ void __launch_bounds__(NT) k_decode_praos(size_t i0, size_t n, const uint8_t* __restrict__ arena,
                                                     uint64_t arena_len, const uint64_t* __restrict__ hoff,
                                                     const uint32_t* __restrict__ hlen, DecOut o, int allow_tp,
                                                     uint32_t stride) {
  const size_t i = i0 + (size_t)blockIdx.x * blockDim.x + threadIdx.x;   // headers [i0, n)
  if (i >= n) return;
  const uint64_t off = hoff[i], len = hlen[i];
  Rd r{arena, off, off + len, 0u, true};
  if (off > arena_len || len > arena_len - off) r.st = PRAOS_DEC_RANGE;
  uint32_t hh[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (!r.st) b2b256_range(hh, arena, off, len);
  store_words(o.header_hash + 32 * i, hh, 8);

  rd_array(r, 2);
  const uint64_t body_start = r.pos;
  r.canon = true;
  const uint64_t arity = rd_expect(r, 4);
  // allow_tp: 0 Praos headers only, 1 Praos or TPraos (block batches), 2 TPraos only
  const bool tp = allow_tp == 2 || (allow_tp == 1 && arity == 15);
  if (!r.st && arity != (tp ? 15u : 10u)) r.st = PRAOS_DEC_SYNTAX;
  const uint64_t block_no = rd_uint(r, ~0ull);
  const uint64_t slot = rd_uint(r, ~0ull);
  uint8_t genesis = 0;
  if (!r.st && r.pos < r.end && arena[r.pos] == 0xF6) {
    r.pos++;
    genesis = 1;
    ((uint4*)(o.prev_hash + 32 * i))[0] = make_uint4(0, 0, 0, 0);
    ((uint4*)(o.prev_hash + 32 * i))[1] = make_uint4(0, 0, 0, 0);
  } else {
    rd_bytes<32>(r, o.prev_hash + 32 * i);
  }
  rd_bytes<32>(r, o.cold_vk + 32 * i);
  rd_bytes<32>(r, o.vrf_vk + 32 * i);
  rd_array(r, 2);
  rd_bytes<64>(r, o.vrf_out + 64 * i);
  rd_bytes<80>(r, o.vrf_proof + 80 * i);
  uint64_t lead_out = 0, lead_proof = 0;     // TPraos leader certificate (arena offsets)
  if (tp) {
    rd_array(r, 2);
    lead_out = rd_skip<64>(r);
    lead_proof = rd_skip<80>(r);
  }
  const uint64_t body_size = rd_uint(r, 0xffffffffull);
  rd_bytes<32>(r, o.body_hash + 32 * i);
  if (!tp) rd_array(r, 4);
  rd_bytes<32>(r, o.hot_vk + 32 * i);
  const uint64_t ocn = rd_uint(r, ~0ull);
  const uint64_t occ0 = rd_uint(r, ~0ull);
  rd_bytes<64>(r, o.ocert_sig + 64 * i);
  if (!tp) rd_array(r, 2);
  const uint64_t pmaj = rd_uint(r, PRAOS_MAX_PROT_MAJOR);   // DecCBOR Version: <= maxVersion
  const uint64_t pmin = rd_uint(r, ~0ull);
  const bool canon = r.canon;
  const uint64_t body_end = r.pos;
  rd_bytes<448>(r, o.kes_sig + 448 * i);
  if (!r.st && r.pos != r.end) r.st = PRAOS_DEC_TRAILING;

  uint8_t* sb = o.signed_body + (size_t)stride * i;
  uint32_t slen = 0xffffffffu;
  if (!r.st) {
    if (canon) {
      // signed bytes = the stored slice (<= 447 bytes for a canonical Praos body,
      // <= 598 for TPraos)
      slen = (uint32_t)(body_end - body_start);
      uint64_t* d = (uint64_t*)sb;
      for (uint32_t k = 0; k < slen; k += 8) {
        uint64_t w = ld64u(arena, body_start + k);
        if (slen - k < 8) w &= (1ull << (8 * (slen - k))) - 1;
        d[k / 8] = w;
      }
    } else {
      Wr w{sb, 0};
      wr_head(w, 4, tp ? 15 : 10);
      wr_head(w, 0, block_no);
      wr_head(w, 0, slot);
      if (genesis) wr_byte(w, 0xF6);
      else wr_bytes(w, o.prev_hash + 32 * i, 32);
      wr_bytes(w, o.cold_vk + 32 * i, 32);
      wr_bytes(w, o.vrf_vk + 32 * i, 32);
      wr_head(w, 4, 2);
      wr_bytes(w, o.vrf_out + 64 * i, 64);
      wr_bytes(w, o.vrf_proof + 80 * i, 80);
      if (tp) {
        wr_head(w, 4, 2);
        wr_bytes(w, arena + lead_out, 64);
        wr_bytes(w, arena + lead_proof, 80);
      }
      wr_head(w, 0, body_size);
      wr_bytes(w, o.body_hash + 32 * i, 32);
      if (!tp) wr_head(w, 4, 4);
      wr_bytes(w, o.hot_vk + 32 * i, 32);
      wr_head(w, 0, ocn);
      wr_head(w, 0, occ0);
      wr_bytes(w, o.ocert_sig + 64 * i, 64);
      if (!tp) wr_head(w, 4, 2);
      wr_head(w, 0, pmaj);
      wr_head(w, 0, pmin);
      slen = w.n;
      for (uint32_t k = slen; k < ((slen + 7) & ~7u); k++) sb[k] = 0;
    }
  }
  {
    // the rest of the row is zero too (a batch reused across calls holds no stale bytes)
    const uint32_t used = slen == 0xffffffffu ? 0u : ((slen + 7) & ~7u);
    uint64_t* d = (uint64_t*)sb;
    for (uint32_t k = used; k < stride; k += 8) d[k / 8] = 0ull;
  }
  const bool ok = r.st == 0;
  if (o.lead_out) {                          // the leader certificate as SoA records (zeros on failure)
    uint64_t* lo = (uint64_t*)(o.lead_out + 64 * i);
    uint64_t* lp = (uint64_t*)(o.lead_proof + 80 * i);
    for (int k = 0; k < 8; k++) lo[k] = ok && tp ? ld64u(arena, lead_out + 8 * k) : 0ull;
    for (int k = 0; k < 10; k++) lp[k] = ok && tp ? ld64u(arena, lead_proof + 8 * k) : 0ull;
  }
  o.status[i] = (uint16_t)(ok ? (canon ? 0u : (uint32_t)PRAOS_DEC_NONCANONICAL) : r.st);
  o.slot[i] = ok ? slot : 0;
  o.block_no[i] = ok ? block_no : 0;
  o.ocert_n[i] = ok ? ocn : 0;
  o.ocert_c0[i] = ok ? occ0 : 0;
  o.body_size[i] = ok ? (uint32_t)body_size : 0;
  o.prot_major[i] = ok ? pmaj : 0;
  o.prot_minor[i] = ok ? pmin : 0;
  o.prev_genesis[i] = ok ? genesis : 0;
  o.body_off[i] = (uint64_t)stride * i;
  o.body_len[i] = slen;
  if (!ok) {
    // a header that does not decode has no fields: zero every record
    const uint4 z = make_uint4(0, 0, 0, 0);
    uint4* q;
    q = (uint4*)(o.prev_hash + 32 * i);  q[0] = z; q[1] = z;
    q = (uint4*)(o.cold_vk + 32 * i);    q[0] = z; q[1] = z;
    q = (uint4*)(o.vrf_vk + 32 * i);     q[0] = z; q[1] = z;
    q = (uint4*)(o.hot_vk + 32 * i);     q[0] = z; q[1] = z;
    q = (uint4*)(o.body_hash + 32 * i);  q[0] = z; q[1] = z;
    q = (uint4*)(o.vrf_out + 64 * i);    for (int k = 0; k < 4; k++) q[k] = z;
    q = (uint4*)(o.ocert_sig + 64 * i);  for (int k = 0; k < 4; k++) q[k] = z;
    q = (uint4*)(o.vrf_proof + 80 * i);  for (int k = 0; k < 5; k++) q[k] = z;
    q = (uint4*)(o.kes_sig + 448 * i);   for (int k = 0; k < 28; k++) q[k] = z;
  }
}

void launch_decode_praos(dim3 grid, dim3 block, hipStream_t stream, size_t n, const uint8_t* arena, uint64_t arena_len,
                         const uint64_t* hoff, const uint32_t* hlen, uint64_t* slot, uint8_t* cold_vk, uint8_t* vrf_vk,
                         uint8_t* vrf_out, uint8_t* vrf_proof, uint8_t* hot_vk, uint8_t* ocert_sig, uint8_t* kes_sig,
                         uint64_t* ocert_n, uint64_t* ocert_c0, uint64_t* body_off, uint32_t* body_len,
                         uint8_t* signed_body, uint64_t* block_no, uint8_t* prev_hash, uint8_t* prev_genesis,
                         uint32_t* body_size, uint8_t* body_hash, uint64_t* prot_major, uint64_t* prot_minor,
                         uint8_t* header_hash, uint16_t* status, int allow_tp, uint32_t stride, uint8_t* lead_out,
                         uint8_t* lead_proof, size_t i0) {
  DecOut o{slot,     cold_vk,   vrf_vk,      vrf_out,  vrf_proof, hot_vk,       ocert_sig, kes_sig,
           ocert_n,  ocert_c0,  body_off,    body_len, signed_body, block_no,   prev_hash, prev_genesis,
           body_size, body_hash, prot_major, prot_minor, header_hash, status, lead_out, lead_proof};
  hipLaunchKernelGGL(k_decode_praos, grid, block, 0, stream, i0, n, arena, arena_len, hoff, hlen, o, allow_tp, stride);
}
