// k_block.hip -- ImmutableDB block-integrity batch.
//
// verifyBlockIntegrity spkp blk = verifyHeaderIntegrity spkp hdr && blockMatchesHeader hdr blk
// (Shelley/Ledger/Integrity.hs:14-20).  The header half is k_kes in header mode
// (t = max(0, kp - c0), Shelley/Protocol/Praos.hs:84-101 and TPraos.hs:59-76) over the
// k_decode SoA (Praos HeaderBody or TPraos BHBody);
// this module supplies the block half:
//   k_block_split   one lane per stored block: the era wrapper [eraTag, [header, s1..sk]]
//                   -- Shelley 2, Allegra 3, Mary 4 (k = 3, TPraos header), Alonzo 5 (k = 4,
//                   TPraos), Babbage 6, Conway 7 (k = 4, Praos header) -- or a bare
//                   [header, s1..s3|s4] with either header kind; every segment must be one
//                   well-formed CBOR item.  Emits the header span (k_decode's input) and
//                   the segment spans, segment-major ([k][i]).
//   k_seg_hash      one lane per (segment k, block i), segment-major so a workgroup hashes
//                   the same segment kind of 256 neighbouring blocks (similar lengths):
//                   Blake2b-256 of the stored segment bytes, message blocks staged through
//                   LDS by coalesced cooperative loads.
//   k_block_join    one lane per block: hashTxSeq = Blake2b-256 of the concatenated segment
//                   hashes (one 96/128-byte compression), compared with hbBodyHash
//                   (blockMatchesHeader, Shelley/Ledger/Block.hs:150-158); folds the KES
//                   and decode bits into the result byte.
// CPU restatement: oracle/block_integrity.py (same decode rules, same result bits).
//
// Roofline: HBM-bound in principle (every block byte is read once by k_seg_hash, the
// header bytes once more by k_decode), but Blake2b is ~12 rounds x 8 G per 128 bytes,
// ~1.4k int ops per 128 B, so at 8 TB/s the integer rate (~39 T ops/s) is the bound:
// ~3.6 TB/s of block bytes.  The KES verify per block dominates for small blocks.
#include "kcommon.hpp"
#include "arena.hpp"

namespace {

constexpr uint32_t MAX_INDEF = 16;          // nested indefinite items (oracle MAX_INDEF)
constexpr uint64_t BIG = 1ull << 62;        // "at an indefinite level" marker for `need`

struct Cur {
  const uint8_t* __restrict__ a;
  uint64_t p, end;
  bool ok;
};

// item head: major type, additional info, argument (indef = true for ai 31)
__device__ __forceinline__ bool head(Cur& c, uint32_t& mt, uint32_t& ai, uint64_t& arg, bool& indef) {
  if (c.p >= c.end) return false;
  const uint32_t ib = c.a[c.p++];
  mt = ib >> 5;
  ai = ib & 31u;
  indef = false;
  if (ai < 24) { arg = ai; return true; }
  if (ai <= 27) {
    const uint32_t nb = 1u << (ai - 24);
    if (nb > c.end - c.p) return false;
    uint64_t v = 0;
    for (uint32_t k = 0; k < nb; k++) v = (v << 8) | c.a[c.p + k];
    c.p += nb;
    arg = v;
    return true;
  }
  if (ai == 31 && (mt == 2 || mt == 3 || mt == 4 || mt == 5 || mt == 7)) { indef = true; arg = 0; return true; }
  return false;   // 28..30 reserved; indefinite uint / nint / tag
}

// advance c.p past ONE well-formed CBOR item (oracle block_integrity.cbor_skip)
__device__ bool cbor_skip(Cur& c) {
  uint64_t need = 1;
  uint64_t st_need[MAX_INDEF];
  uint8_t st_kind[MAX_INDEF];
  uint32_t sp = 0;
  while (need || sp) {
    if (c.p >= c.end) return false;
    if (c.a[c.p] == 0xFF) {
      if (!sp || need != BIG) return false;
      need = st_need[--sp];
      c.p++;
      continue;
    }
    uint32_t mt, ai;
    uint64_t arg;
    bool indef;
    if (!head(c, mt, ai, arg, indef)) return false;
    if (sp && need == BIG && st_kind[sp - 1] != 0 && (mt != st_kind[sp - 1] || indef)) return false;
    if (need != BIG) need -= 1;
    if (mt == 2 || mt == 3) {
      if (indef) {
        if (sp == MAX_INDEF) return false;
        st_need[sp] = need; st_kind[sp] = (uint8_t)mt; sp++;
        need = BIG;
      } else {
        if (arg > c.end - c.p) return false;
        c.p += arg;
      }
    } else if (mt == 4 || mt == 5) {
      if (indef) {
        if (sp == MAX_INDEF) return false;
        st_need[sp] = need; st_kind[sp] = 0; sp++;
        need = BIG;
      } else {
        const uint64_t k = mt == 5 ? 2 * arg : arg;
        if (arg > c.end - c.p || k > c.end - c.p) return false;   // each item takes >= 1 byte
        need += k;
      }
    } else if (mt == 6) {
      need += 1;
    } else if (mt == 7) {
      if (ai == 24 && arg < 32) return false;
    }
  }
  return true;
}

__global__ void __launch_bounds__(NT) k_block_split(size_t n, const uint8_t* __restrict__ arena, uint64_t arena_len,
                                                    uint64_t* __restrict__ off_io, uint32_t* __restrict__ len_io,
                                                    uint64_t* __restrict__ seg_off, uint32_t* __restrict__ seg_len,
                                                    uint8_t* __restrict__ nseg, uint8_t* __restrict__ status) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t off = off_io[i];
  const uint32_t len = len_io[i];
  bool ok = off <= arena_len && len <= arena_len - off;
  Cur c{arena, off, off + len, true};
  uint64_t sp_off[5];
  uint32_t sp_len[5];
  uint32_t nitems = 0;
  if (ok) {
    uint32_t mt, ai;
    uint64_t arg;
    bool indef;
    ok = head(c, mt, ai, arg, indef) && mt == 4 && !indef;
    bool wrapped = false;
    uint64_t arity = 0;   // header body arity the era tag demands (0: bare block, either)
    if (ok && arg == 2) {
      uint64_t tag;
      ok = head(c, mt, ai, tag, indef) && mt == 0 && tag >= 2 && tag <= 7;        // Shelley .. Conway
      ok = ok && head(c, mt, ai, arg, indef) && mt == 4 && !indef && arg == (tag <= 4 ? 4u : 5u);
      arity = tag <= 5 ? 15 : 10;                                                // TPraos / Praos header
      wrapped = true;
    }
    ok = ok && (wrapped || arg == 4 || arg == 5);
    if (ok && arity) {   // the header is [body, kesSig]: peek at the body's arity
      Cur h{arena, c.p, c.end, true};
      uint64_t a2, ab;
      ok = head(h, mt, ai, a2, indef) && mt == 4 && !indef && a2 == 2 && head(h, mt, ai, ab, indef) && mt == 4 &&
           !indef && ab == arity;
    }
    if (ok) {
      nitems = (uint32_t)arg;
      for (uint32_t k = 0; k < nitems && ok; k++) {
        const uint64_t s = c.p;
        ok = cbor_skip(c);
        sp_off[k] = s;
        sp_len[k] = (uint32_t)(c.p - s);
      }
      ok = ok && c.p == c.end;
    }
  }
  if (!ok) {
    off_io[i] = 0;
    len_io[i] = 0;   // k_decode then reports SYNTAX; k_block_join reports DECODE
    nseg[i] = 0;
    status[i] = 1;
    return;
  }
  off_io[i] = sp_off[0];
  len_io[i] = sp_len[0];
  for (uint32_t k = 1; k < 5; k++) {
    seg_off[(size_t)(k - 1) * n + i] = k < nitems ? sp_off[k] : 0;
    seg_len[(size_t)(k - 1) * n + i] = k < nitems ? sp_len[k] : 0;
  }
  nseg[i] = (uint8_t)(nitems - 1);
  status[i] = 0;
}

// Segment hashes with the message blocks staged through LDS: a lane streaming
// its own segment with per-lane 8-byte loads touches 64 different cache lines
// per instruction and the L1 thrashes (each 128-byte line is re-fetched from L2
// for every word).  Here the workgroup loads the next 128-byte block of all 256
// segments cooperatively -- 8 lanes x 16 bytes per block, whole lines per
// instruction -- into LDS (stride 17 words: 2-way bank conflicts at most), and
// each lane compresses its own block from LDS.  The loop runs to the
// workgroup's longest segment; segment-major order keeps neighbours similar.
constexpr uint32_t SEG_STRIDE = 17;   // u64 words per staged block (16 + 1 pad)

__global__ void __launch_bounds__(NT) k_seg_hash(size_t n, const uint8_t* __restrict__ arena,
                                                 const uint64_t* __restrict__ seg_off,
                                                 const uint32_t* __restrict__ seg_len, const uint8_t* __restrict__ nseg,
                                                 uint8_t* __restrict__ seg_hash) {
  __shared__ uint64_t sm[NT * SEG_STRIDE];
  __shared__ uint64_t s_pos[NT];
  __shared__ uint32_t s_len[NT];
  __shared__ uint32_t s_max;
  const uint32_t t = threadIdx.x;
  const size_t j = (size_t)blockIdx.x * NT + t;
  bool act = false;
  uint64_t pos = 0;
  uint32_t len = 0;
  if (j < 4 * n) {
    const size_t k = j / n, i = j - k * n;
    if (k < nseg[i]) { act = true; pos = seg_off[j]; len = seg_len[j]; }
  }
  const uint32_t nblk = act ? (len == 0 ? 1u : (len + 127u) / 128u) : 0u;
  s_pos[t] = pos;
  s_len[t] = len;
  if (t == 0) s_max = 0;
  __syncthreads();
  if (nblk) atomicMax(&s_max, nblk);
  __syncthreads();
  const uint32_t nb = s_max;
  uint64_t h[8];
#pragma unroll
  for (int w = 0; w < 8; w++) h[w] = B2B_IV[w];
  h[0] ^= 0x01010000ULL ^ 32u;
  for (uint32_t b = 0; b < nb; b++) {
#pragma unroll
    for (uint32_t r = 0; r < 8; r++) {
      const uint32_t c = r * NT + t, owner = c >> 3, part = c & 7u;
      const uint32_t olen = s_len[owner];
      const uint64_t o = (uint64_t)b * 128 + 16 * part;
      uint64_t w0 = 0, w1 = 0;
      if (o < olen) {
        const uint64_t opos = s_pos[owner];
        w0 = ld64u(arena, opos + o);
        if (o + 8 < olen) w1 = ld64u(arena, opos + o + 8);
      }
      sm[owner * SEG_STRIDE + 2 * part] = w0;
      sm[owner * SEG_STRIDE + 2 * part + 1] = w1;
    }
    __syncthreads();
    if (b < nblk) {
      uint64_t m[16];
      const uint64_t base = (uint64_t)b * 128;
#pragma unroll
      for (int k = 0; k < 16; k++) {
        const uint64_t o = base + 8 * k;
        uint64_t w = o < len ? sm[t * SEG_STRIDE + k] : 0;
        if (o < len && len - o < 8) w &= (1ull << (8 * (len - o))) - 1;
        m[k] = w;
      }
      const bool last = b + 1 == nblk;
      b2b_compress(h, m, last ? (uint64_t)len : base + 128, last);
    }
    __syncthreads();
  }
  if (!act) return;
  uint32_t out[8];
#pragma unroll
  for (int w = 0; w < 4; w++) { out[2 * w] = (uint32_t)h[w]; out[2 * w + 1] = (uint32_t)(h[w] >> 32); }
  store_words(seg_hash + 32 * j, out, 8);
}

__global__ void __launch_bounds__(NT) k_block_join(size_t n, const uint8_t* __restrict__ nseg,
                                                   const uint8_t* __restrict__ split_status,
                                                   const uint16_t* __restrict__ dec_status,
                                                   const uint16_t* __restrict__ kes_bits,
                                                   const uint8_t* __restrict__ seg_hash,
                                                   const uint8_t* __restrict__ body_hash,
                                                   uint8_t* __restrict__ result, uint8_t* __restrict__ calc_hash) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint4 z = make_uint4(0, 0, 0, 0);
  if (split_status[i] || (dec_status[i] & PRAOS_DEC_FAILED)) {
    result[i] = PRAOS_BLK_DECODE;
    ((uint4*)(calc_hash + 32 * i))[0] = z;
    ((uint4*)(calc_hash + 32 * i))[1] = z;
    return;
  }
  // hashTxSeq: Blake2b-256 of hash(s1) || ... || hash(sk), one 128-byte block
  const uint32_t k = nseg[i];
  uint64_t m[16];
#pragma unroll
  for (uint32_t s = 0; s < 4; s++) {
    const uint4* q = (const uint4*)(seg_hash + 32 * ((size_t)s * n + i));
    const uint4 a = s < k ? q[0] : z, b = s < k ? q[1] : z;
    m[4 * s + 0] = (uint64_t)a.x | ((uint64_t)a.y << 32);
    m[4 * s + 1] = (uint64_t)a.z | ((uint64_t)a.w << 32);
    m[4 * s + 2] = (uint64_t)b.x | ((uint64_t)b.y << 32);
    m[4 * s + 3] = (uint64_t)b.z | ((uint64_t)b.w << 32);
  }
  uint64_t h[8];
#pragma unroll
  for (int w = 0; w < 8; w++) h[w] = B2B_IV[w];
  h[0] ^= 0x01010000ULL ^ 32u;
  b2b_compress(h, m, 32ull * k, true);
  const uint4* e = (const uint4*)(body_hash + 32 * i);
  const uint4 e0 = e[0], e1 = e[1];
  const uint4 c0 = make_uint4((uint32_t)h[0], (uint32_t)(h[0] >> 32), (uint32_t)h[1], (uint32_t)(h[1] >> 32));
  const uint4 c1 = make_uint4((uint32_t)h[2], (uint32_t)(h[2] >> 32), (uint32_t)h[3], (uint32_t)(h[3] >> 32));
  ((uint4*)(calc_hash + 32 * i))[0] = c0;
  ((uint4*)(calc_hash + 32 * i))[1] = c1;
  const bool match = e0.x == c0.x && e0.y == c0.y && e0.z == c0.z && e0.w == c0.w && e1.x == c1.x &&
                     e1.y == c1.y && e1.z == c1.z && e1.w == c1.w;
  uint8_t r = 0;
  if (kes_bits[i] & (PRAOS_BIT_KES_MERKLE | PRAOS_BIT_KES_LEAF | PRAOS_BIT_INPUT)) r |= PRAOS_BLK_KES;
  if (!match) r |= PRAOS_BLK_BODY_HASH;
  result[i] = r;
}

}  // namespace

// ---- host launchers (kernels are only launchable from their own module)
void launch_block_split(dim3 grid, dim3 block, hipStream_t stream, size_t n, const uint8_t* arena,
                        uint64_t arena_len, uint64_t* off_io, uint32_t* len_io, uint64_t* seg_off, uint32_t* seg_len,
                        uint8_t* nseg, uint8_t* status) {
  hipLaunchKernelGGL(k_block_split, grid, block, 0, stream, n, arena, arena_len, off_io, len_io, seg_off, seg_len,
                     nseg, status);
}

void launch_seg_hash(dim3 grid, dim3 block, hipStream_t stream, size_t n, const uint8_t* arena,
                     const uint64_t* seg_off, const uint32_t* seg_len, const uint8_t* nseg, uint8_t* seg_hash) {
  hipLaunchKernelGGL(k_seg_hash, grid, block, 0, stream, n, arena, seg_off, seg_len, nseg, seg_hash);
}

void launch_block_join(dim3 grid, dim3 block, hipStream_t stream, size_t n, const uint8_t* nseg,
                       const uint8_t* split_status, const uint16_t* dec_status, const uint16_t* kes_bits,
                       const uint8_t* seg_hash, const uint8_t* body_hash, uint8_t* result, uint8_t* calc_hash) {
  hipLaunchKernelGGL(k_block_join, grid, block, 0, stream, n, nseg, split_status, dec_status, kes_bits, seg_hash,
                     body_hash, result, calc_hash);
}
