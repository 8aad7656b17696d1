"""Stored-block layout of a synthetic chain (db-synthesizer analogue).

Packs headers produced by ``Context.synthesize(..., body_len=0)`` (genuine
canonical HeaderBody CBOR, Praos/Header.hs:160-185) into the bytes an
ImmutableDB chunk file holds for empty Babbage blocks, and returns the
(offset, length) pairs its secondary index would give for the headers
(blockOffset + headerOffset, headerSize; ImmutableDB/Impl/Index/Secondary.hs:93-128):

    block  = [6, [header, [], [], {}, []]]        (HardForkBlock era tag 6 = Babbage)
    header = [body, kesSig]                       (HeaderRaw, Header.hs:201-210)

so the header of every block starts 3 bytes in, as in the reference's golden
``golden/cardano/disk/Block_Babbage``.  Vectorised with numpy: rows are grouped
by body length and scattered into the arena.
"""
import numpy as np

BLOCK_PREFIX = bytes([0x82, 0x06, 0x85])          # [6, [  (5-element Babbage block)
HEADER_PREFIX = bytes([0x82])                     # [body, kesSig]
SIG_HEAD = bytes([0x59, 0x01, 0xC0])              # bytes(448)
BLOCK_SUFFIX = bytes([0x80, 0x80, 0xA0, 0x80])    # [], [], {}, []
HEADER_OFFSET = len(BLOCK_PREFIX)
OVERHEAD = len(BLOCK_PREFIX) + len(HEADER_PREFIX) + len(SIG_HEAD) + 448 + len(BLOCK_SUFFIX)


def pack_chunk(H, era_tag=6):
    """H: synthesize() output with CBOR bodies.  Returns (arena u8[], off u64[n], len u32[n]).
    era_tag: the HardForkBlock era of the stored blocks (6 Babbage; 5 Alonzo for TPraos
    headers from praos_synthesize_tpraos -- the same 4 segments)."""
    n = len(H["slot"])
    bl = H["body_len"].astype(np.int64)
    blk = bl + OVERHEAD
    start = np.zeros(n, np.int64)
    if n > 1:
        start[1:] = np.cumsum(blk[:-1])
    total = int(blk.sum()) if n else 0
    arena = np.zeros(total, np.uint8)
    body = H["body_bytes"]
    boff = H["body_off"].astype(np.int64)
    for L in np.unique(bl):
        rows = np.nonzero(bl == L)[0]
        for r0 in range(0, len(rows), 65536):
            R = rows[r0:r0 + 65536]
            m = len(R)
            bodies = body[boff[R][:, None] + np.arange(L)[None, :]]
            rec = np.concatenate([
                np.broadcast_to(np.frombuffer(bytes([0x82, era_tag, 0x85]) + HEADER_PREFIX, np.uint8), (m, 4)), bodies,
                np.broadcast_to(np.frombuffer(SIG_HEAD, np.uint8), (m, 3)), H["kes_sig"][R],
                np.broadcast_to(np.frombuffer(BLOCK_SUFFIX, np.uint8), (m, 4))], axis=1)
            arena[start[R][:, None] + np.arange(L + OVERHEAD)[None, :]] = rec
    off = (start + HEADER_OFFSET).astype(np.uint64)
    length = (bl + OVERHEAD - len(BLOCK_PREFIX) - len(BLOCK_SUFFIX)).astype(np.uint32)
    return arena, off, length


SEG_FIXED = (bytes([0x80]), bytes([0xA0]), bytes([0x80]))   # witnesses [], aux {}, invalid txs []


def tx_segment(payload: bytes) -> bytes:
    """Synthetic tx-bodies segment: [payload] as one byte string (4-byte length head)."""
    return bytes([0x81, 0x5A]) + len(payload).to_bytes(4, "big") + payload


def hash_tx_seq(segments):
    """hashTxSeq of a segregated-witness TxSeq: Blake2b-256 over the Blake2b-256 of each
    stored segment (cardano-ledger; pinned against the reference's golden blocks in
    tests/test_block_oracle.py)."""
    import hashlib

    def b2b(m):
        return hashlib.blake2b(m, digest_size=32).digest()
    return b2b(b"".join(b2b(s) for s in segments))


def pack_blocks(H, payloads):
    """Whole stored Babbage blocks [6, [header, [payload], [], {}, []]] from synthesize()
    output with CBOR bodies whose hbBodyHash is hash_tx_seq of these segments.
    Returns (arena u8[], off u64[n], len u32[n]) of the BLOCKS (what
    praos_verify_block_integrity takes)."""
    n = len(H["slot"])
    parts, off, ln, pos = [], np.zeros(n, np.uint64), np.zeros(n, np.uint32), 0
    body = H["body_bytes"]
    for i in range(n):
        bo, bl = int(H["body_off"][i]), int(H["body_len"][i])
        blk = b"".join([BLOCK_PREFIX, HEADER_PREFIX, body[bo:bo + bl].tobytes(), SIG_HEAD,
                        H["kes_sig"][i].tobytes(), tx_segment(payloads[i]), *SEG_FIXED])
        parts.append(blk)
        off[i] = pos
        ln[i] = len(blk)
        pos += len(blk)
    return np.frombuffer(b"".join(parts), np.uint8), off, ln
