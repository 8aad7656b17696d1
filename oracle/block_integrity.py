"""CPU restatement of the ImmutableDB block-integrity batch.

TEST INFRASTRUCTURE ONLY: imported by tests/ as the checker of the GPU path
(k_block.hip + praos_verify_block_integrity).  The product path never imports it.

What it restates:
  * verifyBlockIntegrity spkp blk = verifyHeaderIntegrity spkp hdr && blockMatchesHeader hdr blk
    (ouroboros-consensus-cardano/src/shelley/Ouroboros/Consensus/Shelley/Ledger/Integrity.hs:14-20).
  * verifyHeaderIntegrity for Praos (Shelley/Protocol/Praos.hs:84-101): KES.verifySignedKES
    with t = kp - c0 when kp >= c0, else 0 (kp = slot `div` spkp); no OCert/VRF checks.
  * blockMatchesHeader (Shelley/Ledger/Block.hs:150-158): SL.hashTxSeq txs == header body hash.
    hashTxSeq is cardano-ledger's (not vendored): for the segregated-witness TxSeq the hash is
    Blake2b-256 over the concatenated Blake2b-256 hashes of the stored bytes of each segment
    (bodies, witnesses, auxiliary data[, invalid-tx indices]); Shelley..Mary have 3 segments,
    Alonzo onward 4.  Pinned: the formula reproduces the body hash of every golden block
    (golden/cardano/disk/Block_{Shelley,Allegra,Mary,Alonzo,Babbage,Conway}, golden/shelley/disk/Block;
    tests/test_block_oracle.py).
  * verifyHeaderIntegrity for TPraos (Shelley/Protocol/TPraos.hs:59-76): the same KES check
    (t = kp - c0 when kp >= c0, else 0) over the 15-field BHBody.
  * The on-disk Cardano block is the HardForkBlock wrapper [eraTag, block] (golden files); the
    Shelley-family block is [header, seg_1 .. seg_k].  Era tags: Shelley 2, Allegra 3, Mary 4
    (3 segments, TPraos headers), Alonzo 5 (4 segments, TPraos), Babbage 6, Conway 7 (4
    segments, Praos headers).  Headers are decoded by oracle/cbor_header.py (same rules as
    k_decode.hip).

Restated decode rules (parity unpinned beyond the golden blocks -- the real segment decoders
are the ledger's): a block is either [eraTag, [header, s1..sk]] with eraTag in 2..7, k = 3 for
tags 2-4 and 4 for tags 5-7, the header's body a 15-field BHBody for tags 2-5 and a 10-field
HeaderBody for 6-7; or an unwrapped [header, s1..s3] / [header, s1..s4] with either header
kind; every segment must be ONE well-formed CBOR
item (definite or indefinite lengths, tags, simple values; indefinite strings made of definite
chunks of the same major type; at most MAX_INDEF nested indefinite items); no bytes may follow
the block item.  Anything else sets BLK_DECODE and nothing else.

Result bits per block: 0 = intact; BLK_DECODE, BLK_KES (header integrity false), BLK_BODY_HASH
(body does not match header); KES and body hash are reported independently.
"""
import hashlib

import cbor_header as ch
import oracle as orc

BLK_DECODE = 0x01
BLK_KES = 0x02
BLK_BODY_HASH = 0x04
MAX_INDEF = 16
PRAOS_ERAS = (6, 7)
TPRAOS_ERAS = (2, 3, 4, 5)


def _b2b(m):
    return hashlib.blake2b(m, digest_size=32).digest()


class _Bad(Exception):
    pass


def _head(buf, p, end):
    """(major, info, arg, next) of the item head at p; arg None = indefinite."""
    if p >= end:
        raise _Bad
    ib = buf[p]
    p += 1
    mt, ai = ib >> 5, ib & 31
    if ai < 24:
        return mt, ai, ai, p
    if ai <= 27:
        nb = 1 << (ai - 24)
        if nb > end - p:
            raise _Bad
        return mt, ai, int.from_bytes(buf[p:p + nb], "big"), p + nb
    if ai == 31 and mt in (2, 3, 4, 5, 7):
        return mt, ai, None, p
    raise _Bad  # 28..30 reserved; indefinite 0/1/6


def cbor_skip(buf, p, end):
    """End offset of the single CBOR item at p (within [p, end)); raises _Bad."""
    need = 1
    stack = []  # (saved need, kind): kind 0 = indefinite container, 2/3 = indefinite string
    BIG = 1 << 62
    while need or stack:
        if p >= end:
            raise _Bad
        if buf[p] == 0xFF:
            if not stack or need != BIG:
                raise _Bad
            need, _ = stack.pop()
            p += 1
            continue
        mt, ai, arg, p = _head(buf, p, end)
        if stack and need == BIG and stack[-1][1] in (2, 3):
            if mt != stack[-1][1] or arg is None:
                raise _Bad  # chunk of an indefinite string
        if need != BIG:  # at an indefinite level (need == BIG) items are counted by the break
            need -= 1
        if mt in (0, 1):
            pass
        elif mt in (2, 3):
            if arg is None:
                if len(stack) == MAX_INDEF:
                    raise _Bad
                stack.append((need, mt))
                need = BIG
            else:
                if arg > end - p:
                    raise _Bad
                p += arg
        elif mt in (4, 5):
            if arg is None:
                if len(stack) == MAX_INDEF:
                    raise _Bad
                stack.append((need, 0))
                need = BIG
            else:
                k = arg * (2 if mt == 5 else 1)
                if k > end - p:
                    raise _Bad  # every item takes >= 1 byte
                need += k
        elif mt == 6:
            need += 1
        else:  # 7: simple / float; break handled above
            if ai == 24 and arg < 32:
                raise _Bad
    return p


def _body_arity(buf, p, end):
    """Arity of the header body at p (the header is [body, kesSig])."""
    mt, _, arg, q = _head(buf, p, end)
    if mt != 4 or arg != 2:
        raise _Bad
    mt, _, arg, _ = _head(buf, q, end)
    if mt != 4 or arg is None:
        raise _Bad
    return arg


def split_block(buf, off, length):
    """-> (ok, header_off, header_len, [(seg_off, seg_len)])."""
    if off > len(buf) or length > len(buf) - off:
        return False, 0, 0, []
    end = off + length
    try:
        mt, ai, arg, p = _head(buf, off, end)
        if mt != 4 or arg is None:
            raise _Bad
        arity = None
        if arg == 2:
            mt2, _, tag, q = _head(buf, p, end)
            if mt2 != 0 or tag not in PRAOS_ERAS + TPRAOS_ERAS:
                raise _Bad
            mt, ai, arg, p = _head(buf, q, end)
            if mt != 4 or arg != (4 if tag in (2, 3, 4) else 5):
                raise _Bad
            arity = 15 if tag in TPRAOS_ERAS else 10
        elif arg not in (4, 5):
            raise _Bad
        if arity is not None and _body_arity(buf, p, end) != arity:
            raise _Bad
        spans = []
        for _ in range(arg):
            q = cbor_skip(buf, p, end)
            spans.append((p, q - p))
            p = q
        if p != end:
            raise _Bad
    except _Bad:
        return False, 0, 0, []
    (ho, hl), segs = spans[0], spans[1:]
    return True, ho, hl, segs


def hash_tx_seq(buf, segs):
    return _b2b(b"".join(_b2b(bytes(buf[o:o + n])) for o, n in segs))


def verify_block_integrity(buf, off, length, spkp):
    """-> (bits, computed body hash or zeros)."""
    ok, ho, hl, segs = split_block(buf, off, length)
    if not ok:
        return BLK_DECODE, bytes(32)
    d = ch.decode_header(buf, ho, hl, allow_tpraos=True)
    if d["status"] & ch.DEC_FAIL:
        return BLK_DECODE, bytes(32)
    f = d["fields"]
    bits = 0
    kp = f["slot"] // spkp
    t = kp - f["c0"] if kp >= f["c0"] else 0
    if orc.kes_verify(f["hot_vk"], t, d["signed"], f["kes_sig"]) != 0:
        bits |= BLK_KES
    bh = hash_tx_seq(buf, segs)
    if bh != f["body_hash"]:
        bits |= BLK_BODY_HASH
    return bits, bh
