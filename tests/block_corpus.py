"""Stored-block corpora for the block-integrity tests (test infrastructure).

Blocks are built with the oracle's encoders and signers (oracle/cbor_header.py,
oracle/oracle.py): the header's body hash is hashTxSeq of the block's own
segments and its KES signature is made over the canonical body at
t = max(0, kp - c0), so an unmutated block is intact (Integrity.hs:14-20).
Mutations cover each failure of verifyBlockIntegrity and the envelope/segment
decode edge cases of oracle/block_integrity.py."""
import block_integrity as bi
import cbor_header as ch
import oracle as orc
from helpers import rbytes

H = ch._head


def rand_item(r, depth=0):
    """A random well-formed CBOR item (definite/indefinite, tags, floats, simple)."""
    k = r.randrange(10 if depth < 4 else 4)
    if k == 0:
        return H(0, r.getrandbits(r.choice([3, 8, 16, 40, 64])))
    if k == 1:
        return H(1, r.getrandbits(r.choice([4, 20])))
    if k == 2:
        n = r.choice([0, 5, 28, 32, 64, 200, 1500])
        return H(2, n) + rbytes(r, n)
    if k == 3:
        return r.choice([b"\xf4", b"\xf5", b"\xf6", b"\xf7", b"\xf8\x20", b"\xf9\x3c\x00",
                         b"\xfa\x3f\x80\x00\x00", b"\xfb" + bytes(8)])
    if k in (4, 5):
        n = r.randrange(5)
        items = b"".join(rand_item(r, depth + 1) for _ in range(n))
        return (b"\x9f" + items + b"\xff") if k == 5 else H(4, n) + items
    if k == 6:
        n = r.randrange(4)
        kv = b"".join(rand_item(r, depth + 1) + rand_item(r, depth + 1) for _ in range(n))
        return (b"\xbf" + kv + b"\xff") if r.random() < 0.3 else H(5, n) + kv
    if k == 7:
        return H(6, r.choice([24, 121, 258, 1 << 20])) + rand_item(r, depth + 1)
    if k == 8:  # indefinite byte / text string of definite chunks
        mt = r.choice([2, 3])
        chunks = b"".join(H(mt, m) + (rbytes(r, m) if mt == 2 else b"a" * m)
                          for m in (r.randrange(40) for _ in range(r.randrange(4))))
        return bytes([(mt << 5) | 31]) + chunks + b"\xff"
    n = r.randrange(6)
    return H(4, n) + b"".join(rand_item(r, depth + 1) for _ in range(n))


def rand_segments(r, big=False, pad=0):
    """[tx bodies, witnesses, auxiliary data, invalid txs] (Alonzo+ TxSeq); pad > 0 adds one
    tx body carrying a pad-byte string (mainnet-sized blocks for the bench)."""
    ntx = r.randrange(8 if not big else 60)
    if pad:
        return [H(4, ntx + 1) + H(5, 1) + H(0, 0) + H(2, pad) + rbytes(r, pad) + b"".join(
                    H(5, 1) + H(0, 0) + rand_item(r) for _ in range(ntx)),
                H(4, 1) + H(2, 100) + rbytes(r, 100), H(5, 0), H(4, 0)]
    bodies = H(4, ntx) + b"".join(H(5, 2) + H(0, 0) + rand_item(r) + H(0, 2) + H(0, r.getrandbits(20))
                                  for _ in range(ntx))
    wits = H(4, ntx) + b"".join(rand_item(r) for _ in range(ntx))
    aux = H(5, 1) + H(0, 0) + rand_item(r) if r.random() < 0.5 else H(5, 0)
    inval = H(4, 0)
    return [bodies, wits, aux, inval]


def make_block(r, spkp, era=6, slot=None, c0=None, big=False, wrapped=True, pad=0):
    """-> (block bytes, header fields, KES seed).  era 2..5: a TPraos block (15-field
    BHBody; 3 segments for Shelley/Allegra/Mary, 4 for Alonzo); 6/7: Praos."""
    tp = era in bi.TPRAOS_ERAS
    segs = rand_segments(r, big, pad)
    if era in (2, 3, 4):
        segs = segs[:3]
    bh = bi._b2b(b"".join(bi._b2b(s) for s in segs))
    seed = rbytes(r, 32)
    slot = r.getrandbits(24) if slot is None else slot
    kp = slot // spkp
    if c0 is None:
        c0 = max(0, kp - r.randrange(62))
    t = kp - c0 if kp >= c0 else 0
    f = {"block_no": r.getrandbits(20), "slot": slot, "prev_hash": rbytes(r, 32), "cold_vk": rbytes(r, 32),
         "vrf_vk": rbytes(r, 32), "vrf_out": rbytes(r, 64), "vrf_proof": rbytes(r, 80),
         "body_size": sum(map(len, segs)), "body_hash": bh, "hot_vk": orc.kes_vk(seed), "n": r.getrandbits(8),
         "c0": c0, "ocert_sig": rbytes(r, 64), "prot_major": 9 if not tp else 2 + (era - 2), "prot_minor": 0}
    if tp:
        f["leader_out"], f["leader_proof"] = rbytes(r, 64), rbytes(r, 80)
    body = ch.encode_tpraos_body(f) if tp else ch.encode_body(f)
    kes = orc.kes_sign(seed, min(t, 63), body)  # t > 63: verification must reject
    hdr = H(4, 2) + body + H(2, len(kes)) + kes
    inner = H(4, 1 + len(segs)) + hdr + b"".join(segs)
    blk = (H(4, 2) + H(0, era) + inner) if wrapped else inner
    return blk, f, seed


def _seg_start(blk):
    """Offset of the first segment (after the header) of a wrapped block."""
    _, _, _, p = bi._head(blk, 0, len(blk))
    _, _, _, p = bi._head(blk, p, len(blk))
    _, _, _, p = bi._head(blk, p, len(blk))
    return bi.cbor_skip(blk, p, len(blk))


MUTATIONS = [
    "intact", "seg_byte", "kes_sig", "truncated", "trailing", "era_5", "bare_4", "bad_break",
    "reserved_ai", "deep_indef", "header_trailing", "aux_swap", "empty",
]


def mutate(blk, f, r, kind):
    """The `kind` mutation of a wrapped intact block -> bytes."""
    b = bytearray(blk)
    s0 = _seg_start(blk)
    if kind == "intact":
        return bytes(b)
    if kind == "seg_byte":  # last segment [] -> [0]: still well-formed, body hash differs
        return bytes(b[:-1]) + b"\x81\x00"
    if kind == "kes_sig":
        i = blk.rfind(b"\x59\x01\xc0", 0, s0) + 3 + r.randrange(448)
        b[i] = (b[i] + 1) & 0xFF
        return bytes(b)
    if kind == "truncated":
        return bytes(b[:-1 - r.randrange(min(40, len(b) - 1))])
    if kind == "trailing":
        return bytes(b) + b"\x00"
    if kind == "era_5":
        b[1] = 5
        return bytes(b)
    if kind == "bare_4":  # unwrapped [header, 3 segments]: decodes, hash over 3 segments differs
        return H(4, 4) + bytes(b[3:-1])
    if kind == "bad_break":
        return bytes(b[:-1]) + b"\xff"
    if kind == "reserved_ai":
        return bytes(b[:-1]) + b"\x1c"
    if kind == "deep_indef":
        k = bi.MAX_INDEF + 1
        return bytes(b[:-1]) + b"\x9f" * k + b"\xff" * k
    if kind == "header_trailing":  # header item now [body, sig, 0]: header decode fails
        i = 3
        b[i] = 0x83
        return bytes(b[:s0]) + b"\x00" + bytes(b[s0:])
    if kind == "aux_swap":  # witnesses <-> aux data: well-formed, segment hashes swap places
        p = s0
        spans = []
        for _ in range(4):
            q = bi.cbor_skip(blk, p, len(blk))
            spans.append(blk[p:q])
            p = q
        return bytes(b[:s0]) + spans[0] + spans[2] + spans[1] + spans[3]
    if kind == "empty":
        return b""
    raise ValueError(kind)


def expected_kind(kind):
    return {"intact": 0, "seg_byte": bi.BLK_BODY_HASH, "kes_sig": bi.BLK_KES, "bare_4": bi.BLK_BODY_HASH,
            "aux_swap": bi.BLK_BODY_HASH}.get(kind, bi.BLK_DECODE)
