"""CPU restatement of stored Praos header decoding.

TEST INFRASTRUCTURE ONLY: imported by tests/ and bench.py's self-check as the
checker of the GPU decoder (k_decode.hip).  The product path never imports it.

What it restates (reference: ouroboros-consensus-protocol/src/ouroboros-consensus-
protocol/Ouroboros/Consensus/Protocol/Praos/Header.hs):
  * DecCBOR (Annotator (Header c)) :228-231 -- a header is the CBOR item
    HeaderRaw = [body, kesSig] (:201-210, decodeSignedKES = 448 raw bytes) and
    keeps its stored bytes; headerHash (:147-151) hashes exactly those bytes
    (Blake2b-256, Plain.ToCBOR = encodePreEncoded bytes, :212-213).
  * DecCBOR (HeaderBody) :187-199 / EncCBOR :160-185 -- the 10-field record
    [blockNo, slotNo, prevHash, vk, vrfVk, [vrfOut, vrfProof], bodySize,
     bodyHash, [hotVk, n, c0, sigma], [protMajor, protMinor]].
  * SignableRepresentation HeaderBody :90-94 -- the KES message is the
    RE-serialisation `serialize' hb`, i.e. the canonical (shortest-head,
    definite-length) encoding of the decoded fields, not the stored slice.
    cborg's plain decoders accept non-shortest integer/length heads, so a
    stored body may be non-canonical; the signed bytes are then re-encoded.

TPraos (Shelley..Alonzo) headers, for the block-integrity path: BHeader = [BHBody,
kesSig] with the 15-field BHBody of cardano-protocol-tpraos (BHeader.hs encodeBHBody,
not vendored -- restated from its published encoder and pinned by the golden
Block_{Shelley,Allegra,Mary,Alonzo} files): [blockNo, slotNo, prevHash, vk, vrfVk,
[etaOut, etaProof], [leaderOut, leaderProof], bodySize, bodyHash, hotVk, n, c0, sigma,
protMajor, protMinor] (OCert and ProtVer inlined as groups).  Its KES message is the
same canonical re-serialisation (SignableRepresentation BHBody = serialize').

Status bits (first failure only; NONCANONICAL is informational and only set on
success).  Restated edge rules, parity unpinned (the decoders live in
cardano-binary / cardano-ledger-binary, not vendored): indefinite-length items
and tags are reported UNSUPPORTED (no encoder of the reference emits them),
bodySize must fit Word32 (decodeWord32), every fixed-size field must have its
exact length (rawDeserialise*), prevHash is null (GenesisHash) or 32 bytes.
"""
import hashlib

DEC_RANGE = 0x01
DEC_SYNTAX = 0x02
DEC_SIZE = 0x04
DEC_UNSUPPORTED = 0x08
DEC_TRAILING = 0x10
DEC_NONCANONICAL = 0x20
DEC_OVERFLOW = 0x40
# DecCBOR Version (cardano-ledger-binary, not vendored) rejects a ProtVer major above
# maxVersion; 9 (Conway) at the CHaP index-state of the reference -- parity unpinned.
MAX_PROT_MAJOR = 9
DEC_FAIL = 0x5F               # every bit but NONCANONICAL

SIGNED_STRIDE = 448           # max canonical body = 447 bytes
TP_SIGNED_STRIDE = 640        # max canonical TPraos BHBody = 598 bytes


class _Fail(Exception):
    def __init__(self, bit):
        self.bit = bit


class _R:
    def __init__(self, buf, pos, end):
        self.b, self.pos, self.end = buf, pos, end
        self.canon = True

    def byte(self):
        if self.pos >= self.end:
            raise _Fail(DEC_SYNTAX)
        v = self.b[self.pos]
        self.pos += 1
        return v

    def head(self):
        ib = self.byte()
        mt, ai = ib >> 5, ib & 31
        if ai < 24:
            return mt, ai
        if ai <= 27:
            nb = 1 << (ai - 24)
            v = 0
            for _ in range(nb):
                v = (v << 8) | self.byte()
            if v < (24, 256, 65536, 1 << 32)[ai - 24]:
                self.canon = False
            return mt, v
        if ai == 31:
            raise _Fail(DEC_UNSUPPORTED)
        raise _Fail(DEC_SYNTAX)

    def expect(self, mt_want):
        mt, v = self.head()
        if mt == 6:
            raise _Fail(DEC_UNSUPPORTED)
        if mt != mt_want:
            raise _Fail(DEC_SYNTAX)
        return v

    def array(self, n):
        if self.expect(4) != n:
            raise _Fail(DEC_SYNTAX)

    def uint(self, limit=(1 << 64) - 1):
        v = self.expect(0)
        if v > limit:
            raise _Fail(DEC_OVERFLOW)
        return v

    def bytes_fixed(self, n):
        ln = self.expect(2)
        if ln != n:
            raise _Fail(DEC_SIZE)
        if self.pos + n > self.end:
            raise _Fail(DEC_SYNTAX)
        v = bytes(self.b[self.pos:self.pos + n])
        self.pos += n
        return v


def _head(mt, v, wide=False):
    """Shortest-form CBOR head (cborg's encoders); wide=True gives the 8-byte (or
    for lengths 2-byte) non-canonical form that cborg's decoders still accept."""
    if wide:
        return bytes([(mt << 5) | 27]) + v.to_bytes(8, "big") if mt == 0 else \
            bytes([(mt << 5) | 25]) + v.to_bytes(2, "big")
    if v < 24:
        return bytes([(mt << 5) | v])
    for ai, nb in ((24, 1), (25, 2), (26, 4), (27, 8)):
        if v < (1 << (8 * nb)):
            return bytes([(mt << 5) | ai]) + v.to_bytes(nb, "big")
    raise ValueError(v)


def encode_body(f, wide=()):
    """Canonical EncCBOR HeaderBody (Header.hs:160-185).  `wide` names fields to
    encode with non-shortest heads (test corpora only): any field name, or
    'body' / 'vrf' / 'ocert' / 'pv' for the array heads."""
    def u(k):
        return _head(0, f[k], k in wide)

    def b(k):
        return _head(2, len(f[k]), k in wide) + f[k]
    prev = b"\xf6" if f["prev_hash"] is None else b("prev_hash")
    return b"".join([
        _head(4, 10, "body" in wide), u("block_no"), u("slot"), prev, b("cold_vk"), b("vrf_vk"),
        _head(4, 2, "vrf" in wide), b("vrf_out"), b("vrf_proof"), u("body_size"), b("body_hash"),
        _head(4, 4, "ocert" in wide), b("hot_vk"), u("n"), u("c0"), b("ocert_sig"),
        _head(4, 2, "pv" in wide), u("prot_major"), u("prot_minor")])


def encode_tpraos_body(f, wide=()):
    """Canonical encodeBHBody (15 fields; the OCert and ProtVer groups inlined)."""
    def u(k):
        return _head(0, f[k], k in wide)

    def b(k):
        return _head(2, len(f[k]), k in wide) + f[k]
    prev = b"\xf6" if f["prev_hash"] is None else b("prev_hash")
    return b"".join([
        _head(4, 15, "body" in wide), u("block_no"), u("slot"), prev, b("cold_vk"), b("vrf_vk"),
        _head(4, 2, "vrf" in wide), b("vrf_out"), b("vrf_proof"),
        _head(4, 2, "leader" in wide), b("leader_out"), b("leader_proof"),
        u("body_size"), b("body_hash"), b("hot_vk"), u("n"), u("c0"), b("ocert_sig"),
        u("prot_major"), u("prot_minor")])


def encode_header(f, kes_sig, wide=()):
    """EncCBOR HeaderRaw (Header.hs:201-210): [body, kesSig]."""
    return _head(4, 2) + encode_body(f, wide) + _head(2, len(kes_sig)) + kes_sig


def decode_header(arena, off, length, allow_tpraos=False):
    """Decode header bytes arena[off:off+length].  Returns a dict with 'status',
    the fields (None on failure), 'signed' (canonical body bytes, b'' on failure),
    'header_hash' (Blake2b-256 of the stored bytes; zeros on DEC_RANGE) and 'tpraos'
    (the body had 15 fields; only accepted with allow_tpraos, the block path)."""
    out = {"status": 0, "fields": None, "signed": b"", "header_hash": bytes(32), "tpraos": False}
    if off > len(arena) or length > len(arena) - off:
        out["status"] = DEC_RANGE
        return out
    raw = bytes(arena[off:off + length])
    out["header_hash"] = hashlib.blake2b(raw, digest_size=32).digest()
    r = _R(raw, 0, length)
    try:
        r.array(2)
        body_start = r.pos
        r.canon = True
        arity = r.expect(4)
        tp = allow_tpraos and arity == 15
        if arity != (15 if tp else 10):
            raise _Fail(DEC_SYNTAX)
        f = {"block_no": r.uint(), "slot": r.uint()}
        if r.pos < r.end and r.b[r.pos] == 0xF6:
            r.pos += 1
            f["prev_hash"] = None
        else:
            f["prev_hash"] = r.bytes_fixed(32)
        f["cold_vk"] = r.bytes_fixed(32)
        f["vrf_vk"] = r.bytes_fixed(32)
        r.array(2)
        f["vrf_out"] = r.bytes_fixed(64)
        f["vrf_proof"] = r.bytes_fixed(80)
        if tp:
            r.array(2)
            f["leader_out"] = r.bytes_fixed(64)
            f["leader_proof"] = r.bytes_fixed(80)
        f["body_size"] = r.uint((1 << 32) - 1)
        f["body_hash"] = r.bytes_fixed(32)
        if not tp:
            r.array(4)
        f["hot_vk"] = r.bytes_fixed(32)
        f["n"] = r.uint()
        f["c0"] = r.uint()
        f["ocert_sig"] = r.bytes_fixed(64)
        if not tp:
            r.array(2)
        f["prot_major"] = r.uint(MAX_PROT_MAJOR)
        f["prot_minor"] = r.uint()
        canon = r.canon
        body_end = r.pos
        f["kes_sig"] = r.bytes_fixed(448)
        if r.pos != r.end:
            raise _Fail(DEC_TRAILING)
    except _Fail as e:
        out["status"] = e.bit
        return out
    signed = encode_tpraos_body(f) if tp else encode_body(f)
    assert (signed == raw[body_start:body_end]) == canon
    out["status"] = 0 if canon else DEC_NONCANONICAL
    out["fields"] = f
    out["signed"] = signed
    out["tpraos"] = tp
    return out


def babbage_block(header):
    """An empty Babbage block as stored in an ImmutableDB chunk: the
    HardForkBlock era wrapper [6, block] around [header, [], [], {}, []].
    The header starts at offset 3 (as in golden/cardano/disk/Block_Babbage)."""
    return b"\x82\x06\x85" + header + b"\x80\x80\xa0\x80"


def pack_chunk(headers):
    """Concatenate blocks of the given header bytes; returns (arena, off, len)
    with off/len as the secondary index gives them (blockOffset + headerOffset,
    headerSize; ImmutableDB/Impl/Index/Secondary.hs:93-128)."""
    parts, off, ln, pos = [], [], [], 0
    for h in headers:
        blk = babbage_block(h)
        parts.append(blk)
        off.append(pos + 3)
        ln.append(len(h))
        pos += len(blk)
    return b"".join(parts), off, ln
