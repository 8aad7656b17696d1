"""Stored-header corpora for the decoder tests (test infrastructure).

Every variant is built with the oracle's encoder (oracle/cbor_header.py) from a
field dict, so the expected decode result is the oracle's decode of the same
bytes.  Variants cover the decoder's edge cases: non-canonical heads (the
signed bytes must then be RE-encoded, Header.hs:90-94), GenesisHash prev,
truncation, trailing bytes, wrong fixed sizes, indefinite lengths, tags,
Word32 overflow of bodySize, ProtVer major above maxVersion, wrong major types and out-of-range slices."""
import cbor_header as ch
from helpers import rbytes


def variants(f, kes_sig, k):
    """The k-th mutation of header fields f (k cycles over the corpus).
    Returns (header bytes, name)."""
    g = dict(f)
    h = ch.encode_header(f, kes_sig)
    kinds = [
        ("canonical", lambda: h),
        ("wide_slot", lambda: ch.encode_header(f, kes_sig, ("slot",))),
        ("wide_arrays", lambda: ch.encode_header(f, kes_sig, ("body", "vrf", "ocert", "pv"))),
        ("wide_bytes", lambda: ch.encode_header(f, kes_sig, ("cold_vk", "vrf_proof", "ocert_sig", "n", "c0"))),
        ("genesis_prev", lambda: ch.encode_header(dict(g, prev_hash=None), kes_sig)),
        ("truncated", lambda: h[:-1 - (k % 40)]),
        ("trailing", lambda: h + b"\x00"),
        ("short_vrf_vk", lambda: ch.encode_header(dict(g, vrf_vk=f["vrf_vk"][:31]), kes_sig)),
        ("long_proof", lambda: ch.encode_header(dict(g, vrf_proof=f["vrf_proof"] + b"\x01"), kes_sig)),
        ("short_kes", lambda: ch.encode_header(f, kes_sig[:447])),
        ("indef_body", lambda: h[:1] + b"\x9f" + ch.encode_body(f)[1:] + b"\xff" + h[1 + len(ch.encode_body(f)):]),
        ("tag_slot", lambda: _tag_slot(f, kes_sig)),
        ("body_size_overflow", lambda: ch.encode_header(dict(g, body_size=1 << 32), kes_sig)),
        ("big_ints", lambda: ch.encode_header(dict(g, block_no=(1 << 64) - 1, n=1 << 40, prot_minor=1 << 33), kes_sig)),
        ("neg_slot", lambda: _neg_slot(f, kes_sig)),
        ("body_len_11", lambda: h[:1] + b"\x8b" + h[2:]),
        ("empty", lambda: b""),
        ("prot_major_over", lambda: ch.encode_header(dict(g, prot_major=ch.MAX_PROT_MAJOR + 1), kes_sig)),
    ]
    name, mk = kinds[k % len(kinds)]
    return mk(), name


def _tag_slot(f, kes_sig):
    body = ch.encode_body(f)
    bn = ch._head(0, f["block_no"])
    # tag 2 (bignum) in front of the slot
    body = body[:1 + len(bn)] + b"\xc2" + body[1 + len(bn):]
    return ch._head(4, 2) + body + ch._head(2, 448) + kes_sig


def _neg_slot(f, kes_sig):
    body = ch.encode_body(f)
    bn = ch._head(0, f["block_no"])
    sl = ch._head(0, f["slot"])
    body = body[:1 + len(bn)] + bytes([0x20 | (sl[0] & 31)]) + body[2 + len(bn):]
    return ch._head(4, 2) + body + ch._head(2, 448) + kes_sig


N_KINDS = 18


def random_fields(r):
    return {"block_no": r.getrandbits(r.choice([3, 10, 20, 40])), "slot": r.getrandbits(r.choice([5, 16, 30, 60])),
            "prev_hash": rbytes(r, 32), "cold_vk": rbytes(r, 32), "vrf_vk": rbytes(r, 32), "vrf_out": rbytes(r, 64),
            "vrf_proof": rbytes(r, 80), "body_size": r.getrandbits(r.choice([4, 12, 32])), "body_hash": rbytes(r, 32),
            "hot_vk": rbytes(r, 32), "n": r.getrandbits(r.choice([1, 8, 33])), "c0": r.getrandbits(r.choice([2, 9])),
            "ocert_sig": rbytes(r, 64), "prot_major": r.choice([6, 7, 8, 9]), "prot_minor": r.getrandbits(3)}
