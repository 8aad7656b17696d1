"""GPU header decoding (k_decode.hip) against the oracle
(oracle/cbor_header.py): golden Babbage/Conway headers of the reference, a
mutation corpus of edge cases at unaligned offsets, and the decode -> validate
path (praos_verify_header_bytes / praos_batch_upload_bytes) against the SoA
path on GPU-synthesised chains with genuine CBOR bodies."""
import json
import os
from fractions import Fraction

import numpy as np
import pytest

import cbor_header as ch
from decode_corpus import N_KINDS, random_fields, variants
from helpers import b2b, rbytes, rng

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))

FIELDS_U = ("block_no", "slot", "body_size", "prot_major", "prot_minor")
FIELDS_B = ("cold_vk", "vrf_vk", "vrf_out", "vrf_proof", "body_hash", "hot_vk", "ocert_sig", "kes_sig")


def _check_against_oracle(D, arena, off, ln):
    for i in range(len(off)):
        r = ch.decode_header(bytes(arena), int(off[i]), int(ln[i]))
        assert int(D["status"][i]) == r["status"], (i, int(D["status"][i]), r["status"])
        assert bytes(D["header_hash"][i]) == r["header_hash"], i
        f = r["fields"]
        if f is None:
            assert int(D["signed_len"][i]) == 0xFFFFFFFF
            assert not D["cold_vk"][i].any() and not D["kes_sig"][i].any() and int(D["slot"][i]) == 0
            continue
        for k in FIELDS_U:
            assert int(D[k][i]) == f[k], (i, k)
        assert (int(D["ocert_n"][i]), int(D["ocert_c0"][i])) == (f["n"], f["c0"])
        for k in FIELDS_B:
            assert bytes(D[k][i]) == f[k], (i, k)
        assert int(D["prev_is_genesis"][i]) == (f["prev_hash"] is None)
        assert bytes(D["prev_hash"][i]) == (f["prev_hash"] or bytes(32))
        sl = int(D["signed_len"][i])
        assert bytes(D["signed_body"][i][:sl]) == r["signed"], i


def test_decode_golden_headers(ctx):
    kats = [k for k in json.load(open(os.path.join(HERE, "golden", "reference_kats.json")))["kats"]
            if k["kind"] == "praos"]
    hs = [bytes.fromhex(k["header_cbor"]) for k in kats]
    arena, off, ln = ch.pack_chunk(hs)
    D = ctx.decode_headers(arena, off, ln)
    _check_against_oracle(D, arena, off, ln)
    for i, k in enumerate(kats):
        assert int(D["status"][i]) == 0 and int(D["slot"][i]) == k["slot"]
        assert bytes(D["signed_body"][i][:int(D["signed_len"][i])]).hex() == k["body_cbor"]
        assert bytes(D["header_hash"][i]) == b2b(hs[i])


def test_decode_mutation_corpus(ctx):
    r = rng(2024)
    parts, off, ln, pos = [], [], [], 0
    for k in range(6 * N_KINDS):
        f = random_fields(r)
        h, _ = variants(f, rbytes(r, 448), k)
        gap = rbytes(r, r.randrange(0, 9))          # arbitrary (unaligned) header offsets
        parts.append(gap + h)
        off.append(pos + len(gap))
        ln.append(len(h))
        pos += len(gap) + len(h)
    arena = b"".join(parts)
    off.append(len(arena) - 3)                      # slice past the end: DEC_RANGE
    ln.append(10)
    D = ctx.decode_headers(arena, off, ln)
    _check_against_oracle(D, arena, off, ln)
    st = set(int(s) for s in D["status"])
    assert {0, ch.DEC_NONCANONICAL, ch.DEC_SYNTAX, ch.DEC_SIZE, ch.DEC_UNSUPPORTED, ch.DEC_TRAILING,
            ch.DEC_OVERFLOW, ch.DEC_RANGE} <= st


def _cbor_chain(ctx, n, npools, corrupt, seed=b"\x61" * 32):
    from praos_hip import abi, fixed
    c_raw = fixed.active_slot_log(Fraction(1, 20))
    p = abi.params(slots_per_kes_period=129600, max_kes_evo=62, c_raw=c_raw)
    eta0 = b2b(b"decode-epoch")
    H, pools, corrupted = ctx.synthesize(n, npools, p, eta0, seed, first_slot=5000, slot_stride=20, body_len=0,
                                         corrupt_per_10000=corrupt)
    w = [Fraction(1, i + 10) for i in range(npools)]
    sig = [fixed.from_rational(x / sum(w)) for x in w]
    ctx.set_epoch(eta0, [(h, v, s) for (h, v), s in zip(pools, sig)], p)
    return H, corrupted


def test_verify_header_bytes_matches_soa_path(ctx):
    from praos_hip.chunk import pack_chunk
    H, corrupted = _cbor_chain(ctx, 384, 9, 1500)
    assert all(int(x) <= 447 for x in H["body_len"])
    arena, off, ln = pack_chunk(H)
    soa = ctx.verify_headers(H)
    o, D = ctx.verify_header_bytes(arena, off, ln, decoded=True)
    _check_against_oracle(D, arena, off, ln)
    ok_dec = (D["status"] & ch.DEC_FAIL) == 0
    # headers whose stored bytes still decode to the SoA fields must get identical verdicts
    same = ok_dec & (D["slot"] == H["slot"]) & (D["ocert_n"] == H["ocert_n"]) & (D["ocert_c0"] == H["ocert_c0"])
    for k in ("cold_vk", "vrf_vk", "vrf_out", "vrf_proof", "hot_vk", "ocert_sig", "kes_sig"):
        same &= (D[k] == H[k]).all(axis=1)
    # stored bytes carry every seeded corruption (chunk.py packs the corrupted SoA);
    # only a corrupted body byte (kind 5) may change what the bytes decode to
    assert same[corrupted != 5].all(), np.nonzero(~same)[0][:10]
    for i in np.nonzero(same)[0]:
        sl = int(D["signed_len"][i])
        assert bytes(D["signed_body"][i][:sl]) == bytes(H["body_bytes"][int(H["body_off"][i]):][:int(H["body_len"][i])])
        assert int(o["bits"][i]) == int(soa["bits"][i]), (i, hex(o["bits"][i]), hex(soa["bits"][i]))
        assert bytes(o["beta"][i]) == bytes(soa["beta"][i]) and bytes(o["nonce"][i]) == bytes(soa["nonce"][i])
    # every clean header validates; every header that does not decode is flagged PRAOS_BIT_INPUT
    clean = corrupted == 0
    assert ((o["bits"][clean] & 0x0F1F) == 0).all()
    assert ((o["bits"][~ok_dec] & 0x8000) != 0).all()
    assert ((o["bits"][corrupted != 0] & 0x8F1F) != 0).all()


def test_noncanonical_stored_headers_validate(ctx):
    """A stored body with non-shortest heads decodes to the same HeaderBody, so the
    KES message (serialize' hb) and the verdict are unchanged; headerHash changes."""
    from praos_hip.chunk import pack_chunk
    H, corrupted = _cbor_chain(ctx, 64, 4, 0, seed=b"\x62" * 32)
    arena, off, ln = pack_chunk(H)
    base, Db = ctx.verify_header_bytes(arena, off, ln, decoded=True)
    wides = [("slot",), ("body", "pv"), ("cold_vk", "n"), ("ocert", "vrf_out", "c0")]
    hs = []
    for i in range(64):
        r = ch.decode_header(bytes(arena), int(off[i]), int(ln[i]))
        hs.append(ch.encode_header(r["fields"], r["fields"]["kes_sig"], wides[i % 4]))
    a2, off2, ln2 = ch.pack_chunk(hs)
    o, D = ctx.verify_header_bytes(a2, off2, ln2, decoded=True)
    assert (D["status"] == ch.DEC_NONCANONICAL).all()
    assert (o["bits"] == base["bits"]).all() and ((o["bits"] & 0x0F1F) == 0).all()
    assert (D["signed_body"] == Db["signed_body"]).all() and (D["signed_len"] == Db["signed_len"]).all()
    assert not (D["header_hash"] == Db["header_hash"]).all(axis=1).any()


def test_batch_from_bytes(ctx):
    from praos_hip.chunk import pack_chunk
    H, corrupted = _cbor_chain(ctx, 512, 6, 300, seed=b"\x63" * 32)
    arena, off, ln = pack_chunk(H)
    ref = ctx.verify_header_bytes(arena, off, ln)
    b = ctx.upload_bytes(arena, off, ln)
    try:
        for _ in range(2):                          # re-runs decode + validate from the resident arena
            ctx.run(b)
            ctx.sync()
            assert ctx.kernel_ms(5) > 0.0
        o = ctx.download(b, len(off))
        D = ctx.download_decoded(b, len(off))
    finally:
        ctx.free(b)
    for k in ("bits", "beta", "leader", "nonce", "pool_idx"):
        assert (o[k] == ref[k]).all(), k
    assert (D["slot"] == H["slot"]).all()
