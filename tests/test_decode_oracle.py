"""CPU tests of the header-decoding oracle (oracle/cbor_header.py), pinned to the
reference's golden Babbage/Conway headers (tests/golden/reference_kats.json,
extracted from ouroboros-consensus-cardano/golden/cardano/disk/Block_*), and of
the chunk packer (praos_hip/chunk.py) that lays synthetic chains out as
ImmutableDB blocks."""
import json
import os

import numpy as np

import cbor_header as ch
from decode_corpus import N_KINDS, random_fields as _random_fields, variants
from helpers import rbytes, rng

HERE = os.path.dirname(os.path.abspath(__file__))
KATS = json.load(open(os.path.join(HERE, "golden", "reference_kats.json")))["kats"]
PRAOS = [k for k in KATS if k["kind"] == "praos"]


def test_golden_praos_headers_decode():
    assert len(PRAOS) == 2
    for k in PRAOS:
        h = bytes.fromhex(k["header_cbor"])
        # the block as stored: header at offset 3 of [6, [header, ...]]
        blk = ch.babbage_block(h)
        r = ch.decode_header(blk, 3, len(h))
        assert r["status"] == 0, k["era"]
        f = r["fields"]
        assert f["block_no"] == k["block_no"] and f["slot"] == k["slot"]
        for name in ("cold_vk", "vrf_vk", "hot_vk", "ocert_sig", "kes_sig", "body_hash"):
            assert f[name].hex() == k[name], name
        assert f["vrf_out"].hex() == k["vrf_out"] and f["vrf_proof"].hex() == k["vrf_proof"]
        assert f["body_size"] == k["body_size"] and [f["prot_major"], f["prot_minor"]] == k["prot"]
        assert (f["n"], f["c0"]) == (k["n"], k["c0"])
        # canonical golden body: the signable re-serialisation is the stored slice
        assert r["signed"].hex() == k["body_cbor"]
        assert ch.encode_header(f, f["kes_sig"]) == h


def test_mutation_corpus_statuses():
    r = rng(77)
    seen = {}
    for k in range(3 * N_KINDS):
        f = _random_fields(r)
        sig = rbytes(r, 448)
        h, name = variants(f, sig, k)
        res = ch.decode_header(h, 0, len(h))
        seen[name] = res["status"]
        if res["status"] & ch.DEC_FAIL == 0:
            g = res["fields"]
            assert res["signed"] == ch.encode_body(g)
            assert len(res["signed"]) <= ch.SIGNED_STRIDE - 1
    assert seen["canonical"] == 0 and seen["genesis_prev"] == 0 and seen["big_ints"] == 0
    for name in ("wide_slot", "wide_arrays", "wide_bytes"):
        assert seen[name] == ch.DEC_NONCANONICAL
    assert seen["truncated"] == ch.DEC_SYNTAX and seen["trailing"] == ch.DEC_TRAILING
    assert seen["short_vrf_vk"] == ch.DEC_SIZE and seen["long_proof"] == ch.DEC_SIZE
    assert seen["short_kes"] == ch.DEC_SIZE
    assert seen["indef_body"] == ch.DEC_UNSUPPORTED and seen["tag_slot"] == ch.DEC_UNSUPPORTED
    assert seen["body_size_overflow"] == ch.DEC_OVERFLOW and seen["prot_major_over"] == ch.DEC_OVERFLOW
    assert seen["neg_slot"] == ch.DEC_SYNTAX and seen["body_len_11"] == ch.DEC_SYNTAX and seen["empty"] == ch.DEC_SYNTAX
    assert ch.decode_header(b"\x00" * 10, 8, 5)["status"] == ch.DEC_RANGE


def test_noncanonical_signed_bytes_are_reencoded():
    r = rng(5)
    f = _random_fields(r)
    sig = rbytes(r, 448)
    a = ch.decode_header(ch.encode_header(f, sig), 0, len(ch.encode_header(f, sig)))
    w = ch.encode_header(f, sig, ("slot", "body", "hot_vk"))
    b = ch.decode_header(w, 0, len(w))
    assert b["status"] == ch.DEC_NONCANONICAL
    assert a["signed"] == b["signed"]                 # serialize' hb is encoding-independent
    assert a["header_hash"] != b["header_hash"]       # headerHash hashes the stored bytes


def test_pack_chunk_layout():
    from praos_hip.chunk import pack_chunk
    r = rng(9)
    n = 40
    F = [_random_fields(r) for _ in range(n)]
    bodies = [ch.encode_body(f) for f in F]
    H = {"slot": np.zeros(n, np.uint64), "body_off": np.arange(n, dtype=np.uint64) * 448,
         "body_len": np.array([len(b) for b in bodies], np.uint32), "body_bytes": np.zeros(448 * n + 8, np.uint8),
         "kes_sig": np.frombuffer(b"".join(rbytes(r, 448) for _ in range(n)), np.uint8).reshape(n, 448).copy()}
    for i, b in enumerate(bodies):
        H["body_bytes"][448 * i:448 * i + len(b)] = np.frombuffer(b, np.uint8)
    arena, off, ln = pack_chunk(H)
    ref_arena, ref_off, ref_len = ch.pack_chunk([ch._head(4, 2) + b + ch._head(2, 448) + bytes(H["kes_sig"][i])
                                                 for i, b in enumerate(bodies)])
    assert bytes(arena) == ref_arena and list(off) == ref_off and list(ln) == ref_len
    for i in range(n):
        res = ch.decode_header(bytes(arena), int(off[i]), int(ln[i]))
        assert res["status"] == 0 and res["fields"]["slot"] == F[i]["slot"]
