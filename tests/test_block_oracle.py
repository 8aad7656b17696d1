"""Block-integrity oracle (oracle/block_integrity.py) pinned to the reference's golden
blocks, plus the mutation corpus the GPU test replays (CPU only)."""
import json
import os
import random

import block_corpus as bc
import block_integrity as bi
from golden import cbor_min

KATS = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "reference_kats.json")))["kats"]
SPKP = 129600


def _segments(buf):
    """Generic split of any golden block ([eraTag, blk] or bare blk) with the oracle skipper."""
    _, _, arg, p = bi._head(buf, 0, len(buf))
    if arg == 2:
        _, _, _, p = bi._head(buf, p, len(buf))
        _, _, arg, p = bi._head(buf, p, len(buf))
    spans = []
    for _ in range(arg):
        q = bi.cbor_skip(buf, p, len(buf))
        spans.append((p, q - p))
        p = q
    assert p == len(buf)
    return spans[0], spans[1:]


def test_hash_tx_seq_matches_every_golden_block():
    for k in KATS:
        buf = bytes.fromhex(k["block_cbor"])
        (ho, hl), segs = _segments(buf)
        assert buf[ho:ho + hl].hex() == k["header_cbor"]
        assert len(segs) == (3 if k["era"] in ("Shelley", "Allegra", "Mary", "ShelleyOnly") else 4)
        assert k["expect"]["block_matches_header"]
        assert bi.hash_tx_seq(buf, segs).hex() == k["body_hash"], k["era"]


def test_golden_praos_blocks_integrity_bits():
    # Babbage/Conway: body matches, KES leaf is over the coerced TPraos body (Examples.hs:173-192)
    for k in KATS:
        buf = bytes.fromhex(k["block_cbor"])
        bits, bh = bi.verify_block_integrity(buf, 0, len(buf), SPKP)
        if k["kind"] == "praos":
            assert k["expect"]["kes_result_praos_body"] == 2
            assert bits == bi.BLK_KES, k["era"]
            assert bh.hex() == k["body_hash"]
        else:  # TPraos eras: KES over the 15-field BHBody, body hash -- intact
            assert k["expect"]["kes_result"] == 0
            assert bits == 0, k["era"]
            assert bh.hex() == k["body_hash"]


def test_golden_tpraos_headers_decode():
    """The 15-field BHBody decode reproduces every field the golden TPraos headers hold, and
    its canonical re-encoding is the stored body (the KES message)."""
    import cbor_header as ch
    for k in KATS:
        if k["kind"] != "tpraos":
            continue
        hdr = bytes.fromhex(k["header_cbor"])
        d = ch.decode_header(hdr, 0, len(hdr), allow_tpraos=True)
        assert d["status"] == 0 and d["tpraos"], k["era"]
        f = d["fields"]
        assert (f["block_no"], f["slot"], f["n"], f["c0"]) == (k["block_no"], k["slot"], k["n"], k["c0"])
        for key, fk in (("cold_vk", "cold_vk"), ("vrf_vk", "vrf_vk"), ("vrf_out", "eta_out"),
                        ("vrf_proof", "eta_proof"), ("leader_out", "leader_out"), ("leader_proof", "leader_proof"),
                        ("body_hash", "body_hash"), ("hot_vk", "hot_vk"), ("ocert_sig", "ocert_sig"),
                        ("kes_sig", "kes_sig")):
            assert f[key].hex() == k[fk], (k["era"], key)
        assert hdr[1:1 + len(d["signed"])] == d["signed"]
        # a Praos-only decode rejects the 15-field body
        assert ch.decode_header(hdr, 0, len(hdr))["status"] == ch.DEC_SYNTAX


def test_era_tag_and_header_kind_must_agree():
    """[tag, block]: a TPraos header under a Praos era tag (and vice versa) or a wrong
    segment count for the era does not decode."""
    by = {k["era"]: bytes.fromhex(k["block_cbor"]) for k in KATS}
    shelley, babbage = by["Shelley"], by["Babbage"]
    assert bi.verify_block_integrity(shelley, 0, len(shelley), SPKP)[0] == 0
    for tag in (6, 7):
        b = bytearray(shelley)
        b[1] = tag
        assert bi.verify_block_integrity(bytes(b), 0, len(b), SPKP)[0] == bi.BLK_DECODE
    b = bytearray(shelley)
    b[1] = 5                                   # Alonzo wants 4 segments
    assert bi.verify_block_integrity(bytes(b), 0, len(b), SPKP)[0] == bi.BLK_DECODE
    b = bytearray(babbage)
    b[1] = 5                                   # Alonzo: TPraos header expected
    assert bi.verify_block_integrity(bytes(b), 0, len(b), SPKP)[0] == bi.BLK_DECODE


def test_cbor_skip_agrees_with_generic_decoder():
    r = random.Random(7)
    for _ in range(400):
        item = bc.rand_item(r)
        buf = item + b"\x00\x01"
        assert bi.cbor_skip(buf, 0, len(buf)) == len(item)
        assert cbor_min.decode(buf).end == len(item)


def test_mutation_corpus():
    r = random.Random(0xB10C)
    blk, f, _ = bc.make_block(r, SPKP)
    for kind in bc.MUTATIONS:
        b = bc.mutate(blk, f, r, kind)
        bits, _ = bi.verify_block_integrity(b, 0, len(b), SPKP)
        assert bits == bc.expected_kind(kind), kind


def test_kes_period_clamp():
    # c0 > kp: verifyHeaderIntegrity uses t = 0 (Shelley/Protocol/Praos.hs:97-101)
    r = random.Random(3)
    blk, f, _ = bc.make_block(r, SPKP, slot=5 * SPKP, c0=9)
    assert bi.verify_block_integrity(blk, 0, len(blk), SPKP)[0] == 0
    # t = 67 >= 2^6: SumKES verify only branches on t (t - 2^(l-1) at each level) and the
    # SingleKES leaf's `assert (t == 0)` is compiled out, so the all-ones path (signed at 63)
    # verifies; verifyHeaderIntegrity has no maxKESEvo bound (unlike validateKESSignature)
    blk, f, _ = bc.make_block(r, SPKP, slot=70 * SPKP, c0=3)
    assert bi.verify_block_integrity(blk, 0, len(blk), SPKP)[0] == 0


def test_synthetic_tpraos_blocks():
    """Synthetic TPraos blocks of every TPraos era (and a bare one) are intact; the
    mutation corpus on an Alonzo block gives the same kinds as on Praos blocks."""
    r = random.Random(0x7A)
    for era in (2, 3, 4, 5):
        for wrapped in (True, False):
            blk, _, _ = bc.make_block(r, SPKP, era=era, wrapped=wrapped)
            assert bi.verify_block_integrity(blk, 0, len(blk), SPKP)[0] == 0, (era, wrapped)
    blk, f, _ = bc.make_block(r, SPKP, era=5)
    for kind in bc.MUTATIONS:
        m = bc.mutate(blk, f, r, kind)
        want = 0 if kind == "era_5" else bc.expected_kind(kind)     # already an Alonzo block
        assert bi.verify_block_integrity(m, 0, len(m), SPKP)[0] == want, kind
