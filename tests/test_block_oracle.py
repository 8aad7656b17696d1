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
        else:  # TPraos eras are outside the Praos block path
            assert bits == bi.BLK_DECODE


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
