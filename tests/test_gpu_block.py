"""GPU block-integrity batch (k_block.hip + k_decode + k_kes header mode, SURVEY.md
sec. 8f row 4) against the oracle (oracle/block_integrity.py): the reference's golden
blocks, the mutation corpus at unaligned offsets, large multi-compression segments,
the t = max(0, kp - c0) clamp, and the device-resident re-run path."""
import json
import os
import random

import numpy as np
import pytest

import block_corpus as bc
import block_integrity as bi

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
SPKP = 129600


def _pack(blocks, r=None):
    """Concatenate blocks with random gaps (unaligned offsets, like a chunk file)."""
    parts, off, ln, pos = [], [], [], 0
    for b in blocks:
        gap = r.randrange(8) if r else 0
        parts.append(bytes(gap) + b)
        off.append(pos + gap)
        ln.append(len(b))
        pos += gap + len(b)
    return b"".join(parts), off, ln


def _check(ctx, arena, off, ln):
    res, bh = ctx.verify_block_integrity(arena, off, ln, SPKP)
    for i in range(len(off)):
        bits, h = bi.verify_block_integrity(arena, off[i], ln[i], SPKP)
        assert int(res[i]) == bits, (i, int(res[i]), bits)
        assert bytes(bh[i]) == h, i
    return res


def test_golden_blocks(ctx):
    kats = json.load(open(os.path.join(HERE, "golden", "reference_kats.json")))["kats"]
    blocks = [bytes.fromhex(k["block_cbor"]) for k in kats]
    arena, off, ln = _pack(blocks)
    res = _check(ctx, arena, off, ln)
    for k, r in zip(kats, res):
        # Praos blocks: body matches, KES leaf made over the TPraos body (Examples.hs:173-192);
        # TPraos blocks (Shelley..Alonzo, 15-field BHBody): intact
        assert int(r) == (bi.BLK_KES if k["kind"] == "praos" else 0), k["era"]


def test_mutation_corpus(ctx):
    r = random.Random(0xB10C5)
    blocks, want = [], []
    for j in range(3):
        blk, f, _ = bc.make_block(r, SPKP, era=5 + j)        # Alonzo (TPraos), Babbage, Conway
        for kind in bc.MUTATIONS:
            blocks.append(bc.mutate(blk, f, r, kind))
            want.append(0 if (kind == "era_5" and j == 0) else bc.expected_kind(kind))   # j = 0: Alonzo
    arena, off, ln = _pack(blocks, r)
    res = _check(ctx, arena, off, ln)
    assert [int(x) for x in res] == want


def test_random_blocks_and_clamp(ctx):
    r = random.Random(42)
    blocks = []
    for j in range(96):
        if j % 8 == 0:
            blk, _, _ = bc.make_block(r, SPKP, slot=5 * SPKP + j, c0=9)        # kp < c0: t = 0
        elif j % 8 == 1:
            blk, _, _ = bc.make_block(r, SPKP, big=True)                        # multi-KB segments
        elif j % 8 == 2:
            blk, _, _ = bc.make_block(r, SPKP, wrapped=False)                   # bare 5-item block
        elif j % 8 == 3:
            blk, _, _ = bc.make_block(r, SPKP, era=2 + (j // 8) % 4)             # TPraos eras
        elif j % 8 == 4:
            blk, _, _ = bc.make_block(r, SPKP, era=2, wrapped=False)            # bare Shelley block
        else:
            blk, _, _ = bc.make_block(r, SPKP)
        if j % 5 == 4:
            blk = bc.mutate(blk, None, r, "seg_byte") if j % 10 == 4 else blk
        blocks.append(blk)
    arena, off, ln = _pack(blocks, r)
    res = _check(ctx, arena, off, ln)
    assert (res == 0).sum() >= 80


def test_device_resident_rerun_and_ranges(ctx):
    r = random.Random(9)
    blocks = [bc.make_block(r, SPKP)[0] for _ in range(40)]
    arena, off, ln = _pack(blocks, r)
    off = list(off) + [len(arena) + 1, len(arena) - 3]     # out-of-range spans -> DECODE
    ln = list(ln) + [4, 10]
    b = ctx.upload_blocks(arena, off, ln)
    try:
        for _ in range(3):   # re-runs must not depend on the previous run's header spans
            ctx.run_blocks(b, SPKP)
        res, bh = ctx.download_blocks(b, len(off))
    finally:
        ctx.free(b)
    assert [int(x) for x in res] == [0] * 40 + [bi.BLK_DECODE] * 2
    for i in range(40):
        assert bytes(bh[i]) == bi.verify_block_integrity(arena, off[i], ln[i], SPKP)[1]


def test_empty_batch(ctx):
    res, bh = ctx.verify_block_integrity(b"", [], [], SPKP)
    assert res.shape == (0,)
