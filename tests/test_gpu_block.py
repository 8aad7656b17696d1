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


def _write_chunk(path, blocks, crcs):
    """One ImmutableDB chunk (00000.chunk) and its secondary index: blockOffset and checksum per
    entry (the fields chunk validation reads; Secondary.hs:93-128), the others zero."""
    import zlib  # noqa: F401  (crcs are computed by the caller)
    os.makedirs(path, exist_ok=True)
    data, sec = bytearray(), bytearray()
    for b, c in zip(blocks, crcs):
        sec += len(data).to_bytes(8, "big") + bytes(4) + int(c).to_bytes(4, "big") + bytes(32) + bytes(8)
        data += b
    open(os.path.join(path, "00000.chunk"), "wb").write(bytes(data))
    open(os.path.join(path, "00000.secondary"), "wb").write(bytes(sec))
    return bytes(data)


def _harness_chunk(path, members=3):
    import subprocess
    exe = os.path.join(os.path.dirname(HERE), "integration", "c", "ffi_harness")
    r = subprocess.run([exe, "--chunk", path, "0", str(SPKP), str(members)], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stderr
    return {d["phase"]: d for d in (json.loads(x) for x in r.stdout.splitlines() if x.strip())}


def test_ffi_chunk_validation(tmp_path):
    """Batch.hs verifyChunkIntegrity's call sequence from C (ffi_harness --chunk): the ImmutableDB
    chunk validation of parseChunkFile (Parser.hs:118-141) with its expensive checkIntegrity
    (Validation.hs:379-384 -> verifyBlockIntegrity, Integrity.hs:14-20) batched on the GPU, one
    context and a 3-member group.  (a) every stored checksum wrong: every block is checked, each
    result equals oracle/block_integrity.py, and the chunk is cut at the first corrupt block;
    (b) correct checksums over a chunk damaged on disk in two blocks, plus one stale checksum of an
    intact block: exactly those three are checked, the intact one passes, the chunk is cut at the
    first damaged block."""
    import zlib
    kats = json.load(open(os.path.join(HERE, "golden", "reference_kats.json")))["kats"]
    r = random.Random(0xC4C)
    blocks = [bytes.fromhex(k["block_cbor"]) for k in kats if k["kind"] != "praos"]     # intact TPraos blocks
    for j in range(3):
        blk, f, _ = bc.make_block(r, SPKP, era=5 + j)
        blocks += [blk] + [bc.mutate(blk, f, r, kind) for kind in bc.MUTATIONS]
    blocks += [bytes.fromhex(k["block_cbor"]) for k in kats if k["kind"] == "praos"]    # golden Babbage/Conway
    want = [bi.verify_block_integrity(b, 0, len(b), SPKP)[0] for b in blocks]
    # (a) no usable checksum (every stored one off by a bit)
    data = _write_chunk(str(tmp_path / "a"), blocks, [zlib.crc32(b) ^ 1 for b in blocks])
    out = _harness_chunk(str(tmp_path / "a"))
    first = next(i for i, w in enumerate(want) if w)
    offs = np.cumsum([0] + [len(b) for b in blocks])
    for ph in ("chunk", "chunk_group"):
        o = out[ph]
        assert o["blocks"] == o["checked"] == len(blocks), ph
        assert o["results"] == want, ph
        assert (o["first_corrupt"], o["truncate_at"]) == (first, int(offs[first])), ph
    # (b) correct checksums, then two blocks damaged on disk and one stale checksum
    intact = [i for i, w in enumerate(want) if w == 0]
    assert len(intact) >= 8
    crcs = [zlib.crc32(b) for b in blocks]
    stale = intact[1]
    crcs[stale] ^= 0x5A5A
    data = bytearray(_write_chunk(str(tmp_path / "b"), blocks, crcs))
    d1, d2 = intact[4], intact[7]
    data[int(offs[d1]) + len(blocks[d1]) - 3] ^= 0x01        # a segment byte: hashTxSeq no longer matches
    data[int(offs[d2]) + 200] ^= 0x01                           # inside the header
    open(os.path.join(str(tmp_path / "b"), "00000.chunk"), "wb").write(bytes(data))
    out = _harness_chunk(str(tmp_path / "b"))
    for ph in ("chunk", "chunk_group"):
        o = out[ph]
        checked = [i for i, x in enumerate(o["results"]) if x >= 0]
        assert checked == sorted([stale, d1, d2]), ph
        assert o["results"][stale] == 0, ph
        for d in (d1, d2):
            assert o["results"][d] == bi.verify_block_integrity(bytes(data), int(offs[d]), len(blocks[d]), SPKP)[0] != 0
        assert (o["first_corrupt"], o["truncate_at"]) == (d1, int(offs[d1])), ph


def test_group_block_integrity_equals_single(ctx):
    from praos_hip import abi
    r = random.Random(77)
    blocks = [bc.make_block(r, SPKP)[0] for _ in range(50)]
    blocks[7] = bc.mutate(blocks[7], None, r, "seg_byte")
    arena, off, ln = _pack(blocks, r)
    res1, bh1 = ctx.verify_block_integrity(arena, off, ln, SPKP)
    with abi.Group([0, 0, 0]) as g:
        res3, bh3 = g.verify_block_integrity(arena, off, ln, SPKP)
    assert (res1 == res3).all() and (bh1 == bh3).all() and int(res1[7]) != 0
