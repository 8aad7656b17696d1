"""Host-only checks of the replay driver's ImmutableDB reading (praos_replay_immutable):
the writer's on-disk layout (Secondary.hs:93-128 entries, Primary.hs offsets), and the
reader's error and resume paths, which run before any device work.  The replay itself
(device decode + crypto + fold) is covered by tests/test_gpu_replay.py."""
import os

import numpy as np
import pytest

from helpers import b2b


def _fake_db(path, n=40, chunk_slots=16):
    """n fake 'blocks' [6, [hdr, ...]] with 30-byte headers at slots 3i+1 (not valid
    headers: only the layout matters here)."""
    from praos_hip import immutable
    from praos_hip.chunk import HEADER_OFFSET
    rng = np.random.default_rng(5)
    hdrs = [bytes(rng.integers(0, 256, 30, dtype=np.uint8)) for _ in range(n)]
    blocks = [b"\x82\x06\x85" + h + b"\x80\x80\xa0\x80" for h in hdrs]
    arena = np.frombuffer(b"".join(blocks), np.uint8)
    starts = np.cumsum([0] + [len(b) for b in blocks[:-1]])
    off = (starts + HEADER_OFFSET).astype(np.uint64)
    ln = np.full(n, 30, np.uint32)
    slots = np.arange(n, dtype=np.uint64) * 3 + 1
    hh = np.stack([np.frombuffer(b2b(h), np.uint8) for h in hdrs])
    nch = immutable.write_immutable(str(path), arena, off, ln, slots, hh, chunk_slots)
    return hdrs, slots, hh, nch


def test_writer_layout(tmp_path):
    from praos_hip import immutable
    hdrs, slots, hh, nch = _fake_db(tmp_path)
    assert nch == (int(slots[-1]) // 16) + 1
    seen = 0
    for c in range(nch):
        raw = open(tmp_path / f"{c:05d}.chunk", "rb").read()
        ents = immutable.read_secondary(str(tmp_path), c)
        prim = open(tmp_path / f"{c:05d}.primary", "rb").read()
        offs = [int.from_bytes(prim[1 + 4 * k:5 + 4 * k], "big") for k in range(16 + 2)]
        assert prim[0] == 1 and offs[0] == 0 and offs == sorted(offs) and offs[-1] == 56 * len(ents)
        for e in ents:
            i = seen
            assert e["slot"] == int(slots[i]) and e["header_hash"] == bytes(hh[i])
            assert raw[e["block_offset"] + e["header_offset"]:][:e["header_size"]] == hdrs[i]
            rel = 1 + e["slot"] - 16 * c
            assert offs[rel + 1] - offs[rel] == 56          # the relative slot holds this entry
            seen += 1
    assert seen == len(hdrs)


def _state(eta):
    return {"last_slot": None, "counters": {}, "evolving": eta, "candidate": eta, "epoch_nonce": eta,
            "lab": None, "leb": None}


ENV = {"max_major_pv": 9, "lv_prot_major": 8, "max_header_size": 1100, "max_body_size": 90_112}


@pytest.fixture()
def host_ctx():
    from praos_hip import abi
    c = abi.Context(abi.HOST_ONLY)
    yield c
    c.close()


def test_reader_errors_and_resume(host_ctx, tmp_path):
    from praos_hip import abi
    hdrs, slots, hh, nch = _fake_db(tmp_path)
    p = abi.params()
    pools = [(b"\x01" * 28, b"\x02" * 32, 1)]
    ei = (0, 0, 1000, 100)
    # resume at the last block: everything is skipped, nothing reaches the device
    tip = (int(slots[-1]), 39, bytes(hh[-1]))
    env = dict(ENV, tip=tip)
    st = _state(b"\x07" * 32)
    stats, v = host_ctx.replay_immutable(str(tmp_path), pools, p, ei, st, env)
    assert (stats["skipped"], stats["headers"], stats["validated"], stats["batches"]) == (40, 0, 0, 0)
    assert stats["chunks"] == nch and env["tip"] == tip and st == _state(b"\x07" * 32)
    # a tip that is not in the database
    with pytest.raises(abi.PraosError, match="tip is not a block"):
        host_ctx.replay_immutable(str(tmp_path), pools, p, ei, _state(None), dict(ENV, tip=(tip[0], 39, b"\x00" * 32)))
    # malformed secondary index (not a whole number of entries)
    sec = tmp_path / "00001.secondary"
    raw = open(sec, "rb").read()
    open(sec, "wb").write(raw[:-1])
    with pytest.raises(abi.PraosError, match="malformed secondary index 00001"):
        host_ctx.replay_immutable(str(tmp_path), pools, p, ei, _state(None), dict(ENV, tip=tip))
    # an entry pointing outside its chunk
    bad = bytearray(raw)
    bad[8:10] = (60000).to_bytes(2, "big")
    open(sec, "wb").write(bytes(bad))
    with pytest.raises(abi.PraosError, match="outside its chunk"):
        host_ctx.replay_immutable(str(tmp_path), pools, p, ei, _state(None), dict(ENV, tip=tip))
    # an empty directory: nothing to replay
    empty = tmp_path / "empty"
    os.makedirs(empty)
    stats, _ = host_ctx.replay_immutable(str(empty), pools, p, ei, _state(None), dict(ENV, tip=None))
    assert (stats["headers"], stats["stop_index"], stats["chunks"]) == (0, 0, 0)
