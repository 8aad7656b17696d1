"""Chain replay from an ImmutableDB directory (praos_replay_immutable, SURVEY.md sec. 8
N3; db-analyser's processAllImmutableDB + validateHeader, Analysis.hs:479-607, 815-847).

A linked multi-epoch chain (first-leader-wins under each epoch's own nonce) is written
as chunk + secondary + primary files whose chunk boundaries do not line up with the
epochs, then replayed through the library.  Checked against the oracle's fold run epoch
by epoch (tickChainDepState nonces evolved by the oracle, crypto from the GPU):
every header valid, the final PraosState and tip identical; a corrupted KES signature,
a broken prev-hash link and a damaged secondary index each stop (or fail) where the
reference would; resume from a checkpointed state (CBOR) reaches the same end state."""
import os
import shutil
from fractions import Fraction

import numpy as np
import pytest

from helpers import b2b

pytestmark = pytest.mark.gpu

EPOCHS, EPOCH_LEN, WINDOW, CHUNK_SLOTS = 4, 600, 200, 250
ENV = {"max_major_pv": 9, "lv_prot_major": 8, "max_header_size": 1100, "max_body_size": 90_112}


@pytest.fixture(scope="module")
def chain(ctx, tmp_path_factory):
    from praos_hip import immutable
    cfg = dict(npools=20, stake_offset=1, f=Fraction(1, 2), slots_per_kes_period=129600, max_kes_evo=62,
               eta0=b2b(b"replay-genesis"), seed=b"\x2a" * 32)
    data = immutable.make_multi_epoch_chain(ctx, cfg, EPOCHS, EPOCH_LEN, WINDOW)
    path = str(tmp_path_factory.mktemp("immdb") / "immutable")
    nchunks = immutable.write_immutable(path, data["arena"], data["off"], data["len"], data["slots"],
                                        data["header_hash"], CHUNK_SLOTS)
    data.update(cfg=cfg, path=path, nchunks=nchunks)
    return data


def _genesis_state(eta0):
    return {"last_slot": None, "counters": {}, "evolving": eta0, "candidate": eta0, "epoch_nonce": eta0,
            "lab": None, "leb": None}


def _replay(ctx, data, path=None, state=None, tip=None, batch_max=1 << 16, cap=None):
    st = state if state is not None else _genesis_state(data["cfg"]["eta0"])
    env = dict(ENV, tip=tip)
    n = len(data["off"])
    stats, v = ctx.replay_immutable(path or data["path"], data["pools"], data["params"], data["epoch_info"], st, env,
                                    batch_max=batch_max, verdicts_cap=n if cap is None else cap)
    return stats, v, st, env


def _oracle_fold(ctx, data, upto):
    """The oracle's fold (oracle/chainstate.py) over headers [0, upto), epoch by epoch:
    nonces evolved by the oracle, the crypto of each epoch from the GPU under that nonce."""
    import chainstate as cs
    cfg, arena, off, ln = data["cfg"], data["arena"], data["off"], data["len"]
    st = _genesis_state(cfg["eta0"])
    env = {"tip": None}
    known = {h for h, _, _ in data["pools"]}
    epoch = (data["slots"][:upto] // EPOCH_LEN).astype(int)
    verdicts, etas = [], []
    for e in range(EPOCHS):
        rows = np.nonzero(epoch == e)[0]
        if len(rows) == 0:
            break
        eta = st["epoch_nonce"] if e == 0 else cs.combine(st["candidate"], st["leb"])
        etas.append(eta)
        ctx.set_epoch(eta, data["pools"], data["params"])
        o, D = ctx.verify_header_bytes(arena, off[rows], ln[rows], decoded=True)
        m = len(rows)
        env.update(block_no=D["block_no"], header_hash=D["header_hash"], header_size=ln[rows],
                   body_size=D["body_size"], **ENV)
        hk = [b2b(bytes(c), 28) for c in D["cold_vk"]]
        prev = [None if D["prev_is_genesis"][i] else bytes(D["prev_hash"][i]) for i in range(m)]
        v, stop, done = cs.fold(st, hk, D["slot"], o["bits"], D["ocert_n"], o["nonce"], prev, known, eta, 0, 0,
                                EPOCH_LEN, WINDOW, env=env)
        verdicts += v
        assert done == m
        if stop < m:
            return verdicts, st, env["tip"], etas, int(rows[stop])
    return verdicts, st, env["tip"], etas, upto


def test_immutable_files(chain):
    """The files follow the on-disk layout: secondary entries point at the headers."""
    from praos_hip import immutable
    n = len(chain["off"])
    assert chain["nchunks"] == (int(chain["slots"][-1]) // CHUNK_SLOTS) + 1
    entries = [e for c in range(chain["nchunks"]) for e in immutable.read_secondary(chain["path"], c)]
    assert len(entries) == n
    assert [e["slot"] for e in entries] == [int(s) for s in chain["slots"]]
    assert all(e["header_hash"] == bytes(h) for e, h in zip(entries, chain["header_hash"]))
    e = entries[-1]
    raw = open(os.path.join(chain["path"], f"{chain['nchunks'] - 1:05d}.chunk"), "rb").read()
    hdr = raw[e["block_offset"] + e["header_offset"]:][:e["header_size"]]
    assert b2b(hdr) == e["header_hash"]
    prim = open(os.path.join(chain["path"], "00000.primary"), "rb").read()
    assert prim[0] == 1 and len(prim) == 1 + 4 * (CHUNK_SLOTS + 2)


@pytest.mark.parametrize("batch_max", [1 << 16, 97])
def test_replay_all_valid(ctx, chain, batch_max):
    """Every header valid over 4 epochs; final state and tip = the oracle's; one epoch
    nonce installed per epoch, equal to the ones the chain was forged under."""
    n = len(chain["off"])
    stats, v, st, env = _replay(ctx, chain, batch_max=batch_max)
    assert (stats["headers"], stats["validated"], stats["stop_index"], stats["stop_verdict"]) == (n, n, n, 0)
    assert int((v != 0).sum()) == 0
    assert stats["epochs"] == EPOCHS and stats["chunks"] == chain["nchunks"]
    # batches span epochs (per-header nonces); the first is a quarter of batch_max and the second
    # a half (the nonce chain starts sooner, praos_replay.hip)
    assert stats["batches"] == _expected_batches(n, batch_max)
    assert st == chain["state"]
    assert env["tip"] == (int(chain["slots"][-1]), n - 1, bytes(chain["header_hash"][-1]))
    ov, ost, otip, etas, ostop = _oracle_fold(ctx, chain, n)
    assert ostop == n and etas == chain["nonces"] and len(set(etas)) == EPOCHS
    assert st == ost and env["tip"] == otip


def _expected_batches(n, batch_max):
    """The replay's batch count: a quarter of batch_max first, then a half, then full batches
    (praos_replay.hip)."""
    left, k = n, 0
    while left > 0:
        cap = max(1, batch_max // 4) if k == 0 else max(1, batch_max // 2) if k == 1 else batch_max
        left -= cap
        k += 1
    return k


def _copy_db(chain, tmp_path, name):
    dst = str(tmp_path / name)
    shutil.copytree(chain["path"], dst)
    return dst


def _locate(chain, i):
    """(chunk file, byte offset of header i in it) via the secondary index."""
    from praos_hip import immutable
    c = int(chain["slots"][i]) // CHUNK_SLOTS
    ents = immutable.read_secondary(chain["path"], c)
    e = next(e for e in ents if e["slot"] == int(chain["slots"][i]))
    return f"{c:05d}.chunk", e["block_offset"] + e["header_offset"]


@pytest.mark.parametrize("where", ["kes_sig", "prev_hash"])
def test_replay_stops_at_corruption(ctx, chain, tmp_path, where):
    """A header damaged on disk in epoch 2: the replay stops exactly there with the
    reference's first error (a KES signature byte -> InvalidKesSignatureOCERT; the
    prev-hash field -> UnexpectedPrevHash, the envelope judged first), state and tip =
    the oracle's after the header before."""
    from praos_hip import abi
    n = len(chain["off"])
    k = int(np.nonzero(chain["slots"] >= 2 * EPOCH_LEN)[0][5])
    db = _copy_db(chain, tmp_path, where)
    fname, pos = _locate(chain, k)
    raw = bytearray(open(os.path.join(db, fname), "rb").read())
    hdr = bytes(raw[pos:pos + int(chain["len"][k])])
    if where == "kes_sig":
        at = pos + len(hdr) - 100
    else:
        at = pos + hdr.index(bytes(chain["header_hash"][k - 1])) + 7
    raw[at] ^= 0x40
    open(os.path.join(db, fname), "wb").write(bytes(raw))
    stats, v, st, env = _replay(ctx, chain, path=db)
    want = abi.V_KES_SIG if where == "kes_sig" else abi.V_ENV_PREV_HASH
    assert (stats["stop_index"], stats["stop_verdict"], stats["validated"]) == (k, want, k)
    assert int((v[:k] != 0).sum()) == 0 and v[k] == want
    # the oracle, over the first k headers, reaches the same state
    _, ost, otip, _, ostop = _oracle_fold(ctx, chain, k)
    assert ostop == k and st == ost and env["tip"] == otip
    assert n > k


def test_replay_early_stop_twice_then_clean(ctx, chain, tmp_path):
    """A header damaged early in a replay of small batches: the fold stops while later batches'
    crypto is already queued.  Those batches go back to the context (rp_batch_keep) only after
    their runs end, and the next call's uploads are ordered after them: the same damaged
    database replayed again gives the same stop, and the clean database then replays whole."""
    from praos_hip import abi
    n = len(chain["off"])
    k = 40
    db = _copy_db(chain, tmp_path, "early")
    fname, pos = _locate(chain, k)
    raw = bytearray(open(os.path.join(db, fname), "rb").read())
    raw[pos + int(chain["len"][k]) - 100] ^= 0x40
    open(os.path.join(db, fname), "wb").write(bytes(raw))
    for _ in range(2):
        stats, v, st, env = _replay(ctx, chain, path=db, batch_max=61)
        assert (stats["stop_index"], stats["stop_verdict"], stats["validated"]) == (k, abi.V_KES_SIG, k)
        assert int((v[:k] != 0).sum()) == 0
    stats, v, st, env = _replay(ctx, chain, batch_max=61)
    assert (stats["headers"], stats["validated"], stats["stop_index"]) == (n, n, n)
    assert st == chain["state"]


def test_replay_bad_secondary(ctx, chain, tmp_path):
    """A secondary index whose size is not a whole number of entries, and one whose entry
    points past its chunk, are reported as errors (no silent partial replay)."""
    from praos_hip import abi
    db = _copy_db(chain, tmp_path, "badsec")
    sec = os.path.join(db, "00001.secondary")
    raw = open(sec, "rb").read()
    open(sec, "wb").write(raw[:-3])
    with pytest.raises(abi.PraosError, match="secondary"):
        _replay(ctx, chain, path=db)
    bad = bytearray(raw)
    bad[0:8] = (1 << 40).to_bytes(8, "big")
    open(sec, "wb").write(bytes(bad))
    with pytest.raises(abi.PraosError, match="outside its chunk"):
        _replay(ctx, chain, path=db)


def test_replay_resume_from_checkpoint(ctx, chain, tmp_path):
    """Checkpoint/resume: replay a database holding the first m blocks, serialise the
    PraosState (CBOR) and the tip, decode it and resume over the full database -- the
    end state equals the one-pass replay."""
    from praos_hip import abi, immutable
    n = len(chain["off"])
    m = int(np.nonzero(chain["slots"] >= EPOCH_LEN + 350)[0][0])      # mid-epoch 1, past the window
    part = str(tmp_path / "part")
    immutable.write_immutable(part, chain["arena"], chain["off"][:m], chain["len"][:m], chain["slots"][:m],
                              chain["header_hash"][:m], CHUNK_SLOTS)
    stats, _, st, env = _replay(ctx, chain, path=part)
    assert stats["validated"] == m
    blob = abi.state_encode(st)
    st2 = abi.state_decode(blob)
    assert st2 == st
    stats2, v2, st2, env2 = _replay(ctx, chain, state=st2, tip=env["tip"])
    assert stats2["skipped"] == m and stats2["validated"] == n - m and stats2["stop_index"] == n - m
    assert int((v2[:n - m] != 0).sum()) == 0
    assert st2 == chain["state"] and env2["tip"][2] == bytes(chain["header_hash"][-1])
    with pytest.raises(abi.PraosError, match="tip is not a block"):
        _replay(ctx, chain, state=dict(st), tip=(env["tip"][0], env["tip"][1], b"\x00" * 32))


def test_multi_epoch_batch_nonces(ctx, chain):
    """One device batch over all four epochs with per-header nonces (praos_batch_set_nonces)
    gives the same outputs as per-epoch batches under praos_set_epoch; the fold over it
    with those nonces (praos_validate_headers_nonces) ends in the generator's state; a
    header verified under the wrong nonce ends the fold there (processed < n)."""
    arena, off, ln = chain["arena"], chain["off"], chain["len"]
    n = len(off)
    epoch = (chain["slots"] // EPOCH_LEN).astype(np.uint8)
    ctx.set_epoch(chain["nonces"][0], chain["pools"], chain["params"])
    b = ctx.upload_bytes(arena, off, ln)
    try:
        ctx.batch_decode(b)
        D = ctx.download_decoded(b, n)
        ctx.set_nonces(b, chain["nonces"], epoch)
        ctx.run(b)
        o = ctx.download(b, n)
    finally:
        ctx.free(b)
    assert int((o["bits"] != 0).sum()) == 0
    for e in range(EPOCHS):
        rows = np.nonzero(epoch == e)[0]
        ctx.set_epoch(chain["nonces"][e], chain["pools"], chain["params"])
        oe = ctx.verify_header_bytes(arena, off[rows], ln[rows])
        for k in ("bits", "pool_idx", "beta", "leader", "nonce"):
            assert np.array_equal(oe[k], o[k][rows]), (e, k)
    st = _genesis_state(chain["cfg"]["eta0"])
    v, stop, done = ctx.update_chain_dep_state(_soa(D, n), o, D["prev_hash"], st, chain["epoch_info"],
                                               prev_is_genesis=D["prev_is_genesis"], etas=chain["nonces"],
                                               eta_idx=epoch)
    assert (stop, done) == (n, n) and st == chain["state"]
    # epoch 2's headers claimed under epoch 1's nonce: the fold stops at the first of them
    bad = epoch.copy()
    first2 = int(np.nonzero(epoch == 2)[0][0])
    bad[epoch == 2] = 1
    st = _genesis_state(chain["cfg"]["eta0"])
    v, stop, done = ctx.update_chain_dep_state(_soa(D, n), o, D["prev_hash"], st, chain["epoch_info"],
                                               prev_is_genesis=D["prev_is_genesis"], etas=chain["nonces"],
                                               eta_idx=bad)
    assert done == first2 and stop == first2


def _soa(D, n):
    """praos_headers view of decoded fields (the fold reads slot, cold_vk, ocert_n)."""
    z = lambda shape, dt: np.zeros(shape, dt)  # noqa: E731
    return {"slot": D["slot"], "cold_vk": D["cold_vk"], "vrf_vk": D["vrf_vk"], "vrf_out": D["vrf_out"],
            "vrf_proof": D["vrf_proof"], "hot_vk": D["hot_vk"], "ocert_n": D["ocert_n"], "ocert_c0": D["ocert_c0"],
            "ocert_sig": D["ocert_sig"], "kes_sig": D["kes_sig"], "body_off": z(n, np.uint64),
            "body_len": z(n, np.uint32), "body_bytes": z(8, np.uint8)}


# ---------------------------------------------------------------- TPraos (Shelley..Alonzo)
TP_EXTRA = b2b(b"tpraos-extra-entropy")


@pytest.fixture(scope="module")
def tchain(ctx, tmp_path_factory):
    """A linked TPraos chain over 3 epochs (TPraos leader schedule, BHeaders in Alonzo
    blocks, TICKN with an extra entropy nonce), written as an ImmutableDB."""
    from praos_hip import immutable
    cfg = dict(npools=12, stake_offset=1, f=Fraction(1, 2), slots_per_kes_period=129600, max_kes_evo=62,
               eta0=b2b(b"tpraos-replay-genesis"), seed=b"\x2b" * 32)
    data = immutable.make_multi_epoch_chain(ctx, cfg, 3, EPOCH_LEN, WINDOW, tpraos=True, extra_entropy=TP_EXTRA)
    path = str(tmp_path_factory.mktemp("immdb_tp") / "immutable")
    nchunks = immutable.write_immutable(path, data["arena"], data["off"], data["len"], data["slots"],
                                        data["header_hash"], CHUNK_SLOTS)
    data.update(cfg=cfg, path=path, nchunks=nchunks)
    return data


def _tp_replay(ctx, data, path=None, batch_max=1 << 16):
    st = _genesis_state(data["cfg"]["eta0"])
    env = dict(ENV, tip=None, lv_prot_major=6)
    n = len(data["off"])
    stats, v, f = ctx.replay_immutable(path or data["path"], data["pools"], data["params"], data["epoch_info"], st,
                                       env, batch_max=batch_max, verdicts_cap=n, tpraos=True,
                                       extra_entropy=TP_EXTRA)
    return stats, v, f, st, env


def _tp_oracle_fold(ctx, data, upto):
    """oracle/tpraos.py's fold (TICKN with the extra entropy, PRTCL failure sets) epoch by
    epoch over headers [0, upto), the TPraos crypto of each epoch from the GPU (stored bytes,
    praos_verify_tpraos_header_bytes) under that epoch's nonce."""
    import chainstate as cs
    import tpraos as tp
    st = _genesis_state(data["cfg"]["eta0"])
    known = {h for h, _, _ in data["pools"]}
    epoch = (data["slots"][:upto] // EPOCH_LEN).astype(int)
    verdicts, fails, etas = [], [], []
    for e in range(3):
        rows = np.nonzero(epoch == e)[0]
        if len(rows) == 0:
            break
        eta = st["epoch_nonce"] if e == 0 else cs.combine(cs.combine(st["candidate"], st["leb"]), TP_EXTRA)
        etas.append(eta)
        ctx.set_epoch(eta, data["pools"], data["params"])
        o, D = ctx.verify_tpraos_header_bytes(data["arena"], data["off"][rows], data["len"][rows], decoded=True)
        hk = [b2b(bytes(c), 28) for c in D["cold_vk"]]
        prev = [None if D["prev_is_genesis"][i] else bytes(D["prev_hash"][i]) for i in range(len(rows))]
        v, f, stop, done = tp.fold(st, hk, D["slot"], o["bits"], D["ocert_n"], o["nonce"], prev, known, eta, 0, 0,
                                   EPOCH_LEN, WINDOW, extra_entropy=TP_EXTRA)
        verdicts += v
        fails += f
        assert done == len(rows)
        if stop < len(rows):
            return verdicts, fails, st, etas, int(rows[stop])
    return verdicts, fails, st, etas, upto


@pytest.mark.parametrize("batch_max", [1 << 16, 61])
def test_tpraos_replay_all_valid(ctx, tchain, batch_max):
    """praos_replay_immutable_tpraos over the whole TPraos database: every header valid, the
    final state = the generator's and the oracle's fold, the epoch nonces include TICKN's
    extra entropy."""
    n = len(tchain["off"])
    stats, v, f, st, env = _tp_replay(ctx, tchain, batch_max=batch_max)
    assert (stats["headers"], stats["validated"], stats["stop_index"], stats["stop_verdict"]) == (n, n, n, 0)
    assert int((v != 0).sum()) == 0 and int((f != 0).sum()) == 0
    assert stats["epochs"] == 3 and stats["batches"] == _expected_batches(n, batch_max)
    assert st == tchain["state"]
    assert env["tip"] == (int(tchain["slots"][-1]), n - 1, bytes(tchain["header_hash"][-1]))
    ov, of, ost, etas, ostop = _tp_oracle_fold(ctx, tchain, n)
    assert ostop == n and etas == tchain["nonces"] and len(set(etas)) == 3
    assert st == ost


def test_tpraos_replay_stops_at_corruption(ctx, tchain, tmp_path):
    """A KES signature damaged on disk in epoch 1: the replay stops there with the PRTCL
    failure set {InvalidKesSignatureOCERT} (PRAOS_V_TPRAOS), state = the oracle's."""
    from praos_hip import abi
    k = int(np.nonzero(tchain["slots"] >= EPOCH_LEN)[0][7])
    db = _copy_db(tchain, tmp_path, "tp_kes")
    fname, pos = _locate(tchain, k)
    raw = bytearray(open(os.path.join(db, fname), "rb").read())
    raw[pos + int(tchain["len"][k]) - 100] ^= 0x40
    open(os.path.join(db, fname), "wb").write(bytes(raw))
    stats, v, f, st, env = _tp_replay(ctx, tchain, path=db)
    assert (stats["stop_index"], stats["stop_verdict"], stats["validated"]) == (k, abi.V_TPRAOS, k)
    assert int((v[:k] != 0).sum()) == 0 and f[k] == abi.TPF_KES_SIG
    _, _, ost, _, ostop = _tp_oracle_fold(ctx, tchain, k)
    assert ostop == k and st == ost


# ---------------------------------------------------------------- the replay over a group (several GPUs)
_TIMES = ("ms_io", "ms_device", "ms_fold", "ms_nonce")


def _same_replay(a, b, ignore=()):
    """Two replays' (stats, verdicts, state, envelope) agree except for the timings (and, for a
    replay that stopped early, the counts of batches whose crypto was already queued and of chunk
    files the reader had opened by then: they depend on how many batches the pipeline keeps in
    flight -- RP_SLOTS, 4 per context -- and on how far the reader got before the stop)."""
    (sa, va, sta, ea), (sb, vb, stb, eb) = a, b
    stopped = sa["stop_index"] < sa["headers"] + sa["skipped"] or sa["stop_verdict"]
    skip = _TIMES + (("batches", "chunks") if stopped else ()) + tuple(ignore)
    assert {k: v for k, v in sa.items() if k not in skip} == {k: v for k, v in sb.items() if k not in skip}
    assert np.array_equal(va, vb) and sta == stb and ea["tip"] == eb["tip"]


def _group_replay(g, data, path=None, state=None, tip=None, batch_max=1 << 16):
    st = state if state is not None else _genesis_state(data["cfg"]["eta0"])
    env = dict(ENV, tip=tip)
    stats, v = g.replay_immutable(path or data["path"], data["pools"], data["params"], data["epoch_info"], st, env,
                                  batch_max=batch_max, verdicts_cap=len(data["off"]))
    return stats, v, st, env


@pytest.mark.parametrize("members,batch_max", [(2, 97), (3, 61), (4, 1 << 16)])
def test_group_replay_equals_single(ctx, chain, members, batch_max):
    """praos_group_replay_immutable (batches dealt to the members in turn, one nonce chain and one
    fold in chain order) over members contexts on device 0: stats, verdicts, PraosState and tip
    equal to the one-context replay's; with 97-header batches every member runs several."""
    from praos_hip import abi
    single = _replay(ctx, chain, batch_max=batch_max)
    with abi.Group([0] * members) as g:
        grp = _group_replay(g, chain, batch_max=batch_max)
        again = _group_replay(g, chain, batch_max=batch_max)          # the members keep their batches
    _same_replay(single, grp)
    _same_replay(single, again)
    assert grp[0]["batches"] >= (members if batch_max < 1000 else 1)
    assert grp[2] == chain["state"]


def test_group_replay_early_stop_then_resume(ctx, chain, tmp_path):
    """A header damaged at index 40 of a replay in 29-header batches over a 3-member group: the
    group stops where one context stops (later batches' crypto already queued on other
    members), twice; a database holding the blocks before it, replayed by the group, then
    checkpointed (CBOR) and resumed by the group over the clean database, ends in the
    generator's state."""
    from praos_hip import abi, immutable
    n = len(chain["off"])
    k = 40
    db = _copy_db(chain, tmp_path, "gearly")
    fname, pos = _locate(chain, k)
    raw = bytearray(open(os.path.join(db, fname), "rb").read())
    raw[pos + int(chain["len"][k]) - 100] ^= 0x40
    open(os.path.join(db, fname), "wb").write(bytes(raw))
    single = _replay(ctx, chain, path=db, batch_max=29)
    assert (single[0]["stop_index"], single[0]["stop_verdict"]) == (k, abi.V_KES_SIG)
    part = str(tmp_path / "gpart")
    m = int(np.nonzero(chain["slots"] >= EPOCH_LEN + 350)[0][0])
    immutable.write_immutable(part, chain["arena"], chain["off"][:m], chain["len"][:m], chain["slots"][:m],
                              chain["header_hash"][:m], CHUNK_SLOTS)
    with abi.Group([0, 0, 0]) as g:
        for _ in range(2):
            _same_replay(single, _group_replay(g, chain, path=db, batch_max=29))
        stats, _, st, env = _group_replay(g, chain, path=part, batch_max=29)
        assert stats["validated"] == m
        st2 = abi.state_decode(abi.state_encode(st))
        stats2, v2, st2, env2 = _group_replay(g, chain, state=st2, tip=env["tip"], batch_max=29)
    assert stats2["skipped"] == m and stats2["validated"] == n - m and int((v2[:n - m] != 0).sum()) == 0
    assert st2 == chain["state"] and env2["tip"][2] == bytes(chain["header_hash"][-1])


def test_group_replay_tpraos_equals_single(ctx, tchain):
    """praos_group_replay_immutable_tpraos over 2 members = the one-context TPraos replay
    (verdicts, PRTCL failure sets, state)."""
    from praos_hip import abi
    n = len(tchain["off"])
    s1, v1, f1, st1, e1 = _tp_replay(ctx, tchain, batch_max=61)
    with abi.Group([0, 0]) as g:
        st2 = _genesis_state(tchain["cfg"]["eta0"])
        e2 = dict(ENV, tip=None, lv_prot_major=6)
        s2, v2, f2 = g.replay_immutable(tchain["path"], tchain["pools"], tchain["params"], tchain["epoch_info"], st2,
                                        e2, batch_max=61, verdicts_cap=n, tpraos=True, extra_entropy=TP_EXTRA)
    assert {k: v for k, v in s1.items() if k not in _TIMES} == {k: v for k, v in s2.items() if k not in _TIMES}
    assert np.array_equal(v1, v2) and np.array_equal(f1, f2) and st1 == st2 == tchain["state"]
    assert e1["tip"] == e2["tip"]


def test_fresh_context_store_on_first_call_replay(chain):
    """Pool-key store regression (round 4's first box fault): a fresh context whose first call is
    a replay (the store on by default there, allocated and initialised on the cache's stream
    inside that call) gives the generator's state; a second replay on it, with the store full
    of the first one's keys, too."""
    import praos_hip
    c = praos_hip.Context(0)
    try:
        for _ in range(2):
            stats, v, st, env = _replay(c, chain)
            assert stats["validated"] == len(chain["off"]) and st == chain["state"]
    finally:
        c.close()


def test_reused_batches_alternate_replay_and_pipeline(chain):
    """The batches a context keeps between calls (the replay's, with per-header epoch nonces; the
    stored-bytes pipeline's, here forced to 4 chunks) are reset by one routine whenever they are
    taken again (batch_reuse_reset).  One context alternates replay / pipeline / replay in small
    batches / pipeline / replay under different epoch nonces: every pipeline call equals the same
    call on a fresh context, bit for bit, and every replay ends in the generator's state."""
    import praos_hip
    from praos_hip import abi
    ep = (chain["slots"] // EPOCH_LEN).astype(int)

    def pipeline_call(c, e):
        rows = np.nonzero(ep == e)[0]
        c.set_epoch(chain["nonces"][e], chain["pools"], chain["params"])
        o, D = c.verify_header_bytes(chain["arena"], chain["off"][rows], chain["len"][rows], decoded=True)
        return {k: np.array(v) for k, v in o.items()}, {k: np.array(D[k]) for k in ("slot", "header_hash", "cold_vk")}

    def fresh(e):
        f = praos_hip.Context(0)
        try:
            f.set_option(abi.OPT_PIPELINE, 4)
            return pipeline_call(f, e)
        finally:
            f.close()

    want = {e: fresh(e) for e in (2, 0)}
    c = praos_hip.Context(0)
    try:
        c.set_option(abi.OPT_PIPELINE, 4)
        for step, (kind, arg) in enumerate([("replay", 1 << 16), ("pipe", 2), ("replay", 61), ("pipe", 0),
                                            ("replay", 97)]):
            if kind == "replay":
                stats, v, st, env = _replay(c, chain, batch_max=arg)
                assert stats["validated"] == len(chain["off"]) and st == chain["state"], step
            else:
                o, D = pipeline_call(c, arg)
                wo, wD = want[arg]
                for k in ("bits", "pool_idx", "beta", "leader", "nonce"):
                    assert (o[k] == wo[k]).all(), (step, k)
                for k in D:
                    assert (D[k] == wD[k]).all(), (step, k)
                assert int((o["bits"] != 0).sum()) == 0, step
    finally:
        c.close()


@pytest.mark.parametrize("env", [{"PRAOS_REPLAY_EARLY": "1"}, {"PRAOS_REPLAY_EARLY": "2"},
                                 {"PRAOS_REPLAY_PIN": "1"}, {"PRAOS_CSTREAM_PRIO": "1"},
                                 {"PRAOS_PARSE_THREADS": "0"}, {"PRAOS_PARSE_THREADS": "1"},
                                 {"PRAOS_REPLAY_RAMP": "0"}, {"PRAOS_REPLAY_RAMP": "2"}])
def test_replay_schedule_options_equal_default(ctx, chain, tmp_path, monkeypatch, env):
    """Host-schedule options of the replay give the default replay's stats, verdicts, state and tip:
    crypto launched as soon as the batch's epoch nonces are published (PRAOS_REPLAY_EARLY 1; 2: and
    the next batch decoded), pinned threads (PRAOS_REPLAY_PIN), the copy / decode stream at the
    greatest priority (PRAOS_CSTREAM_PRIO, read when a context opens), the nonce chain on the
    device decode's fields instead of the host's reading of the headers (PRAOS_PARSE_THREADS=0), or
    that reading on one worker, other batch-size ramps (PRAOS_REPLAY_RAMP 0 / 2: the batch count
    differs) -- over the
    clean 4-epoch database (one context, 97-header batches; a 3-member group) and over one damaged
    in epoch 2 (the stop, its verdict and the state before it)."""
    from praos_hip import abi
    k = int(np.nonzero(chain["slots"] >= 2 * EPOCH_LEN)[0][5])
    db = _copy_db(chain, tmp_path, "bad")
    fname, pos = _locate(chain, k)
    raw = bytearray(open(os.path.join(db, fname), "rb").read())
    raw[pos + int(chain["len"][k]) - 100] ^= 0x40                   # a KES signature byte
    open(os.path.join(db, fname), "wb").write(bytes(raw))
    base = [_replay(ctx, chain, batch_max=97), _replay(ctx, chain, batch_max=1 << 16), _replay(ctx, chain, path=db)]
    with abi.Group([0] * 3) as g:
        gbase = _group_replay(g, chain, batch_max=61)
    for key, val in env.items():
        monkeypatch.setenv(key, val)
    import praos_hip
    c2 = praos_hip.Context(0)                                            # (context-open settings)
    try:
        got = [_replay(c2, chain, batch_max=97), _replay(c2, chain, batch_max=1 << 16), _replay(c2, chain, path=db)]
    finally:
        c2.close()
    with abi.Group([0] * 3) as g:
        ggot = _group_replay(g, chain, batch_max=61)
    for a, b in list(zip(base, got)) + [(gbase, ggot)]:
        _same_replay(a, b, ("batches",) if "PRAOS_REPLAY_RAMP" in env else ())
    assert got[2][0]["stop_index"] == k and got[2][0]["stop_verdict"] == abi.V_KES_SIG
    assert got[0][2] == chain["state"] and ggot[2] == chain["state"]


def test_tpraos_replay_early_launch_equals_default(ctx, tchain, monkeypatch):
    """TPraos replay with early launches (the published epoch nonces carry TICKN's extra entropy):
    the default replay's stats, verdicts, failure sets and state."""
    a = _tp_replay(ctx, tchain, batch_max=61)
    monkeypatch.setenv("PRAOS_REPLAY_EARLY", "1")
    b = _tp_replay(ctx, tchain, batch_max=61)
    assert {k: v for k, v in a[0].items() if k not in _TIMES} == {k: v for k, v in b[0].items() if k not in _TIMES}
    assert np.array_equal(a[1], b[1]) and np.array_equal(a[2], b[2]) and a[3] == b[3] == tchain["state"]
