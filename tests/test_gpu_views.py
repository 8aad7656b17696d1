"""A ledger view per epoch: db-analyser forecasts each
header's LedgerView from the ledger state it advances block by block (Analysis.hs:564-572,
ledgerViewForecastAt; Shelley/Ledger/SupportsProtocol.hs:100-125: lvPoolDistr = nesPd), and the
PoolDistr changes at every epoch boundary (NEWEPOCH).

The chain here is forged under a stake distribution that changes between epochs -- a pool leaves
the PoolDistr, stakes are re-weighted, the pool comes back and another leaves -- with each
epoch's leader schedule searched under that epoch's stake.  Checked:
  * praos_replay_immutable_views with the per-epoch views accepts every header and ends in the
    generator's state, equal to the oracle's fold run epoch by epoch under each epoch's view;
  * the same database replayed with epoch 0's view throughout stops in a later epoch (the
    PoolDistr change is load-bearing);
  * the group form, small batches and a damaged header agree with the single call;
  * the db-analyser analysis' call sequence from C (integration/c/ffi_harness.c phase
    "analysis": forecast -> praos_ticked_epoch_nonce -> praos_set_epoch -> praos_verify_header_bytes
    -> praos_validate_headers per epoch, epoch e on a worker while epoch e+1 streams) equals the
    single views replay, on one context and on a group."""
import os
import shutil
from fractions import Fraction

import numpy as np
import pytest

from helpers import b2b
from test_gpu_ffi import _run_harness
from test_gpu_replay import ENV, _genesis_state

pytestmark = pytest.mark.gpu

EPOCHS, EPOCH_LEN, WINDOW, CHUNK_SLOTS = 4, 600, 200, 250
NPOOLS = 20
# the LedgerView's envelope part changes too: epoch 2 on raises the protocol version
LIMITS = {0: dict(lv_prot_major=8, max_header_size=1100, max_body_size=90_112),
          1: dict(lv_prot_major=8, max_header_size=1100, max_body_size=90_112),
          2: dict(lv_prot_major=9, max_header_size=1200, max_body_size=90_112)}


def _stakes(e):
    """Per-pool stake of epoch e (Fixed E34; 0 = not in the PoolDistr).  Epoch 3 keeps epoch 2's
    distribution (a view holds until the next one)."""
    from praos_hip import fixed
    if e == 0:
        w = [Fraction(1, i + 1) for i in range(NPOOLS)]
    elif e == 1:                                   # pool 0 retired; the order of stakes reversed
        w = [Fraction(0)] + [Fraction(1, NPOOLS - i) for i in range(1, NPOOLS)]
    else:                                          # pool 0 back, pool 1 retired, flatter weights
        w = [Fraction(1, i + 3) if i != 1 else Fraction(0) for i in range(NPOOLS)]
    tot = sum(w)
    return [fixed.from_rational(x / tot) if x else 0 for x in w]


@pytest.fixture(scope="module")
def vchain(ctx, tmp_path_factory):
    from praos_hip import immutable
    cfg = dict(npools=NPOOLS, stake_offset=1, f=Fraction(1, 2), slots_per_kes_period=129600, max_kes_evo=62,
               eta0=b2b(b"views-genesis"), seed=b"\x3c" * 32)
    data = immutable.make_multi_epoch_chain(ctx, cfg, EPOCHS, EPOCH_LEN, WINDOW, stakes=_stakes)
    path = str(tmp_path_factory.mktemp("immdb_views") / "immutable")
    immutable.write_immutable(path, data["arena"], data["off"], data["len"], data["slots"], data["header_hash"],
                              CHUNK_SLOTS)
    data.update(cfg=cfg, path=path)
    # the ledger views a replay gets: epochs 0, 1, 2 (epoch 3 under epoch 2's)
    data["lviews"] = [(e, data["views"][e][1], LIMITS[e]) for e in range(3)]
    return data


def _views_replay(ctx, data, path=None, batch_max=1 << 16, state=None, tip=None):
    st = state if state is not None else _genesis_state(data["cfg"]["eta0"])
    env = {"max_major_pv": ENV["max_major_pv"], "tip": tip}
    n = len(data["off"])
    stats, v = ctx.replay_immutable_views(path or data["path"], data["lviews"], data["params"], data["epoch_info"],
                                          st, env, batch_max=batch_max, verdicts_cap=n)
    return stats, v, st, env


def _oracle_fold_views(ctx, data, upto):
    """oracle/chainstate.py's fold over headers [0, upto), epoch by epoch, each epoch under its own
    ledger view (pools for the crypto and the counters' PoolDistr membership, envelope limits)."""
    import chainstate as cs
    cfg, arena, off, ln = data["cfg"], data["arena"], data["off"], data["len"]
    st = _genesis_state(cfg["eta0"])
    env = {"tip": None}
    epoch = (data["slots"][:upto] // EPOCH_LEN).astype(int)
    for e in range(EPOCHS):
        rows = np.nonzero(epoch == e)[0]
        if len(rows) == 0:
            break
        _, pools, lim = data["lviews"][min(e, 2)]
        eta = st["epoch_nonce"] if e == 0 else cs.combine(st["candidate"], st["leb"])
        ctx.set_epoch(eta, pools, data["params"])
        o, D = ctx.verify_header_bytes(arena, off[rows], ln[rows], decoded=True)
        m = len(rows)
        env.update(block_no=D["block_no"], header_hash=D["header_hash"], header_size=ln[rows],
                   body_size=D["body_size"], max_major_pv=ENV["max_major_pv"], **lim)
        hk = [b2b(bytes(c), 28) for c in D["cold_vk"]]
        prev = [None if D["prev_is_genesis"][i] else bytes(D["prev_hash"][i]) for i in range(m)]
        known = {h for h, _, _ in pools}
        _, stop, done = cs.fold(st, hk, D["slot"], o["bits"], D["ocert_n"], o["nonce"], prev, known, eta, 0, 0,
                                EPOCH_LEN, WINDOW, env=env)
        assert done == m
        if stop < m:
            return st, env["tip"], int(rows[stop])
    return st, env["tip"], upto


def _epoch_file(path, data):
    p = data["params"]
    lines = [f"eta0 {data['cfg']['eta0'].hex()}",
             f"params {p.slots_per_kes_period} {p.max_kes_evo} {p.f_is_one} {p.vrf_check_output} {bytes(p.c_raw).hex()}",
             "epoch " + " ".join(str(x) for x in data["epoch_info"]),
             f"env {ENV['max_major_pv']} {LIMITS[0]['lv_prot_major']} {LIMITS[0]['max_header_size']} "
             f"{LIMITS[0]['max_body_size']}"]
    for e, pools, lim in data["lviews"]:
        if e:
            lines.append(f"view {e} {lim['lv_prot_major']} {lim['max_header_size']} {lim['max_body_size']}")
        lines += [f"pool {h.hex()} {v.hex()} {int(s).to_bytes(16, 'little').hex()}" for h, v, s in pools]
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")


def test_views_chain_changes_pooldistr(vchain):
    """The fixture is what it claims: the PoolDistr differs between epochs 0, 1 and 2."""
    hs = [{h for h, _, _ in vchain["views"][e][1]} for e in range(EPOCHS)]
    assert len(hs[0]) == NPOOLS and len(hs[1]) == NPOOLS - 1 and hs[1] != hs[2] and hs[2] == hs[3]
    assert all(int((vchain["slots"] // EPOCH_LEN == e).sum()) > 100 for e in range(EPOCHS))


def test_views_replay_all_valid_and_equals_oracle(ctx, vchain):
    from praos_hip import abi
    n = len(vchain["off"])
    stats, v, st, env = _views_replay(ctx, vchain)
    assert (stats["headers"], stats["validated"], stats["stop_index"]) == (n, n, n)
    assert int((v != 0).sum()) == 0 and stats["epochs"] == EPOCHS
    assert st == vchain["state"]
    ost, otip, ostop = _oracle_fold_views(ctx, vchain, n)
    assert ostop == n and st == ost and env["tip"] == otip
    assert abi.state_encode(st) == abi.state_encode(ost)


def test_single_view_diverges(ctx, vchain):
    """Epoch 0's view for the whole database (praos_replay_immutable): the replay stops in a later
    epoch -- the per-epoch PoolDistr is load-bearing -- and the oracle under the same single view
    stops at the same header with the same state."""
    from praos_hip import abi
    n = len(vchain["off"])
    st = _genesis_state(vchain["cfg"]["eta0"])
    env = dict(ENV, tip=None)
    stats, v = ctx.replay_immutable(vchain["path"], vchain["lviews"][0][1], vchain["params"], vchain["epoch_info"],
                                    st, env, verdicts_cap=n)
    k = stats["stop_index"]
    assert k < n and int(vchain["slots"][k]) >= EPOCH_LEN
    assert stats["stop_verdict"] in (abi.V_LEADER_TOO_BIG, abi.V_VRF_KEY_UNKNOWN, abi.V_ENV_OBSOLETE_NODE)
    ost, otip, ostop = _oracle_fold_views(ctx, dict(vchain, lviews=[vchain["lviews"][0]] * 3), n)
    assert ostop == k and st == ost and env["tip"] == otip


@pytest.mark.parametrize("members,batch_max", [(1, 61), (3, 97), (2, 1 << 16)])
def test_views_replay_group_and_batches(ctx, vchain, members, batch_max):
    """A group (batches dealt round robin, a view's tables built per member on first use) and
    batches far smaller than an epoch: the single call's result."""
    from praos_hip import abi
    n = len(vchain["off"])
    if members == 1:
        stats, v, st, env = _views_replay(ctx, vchain, batch_max=batch_max)
    else:
        with abi.Group([0] * members) as g:
            st = _genesis_state(vchain["cfg"]["eta0"])
            env = {"max_major_pv": ENV["max_major_pv"], "tip": None}
            stats, v = g.replay_immutable_views(vchain["path"], vchain["lviews"], vchain["params"],
                                                vchain["epoch_info"], st, env, batch_max=batch_max, verdicts_cap=n)
    assert (stats["validated"], stats["stop_index"]) == (n, n) and int((v != 0).sum()) == 0
    assert st == vchain["state"]


def test_views_replay_stops_and_resumes(ctx, vchain, tmp_path):
    """A KES signature damaged in epoch 2 (under the third view): the views replay stops there, as
    the oracle does; resuming from a checkpoint taken at the end of epoch 1 over the clean database
    reaches the one-pass end state."""
    from praos_hip import abi, immutable
    n = len(vchain["off"])
    k = int(np.nonzero(vchain["slots"] >= 2 * EPOCH_LEN)[0][9])
    db = str(tmp_path / "bad")
    shutil.copytree(vchain["path"], db)
    c = int(vchain["slots"][k]) // CHUNK_SLOTS
    e = next(x for x in immutable.read_secondary(db, c) if x["slot"] == int(vchain["slots"][k]))
    f = os.path.join(db, f"{c:05d}.chunk")
    raw = bytearray(open(f, "rb").read())
    raw[e["block_offset"] + e["header_offset"] + int(vchain["len"][k]) - 100] ^= 0x40
    open(f, "wb").write(bytes(raw))
    stats, v, st, env = _views_replay(ctx, vchain, path=db, batch_max=97)
    assert (stats["stop_index"], stats["stop_verdict"], stats["validated"]) == (k, abi.V_KES_SIG, k)
    ost, otip, ostop = _oracle_fold_views(ctx, vchain, k)
    assert ostop == k and st == ost and env["tip"] == otip
    m = int(np.nonzero(vchain["slots"] >= 2 * EPOCH_LEN)[0][0])
    part = str(tmp_path / "part")
    immutable.write_immutable(part, vchain["arena"], vchain["off"][:m], vchain["len"][:m], vchain["slots"][:m],
                              vchain["header_hash"][:m], CHUNK_SLOTS)
    s1, _, st1, env1 = _views_replay(ctx, vchain, path=part)
    assert s1["validated"] == m
    s2, v2, st2, env2 = _views_replay(ctx, vchain, state=abi.state_decode(abi.state_encode(st1)), tip=env1["tip"])
    assert s2["skipped"] == m and s2["validated"] == n - m and st2 == vchain["state"]


def test_views_replay_rejects_missing_view(ctx, vchain):
    from praos_hip import abi
    bad = dict(vchain, lviews=[(1, vchain["lviews"][1][1], LIMITS[1])])     # nothing covers epoch 0
    with pytest.raises(abi.PraosError, match="no ledger view"):
        _views_replay(ctx, bad)


def test_ffi_analysis_sequence_matches_views_replay(ctx, vchain, tmp_path):
    """integration/c/ffi_harness.c phase "analysis" (the db-analyser analysis' per-epoch
    forecast -> set_epoch -> verify -> fold, pipelined with the stream) on one context and on a
    4-member group, and praos_[group_]replay_immutable_views, all end in the Python views replay's
    state and tip; the single-view phases stop where the single-view replay stops."""
    from praos_hip import abi
    ef = str(tmp_path / "epoch_views.txt")
    _epoch_file(ef, vchain)
    out = _run_harness(vchain["path"], ef)
    n = len(vchain["off"])
    stats, _, st, env = _views_replay(ctx, vchain)
    cbor = abi.state_encode(st).hex()
    for phase in ("analysis", "analysis_group", "replay_views", "replay_views_group"):
        o = out[phase]
        assert (o["validated"], o["stop_index"], o["stop_verdict"]) == (n, n, 0), phase
        assert o["state_cbor"] == cbor, phase
        assert (o["tip_slot"], o["tip_block_no"], bytes.fromhex(o["tip_hash"])) == env["tip"], phase
    assert out["analysis"]["epochs"] == EPOCHS
    st1 = _genesis_state(vchain["cfg"]["eta0"])
    env1 = dict(ENV, tip=None)
    s1, _ = ctx.replay_immutable(vchain["path"], vchain["lviews"][0][1], vchain["params"], vchain["epoch_info"],
                                 st1, env1)
    assert s1["stop_index"] < n
    for phase in ("binding", "typed", "typed_group", "replay", "replay_group"):
        assert (out[phase]["stop_index"], out[phase]["stop_verdict"]) == (s1["stop_index"], s1["stop_verdict"]), phase
        assert out[phase]["state_cbor"] == abi.state_encode(st1).hex(), phase
