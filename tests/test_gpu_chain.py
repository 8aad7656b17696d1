"""Leader-valid synthetic chains: the db-synthesizer slot loop (first leader wins,
Forging.hs:139-148, checkIsLeader Praos.hs:375-397 / meetsLeaderThreshold :505-526)
run on the GPU (praos_leader_schedule), checked against the oracle's restatement,
and the chains signed from it validated end to end (configs[0] and a configs[4]-shaped
batch at the full 3000-pool distribution)."""
from fractions import Fraction

import numpy as np
import pytest

from helpers import b2b

pytestmark = pytest.mark.gpu


def _small_cfg(npools, f, seed):
    return dict(npools=npools, stake_offset=1, f=f, slots_per_kes_period=129600, max_kes_evo=62,
                eta0=b2b(b"schedule-test"), seed=seed)


@pytest.mark.parametrize("tpraos", [False, True])
def test_leader_schedule_vs_oracle(ctx, oracle, tpraos):
    """f = 1/2 so that most slots have a leader and later forgers win some of them."""
    from praos_hip import chains, fixed
    cfg = _small_cfg(8 if not tpraos else 5, Fraction(1, 2), b"\x17" * 32)
    sig = chains.stake(cfg["npools"], 1)
    c_raw = fixed.active_slot_log(cfg["f"])
    first, n = 70_000, (48 if not tpraos else 24)
    got = ctx.leader_schedule(cfg["seed"], sig, chains.params(cfg), cfg["eta0"], first, n, tpraos=tpraos)
    want = oracle.leader_schedule(cfg["seed"], sig, c_raw, cfg["eta0"], range(first, first + n), tpraos=tpraos)
    assert list(got) == want
    assert -1 in want and max(want) > 0 and sum(1 for w in want if w >= 0) >= n // 4


def test_leader_schedule_f_one(ctx):
    """activeSlotVal f == maxBound: checkLeaderNatValue is True, so pool 0 forges every slot."""
    from praos_hip import chains
    cfg = _small_cfg(4, Fraction(1), b"\x18" * 32)
    got = ctx.leader_schedule(cfg["seed"], chains.stake(4, 1), chains.params(cfg), cfg["eta0"], 5, 40)
    assert (got == 0).all()


def _oracle_header(oracle, ep, H, i):
    off, ln = int(H["body_off"][i]), int(H["body_len"][i])
    return oracle.praos_header(ep, {
        "slot": int(H["slot"][i]), "cold_vk": bytes(H["cold_vk"][i]), "vrf_vk": bytes(H["vrf_vk"][i]),
        "vrf_out": bytes(H["vrf_out"][i]), "vrf_proof": bytes(H["vrf_proof"][i]), "hot_vk": bytes(H["hot_vk"][i]),
        "n": int(H["ocert_n"][i]), "c0": int(H["ocert_c0"][i]), "ocert_sig": bytes(H["ocert_sig"][i]),
        "kes_sig": bytes(H["kes_sig"][i]), "body": bytes(H["body_bytes"][off:off + ln])})


def _check_first_leader_wins(oracle, cfg, sig, c_raw, slot, forger):
    """Oracle: the forger leads the slot and no earlier forger does (forger = -1: nobody)."""
    upto = cfg["npools"] if forger < 0 else forger + 1
    for p in range(upto):
        seed = oracle.synth_seed(cfg["seed"], 2, p)
        lead = oracle.is_leader_at(seed, int(slot), cfg["eta0"], sig[p], c_raw)
        assert lead == (p == forger), (slot, p, forger)


def test_c1_chain(ctx, oracle):
    """configs[0]: the first 10,000 blocks of a 100-pool first-leader-wins chain from slot 0
    under the tools-test genesis.  Every header is valid (incl. the leader check), blocks
    are stake-shaped, and the chain state folds over all of it."""
    from praos_hip import chains, fixed
    cfg = chains.CONFIGS["c1"]
    slots, pools = chains.search_schedule(ctx, cfg, cfg["blocks"])
    assert len(slots) == 10_000 and (np.diff(slots.astype(np.int64)) > 0).all()
    assert 150_000 < int(slots[-1]) < 250_000                     # ~1/f slots per block
    sig = chains.stake(cfg["npools"], cfg["stake_offset"])
    share0 = sig[0] / fixed.R
    cnt = np.bincount(pools, minlength=cfg["npools"])
    assert abs(cnt[0] - 10_000 * share0) < 6 * np.sqrt(10_000 * share0)   # stake-proportional
    H, pool_list, corrupted, p = chains.make_chain(ctx, cfg, (slots, pools))
    assert (corrupted == 0).all()
    ctx.set_epoch(cfg["eta0"], pool_list, p)
    o = ctx.verify_headers(H)
    assert int((o["bits"] != 0).sum()) == 0
    assert list(o["pool_idx"]) == list(pools)
    # oracle on a sample of headers (bits, beta, leader value, nonce)
    c_raw = fixed.active_slot_log(cfg["f"])
    ep = oracle.make_epoch(cfg["eta0"], cfg["slots_per_kes_period"], cfg["max_kes_evo"], c_raw, pool_list)
    for i in np.linspace(0, 9_999, 60).astype(int):
        r = _oracle_header(oracle, ep, H, i)
        assert r["bits"] == 0
        assert bytes(o["beta"][i]) == r["beta"] and bytes(o["leader"][i]) == r["leader"]
        assert bytes(o["nonce"][i]) == r["nonce"]
    # first leader wins, on the oracle: two blocks and two empty slots
    for i in (3, 4_321):
        _check_first_leader_wins(oracle, cfg, sig, c_raw, slots[i], int(pools[i]))
    empty = sorted(set(range(int(slots[0]) + 1, int(slots[0]) + 60)) - set(int(s) for s in slots[:20]))[:2]
    for s in empty:
        _check_first_leader_wins(oracle, cfg, sig, c_raw, s, -1)
    # the whole chain folds: every header OK, one counter per issuing pool
    n = len(slots)
    st = {"last_slot": None, "counters": {}, "evolving": cfg["eta0"], "candidate": cfg["eta0"],
          "epoch_nonce": cfg["eta0"], "lab": None, "leb": None}
    v, stop, done = ctx.update_chain_dep_state(H, o, np.zeros((n, 32), np.uint8), st,
                                               (0, 0, cfg["epoch_length"], 129_600))
    assert (done, stop) == (n, n) and int((v != 0).sum()) == 0
    assert len(st["counters"]) == len(set(pools.tolist())) and st["last_slot"] == int(slots[-1])


def test_c5_schedule_fixture(ctx, oracle):
    """The shipped configs[4] schedule is the GPU's own first-leader-wins search: two
    windows re-searched on the GPU, two blocks re-checked on the oracle."""
    from praos_hip import chains, fixed
    cfg = chains.CONFIGS["c5"]
    slots, pools = chains.load_schedule("c5")
    assert len(slots) == cfg["blocks"] and (np.diff(slots.astype(np.int64)) > 0).all()
    assert int(slots[-1]) < cfg["epoch_length"]
    sig = chains.stake(cfg["npools"], cfg["stake_offset"])
    p = chains.params(cfg)
    for first in (0, int(slots[200_000]) - 1500):
        lead = ctx.leader_schedule(cfg["seed"], sig, p, cfg["eta0"], first, 3000)
        idx = np.nonzero(lead >= 0)[0]
        sel = (slots >= first) & (slots < first + 3000)
        assert list(first + idx) == list(slots[sel]) and list(lead[idx]) == list(pools[sel])
    c_raw = fixed.active_slot_log(cfg["f"])
    small = [i for i in range(2000) if pools[i] < 40][:2]
    for i in small:
        _check_first_leader_wins(oracle, cfg, sig, c_raw, slots[i], int(pools[i]))


def test_c5_shaped_batch(ctx, oracle):
    """60,000 headers of the configs[4] chain (3000-pool table, binary search, key cache at
    scale) with 1 % seeded corruptions: clean headers all valid, corrupted ones caught,
    and a sample of 300 headers bit-exact against the oracle."""
    from praos_hip import abi, chains, fixed
    cfg = chains.CONFIGS["c5"]
    sched = chains.load_schedule("c5")
    n = 60_000
    H, pool_list, corrupted, p = chains.make_chain(ctx, cfg, sched, n=n, corrupt_per_10000=100)
    ctx.set_epoch(cfg["eta0"], pool_list, p)
    b = ctx.upload(H)
    ctx.run(b)
    ctx.sync()
    o = ctx.download(b, n)
    st = ctx.batch_stats(b)
    dd = ctx.dedup_stats(b)
    ctx.free(b)
    clean = corrupted == 0
    assert int((o["bits"][clean] != 0).sum()) == 0
    assert int((o["bits"][~clean] == 0).sum()) == 0
    # OCert dedup: ~one distinct OCert per pool (+ the corrupted ones); the cold-key
    # cache sees only those; the VRF key cache sees every header
    assert dd["headers"] == n and 2000 < dd["ocert_unique"] < 4000, dd
    assert st["cold_hits"] + st["cold_misses"] == dd["ocert_unique"]
    assert st["vrf_hits"] + st["vrf_misses"] == n and st["vrf_keys"] > 2000
    assert list(o["pool_idx"][clean]) == list(sched[1][:n][clean])
    c_raw = fixed.active_slot_log(cfg["f"])
    ep = oracle.make_epoch(cfg["eta0"], cfg["slots_per_kes_period"], cfg["max_kes_evo"], c_raw, pool_list)
    hash_of = {h: i for i, (h, _, _) in enumerate(pool_list)}
    sample = sorted(set(np.linspace(0, n - 1, 200).astype(int).tolist()) | set(np.nonzero(~clean)[0][:100].tolist()))
    for i in sample:
        r = _oracle_header(oracle, ep, H, i)
        assert int(o["bits"][i]) & 0x1F1F == r["bits"], (i, hex(o["bits"][i]), hex(r["bits"]), corrupted[i])
        assert bytes(o["beta"][i]) == r["beta"] and bytes(o["leader"][i]) == r["leader"]
        assert bytes(o["nonce"][i]) == r["nonce"]
        assert int(o["pool_idx"][i]) == hash_of.get(r["issuer_hash"], -1)
    assert abi.BIT_LEADER not in {int(x) & abi.BIT_LEADER for x in o["bits"][clean]}


def _validate_from_bytes(ctx, cfg, H, tip=None):
    """Stored headers -> GPU decode + crypto -> praos_validate_headers (envelope + protocol)."""
    import hashlib
    from praos_hip.chunk import pack_chunk
    arena, off, ln = pack_chunk(H)
    o, D = ctx.verify_header_bytes(arena, off, ln, decoded=True)
    n = len(off)
    eta = cfg["eta0"]
    st = {"last_slot": None, "counters": {}, "evolving": eta, "candidate": eta, "epoch_nonce": eta, "lab": None,
          "leb": None}
    env = {"block_no": D["block_no"], "header_hash": D["header_hash"], "header_size": ln,
           "body_size": D["body_size"], "tip": tip, "max_major_pv": 9, "lv_prot_major": 8, "max_header_size": 1100,
           "max_body_size": 90_112}
    Hs = dict(H, slot=D["slot"], ocert_n=D["ocert_n"])
    ref_in = (dict(st), dict(env))
    v, stop, done = ctx.update_chain_dep_state(Hs, o, D["prev_hash"], st, (0, 0, cfg["epoch_length"], 129_600),
                                               prev_is_genesis=D["prev_is_genesis"], envelope=env)
    return o, D, v, stop, done, st, env, ref_in, ln


def test_linked_chain_validate_headers(ctx, oracle):
    """A real chain (hbPrev = headerHash of the previous block, GenesisHash first) of the
    configs[0] pools: stored bytes -> GPU decode + crypto -> validateHeader over the batch
    (envelope + updateChainDepState): every header valid, the tip is the last header; the
    same with seeded corruptions stops exactly at the first corrupted header, verdicts and
    state equal to the oracle's fold."""
    import chainstate as cs
    from praos_hip import chains
    cfg = chains.CONFIGS["c1"]
    sched = chains.search_schedule(ctx, cfg, 1500, window=40_000)
    H, pool_list, corrupted, p = chains.make_chain(ctx, cfg, sched, link=True)
    ctx.set_epoch(cfg["eta0"], pool_list, p)
    o, D, v, stop, done, st, env, _, ln = _validate_from_bytes(ctx, cfg, H)
    n = len(sched[0])
    assert (D["status"] & 0x5F == 0).all() and D["prev_is_genesis"][0] == 1 and D["prev_is_genesis"][1:].sum() == 0
    assert (D["header_hash"] == H["header_hash"]).all()
    assert (D["prev_hash"][1:] == D["header_hash"][:-1]).all()
    assert int((o["bits"] != 0).sum()) == 0
    assert (done, stop) == (n, n) and int((v != 0).sum()) == 0
    assert env["tip"] == (int(sched[0][-1]), n - 1, bytes(D["header_hash"][-1]))
    # corrupted copy: the chain stops at the first corrupted header
    H2, _, corrupted2, _ = chains.make_chain(ctx, cfg, sched, link=True, corrupt_per_10000=150)
    o2, D2, v2, stop2, done2, st2, env2, (ref_st, ref_env), _ = _validate_from_bytes(ctx, cfg, H2)
    first_bad = int(np.nonzero(corrupted2)[0][0])
    assert stop2 == first_bad and v2[first_bad] != 0 and int((v2[:first_bad] != 0).sum()) == 0
    hk = [oracle.blake2b(bytes(c), 28) for c in D2["cold_vk"]]
    prev = [None if D2["prev_is_genesis"][i] else bytes(D2["prev_hash"][i]) for i in range(n)]
    wv, wstop, wdone = cs.fold(ref_st, hk, D2["slot"], o2["bits"], D2["ocert_n"], o2["nonce"], prev,
                               {h for h, _, _ in pool_list}, cfg["eta0"], 0, 0, cfg["epoch_length"], 129_600,
                               env=ref_env)
    assert (wdone, wstop) == (done2, stop2) and list(v2) == wv
    assert st2 == ref_st and env2["tip"] == ref_env["tip"]


def test_decode_failure_is_input_with_kernel_mask(ctx):
    """A stored header that does not decode reports PRAOS_BIT_INPUT even when the KES
    kernel (which used to carry that bit) is masked out (praos_set_option KERNELS)."""
    from praos_hip import abi, chains
    from praos_hip.chunk import pack_chunk
    cfg = chains.CONFIGS["c1"]
    sched = chains.search_schedule(ctx, cfg, 40, window=2_000)
    H, pool_list, _, p = chains.make_chain(ctx, cfg, sched)
    arena, off, ln = pack_chunk(H)
    ln = ln.copy()
    ln[7] -= 5                                      # truncated: DEC_SYNTAX
    ctx.set_epoch(cfg["eta0"], pool_list, p)
    try:
        for mask in (1, 4, 5):
            ctx.set_option(abi.OPT_KERNELS, mask)
            o = ctx.verify_header_bytes(arena, off, ln)
            assert o["bits"][7] & abi.BIT_INPUT and int((o["bits"][:7] & abi.BIT_INPUT).sum()) == 0
    finally:
        ctx.set_option(abi.OPT_KERNELS, 7)
