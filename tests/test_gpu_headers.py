"""End-to-end header batches: GPU-synthesised chains (with seeded corruptions),
validated by the GPU pipeline, checked header-by-header against the oracle's
restatement of Praos.hs:558-606 / :528-556, and the sequential verdict order
(praos_apply_batch) against a Python restatement of updateChainDepState."""
from fractions import Fraction

import numpy as np
import pytest

from helpers import arr, b2b, corrupt, rbytes, rng

pytestmark = pytest.mark.gpu

BITS_FROM_ORACLE = 0x0001 | 0x0002 | 0x0004 | 0x0008 | 0x0010 | 0x0100 | 0x0200 | 0x0400 | 0x0800 | 0x1000


def _chain(ctx, n, npools, corrupt_per_10000, seed=b"\x42" * 32, f=Fraction(1, 20), eta0=None,
           stride=20, body_len=397):
    from praos_hip import abi, fixed
    c_raw = fixed.active_slot_log(f)
    p = abi.params(slots_per_kes_period=129600, max_kes_evo=62, c_raw=c_raw)
    eta0 = eta0 if eta0 is not None else b2b(b"genesis")
    H, pools, corrupted = ctx.synthesize(n, npools, p, eta0, seed, first_slot=1000, slot_stride=stride,
                                         body_len=body_len, corrupt_per_10000=corrupt_per_10000)
    # stake: sigma_i ~ 1/(i+10), exact rationals, normalised
    w = [Fraction(1, i + 10) for i in range(npools)]
    tot = sum(w)
    sig = [fixed.from_rational(x / tot) for x in w]
    pool_list = [(h, v, s) for (h, v), s in zip(pools, sig)]
    ctx.set_epoch(eta0, pool_list, p)
    return H, pool_list, corrupted, p, c_raw, eta0


def _oracle_bits(oracle, H, pool_list, c_raw, eta0):
    ep = oracle.make_epoch(eta0, 129600, 62, c_raw, pool_list)
    out = []
    for i in range(len(H["slot"])):
        off, ln = int(H["body_off"][i]), int(H["body_len"][i])
        h = {"slot": int(H["slot"][i]), "cold_vk": bytes(H["cold_vk"][i]), "vrf_vk": bytes(H["vrf_vk"][i]),
             "vrf_out": bytes(H["vrf_out"][i]), "vrf_proof": bytes(H["vrf_proof"][i]),
             "hot_vk": bytes(H["hot_vk"][i]), "n": int(H["ocert_n"][i]), "c0": int(H["ocert_c0"][i]),
             "ocert_sig": bytes(H["ocert_sig"][i]), "kes_sig": bytes(H["kes_sig"][i]),
             "body": bytes(H["body_bytes"][off:off + ln])}
        out.append(oracle.praos_header(ep, h))
    return out


def test_synth_chain_parity(ctx, oracle):
    H, pool_list, corrupted, p, c_raw, eta0 = _chain(ctx, 300, 7, 1500)
    o = ctx.verify_headers(H)
    ref = _oracle_bits(oracle, H, pool_list, c_raw, eta0)
    hash_of = {h: i for i, (h, _, _) in enumerate(pool_list)}
    for i, r in enumerate(ref):
        assert int(o["bits"][i]) & BITS_FROM_ORACLE == r["bits"], (i, hex(o["bits"][i]), hex(r["bits"]), corrupted[i])
        assert bytes(o["beta"][i]) == r["beta"]
        assert bytes(o["leader"][i]) == r["leader"]
        assert bytes(o["nonce"][i]) == r["nonce"]
        assert int(o["pool_idx"][i]) == hash_of.get(r["issuer_hash"], -1)
    # uncorrupted headers carry valid crypto (only the leader check may fail)
    clean = [i for i in range(len(ref)) if corrupted[i] == 0]
    assert clean and all(int(o["bits"][i]) & ~0x1000 == 0 for i in clean)
    assert any(corrupted) and any(int(o["bits"][i]) != 0 for i in range(len(ref)) if corrupted[i])


def _run_batch(ctx, H, keycache, dedup=0, want_dedup_stats=False):
    from praos_hip import abi
    ctx.set_option(abi.OPT_KEYCACHE, keycache)
    ctx.set_option(abi.OPT_DEDUP, dedup)
    try:
        b = ctx.upload(H)
        ctx.run(b)
        ctx.sync()
        st = ctx.batch_stats(b)
        dd = ctx.dedup_stats(b)
        o = ctx.download(b, len(H["slot"]))
        ctx.free(b)
    finally:
        ctx.set_option(abi.OPT_KEYCACHE, 2)
        ctx.set_option(abi.OPT_DEDUP, 1)
    return (o, st, dd) if want_dedup_stats else (o, st)


def test_keycache_equivalence(ctx, oracle):
    """Per-batch key cache (k_keys.hip): cached and uncached chains give identical
    outputs, including repeated invalid keys (small order, non-canonical, not on
    the curve) that take the cached path with their validity flags."""
    H, pool_list, corrupted, p, c_raw, eta0 = _chain(ctx, 1500, 23, 1500, seed=b"\x33" * 32)
    p_plus_2 = (2 ** 255 - 19 + 2).to_bytes(32, "little")            # non-canonical y
    ident = (1).to_bytes(32, "little")                                 # small order (identity)
    not_on_curve = None
    for y in range(2, 200):                                            # first y with no x
        if not oracle.decode_ok(y.to_bytes(32, "little")):
            not_on_curve = y.to_bytes(32, "little")
            break
    assert not_on_curve is not None
    for k, bad in enumerate((p_plus_2, ident, not_on_curve)):
        for j in range(3):                                             # repeated: cached
            H["cold_vk"][10 + 3 * k + j] = np.frombuffer(bad, np.uint8)
            H["vrf_vk"][40 + 3 * k + j] = np.frombuffer(bad, np.uint8)
    o1, st1 = _run_batch(ctx, H, 2)
    o0, st0 = _run_batch(ctx, H, 0)
    assert st1["cold_keys"] >= 23 and st1["cold_hits"] > 1300 and st1["vrf_hits"] > 1300
    assert st0["cold_keys"] == 0 and st0["cold_hits"] == 0
    assert st1["cold_hits"] + st1["cold_misses"] == len(H["slot"])
    for key in ("bits", "beta", "leader", "nonce", "pool_idx"):
        assert np.array_equal(o1[key], o0[key]), key
    ref = _oracle_bits(oracle, H, pool_list, c_raw, eta0)
    for i, r in enumerate(ref):
        assert int(o1["bits"][i]) & BITS_FROM_ORACLE == r["bits"], (i, hex(o1["bits"][i]), hex(r["bits"]))
        assert bytes(o1["beta"][i]) == r["beta"]
    assert all(int(o1["bits"][10 + j]) & 0x0004 for j in range(9))    # OCert rejected for the bad cold keys


def test_stream_schedule_equivalence(ctx, oracle):
    """The concurrent schedule of praos_batch_run (OCert / KES / VRF side streams, the
    VRF stream at high priority, miss lists on the main stream, the OCert misses and
    the dedup fanout at the end of its queue) gives the serial schedule's outputs bit
    for bit, on a batch with cache hits AND misses in all three caches."""
    from praos_hip import abi
    H, pool_list, corrupted, p, c_raw, eta0 = _chain(ctx, 1500, 23, 1500, seed=b"\x5a" * 32)
    r = rng(77)
    for j in range(0, 60, 3):                       # single-use cold / VRF keys: cache misses
        H["cold_vk"][100 + j] = np.frombuffer(rbytes(r, 32), np.uint8)
        H["vrf_vk"][400 + j] = np.frombuffer(rbytes(r, 32), np.uint8)
        H["slot"][700 + j] += 129600 * (1 + j % 3)  # another KES period: a single-use leaf key
    outs = []
    try:
        ctx.set_option(abi.OPT_POOL_KEYS, 0)        # per-batch caches: the single-use keys are misses
        ctx.set_option(abi.OPT_KES_NOCACHE, 0)      # the KES leaf-key cache at this size too
        for conc in (0, 1, 1):
            ctx.set_option(abi.OPT_CONCURRENT, conc)
            o, st, dd = _run_batch(ctx, H, 2, dedup=1, want_dedup_stats=True)
            outs.append(o)
    finally:
        ctx.set_option(abi.OPT_CONCURRENT, 1)
        ctx.set_option(abi.OPT_POOL_KEYS, -1)
        ctx.set_option(abi.OPT_KES_NOCACHE, -1)
    assert st["cold_misses"] > 0 and st["vrf_misses"] > 0 and st["kes_misses"] > 0, st
    assert st["cold_hits"] > 0 and st["vrf_hits"] > 0 and st["kes_hits"] > 0, st
    for o in outs[1:]:
        for key in ("bits", "beta", "leader", "nonce", "pool_idx"):
            assert np.array_equal(o[key], outs[0][key]), key
    ref = _oracle_bits(oracle, H, pool_list, c_raw, eta0)
    for i, rr in enumerate(ref):
        assert int(outs[1]["bits"][i]) & BITS_FROM_ORACLE == rr["bits"], (i, hex(outs[1]["bits"][i]), hex(rr["bits"]))


def test_header_edge_inputs(ctx, oracle):
    """Unknown issuer, wrong VRF key, KES period out of range, neutral nonce."""
    H, pool_list, corrupted, p, c_raw, eta0 = _chain(ctx, 64, 5, 0, seed=b"\x07" * 32)
    n = len(H["slot"])
    H["cold_vk"][1] = H["cold_vk"][0] if bytes(H["cold_vk"][0]) != bytes(H["cold_vk"][1]) else H["cold_vk"][2]
    H["vrf_vk"][2] = np.frombuffer(b2b(b"x"), np.uint8)
    H["ocert_c0"][3] = 10 ** 6                       # KESBeforeStart
    H["slot"][4] = 129600 * 70                       # KESAfterEnd (kp - c0 >= 62)
    H["cold_vk"][5] = np.frombuffer(b2b(b"nobody"), np.uint8)   # unknown pool
    pools_wrong_vrf = list(pool_list)
    o = ctx.verify_headers(H)
    ref = _oracle_bits(oracle, H, pool_list, c_raw, eta0)
    for i, r in enumerate(ref):
        assert int(o["bits"][i]) & BITS_FROM_ORACLE == r["bits"], i
    assert int(o["bits"][5]) & 0x0100
    assert int(o["bits"][3]) & 0x0001 and int(o["bits"][4]) & 0x0002
    # neutral epoch nonce: alpha = Blake2b256(BE64 slot)
    ctx.set_epoch(None, pools_wrong_vrf, p)
    o2 = ctx.verify_headers(H)
    ref2 = _oracle_bits(oracle, H, pool_list, c_raw, None)
    for i, r in enumerate(ref2):
        assert int(o2["bits"][i]) & BITS_FROM_ORACLE == r["bits"], i


def _apply_python(H, bits, pool_idx, pool_list, counters):
    """Restatement of the first-error order of Praos.updateChainDepState."""
    from praos_hip import abi
    known = {h for h, _, _ in pool_list}
    cm = dict(counters)
    verdicts, stop = [], None
    for i in range(len(H["slot"])):
        b = int(bits[i])
        hk = pool_list[pool_idx[i]][0] if pool_idx[i] >= 0 else b2b(bytes(H["cold_vk"][i]), 28)
        n = int(H["ocert_n"][i])
        if b & abi.BIT_INPUT:
            v = abi.V_INPUT
        elif b & abi.BIT_KES_BEFORE_START:
            v = abi.V_KES_BEFORE_START
        elif b & abi.BIT_KES_AFTER_END:
            v = abi.V_KES_AFTER_END
        elif b & abi.BIT_OCERT_SIG:
            v = abi.V_OCERT_SIG
        elif b & (abi.BIT_KES_MERKLE | abi.BIT_KES_LEAF):
            v = abi.V_KES_SIG
        else:
            m = cm.get(hk, 0 if hk in known else None)
            if m is None:
                v = abi.V_COUNTER_MISSING
            elif not m <= n:
                v = abi.V_COUNTER_TOO_SMALL
            elif not n <= m + 1:
                v = abi.V_COUNTER_OVER_INC
            elif b & abi.BIT_VRF_KEY_UNKNOWN:
                v = abi.V_VRF_KEY_UNKNOWN
            elif b & abi.BIT_VRF_KEY_WRONG:
                v = abi.V_VRF_KEY_WRONG
            elif b & (abi.BIT_VRF_PROOF | abi.BIT_VRF_OUTPUT):
                v = abi.V_VRF_BAD_PROOF
            elif b & abi.BIT_LEADER:
                v = abi.V_LEADER_TOO_BIG
            else:
                v = abi.V_OK
        verdicts.append(v)
        if v == abi.V_OK:
            cm[hk] = n
        elif stop is None:
            stop = i
    return verdicts, (stop if stop is not None else len(H["slot"])), cm


def test_apply_batch_order(ctx):
    from praos_hip import abi, fixed
    H, pool_list, corrupted, p, c_raw, eta0 = _chain(ctx, 200, 6, 800, seed=b"\x09" * 32, f=Fraction(9, 10))
    o = ctx.verify_headers(H)
    r = rng(3)
    # counters: some pools ahead (CounterTooSmall), some behind by 2 (OverIncremented)
    counters = {pool_list[0][0]: 5, pool_list[1][0]: 0, b2b(b"retired", 28): 3}
    H["ocert_n"][10] = 7
    verdict, stop, cm = ctx.apply_batch(H, o, counters)
    want, want_stop, want_cm = _apply_python(H, o["bits"], o["pool_idx"], pool_list, counters)
    assert list(verdict) == want
    assert stop == want_stop
    for k in counters:
        assert cm[k] == want_cm[k]
    assert abi.V_OK in want and len(set(want)) >= 3


def test_chain_dep_state_fold_gpu(ctx):
    """praos_update_chain_dep_state over a GPU-verified synthetic chain: the nonce fold
    uses the GPU's vrfNonceValue outputs; checked against oracle/chainstate.py."""
    import chainstate as cs
    H, pool_list, corrupted, p, c_raw, eta0 = _chain(ctx, 300, 5, 300, seed=b"\x0b" * 32, f=Fraction(9, 10))
    o = ctx.verify_headers(H)
    n = len(H["slot"])
    prev = np.stack([np.frombuffer(b2b(i.to_bytes(8, "big")), np.uint8) for i in range(n)])
    st = {"last_slot": None, "counters": {}, "evolving": eta0, "candidate": eta0, "epoch_nonce": eta0,
          "lab": None, "leb": None}
    ref = dict(st, counters={})
    base = int(H["slot"][0]) - int(H["slot"][0]) % 432000
    ei = (base, 0, 432000, 129600)
    v, stop, done = ctx.update_chain_dep_state(H, o, prev, st, ei)
    hk = [pool_list[pi][0] if pi >= 0 else b2b(bytes(H["cold_vk"][i]), 28) for i, pi in enumerate(o["pool_idx"])]
    wv, wstop, wdone = cs.fold(ref, hk, H["slot"], o["bits"], H["ocert_n"], o["nonce"], [bytes(x) for x in prev],
                               {q[0] for q in pool_list}, eta0, base, 0, 432000, 129600)
    assert (done, stop) == (wdone, wstop) and list(v) == wv and st == ref


def test_ocert_dedup_equivalence(ctx, oracle):
    """OCert dedup (PRAOS_OPT_DEDUP, k_keys.hip k_ocert_dedup / k_ocert_fanout): every
    header's outputs are identical with and without it, with and without the key
    cache -- including invalid tuples repeated over several headers, and headers
    sharing a tuple whose KES-period checks differ (slot-dependent, per header)."""
    H, pool_list, corrupted, p, c_raw, eta0 = _chain(ctx, 1500, 23, 1500, seed=b"\x5a" * 32)
    bad = [i for i in range(1500) if corrupted[i]]
    assert bad
    # an invalid OCert signature carried by five headers (copies of one tuple)
    src = 100
    H["ocert_sig"][src][3] ^= 0x40
    for j in range(101, 105):
        for f in ("cold_vk", "hot_vk", "ocert_sig"):
            H[f][j] = H[f][src]
        H["ocert_n"][j] = H["ocert_n"][src]
        H["ocert_c0"][j] = H["ocert_c0"][src]
    # a header sharing its pool's tuple, in a KES period past the OCert's end
    H["slot"][201] = int(H["slot"][201]) + 129600 * 70
    outs = {}
    for kc in (2, 0):
        for dd in (1, 0):
            outs[(kc, dd)] = _run_batch(ctx, H, kc, dedup=dd, want_dedup_stats=True)
    o_ref = outs[(0, 0)][0]
    for key, (o, st, d) in outs.items():
        for f in ("bits", "beta", "leader", "nonce", "pool_idx"):
            assert np.array_equal(o[f], o_ref[f]), (key, f)
        if key[1]:
            assert d["headers"] == 1500 and 23 <= d["ocert_unique"] < 400, d
        else:
            assert d["ocert_unique"] == 0
    assert all(int(o_ref["bits"][j]) & 0x0004 for j in range(100, 105))
    assert int(o_ref["bits"][201]) & 0x0002
    ref = _oracle_bits(oracle, H, pool_list, c_raw, eta0)
    for i, r in enumerate(ref):
        assert int(o_ref["bits"][i]) & BITS_FROM_ORACLE == r["bits"], (i, hex(o_ref["bits"][i]), hex(r["bits"]))
