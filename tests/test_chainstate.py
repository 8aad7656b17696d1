"""The host-side sequential part (Praos.hs:407-502) through the C ABI on a host-only
context (no GPU: crypto bits are synthetic), against oracle/chainstate.py."""
import hashlib
import random
from fractions import Fraction

import numpy as np
import pytest

import chainstate as cs


def _b2b(m, n=32):
    return hashlib.blake2b(m, digest_size=n).digest()


@pytest.fixture(scope="module")
def hctx():
    from praos_hip import abi
    c = abi.Context(abi.HOST_ONLY)
    yield c
    c.close()


def _batch(r, n, pools, first_slot, stride):
    H = {"slot": np.array([first_slot + i * stride + r.randrange(stride) for i in range(n)], np.uint64),
         "cold_vk": np.frombuffer(bytes(r.getrandbits(8) for _ in range(32 * n)), np.uint8).reshape(n, 32).copy(),
         "vrf_vk": np.zeros((n, 32), np.uint8), "vrf_out": np.zeros((n, 64), np.uint8),
         "vrf_proof": np.zeros((n, 80), np.uint8), "hot_vk": np.zeros((n, 32), np.uint8),
         "ocert_n": np.zeros(n, np.uint64), "ocert_c0": np.zeros(n, np.uint64),
         "ocert_sig": np.zeros((n, 64), np.uint8), "kes_sig": np.zeros((n, 448), np.uint8),
         "body_off": np.zeros(n, np.uint64), "body_len": np.zeros(n, np.uint32), "body_bytes": np.zeros(8, np.uint8)}
    weights = [(0, 80), (cs.BIT_OCERT_SIG, 2), (cs.BIT_KES_LEAF, 2), (cs.BIT_VRF_PROOF, 2), (cs.BIT_LEADER, 3),
               (cs.BIT_VRF_KEY_WRONG, 1), (cs.BIT_KES_AFTER_END, 1), (cs.BIT_INPUT, 1)]
    bits = np.array([r.choices([b for b, _ in weights], [w for _, w in weights])[0] for _ in range(n)], np.uint16)
    pidx = np.array([r.randrange(len(pools)) if r.random() > 0.02 else -1 for _ in range(n)], np.int32)
    for i in range(n):
        H["ocert_n"][i] = r.choice([0, 0, 1, 1, 2, 5])
    crypto = {"bits": bits, "pool_idx": pidx, "beta": np.zeros((n, 64), np.uint8),
              "leader": np.zeros((n, 32), np.uint8),
              "nonce": np.frombuffer(bytes(r.getrandbits(8) for _ in range(32 * n)), np.uint8).reshape(n, 32).copy()}
    prev = np.frombuffer(bytes(r.getrandbits(8) for _ in range(32 * n)), np.uint8).reshape(n, 32).copy()
    hk = [pools[p][0] if p >= 0 else _b2b(bytes(H["cold_vk"][i]), 28) for i, p in enumerate(pidx)]
    return H, crypto, prev, hk


def _pools(r, k):
    from praos_hip import fixed
    return [(_b2b(b"pool" + bytes([i]), 28), _b2b(b"vrf" + bytes([i])), fixed.from_rational(Fraction(1, k)))
            for i in range(k)]


def _params():
    from praos_hip import abi, fixed
    return abi.params(c_raw=fixed.active_slot_log(Fraction(1, 20)))


def test_apply_batch_host_only(hctx):
    r = random.Random(5)
    pools = _pools(r, 8)
    hctx.set_epoch(_b2b(b"e"), pools, _params())
    H, crypto, prev, hk = _batch(r, 400, pools, 1000, 7)
    counters = {pools[0][0]: 1, pools[1][0]: 4, _b2b(b"gone", 28): 2}
    v, stop, cm = hctx.apply_batch(H, crypto, counters)
    want, want_stop, want_cm = cs.apply_batch(hk, crypto["bits"], H["ocert_n"], {p[0] for p in pools}, counters)
    assert list(v) == want and stop == want_stop
    assert all(cm[k] == want_cm[k] for k in counters)
    assert len(set(want)) >= 6


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_chain_dep_state_stops_at_first_invalid(hctx, seed):
    """A batch with invalid headers: the returned state is the state after the last
    valid header before the first invalid one (the reference stops the chain there,
    Praos.hs:441-459 in Except); later headers still get would-be verdicts."""
    r = random.Random(100 + seed)
    pools = _pools(r, 6)
    base, length, window = 3000, 6000, 180
    H, crypto, prev, hk = _batch(r, 200, pools, base + 40, 7)
    eta = _b2b(b"epoch-a")
    st = {"last_slot": None, "counters": {pools[2][0]: 0}, "evolving": _b2b(b"ev"), "candidate": _b2b(b"cand"),
          "epoch_nonce": eta, "lab": None, "leb": _b2b(b"leb")}
    ref = {k: (dict(v) if isinstance(v, dict) else v) for k, v in st.items()}
    hctx.set_epoch(eta, pools, _params())
    v, stop, done = hctx.update_chain_dep_state(H, crypto, prev, st, (base, 0, length, window))
    wv, wstop, wdone = cs.fold(ref, hk, H["slot"], crypto["bits"], H["ocert_n"], crypto["nonce"],
                               [bytes(p) for p in prev], {p[0] for p in pools}, eta, base, 0, length, window)
    assert (done, stop) == (wdone, wstop) == (200, wstop)
    assert stop < 200 and list(v) == wv
    assert st == ref
    assert st["last_slot"] == (int(H["slot"][stop - 1]) if stop > 0 else None)


def test_failed_set_epoch_leaves_no_epoch(hctx):
    """A praos_set_epoch that fails (here: x_raw out of range) must not leave the previous
    epoch's tables behind: the next call needing an epoch returns PRAOS_E_STATE."""
    from praos_hip import abi
    r = random.Random(11)
    pools = _pools(r, 3)
    hctx.set_epoch(_b2b(b"ok"), pools, _params())
    bad = [(h, v, 1 << 127) for h, v, _ in pools]        # sigma ~ 1.7e4: x_raw > 16 * 10^34
    with pytest.raises(abi.PraosError):
        hctx.set_epoch(_b2b(b"bad"), bad, _params())
    H, crypto, prev, hk = _batch(r, 8, pools, 0, 5)
    with pytest.raises(abi.PraosError, match="rc=-4"):
        hctx.apply_batch(H, crypto, {})


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_chain_dep_state_fold_across_epochs(hctx, seed):
    """Two epochs of 600 slots, stability window 180, all headers valid: the fold stops
    at the boundary (the ticked epoch nonce differs from the context's), resumes after
    set_epoch with the nonce the state computed, and matches the restatement step for step."""
    r = random.Random(seed)
    pools = _pools(r, 6)
    base, length, window = 3000, 600, 180
    H, crypto, prev, hk = _batch(r, 160, pools, base + 40, 7)      # slots 3040 .. ~4160: epochs 0, 1
    crypto["bits"][:] = 0
    for i in range(160):                                             # known issuers, valid counters
        H["ocert_n"][i] = 0
        if crypto["pool_idx"][i] < 0:
            crypto["pool_idx"][i] = 0
            hk[i] = pools[0][0]
    genesis = np.zeros(160, np.uint8)
    genesis[0] = 1
    eta_a = _b2b(b"epoch-a")
    st = {"last_slot": None, "counters": {pools[2][0]: 0}, "evolving": _b2b(b"ev"), "candidate": _b2b(b"cand"),
          "epoch_nonce": eta_a, "lab": None, "leb": _b2b(b"leb")}
    ref = {k: (dict(v) if isinstance(v, dict) else v) for k, v in st.items()}
    known = {p[0] for p in pools}
    ei = (base, 0, length, window)
    prev_l = [None if genesis[i] else bytes(prev[i]) for i in range(160)]
    done_total, calls = 0, 0
    eta = eta_a
    for _ in range(3):
        calls += 1
        hctx.set_epoch(eta, pools, _params())
        sl = slice(done_total, None)
        Hs = {k: (v[sl] if k not in ("body_bytes",) else v) for k, v in H.items()}
        Hs = {k: np.ascontiguousarray(v) for k, v in Hs.items()}
        cr = {k: np.ascontiguousarray(v[sl]) for k, v in crypto.items()}
        v, stop, done = hctx.update_chain_dep_state(Hs, cr, prev[sl], st, ei, prev_is_genesis=genesis[sl])
        wv, wstop, wdone = cs.fold(ref, hk[sl], Hs["slot"], cr["bits"], Hs["ocert_n"], cr["nonce"], prev_l[sl],
                                   known, eta, base, 0, length, window)
        assert done == wdone and stop == wstop
        assert list(v[:done]) == wv
        assert st == ref
        done_total += done
        if done_total == 160:
            break
        # the state ticks into the next epoch: eta = candidate ⭒ lastEpochBlock
        eta = cs.combine(ref["candidate"], ref["leb"])
    assert done_total == 160 and calls == 2
    assert ref["epoch_nonce"] == eta != eta_a


@pytest.mark.parametrize("seed", [4, 5])
def test_fold_with_per_header_nonces(hctx, seed):
    """praos_validate_headers_nonces (update_chain_dep_state with etas/eta_idx, no envelope):
    the same two-epoch batch as above folds in ONE call when every header carries the
    nonce of its epoch, and matches the restatement epoch by epoch; a header labelled
    with the wrong nonce ends the fold exactly there (processed), with the state of the
    headers before it; praos_ticked_epoch_nonce gives the second epoch's nonce."""
    from praos_hip import abi
    r = random.Random(seed)
    pools = _pools(r, 6)
    base, length, window = 3000, 600, 180
    n = 160
    H, crypto, prev, hk = _batch(r, n, pools, base + 40, 7)
    crypto["bits"][:] = 0
    for i in range(n):
        H["ocert_n"][i] = 0
        if crypto["pool_idx"][i] < 0:
            crypto["pool_idx"][i] = 0
            hk[i] = pools[0][0]
    genesis = np.zeros(n, np.uint8)
    genesis[0] = 1
    eta_a = _b2b(b"epoch-a")
    st0 = {"last_slot": None, "counters": {}, "evolving": _b2b(b"ev"), "candidate": _b2b(b"cand"),
           "epoch_nonce": eta_a, "lab": None, "leb": _b2b(b"leb")}
    known = {p[0] for p in pools}
    ei = (base, 0, length, window)
    prev_l = [None if genesis[i] else bytes(prev[i]) for i in range(n)]
    epoch = ((H["slot"] - base) // length).astype(np.uint8)
    k1 = int(np.nonzero(epoch == 1)[0][0])
    # the restatement, epoch by epoch, gives the second nonce and the final state
    ref = {k: (dict(v) if isinstance(v, dict) else v) for k, v in st0.items()}
    cs.fold(ref, hk[:k1], H["slot"][:k1], crypto["bits"][:k1], H["ocert_n"][:k1], crypto["nonce"][:k1],
            prev_l[:k1], known, eta_a, base, 0, length, window)
    eta_b = cs.combine(ref["candidate"], ref["leb"])
    assert abi.ticked_epoch_nonce(ref, ei, int(H["slot"][k1])) == eta_b
    cs.fold(ref, hk[k1:], H["slot"][k1:], crypto["bits"][k1:], H["ocert_n"][k1:], crypto["nonce"][k1:],
            prev_l[k1:], known, eta_b, base, 0, length, window)
    hctx.set_epoch(eta_a, pools, _params())
    st = {k: (dict(v) if isinstance(v, dict) else v) for k, v in st0.items()}
    v, stop, done = hctx.update_chain_dep_state(H, crypto, prev, st, ei, prev_is_genesis=genesis,
                                                etas=[eta_a, eta_b], eta_idx=epoch)
    assert (stop, done) == (n, n) and int((v != 0).sum()) == 0 and st == ref
    # epoch 1 claimed under epoch 0's nonce: the fold ends at its first header
    st = {k: (dict(v) if isinstance(v, dict) else v) for k, v in st0.items()}
    wrong = epoch.copy()
    wrong[k1:] = 0
    v, stop, done = hctx.update_chain_dep_state(H, crypto, prev, st, ei, prev_is_genesis=genesis,
                                                etas=[eta_a, eta_b], eta_idx=wrong)
    assert done == k1 and stop == k1 and st["last_slot"] == int(H["slot"][k1 - 1])
    with pytest.raises(abi.PraosError):          # an index past the table
        bad = epoch.copy()
        bad[3] = 7
        hctx.update_chain_dep_state(H, crypto, prev, dict(st0), ei, prev_is_genesis=genesis,
                                    etas=[eta_a, eta_b], eta_idx=bad)


def test_host_only_refuses_gpu_calls(hctx):
    from praos_hip import abi
    r = random.Random(9)
    pools = _pools(r, 2)
    hctx.set_epoch(None, pools, _params())
    H, crypto, prev, hk = _batch(r, 4, pools, 0, 5)
    with pytest.raises(abi.PraosError):
        hctx.verify_headers(H)


def _envelope_chain(r, n, first_slot, tip, kind, at):
    """Block numbers / slots / header hashes of a linked chain after `tip`; header `at`
    mutated by `kind` (every later header then fails too: the tip stays before it)."""
    bn0 = 0 if tip is None else tip[1] + 1
    block_no = np.array([bn0 + i for i in range(n)], np.uint64)
    slots = np.array([first_slot + 3 * i + r.randrange(3) for i in range(n)], np.uint64)
    hh = [_b2b(b"hdr" + bytes([i % 256, i // 256])) for i in range(n)]
    prev = [tip[2] if tip is not None else None] + hh[:-1]
    hsize = np.array([r.choice([600, 849, 1100]) for _ in range(n)], np.uint32)
    bsize = np.array([r.randrange(0, 90_000) for _ in range(n)], np.uint32)
    if kind == "block_no":
        block_no[at] += r.choice([1, 2])
    elif kind == "slot":
        slots[at] = slots[at - 1]
    elif kind == "prev":
        prev[at] = _b2b(b"fork")
    elif kind == "genesis":
        prev[at] = None
    elif kind == "hsize":
        hsize[at] = 1101
    elif kind == "bsize":
        bsize[at] = 90_113
    return block_no, slots, hh, prev, hsize, bsize


ENV_KINDS = {"ok": 0, "block_no": 13, "slot": 14, "prev": 15, "genesis": 15, "hsize": 17, "bsize": 18}


@pytest.mark.parametrize("origin", [True, False])
@pytest.mark.parametrize("kind", sorted(ENV_KINDS))
def test_validate_headers_envelope(hctx, kind, origin):
    """praos_validate_headers = validateEnvelope + Praos envelopeChecks, then the protocol
    verdicts (HeaderValidation.hs:413-432), against the oracle restatement: verdicts,
    the chain state and the tip at the chain stop."""
    r = random.Random(sum(map(ord, kind)) * 2 + origin)
    pools = _pools(r, 5)
    n, at = 60, 25
    tip = None if origin else (4000, 77, _b2b(b"tip"))
    H, crypto, _, hk = _batch(r, n, pools, 4100, 7)
    block_no, slots, hh, prev, hsize, bsize = _envelope_chain(r, n, 4100, tip, kind, at)
    H["slot"] = slots
    crypto["bits"][:] = 0
    crypto["bits"][40] = cs.BIT_VRF_PROOF             # a protocol failure after the envelope one
    for i in range(n):
        H["ocert_n"][i] = 0
        if crypto["pool_idx"][i] < 0:
            crypto["pool_idx"][i] = 0
            hk[i] = pools[0][0]
    prev_arr = np.array([list(p) if p is not None else [0] * 32 for p in prev], np.uint8)
    genesis = np.array([p is None for p in prev], np.uint8)
    eta = _b2b(b"epoch-env")
    st = {"last_slot": None, "counters": {}, "evolving": eta, "candidate": eta, "epoch_nonce": eta, "lab": None,
          "leb": None}
    ref = {k: (dict(v) if isinstance(v, dict) else v) for k, v in st.items()}
    env = {"block_no": block_no, "header_hash": np.array([list(x) for x in hh], np.uint8), "header_size": hsize,
           "body_size": bsize, "tip": tip, "max_major_pv": 9, "lv_prot_major": 8, "max_header_size": 1100,
           "max_body_size": 90_112}
    renv = dict(env)
    hctx.set_epoch(eta, pools, _params())
    v, stop, done = hctx.update_chain_dep_state(H, crypto, prev_arr, st, (0, 0, 1_000_000, 129_600),
                                                prev_is_genesis=genesis, envelope=env)
    wv, wstop, wdone = cs.fold(ref, hk, slots, crypto["bits"], H["ocert_n"], crypto["nonce"], prev,
                               {p[0] for p in pools}, eta, 0, 0, 1_000_000, 129_600, env=renv)
    assert (done, stop) == (wdone, wstop) and list(v) == wv
    assert st == ref and env["tip"] == renv["tip"]
    want_stop = at if kind != "ok" else 40
    assert stop == want_stop and wv[want_stop] == (ENV_KINDS[kind] if kind != "ok" else cs.V_VRF_BAD_PROOF)
    assert all(x == cs.V_OK for x in wv[:want_stop])
    assert env["tip"] == (int(slots[want_stop - 1]), int(block_no[want_stop - 1]), hh[want_stop - 1])
    if kind == "ok":
        # ObsoleteNode: the ledger view's protocol version above the node's maximum fails every header
        env2 = dict(env, tip=tip, lv_prot_major=10)
        st2 = {"last_slot": None, "counters": {}, "evolving": eta, "candidate": eta, "epoch_nonce": eta,
               "lab": None, "leb": None}
        v2, stop2, _ = hctx.update_chain_dep_state(H, crypto, prev_arr, st2, (0, 0, 1_000_000, 129_600),
                                                   prev_is_genesis=genesis, envelope=env2)
        assert stop2 == 0 and env2["tip"] == tip and v2[0] == cs.V_ENV_OBSOLETE_NODE


def test_praos_state_codec_golden():
    """praos_state_encode / _decode against the reference's golden PraosState encodings
    (ChainDepState_{Babbage,Conway}, extracted by tests/golden/make_state_golden.py):
    decode gives the example's values, re-encoding gives the same bytes."""
    import json
    import os
    from praos_hip import abi
    G = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "praos_state.json")))["states"]
    assert len(G) == 2
    for g in G:
        raw = bytes.fromhex(g["cbor"])
        st = abi.state_decode(raw)
        assert st["last_slot"] == g["last_slot"]
        assert {k.hex(): v for k, v in st["counters"].items()} == g["counters"]
        for k in ("evolving", "candidate", "epoch_nonce", "lab", "leb"):
            assert (st[k].hex() if st[k] is not None else None) == g[k]
        assert abi.state_encode(st) == raw
    # Origin / empty map / all-neutral round trip, and rejection of malformed input
    z = {"last_slot": None, "counters": {}, "evolving": None, "candidate": None, "epoch_nonce": None, "lab": None,
         "leb": None}
    e = abi.state_encode(z)
    assert e == bytes.fromhex("820087" "8100" "a0" + "8100" * 5) and abi.state_decode(e) == z
    r = random.Random(3)
    big = {"last_slot": 2 ** 40, "counters": {_b2b(bytes([i]), 28): r.getrandbits(64) for i in range(40)},
           "evolving": _b2b(b"e"), "candidate": None, "epoch_nonce": _b2b(b"n"), "lab": _b2b(b"l"), "leb": None}
    assert abi.state_decode(abi.state_encode(big)) == big
    for bad in (raw[:-1], raw + b"\x00", b"\x82\x01" + raw[2:]):
        with pytest.raises(abi.PraosError):
            abi.state_decode(bad)
