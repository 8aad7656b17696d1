"""TPraos decentralisation overlay and chain-state fold through the C ABI on a host-only
context (praos_set_overlay, praos_overlay_classify, praos_tpraos_update_chain_dep_state;
crypto bits synthetic), against oracle/tpraos.py (restated cardano-protocol-tpraos
Rules/Overlay.hs, OCert.hs, Prtcl.hs, Tickn.hs -- parity unpinned: no reference fixture
covers d > 0)."""
import hashlib
import random
from fractions import Fraction

import numpy as np
import pytest

import chainstate as cs
import tpraos as tp


def _b2b(m, n=32):
    return hashlib.blake2b(m, digest_size=n).digest()


@pytest.fixture(scope="module")
def hctx():
    from praos_hip import abi
    c = abi.Context(abi.HOST_ONLY)
    yield c
    c.close()


def _gen(r, k, delegates=None):
    g = []
    for i in range(k):
        dl = delegates[i] if delegates else _b2b(b"dlg" + bytes([i]), 28)
        g.append((_b2b(b"gen" + bytes([r.randrange(256)]) + bytes([i]), 28), dl, _b2b(b"gvrf" + bytes([i]))))
    return g


@pytest.mark.parametrize("d,f", [(Fraction(1, 2), Fraction(1, 20)), (Fraction(1), Fraction(1, 20)),
                                 (Fraction(7, 10), Fraction(1, 2)), (Fraction(3, 1000), Fraction(1, 20)),
                                 (Fraction(2, 4), Fraction(3, 7)), (Fraction(9, 10), Fraction(1)),
                                 (Fraction(0), Fraction(1, 20))])
def test_overlay_classify_vs_oracle(hctx, d, f):
    r = random.Random(hash((d, f)) & 0xffff)
    base, length = 4492800, 432000
    gen = _gen(r, 7)
    hctx.set_overlay(d, f, base, length, gen)
    slots = [base + r.randrange(3 * length) for _ in range(3000)] + [base + k for k in range(400)] + \
            [base + length - 1, base + length, base + 2 * length + 1, base + (1 << 40) + 17]
    got = hctx.overlay_classify(np.array(slots, np.uint64))
    want = [tp.classify(s, d, f, base, length, len(gen)) for s in slots]
    assert list(got) == want
    if d > 0:
        assert (got == -1).any() or d == 1
        assert (got >= 0).any()
    else:
        assert (got == -1).all()
    hctx.set_overlay(None, None, 0, 1, [])
    assert (hctx.overlay_classify(np.array(slots[:50], np.uint64)) == -1).all()


def test_overlay_rejects_bad_arguments(hctx):
    from praos_hip.abi import PraosError
    r = random.Random(3)
    gen = _gen(r, 3)
    for d, f, g in ((Fraction(3, 2), Fraction(1, 20), gen), (Fraction(1, 2), Fraction(1, 20), []),
                    (Fraction(1, 2), Fraction(1, 20), [gen[0], gen[0]])):
        with pytest.raises(PraosError):
            hctx.set_overlay(d, f, 0, 100, g)
    hctx.set_overlay(None, None, 0, 1, [])


def _batch(r, n, pools, dlg_vks, base, length):
    H = {"slot": np.array(sorted(base + r.randrange(2 * length) for _ in range(n)), np.uint64),
         "cold_vk": np.frombuffer(bytes(r.getrandbits(8) for _ in range(32 * n)), np.uint8).reshape(n, 32).copy(),
         "vrf_vk": np.zeros((n, 32), np.uint8), "vrf_out": np.zeros((n, 64), np.uint8),
         "vrf_proof": np.zeros((n, 80), np.uint8), "hot_vk": np.zeros((n, 32), np.uint8),
         "ocert_n": np.array([r.choice([0, 0, 1, 1, 2, 4]) for _ in range(n)], np.uint64),
         "ocert_c0": np.zeros(n, np.uint64), "ocert_sig": np.zeros((n, 64), np.uint8),
         "kes_sig": np.zeros((n, 448), np.uint8), "body_off": np.zeros(n, np.uint64),
         "body_len": np.zeros(n, np.uint32), "body_bytes": np.zeros(8, np.uint8),
         "leader_out": np.zeros((n, 64), np.uint8), "leader_proof": np.zeros((n, 80), np.uint8)}
    # bit patterns a TPraos batch can carry: Praos-slot VRF failures, overlay slots (active,
    # with genesis-key mismatches, or non-active), OCERT failures alone or combined
    pats = [(0, 60), (tp.BIT_TP_OVERLAY, 12), (tp.BIT_TP_OVERLAY | tp.BIT_TP_GEN_COLD, 2),
            (tp.BIT_TP_OVERLAY | tp.BIT_TP_GEN_VRF | tp.BIT_TP_NONCE, 2),
            (tp.BIT_TP_OVERLAY | tp.BIT_TP_NONCE | tp.BIT_TP_LEADER, 2), (tp.BIT_TP_NOT_ACTIVE, 2),
            (tp.BIT_TP_NOT_ACTIVE | tp.BIT_OCERT_SIG, 1), (tp.BIT_VRF_KEY_UNKNOWN | tp.BIT_TP_NONCE, 2),
            (tp.BIT_VRF_KEY_WRONG | tp.BIT_LEADER, 1), (tp.BIT_TP_LEADER | tp.BIT_LEADER, 1), (tp.BIT_LEADER, 3),
            (tp.BIT_KES_AFTER_END | tp.BIT_KES_LEAF | tp.BIT_OCERT_SIG, 1), (tp.BIT_KES_BEFORE_START, 1),
            (tp.BIT_INPUT, 1)]
    bits = np.array([r.choices([b for b, _ in pats], [w for _, w in pats])[0] for _ in range(n)], np.uint16)
    pidx = np.full(n, -1, np.int32)
    for i in range(n):
        if bits[i] & (tp.BIT_TP_OVERLAY | tp.BIT_TP_NOT_ACTIVE):
            if r.random() < 0.8:                                     # a genesis delegate forges
                H["cold_vk"][i] = np.frombuffer(r.choice(dlg_vks), np.uint8)
        elif r.random() > 0.03:
            pidx[i] = r.randrange(len(pools))
    crypto = {"bits": bits, "pool_idx": pidx,
              "nonce": np.frombuffer(bytes(r.getrandbits(8) for _ in range(32 * n)), np.uint8).reshape(n, 32).copy()}
    prev = np.frombuffer(bytes(r.getrandbits(8) for _ in range(32 * n)), np.uint8).reshape(n, 32).copy()
    hk = [pools[p][0] if p >= 0 else _b2b(bytes(H["cold_vk"][i]), 28) for i, p in enumerate(pidx)]
    return H, crypto, prev, hk


@pytest.mark.parametrize("seed,extra", [(1, None), (2, b"\x07" * 32), (3, None)])
def test_tpraos_fold_host_only(hctx, seed, extra):
    from praos_hip import abi, fixed
    r = random.Random(seed)
    pools = [(_b2b(b"pool" + bytes([i]), 28), _b2b(b"vrf" + bytes([i])), fixed.from_rational(Fraction(1, 6)))
             for i in range(6)]
    dlg_vks = [_b2b(b"delegate-vk" + bytes([i])) for i in range(3)]
    dlg_hashes = [_b2b(v, 28) for v in dlg_vks]
    base, length, window = 1000, 5000, 1500
    hctx.set_overlay(Fraction(1, 2), Fraction(1, 20), base, length, _gen(r, 3, dlg_hashes))
    eta0 = _b2b(b"tp-eta0")
    hctx.set_epoch(eta0, pools, abi.params(c_raw=fixed.active_slot_log(Fraction(1, 20))))
    n = 600
    H, crypto, prev, hk = _batch(r, n, pools, dlg_vks, base, length)
    H["slot"][:] = np.sort(np.array([base + r.randrange(length) for _ in range(n)], np.uint64))   # one epoch
    state = {"last_slot": None, "counters": {pools[0][0]: 1, dlg_hashes[1]: 2}, "evolving": _b2b(b"ev"),
             "candidate": _b2b(b"cand"), "epoch_nonce": eta0, "lab": None, "leb": _b2b(b"leb")}
    ref_state = {k: (dict(v) if isinstance(v, dict) else v) for k, v in state.items()}
    ei = (base, 0, length, window)
    v, fails, stop, done = hctx.tpraos_update_chain_dep_state(H, crypto, prev, state, ei, extra_entropy=extra)
    known = {p[0] for p in pools} | set(dlg_hashes)
    rv, rf, rstop, rdone = tp.fold(ref_state, hk, H["slot"], crypto["bits"], H["ocert_n"], crypto["nonce"],
                                   [bytes(x) for x in prev], known, eta0, base, 0, length, window, extra)
    assert done == rdone == n
    assert list(v[:done]) == rv
    assert list(fails[:done]) == rf
    assert stop == rstop
    assert state == ref_state
    assert any(x == tp.V_OK for x in rv) and any(x == tp.V_TPRAOS for x in rv)
    assert any(f & tp.TPF_NOT_ACTIVE for f in rf) and any(f & tp.TPF_GEN_COLD for f in rf)
    hctx.set_overlay(None, None, 0, 1, [])


def test_tpraos_fold_epoch_boundary_extra_entropy(hctx):
    """A valid run across an epoch boundary: the ticked nonce includes the extra entropy
    (TICKN: eta_c ⭒ eta_h ⭒ extraEntropy), so the fold stops where that nonce differs from
    the context's, exactly as the restatement does."""
    from praos_hip import abi, fixed
    r = random.Random(11)
    pools = [(_b2b(b"pool" + bytes([i]), 28), _b2b(b"vrf" + bytes([i])), fixed.from_rational(Fraction(1, 4)))
             for i in range(4)]
    base, length, window = 0, 1000, 300
    extra = _b2b(b"extra")
    eta0 = _b2b(b"e0")
    hctx.set_overlay(None, None, 0, 1, [])
    n = 60
    H, crypto, prev, hk = _batch(r, n, pools, [bytes(32)], base, length)
    H["slot"][:] = np.array([100 + 30 * i for i in range(n)], np.uint64)      # crosses slot 1000
    crypto["bits"][:] = 0
    crypto["pool_idx"][:] = [i % 4 for i in range(n)]
    hk = [pools[i % 4][0] for i in range(n)]
    H["ocert_n"][:] = 0
    st0 = {"last_slot": None, "counters": {}, "evolving": _b2b(b"ev"), "candidate": _b2b(b"c"),
           "epoch_nonce": eta0, "lab": None, "leb": None}
    for ext in (None, extra):
        hctx.set_epoch(eta0, pools, abi.params(c_raw=fixed.active_slot_log(Fraction(1, 20))))
        st, ref = dict(st0, counters={}), dict(st0, counters={})
        v, fails, stop, done = hctx.tpraos_update_chain_dep_state(H, crypto, prev, st, (base, 0, length, window),
                                                                  extra_entropy=ext)
        rv, rf, rstop, rdone = tp.fold(ref, hk, H["slot"], crypto["bits"], H["ocert_n"], crypto["nonce"],
                                       [bytes(x) for x in prev], {p[0] for p in pools}, eta0, base, 0, length,
                                       window, ext)
        assert (done, stop) == (rdone, rstop) and list(v[:done]) == rv and st == ref
        assert done < n                                                   # the tick to epoch 1 ends the fold
        # continue in epoch 1 under the ticked nonce (with the extra entropy folded in)
        nxt = cs.combine(cs.combine(st["candidate"], st["leb"]), ext)
        hctx.set_epoch(nxt, pools, abi.params(c_raw=fixed.active_slot_log(Fraction(1, 20))))
        Hs = {k: (a[done:] if isinstance(a, np.ndarray) and len(a) == n else a) for k, a in H.items()}
        Cs = {k: a[done:] for k, a in crypto.items()}
        v2, f2, stop2, done2 = hctx.tpraos_update_chain_dep_state(Hs, Cs, prev[done:], st,
                                                                   (base, 0, length, window), extra_entropy=ext)
        rv2, rf2, rstop2, rdone2 = tp.fold(ref, hk[done:], Hs["slot"], Cs["bits"], Hs["ocert_n"], Cs["nonce"],
                                           [bytes(x) for x in prev[done:]], {p[0] for p in pools}, nxt, base, 0,
                                           length, window, ext)
        assert done2 == rdone2 == n - done and list(v2) == rv2 and st == ref and all(x == 0 for x in rv2)
