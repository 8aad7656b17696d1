"""GPU parity of the verification batches (C ABI) against the oracle and the
reference's golden KATs (tests/golden/reference_kats.json).  Bit-exact on
verdicts, VRF outputs and leader decisions."""
import json
import os
from fractions import Fraction

import numpy as np
import pytest

from helpers import L, P, arr, b2b, corrupt, rbytes, rng

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
KATS = json.load(open(os.path.join(HERE, "golden", "reference_kats.json")))["kats"]
H = bytes.fromhex


def _ocert_msg(hot, n, c0):
    return hot + n.to_bytes(8, "big") + c0.to_bytes(8, "big")


# ---------------------------------------------------------------- OCert / Ed25519
def _ocert_vectors(oracle, seed, n):
    r = rng(seed)
    cold, hot, ns, c0s, sig = [], [], [], [], []
    for i in range(n):
        sk = rbytes(r, 32)
        pk = oracle.ed25519_pk(sk)
        hv = rbytes(r, 32)
        nn, cc = r.getrandbits(16), r.randrange(600)
        s = oracle.ed25519_sign(sk, _ocert_msg(hv, nn, cc))
        kind = i % 10
        if kind == 1:
            s = corrupt(s, r.getrandbits(16))
        elif kind == 2:
            pk = corrupt(pk, r.getrandbits(16))
        elif kind == 3:
            hv = corrupt(hv, r.getrandbits(16))
        elif kind == 4:  # S + L (non-canonical S, same point equation)
            S = int.from_bytes(s[32:], "little") + L
            if S < 2 ** 256:
                s = s[:32] + S.to_bytes(32, "little")
        elif kind == 5:  # small-order R
            s = bytes(32) + s[32:]
        elif kind == 6:  # small-order A
            pk = (P - 1).to_bytes(32, "little")
        elif kind == 7:  # non-canonical A encoding (y + p) when representable
            y = int.from_bytes(pk, "little") & (2 ** 255 - 1)
            if y + P < 2 ** 255:
                pk = ((y + P) | (int.from_bytes(pk, "little") & 2 ** 255)).to_bytes(32, "little")
            else:
                pk = (P + 3).to_bytes(32, "little")
        elif kind == 8:  # flip sign of A
            pk = pk[:31] + bytes([pk[31] ^ 0x80])
        cold.append(pk); hot.append(hv); ns.append(nn); c0s.append(cc); sig.append(s)
    return cold, hot, ns, c0s, sig


def test_ocert_batch_vs_oracle(ctx, oracle):
    cold, hot, ns, c0s, sig = _ocert_vectors(oracle, 11, 600)
    ok = ctx.verify_ocert(arr(cold, 32), arr(hot, 32), np.array(ns, np.uint64), np.array(c0s, np.uint64),
                          arr(sig, 64))
    want = [oracle.ed25519_verify(c, _ocert_msg(h, n, c0), s) for c, h, n, c0, s in zip(cold, hot, ns, c0s, sig)]
    assert [bool(x) for x in ok] == want
    assert sum(want) >= 100 and sum(want) < len(want)


def test_ocert_reference_kats(ctx):
    ok = ctx.verify_ocert(arr([H(k["cold_vk"]) for k in KATS], 32), arr([H(k["hot_vk"]) for k in KATS], 32),
                          np.array([k["n"] for k in KATS], np.uint64), np.array([k["c0"] for k in KATS], np.uint64),
                          arr([H(k["ocert_sig"]) for k in KATS], 64))
    assert all(ok == 1)


# ---------------------------------------------------------------- KES
def test_kes_reference_kats(ctx):
    vk, per, sig, msgs, want = [], [], [], [], []
    for k in KATS:
        vk.append(H(k["hot_vk"])); per.append(0); sig.append(H(k["kes_sig"])); msgs.append(H(k["body_cbor"]))
        want.append(0 if k["kind"] == "tpraos" else 2)
        if k["kind"] == "praos":  # the leaf verifies over the reconstructed TPraos body
            vk.append(H(k["hot_vk"])); per.append(0); sig.append(H(k["kes_sig"])); msgs.append(H(k["kes_recon_body"]))
            want.append(0)
    res = ctx.verify_kes(arr(vk, 32), np.array(per, np.uint32), arr(sig, 448), msgs)
    assert list(res) == want


def test_kes_vs_oracle(ctx, oracle):
    r = rng(12)
    vk, per, sig, msgs = [], [], [], []
    for key in range(4):
        seed = rbytes(r, 32)
        v = oracle.kes_vk(seed)
        for j in range(12):
            t = r.randrange(64)
            m = rbytes(r, r.choice([0, 1, 63, 64, 100, 397, 500]))
            s = oracle.kes_sign(seed, t, m)
            kind = j % 6
            tt = t
            if kind == 1:
                s = corrupt(s, r.getrandbits(16))
            elif kind == 2:
                tt = (t + 1) % 64            # wrong period -> wrong branch (Reject or leaf failure)
            elif kind == 3 and m:
                m = corrupt(m, r.getrandbits(16))
            elif kind == 4:
                tt = t + 64 * r.randrange(1, 4)   # Word period beyond 2^6 (reference semantics)
            vk.append(v); per.append(tt); sig.append(s); msgs.append(m)
    res = ctx.verify_kes(arr(vk, 32), np.array(per, np.uint32), arr(sig, 448), msgs)
    want = [oracle.kes_verify(v, t, m, s) for v, t, m, s in zip(vk, per, msgs, sig)]
    assert list(res) == want
    assert 0 in want and 1 in want and 2 in want


# ---------------------------------------------------------------- VRF
def test_vrf_reference_kats(ctx):
    vk, pr, al, out = [], [], [], []
    for k in KATS:
        if k["kind"] == "tpraos":
            for p, o, a in ((k["eta_proof"], k["eta_out"], k["expect"]["eta_alpha"]),
                            (k["leader_proof"], k["leader_out"], k["expect"]["leader_alpha"])):
                vk.append(H(k["vrf_vk"])); pr.append(H(p)); al.append(H(a)); out.append(H(o))
        else:
            vk.append(H(k["vrf_vk"])); pr.append(H(k["vrf_proof"])); al.append(H(k["expect"]["vrf_alpha"]))
            out.append(H(k["vrf_out"]))
    ok, beta = ctx.verify_vrf(arr(vk, 32), arr(pr, 80), arr(al, 32))
    assert all(ok == 1)
    assert [bytes(b) for b in beta] == out
    # wrong alpha (mkInputVRF instead of the example's dummy seed) -> VRFKeyBadProof
    bad = [b2b(b"\x07" + a) for a in al]
    ok2, beta2 = ctx.verify_vrf(arr(vk, 32), arr(pr, 80), arr(bad, 32))
    assert all(ok2 == 0)
    assert [bytes(b) for b in beta2] == out      # proof_to_hash does not depend on alpha


def test_vrf_vs_oracle(ctx, oracle):
    r = rng(13)
    vk, pr, al = [], [], []
    for i in range(160):
        sk = rbytes(r, 32)
        pk = oracle.vrf_pk(sk)
        a = rbytes(r, 32)
        proof = oracle.vrf_prove(sk, a)
        kind = i % 8
        if kind == 1:
            proof = corrupt(proof, r.getrandbits(16))
        elif kind == 2:
            a = corrupt(a, r.getrandbits(16))
        elif kind == 3:
            pk = corrupt(pk, r.getrandbits(16))
        elif kind == 4:  # s + L: still valid (s is reduced, not canonicity-checked)
            s = int.from_bytes(proof[48:], "little") + L
            if s < 2 ** 256:
                proof = proof[:48] + s.to_bytes(32, "little")
        elif kind == 5:  # small-order pk
            pk = bytes([1] + [0] * 31)
        elif kind == 6:  # undecodable Gamma
            while True:
                g = rbytes(r, 32)
                if not oracle.decode_ok(g):
                    break
            proof = g + proof[32:]
        vk.append(pk); pr.append(proof); al.append(a)
    ok, beta = ctx.verify_vrf(arr(vk, 32), arr(pr, 80), arr(al, 32))
    for pk, p, a, k, b in zip(vk, pr, al, ok, beta):
        want = oracle.vrf_verify(pk, p, a)
        assert bool(k) == (want is not None), (pk.hex(), p.hex())
        if want is not None:
            assert bytes(b) == want
        p2h = oracle.vrf_proof_to_hash(p)
        assert bytes(b) == (p2h if p2h is not None else bytes(64))
    assert 0 < int(ok.sum()) < len(ok)


# ---------------------------------------------------------------- leader
def _leader_python(l, sigma_fp, c_raw):
    """Independent exact restatement of checkLeaderNatValue (pure Python ints)."""
    R = 10 ** 34
    x = -((sigma_fp * c_raw) // R)
    q = (2 ** 256 * R) // (2 ** 256 - l)
    err, acc, n = x, R, 0
    while True:
        if n == 1000:
            return False
        k = n + 2
        errp = ((err * x) // R) // k
        accp = acc + err
        e = 3 * errp
        if q >= accp + e:
            return False
        if q < accp - e:
            return True
        err, acc, n = errp, accp, n + 1


def test_leader_vs_oracle(ctx, oracle):
    from praos_hip import abi, fixed
    r = rng(14)
    c_raw = fixed.active_slot_log(Fraction(1, 20))
    ls, sig = [], []
    sigmas = [Fraction(1, 3000), Fraction(1, 100), Fraction(1, 2), Fraction(1), Fraction(0), Fraction(17, 10007)]
    for i in range(400):
        s = sigmas[i % len(sigmas)] if i < 60 else Fraction(r.randrange(1, 10 ** 6), 10 ** 6 + r.randrange(10 ** 6))
        sf = fixed.from_rational(s)
        if i % 3 == 0:
            # leader value at the threshold: p = 1 - (1-f)^sigma
            import math
            p = 1 - math.exp(float(s) * math.log(0.95))
            l = int(p * 2 ** 256) + r.randrange(-3, 4) * 2 ** 200
            l = min(max(l, 0), 2 ** 256 - 1)
        else:
            l = r.getrandbits(256) >> r.randrange(0, 32)
        ls.append(l.to_bytes(32, "big")); sig.append(sf)
    res = ctx.check_leader(arr(ls, 32), arr([s.to_bytes(16, "little") for s in sig], 16),
                           abi.params(c_raw=c_raw))
    for lb, sf, got in zip(ls, sig, res):
        want_c, _ = oracle.check_leader(lb, sf, c_raw)
        want_py = _leader_python(int.from_bytes(lb, "big"), sf, c_raw)
        assert want_c == want_py
        assert bool(got) == want_c
    assert 0 < int(res.sum()) < len(res)


def test_leader_f_is_one(ctx):
    from praos_hip import abi
    res = ctx.check_leader(arr([bytes([0xff] * 32)], 32), arr([bytes(16)], 16), abi.params(f_is_one=True))
    assert list(res) == [1]


def test_leader_boundary_vectors(ctx):
    """Bisected decision boundaries (tests/golden/leader_boundary.json): for each (sigma, f)
    the leader values l*-2, l*-1 (leader) and l*, l*+1 (not leader), 256-bit (Praos) and
    512-bit (TPraos) forms; decisions and Taylor iteration counts bit-exact."""
    import json
    import os
    R = 10 ** 34
    cases = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "leader_boundary.json")))["cases"]
    for bits in (256, 512):
        ls, xs, want, want_it = [], [], [], []
        for c in (c for c in cases if c["bits"] == bits):
            x = -((int(c["sigma_fp"]) * int(c["c_raw"])) // R)
            for v in c["vectors"]:
                ls.append(int(v["leader_value"], 16).to_bytes(bits // 8, "big"))
                xs.append(x.to_bytes(16, "little"))
                want.append(int(v["is_leader"]))
                want_it.append(v["iterations"])
        fn = ctx.debug_leader if bits == 256 else ctx.debug_leader512
        res, it = fn(arr(ls, bits // 8), arr(xs, 16))
        assert list(res) == want and list(it) == want_it
