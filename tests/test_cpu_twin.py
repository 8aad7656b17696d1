"""The CPU twin (libpraos_cpu.so, the timed CPU baseline) against the oracle, bit for
bit: the same vector families as the GPU parity tests (Ed25519 edge rules, Sum6KES
incl. Word periods, draft-03 VRF incl. undecodable keys / Gamma, the leader test
and its bisected boundary vectors), the reference's golden KATs, and whole Praos
headers signed by the oracle (Praos.hs:558-606 / :528-556 restated in
oracle/praos.c).  Runs on the CPU (no GPU needed)."""
import json
import os
from fractions import Fraction

import numpy as np
import pytest

import test_gpu_verify as G
from helpers import arr, b2b, corrupt, rbytes, rng


@pytest.fixture(scope="module")
def cpu():
    from praos_hip import cpu as C
    c = C.CpuContext(threads=4)
    yield c
    c.close()


def test_ocert_vs_oracle(cpu, oracle):
    G.test_ocert_batch_vs_oracle(cpu, oracle)
    G.test_ocert_reference_kats(cpu)


def test_kes_vs_oracle(cpu, oracle):
    G.test_kes_vs_oracle(cpu, oracle)
    G.test_kes_reference_kats(cpu)


def test_vrf_vs_oracle(cpu, oracle):
    G.test_vrf_vs_oracle(cpu, oracle)
    G.test_vrf_reference_kats(cpu)


def test_leader_vs_oracle(cpu, oracle):
    G.test_leader_vs_oracle(cpu, oracle)
    G.test_leader_f_is_one(cpu)


def test_leader_boundary_vectors(cpu):
    from praos_hip import abi
    cases = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "leader_boundary.json")))["cases"]
    for c in (c for c in cases if c["bits"] == 256):
        ls = [int(v["leader_value"], 16).to_bytes(32, "big") for v in c["vectors"]]
        sig = [int(c["sigma_fp"]).to_bytes(16, "little")] * len(ls)
        res = cpu.check_leader(arr(ls, 32), arr(sig, 16), abi.params(c_raw=int(c["c_raw"])))
        assert list(res) == [int(v["is_leader"]) for v in c["vectors"]]


def _oracle_chain(oracle, r, n, npools, eta0, c_raw):
    """n Praos headers signed by the oracle (pools by round robin), with corruptions."""
    from praos_hip import fixed
    pools = []
    for p in range(npools):
        cold, vrf, kes = rbytes(r, 32), rbytes(r, 32), rbytes(r, 32)
        pools.append((cold, vrf, kes, oracle.ed25519_pk(cold), oracle.vrf_pk(vrf), oracle.kes_vk(kes)))
    H = {k: [] for k in ("slot", "cold_vk", "vrf_vk", "vrf_out", "vrf_proof", "hot_vk", "ocert_n", "ocert_c0",
                         "ocert_sig", "kes_sig", "body")}
    for i in range(n):
        cold, vrf, kes, cpk, vpk, kvk = pools[i % npools]
        slot = 1000 + 37 * i
        kp = slot // 129600
        c0 = kp if i % 7 else kp + 1          # every 7th: KESBeforeStartOCERT
        nn = i % 4
        sig = oracle.ed25519_sign(cold, kvk + nn.to_bytes(8, "big") + c0.to_bytes(8, "big"))
        body = rbytes(r, r.choice([1, 100, 397]))
        t = max(kp - c0, 0)
        ks = oracle.kes_sign(kes, min(t, 63), body)
        alpha = oracle.mk_input_vrf(slot, eta0)
        proof = oracle.vrf_prove(vrf, alpha)
        out = oracle.vrf_proof_to_hash(proof)
        kind = i % 9
        if kind == 1:
            sig = corrupt(sig, r.getrandbits(16))
        elif kind == 2:
            ks = corrupt(ks, r.getrandbits(16))
        elif kind == 3:
            proof = corrupt(proof, r.getrandbits(16))
        elif kind == 4:
            out = corrupt(out, r.getrandbits(16))
        elif kind == 5:
            body = corrupt(body, r.getrandbits(16))
        elif kind == 6:
            cpk = rbytes(r, 32)                   # unknown issuer
        for k, v in (("slot", slot), ("cold_vk", cpk), ("vrf_vk", vpk), ("vrf_out", out), ("vrf_proof", proof),
                     ("hot_vk", kvk), ("ocert_n", nn), ("ocert_c0", c0), ("ocert_sig", sig), ("kes_sig", ks),
                     ("body", body)):
            H[k].append(v)
    sig = [fixed.from_rational(Fraction(1, npools + 1))] * npools
    sig[0] = fixed.from_rational(Fraction(1, 1))   # a pool with all the stake
    pool_list = [(b2b(p[3], 28), b2b(p[4]), s) for p, s in zip(pools, sig)]
    return H, pool_list


def test_headers_vs_oracle(cpu, oracle):
    from praos_hip import abi, fixed
    r = rng(31)
    eta0 = b2b(b"cpu-twin-epoch")
    c_raw = fixed.active_slot_log(Fraction(9, 10))    # pool 0 (all the stake) leads 90 % of slots
    H, pool_list = _oracle_chain(oracle, r, 45, 4, eta0, c_raw)
    n = len(H["slot"])
    bodies = H["body"]
    off = np.cumsum([0] + [len(b) for b in bodies[:-1]]).astype(np.uint64)
    S = {"slot": np.array(H["slot"], np.uint64), "cold_vk": arr(H["cold_vk"], 32), "vrf_vk": arr(H["vrf_vk"], 32),
         "vrf_out": arr(H["vrf_out"], 64), "vrf_proof": arr(H["vrf_proof"], 80), "hot_vk": arr(H["hot_vk"], 32),
         "ocert_n": np.array(H["ocert_n"], np.uint64), "ocert_c0": np.array(H["ocert_c0"], np.uint64),
         "ocert_sig": arr(H["ocert_sig"], 64), "kes_sig": arr(H["kes_sig"], 448), "body_off": off,
         "body_len": np.array([len(b) for b in bodies], np.uint32),
         "body_bytes": np.frombuffer(b"".join(bodies) + bytes(8), np.uint8).copy()}
    p = abi.params(c_raw=c_raw)
    cpu.set_epoch(eta0, pool_list, p)
    o = cpu.verify_headers(S)
    ep = oracle.make_epoch(eta0, 129600, 62, c_raw, pool_list)
    hash_of = {h: i for i, (h, _, _) in enumerate(pool_list)}
    seen = set()
    for i in range(n):
        h = {"slot": H["slot"][i], "cold_vk": H["cold_vk"][i], "vrf_vk": H["vrf_vk"][i], "vrf_out": H["vrf_out"][i],
             "vrf_proof": H["vrf_proof"][i], "hot_vk": H["hot_vk"][i], "n": H["ocert_n"][i], "c0": H["ocert_c0"][i],
             "ocert_sig": H["ocert_sig"][i], "kes_sig": H["kes_sig"][i], "body": bodies[i]}
        ref = oracle.praos_header(ep, h)
        assert int(o["bits"][i]) == ref["bits"], (i, hex(o["bits"][i]), hex(ref["bits"]))
        assert bytes(o["beta"][i]) == ref["beta"] and bytes(o["leader"][i]) == ref["leader"]
        assert bytes(o["nonce"][i]) == ref["nonce"]
        assert int(o["pool_idx"][i]) == hash_of.get(ref["issuer_hash"], -1)
        seen.add(ref["bits"])
    assert 0 in seen and len(seen) >= 6


def _oracle_tpraos_chain(oracle, r, n, npools, eta0):
    """n TPraos headers signed by the oracle: both certificates proved over mkSeed seedEta /
    seedL (oracle.tpraos_seed), with corruptions in every checked field."""
    pools = []
    for p in range(npools):
        cold, vrf, kes = rbytes(r, 32), rbytes(r, 32), rbytes(r, 32)
        pools.append((cold, vrf, kes, oracle.ed25519_pk(cold), oracle.vrf_pk(vrf), oracle.kes_vk(kes)))
    H = {k: [] for k in ("slot", "cold_vk", "vrf_vk", "vrf_out", "vrf_proof", "hot_vk", "ocert_n", "ocert_c0",
                         "ocert_sig", "kes_sig", "body", "leader_out", "leader_proof")}
    for i in range(n):
        cold, vrf, kes, cpk, vpk, kvk = pools[i % npools]
        slot = 2000 + 41 * i
        kp = slot // 129600
        c0 = kp if i % 11 else kp + 1
        nn = i % 3
        sig = oracle.ed25519_sign(cold, kvk + nn.to_bytes(8, "big") + c0.to_bytes(8, "big"))
        body = rbytes(r, r.choice([50, 560]))
        ks = oracle.kes_sign(kes, min(max(kp - c0, 0), 63), body)
        pe = oracle.vrf_prove(vrf, oracle.tpraos_seed(slot, eta0, 0))
        pl = oracle.vrf_prove(vrf, oracle.tpraos_seed(slot, eta0, 1))
        oe, ol = oracle.vrf_proof_to_hash(pe), oracle.vrf_proof_to_hash(pl)
        kind = i % 10
        if kind == 1:
            sig = corrupt(sig, r.getrandbits(16))
        elif kind == 2:
            ks = corrupt(ks, r.getrandbits(16))
        elif kind == 3:
            pe = corrupt(pe, r.getrandbits(16))
        elif kind == 4:
            oe = corrupt(oe, r.getrandbits(16))
        elif kind == 5:
            pl = corrupt(pl, r.getrandbits(16))
        elif kind == 6:
            ol = corrupt(ol, r.getrandbits(16))
        elif kind == 7:
            cpk = rbytes(r, 32)
        for k, v in (("slot", slot), ("cold_vk", cpk), ("vrf_vk", vpk), ("vrf_out", oe), ("vrf_proof", pe),
                     ("hot_vk", kvk), ("ocert_n", nn), ("ocert_c0", c0), ("ocert_sig", sig), ("kes_sig", ks),
                     ("body", body), ("leader_out", ol), ("leader_proof", pl)):
            H[k].append(v)
    return H, pools


def _soa(H):
    bodies = H["body"]
    off = np.cumsum([0] + [len(b) for b in bodies[:-1]]).astype(np.uint64)
    S = {"slot": np.array(H["slot"], np.uint64), "cold_vk": arr(H["cold_vk"], 32), "vrf_vk": arr(H["vrf_vk"], 32),
         "vrf_out": arr(H["vrf_out"], 64), "vrf_proof": arr(H["vrf_proof"], 80), "hot_vk": arr(H["hot_vk"], 32),
         "ocert_n": np.array(H["ocert_n"], np.uint64), "ocert_c0": np.array(H["ocert_c0"], np.uint64),
         "ocert_sig": arr(H["ocert_sig"], 64), "kes_sig": arr(H["kes_sig"], 448), "body_off": off,
         "body_len": np.array([len(b) for b in bodies], np.uint32),
         "body_bytes": np.frombuffer(b"".join(bodies) + bytes(8), np.uint8).copy()}
    if "leader_out" in H:
        S["leader_out"], S["leader_proof"] = arr(H["leader_out"], 64), arr(H["leader_proof"], 80)
    return S


def test_tpraos_headers_vs_oracle(cpu, oracle):
    """The twin's praos_verify_tpraos_headers (TPraos.hs:378-387: OCERT + praosVrfChecks with
    both mkSeed certificates, 2^512 leader bound) bit for bit against oracle/praos.c
    orc_tpraos_header on oracle-signed headers, every output field."""
    from praos_hip import abi, fixed
    r = rng(37)
    eta0 = b2b(b"cpu-twin-tpraos-epoch")
    c_raw = fixed.active_slot_log(Fraction(1, 2))
    H, pools = _oracle_tpraos_chain(oracle, r, 50, 4, eta0)
    sig = [fixed.from_rational(Fraction(3, 4))] * 4
    pool_list = [(b2b(p[3], 28), b2b(p[4]), s) for p, s in zip(pools, sig)]
    cpu.set_epoch(eta0, pool_list, abi.params(c_raw=c_raw))
    o = cpu.verify_tpraos_headers(_soa(H))
    ep = oracle.make_epoch(eta0, 129600, 62, c_raw, pool_list)
    hash_of = {h: i for i, (h, _, _) in enumerate(pool_list)}
    seen = set()
    for i in range(len(H["slot"])):
        h = {k: H[k][i] for k in H}
        h["n"], h["c0"] = h.pop("ocert_n"), h.pop("ocert_c0")
        ref = oracle.tpraos_header(ep, h)
        assert int(o["bits"][i]) == ref["bits"], (i, hex(o["bits"][i]), hex(ref["bits"]))
        assert bytes(o["beta_eta"][i]) == ref["beta_eta"] and bytes(o["beta_leader"][i]) == ref["beta_leader"]
        assert bytes(o["nonce"][i]) == ref["nonce"]
        assert int(o["pool_idx"][i]) == hash_of.get(b2b(h["cold_vk"], 28), -1)       # caller order
        seen.add(ref["bits"])
    # clean headers (some leaders, some not at sigma 3/4, f 1/2) and every corruption kind
    assert {0, 0x1000} <= seen and len(seen) >= 8, sorted(hex(x) for x in seen)


def test_tpraos_golden_blocks(cpu):
    """The reference's golden TPraos blocks through the twin: OCERT passes, both certificates'
    proof_to_hash equal the stored outputs (their VRF inputs are dummy seeds, so with no pool
    distribution the key is unknown), nonce = Blake2b-256 of the eta output."""
    import test_gpu_tpraos as T
    from praos_hip import abi
    cpu.set_epoch(None, [], abi.params(c_raw=T._params()[1]))
    Hx = bytes.fromhex
    K = T.KATS
    bodies = [Hx(k["body_cbor"]) for k in K]
    H = {"slot": [k["slot"] for k in K], "cold_vk": [Hx(k["cold_vk"]) for k in K],
         "vrf_vk": [Hx(k["vrf_vk"]) for k in K], "vrf_out": [Hx(k["eta_out"]) for k in K],
         "vrf_proof": [Hx(k["eta_proof"]) for k in K], "hot_vk": [Hx(k["hot_vk"]) for k in K],
         "ocert_n": [k["n"] for k in K], "ocert_c0": [k["c0"] for k in K],
         "ocert_sig": [Hx(k["ocert_sig"]) for k in K], "kes_sig": [Hx(k["kes_sig"]) for k in K], "body": bodies,
         "leader_out": [Hx(k["leader_out"]) for k in K], "leader_proof": [Hx(k["leader_proof"]) for k in K]}
    o = cpu.verify_tpraos_headers(_soa(H))
    for i, k in enumerate(K):
        assert int(o["bits"][i]) & 0x001F == 0, k["era"]
        assert int(o["bits"][i]) & 0x0100
        assert bytes(o["beta_eta"][i]) == Hx(k["eta_out"]) and bytes(o["beta_leader"][i]) == Hx(k["leader_out"])
        assert bytes(o["nonce"][i]) == b2b(Hx(k["eta_out"]))
