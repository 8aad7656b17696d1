"""TPraos (Shelley..Alonzo, d = 0) header batches through praos_verify_tpraos_headers,
bit-exact against the oracle's restatement (cardano-protocol-tpraos OVERLAY
praosVrfChecks + OCERT) and the reference's golden TPraos blocks."""
import json
import os
from fractions import Fraction

import numpy as np
import pytest

from helpers import arr, b2b

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
KATS = [k for k in json.load(open(os.path.join(HERE, "golden", "reference_kats.json")))["kats"]
        if k["kind"] == "tpraos"]
TP_BITS = 0x0001 | 0x0002 | 0x0004 | 0x0008 | 0x0010 | 0x0100 | 0x0200 | 0x0400 | 0x0800 | 0x1000


def _params(f=Fraction(1, 20)):
    from praos_hip import abi, fixed
    c_raw = fixed.active_slot_log(f)
    return abi.params(c_raw=c_raw), c_raw


def test_tpraos_synth_chain_parity(ctx, oracle):
    from praos_hip import fixed
    p, c_raw = _params(Fraction(1, 2))
    eta0 = b2b(b"tpraos-epoch")
    H, pools, corrupted = ctx.synthesize(256, 6, p, eta0, b"\x33" * 32, first_slot=5000, slot_stride=3,
                                         corrupt_per_10000=1500, tpraos=True)
    sig = [fixed.from_rational(Fraction(1, 6))] * 6
    pool_list = [(h, v, s) for (h, v), s in zip(pools, sig)]
    ctx.set_epoch(eta0, pool_list, p)
    o = ctx.verify_tpraos_headers(H)
    ep = oracle.make_epoch(eta0, 129600, 62, c_raw, pool_list)
    for i in range(len(H["slot"])):
        off, ln = int(H["body_off"][i]), int(H["body_len"][i])
        h = {"slot": int(H["slot"][i]), "cold_vk": bytes(H["cold_vk"][i]), "vrf_vk": bytes(H["vrf_vk"][i]),
             "vrf_out": bytes(H["vrf_out"][i]), "vrf_proof": bytes(H["vrf_proof"][i]),
             "hot_vk": bytes(H["hot_vk"][i]), "n": int(H["ocert_n"][i]), "c0": int(H["ocert_c0"][i]),
             "ocert_sig": bytes(H["ocert_sig"][i]), "kes_sig": bytes(H["kes_sig"][i]),
             "body": bytes(H["body_bytes"][off:off + ln]), "leader_out": bytes(H["leader_out"][i]),
             "leader_proof": bytes(H["leader_proof"][i])}
        r = oracle.tpraos_header(ep, h)
        assert int(o["bits"][i]) & TP_BITS == r["bits"], (i, hex(o["bits"][i]), hex(r["bits"]), corrupted[i])
        assert bytes(o["beta_eta"][i]) == r["beta_eta"]
        assert bytes(o["beta_leader"][i]) == r["beta_leader"]
        assert bytes(o["nonce"][i]) == r["nonce"]
    clean = [i for i in range(256) if corrupted[i] == 0]
    assert all(int(o["bits"][i]) & ~0x1000 == 0 for i in clean)
    # with sigma = 1/6 and f = 1/2 a good share of the 512-bit leader values pass
    assert 0 < sum(1 for i in clean if not int(o["bits"][i]) & 0x1000) < len(clean)


def test_tpraos_staged_equals_one_kernel(ctx):
    """The staged TPraos VRF (stage V per certificate with its mkSeed input, U against the VRF
    key cache -- hits and per-lane misses --, k_vrf_join_tp) against the one-kernel k_vrf_tp
    (PRAOS_TP_STAGED=0, two uncached certificates per lane) on the same corrupted chain:
    every output bit for bit."""
    import praos_hip
    from praos_hip import fixed
    p, c_raw = _params(Fraction(1, 2))
    eta0 = b2b(b"tpraos-staged")
    n, npools = 3000, 1500          # ~2 headers per VRF key: about a quarter used once (cache misses)
    H, pools, corrupted = ctx.synthesize(n, npools, p, eta0, b"\x35" * 32, first_slot=9000, slot_stride=2,
                                         corrupt_per_10000=1200, tpraos=True)
    pool_list = [(h, v, fixed.from_rational(Fraction(1, npools))) for (h, v) in pools]
    ctx.set_epoch(eta0, pool_list, p)
    o = ctx.verify_tpraos_headers(H)
    os.environ["PRAOS_TP_STAGED"] = "0"
    try:
        c2 = praos_hip.Context(0)
    finally:
        del os.environ["PRAOS_TP_STAGED"]
    try:
        c2.set_epoch(eta0, pool_list, p)
        o2 = c2.verify_tpraos_headers(H)
    finally:
        c2.close()
    # and the staged form with every kernel on the ctx stream (no side / V streams)
    from praos_hip import abi
    ctx.set_option(abi.OPT_CONCURRENT, 0)
    try:
        o3 = ctx.verify_tpraos_headers(H)
    finally:
        ctx.set_option(abi.OPT_CONCURRENT, 1)
    for oo in (o2, o3):
        assert set(o) == set(oo)
        for k in o:
            assert np.array_equal(np.asarray(o[k]), np.asarray(oo[k])), k
    assert np.count_nonzero(corrupted) and any(int(x) & (0x0400 | 0x0800) for x in o["bits"])


def test_tpraos_ocert_dedup_equals_off(ctx):
    """The OCert dedup (PRAOS_OPT_DEDUP: each distinct (cold vk, hot vk, n, c0, sigma) tuple of
    the batch verified once, its verdict fanned out with each header's own KES-period checks)
    on a TPraos batch with corrupted OCert signatures and KES periods out of range: every
    output equal to verifying each header's OCert on its own, and the dedup did collapse the
    pools' repeated certificates."""
    from praos_hip import abi, fixed
    p, c_raw = _params(Fraction(1, 2))
    eta0 = b2b(b"tpraos-dedup")
    n, npools = 4000, 300           # ~13 headers per pool: one OCert tuple repeated per pool
    H, pools, corrupted = ctx.synthesize(n, npools, p, eta0, b"\x36" * 32, first_slot=9000, slot_stride=2,
                                         corrupt_per_10000=900, tpraos=True)
    H["ocert_c0"][::97] += 10 ** 6                   # KESBeforeStart on some headers of a shared tuple
    pool_list = [(h, v, fixed.from_rational(Fraction(1, npools))) for (h, v) in pools]
    ctx.set_epoch(eta0, pool_list, p)
    outs = []
    for dd in (1, 0):
        ctx.set_option(abi.OPT_DEDUP, dd)
        try:
            outs.append(ctx.verify_tpraos_headers(H))
        finally:
            ctx.set_option(abi.OPT_DEDUP, 1)
    o, o0 = outs
    for k in o:
        assert np.array_equal(np.asarray(o[k]), np.asarray(o0[k])), k
    assert any(int(x) & 0x0004 for x in o["bits"]) and any(int(x) & 0x0001 for x in o["bits"])


def test_tpraos_golden_blocks(ctx):
    """The golden TPraos blocks: OCert and KES verify, both certificates' proof_to_hash
    equal the stored outputs.  Their VRF inputs are the example's dummy seeds, not
    mkSeed, so both VRF bits are set under a real epoch nonce (and the key is unknown)."""
    p, c_raw = _params()
    ctx.set_epoch(None, [], p)
    H = bytes.fromhex
    n = len(KATS)
    bodies = [H(k["body_cbor"]) for k in KATS]
    offs = np.cumsum([0] + [len(b) for b in bodies[:-1]]).astype(np.uint64)
    Hd = {"slot": np.array([k["slot"] for k in KATS], np.uint64), "cold_vk": arr([H(k["cold_vk"]) for k in KATS], 32),
          "vrf_vk": arr([H(k["vrf_vk"]) for k in KATS], 32), "vrf_out": arr([H(k["eta_out"]) for k in KATS], 64),
          "vrf_proof": arr([H(k["eta_proof"]) for k in KATS], 80), "hot_vk": arr([H(k["hot_vk"]) for k in KATS], 32),
          "ocert_n": np.array([k["n"] for k in KATS], np.uint64), "ocert_c0": np.array([k["c0"] for k in KATS], np.uint64),
          "ocert_sig": arr([H(k["ocert_sig"]) for k in KATS], 64), "kes_sig": arr([H(k["kes_sig"]) for k in KATS], 448),
          "body_off": offs, "body_len": np.array([len(b) for b in bodies], np.uint32),
          "body_bytes": np.frombuffer(b"".join(bodies) + b"\0" * 8, np.uint8).copy(),
          "leader_out": arr([H(k["leader_out"]) for k in KATS], 64),
          "leader_proof": arr([H(k["leader_proof"]) for k in KATS], 80)}
    o = ctx.verify_tpraos_headers(Hd)
    for i, k in enumerate(KATS):
        assert int(o["bits"][i]) & 0x001F == 0, k["era"]               # OCERT rule passes
        assert int(o["bits"][i]) & 0x0100                                # no pool distribution given
        assert bytes(o["beta_eta"][i]) == H(k["eta_out"])
        assert bytes(o["beta_leader"][i]) == H(k["leader_out"])
        assert bytes(o["nonce"][i]) == b2b(H(k["eta_out"]))


def test_leader512_vs_oracle(ctx, oracle):
    """The 2^512-bound leader test (TPraos checkLeaderValue) against the oracle."""
    import random
    from praos_hip import fixed
    r = random.Random(21)
    p, c_raw = _params()
    pools = []
    for i in range(200):
        s = Fraction(r.randrange(1, 1000), 1000)
        pools.append((b2b(i.to_bytes(4, "big"), 28), b2b(b"v" + i.to_bytes(4, "big")), fixed.from_rational(s)))
    # drive k_leader through the TPraos batch with synthetic leader outputs: reuse a synth chain
    H, pl, corrupted = ctx.synthesize(200, 200, p, None, b"\x44" * 32, tpraos=True)
    pool_list = [(h, v, s) for (h, v), (_, _, s) in zip(pl, pools)]
    ctx.set_epoch(None, pool_list, p)
    for i in range(200):
        l = r.getrandbits(512) >> r.randrange(0, 16)
        H["leader_out"][i] = np.frombuffer(l.to_bytes(64, "big"), np.uint8)
    o = ctx.verify_tpraos_headers(H)
    for i in range(200):
        idx = int(o["pool_idx"][i])
        want, _ = oracle.check_leader512(bytes(H["leader_out"][i]), pool_list[idx][2], c_raw)
        assert bool(int(o["bits"][i]) & 0x1000) == (not want)


def test_tpraos_overlay_chain_parity(ctx, oracle):
    """d = 1/2 overlay schedule (praos_set_overlay): active overlay slots forged by the
    scheduled genesis delegate (or, seeded, by a wrong pool), non-active overlay slots,
    and Praos slots, all through praos_verify_tpraos_headers and the TPraos fold, against
    oracle/tpraos.py (overlay classification, pbftVrfChecks / praosVrfChecks, OCERT) on top
    of the oracle's per-header crypto."""
    import random
    import tpraos as tp
    from praos_hip import fixed
    r = random.Random(77)
    p, c_raw = _params(Fraction(1, 2))
    eta0 = b2b(b"tpraos-overlay-epoch")
    d, f = Fraction(1, 2), Fraction(1, 20)
    base, length = 0, 432000
    npools, n = 8, 256
    genesis = [b2b(b"genesis-key" + bytes([k]), 28) for k in range(3)]
    order = sorted(range(3), key=lambda k: genesis[k])                 # Set.elemAt order
    slots = sorted(r.sample(range(40, 4000), n))
    cls = [tp.classify(s, d, f, base, length, 3) for s in slots]
    # forger per header: the delegate of the scheduled genesis key (pools 5..7), sometimes a
    # wrong pool; any pool for non-active and Praos slots
    forger = []
    for c in cls:
        if c >= 0:
            forger.append(5 + order[c] if r.random() < 0.85 else r.randrange(5))
        else:
            forger.append(r.randrange(npools))
    H, pools, corrupted = ctx.synthesize(n, npools, p, eta0, b"\x39" * 32, tpraos=True, corrupt_per_10000=800,
                                         schedule=(np.array(slots, np.uint64), np.array(forger, np.uint32)))
    sig = [fixed.from_rational(Fraction(1, 8))] * npools
    pool_list = [(h, v, s) for (h, v), s in zip(pools, sig)]
    gen = [(genesis[k], pools[5 + k][0], pools[5 + k][1]) for k in range(3)]
    gen_sorted = sorted(gen)
    ctx.set_epoch(eta0, pool_list, p)
    ctx.set_overlay(d, f, base, length, gen)
    try:
        assert list(ctx.overlay_classify(np.array(slots, np.uint64))) == cls
        o = ctx.verify_tpraos_headers(H)
        ep = oracle.make_epoch(eta0, 129600, 62, c_raw, pool_list)
        mask = TP_BITS | 0x2000 | 0x4000
        for i in range(n):
            off, ln = int(H["body_off"][i]), int(H["body_len"][i])
            h = {"slot": int(H["slot"][i]), "cold_vk": bytes(H["cold_vk"][i]), "vrf_vk": bytes(H["vrf_vk"][i]),
                 "vrf_out": bytes(H["vrf_out"][i]), "vrf_proof": bytes(H["vrf_proof"][i]),
                 "hot_vk": bytes(H["hot_vk"][i]), "n": int(H["ocert_n"][i]), "c0": int(H["ocert_c0"][i]),
                 "ocert_sig": bytes(H["ocert_sig"][i]), "kes_sig": bytes(H["kes_sig"][i]),
                 "body": bytes(H["body_bytes"][off:off + ln]), "leader_out": bytes(H["leader_out"][i]),
                 "leader_proof": bytes(H["leader_proof"][i])}
            rr = oracle.tpraos_header(ep, h)
            want = tp.overlay_bits(rr["bits"], cls[i], h["cold_vk"], h["vrf_vk"], gen_sorted)
            assert int(o["bits"][i]) & mask == want, (i, cls[i], hex(o["bits"][i]), hex(want), corrupted[i])
            assert bytes(o["nonce"][i]) == rr["nonce"]
        kinds = {"active": sum(c >= 0 for c in cls), "non_active": cls.count(-2), "praos": cls.count(-1)}
        assert all(v > 5 for v in kinds.values()), kinds
        clean_active = [i for i in range(n) if cls[i] >= 0 and not corrupted[i] and forger[i] >= 5]
        assert clean_active and all(int(o["bits"][i]) & ~0x2000 == 0 for i in clean_active)
        # the TPraos fold over these outputs
        prev = np.frombuffer(bytes(r.getrandbits(8) for _ in range(32 * n)), np.uint8).reshape(n, 32).copy()
        state = {"last_slot": None, "counters": {}, "evolving": None, "candidate": None, "epoch_nonce": eta0,
                 "lab": None, "leb": None}
        ref_state = {k: (dict(v) if isinstance(v, dict) else v) for k, v in state.items()}
        ei = (base, 0, length, 1000)
        v, fails, stop, done = ctx.tpraos_update_chain_dep_state(H, o, prev, state, ei)
        hk = [b2b(bytes(H["cold_vk"][i]), 28) for i in range(n)]
        known = {pl[0] for pl in pool_list} | {g[1] for g in gen}
        rv, rf, rstop, rdone = tp.fold(ref_state, hk, H["slot"], o["bits"], H["ocert_n"], o["nonce"],
                                       [bytes(x) for x in prev], known, eta0, base, 0, length, 1000)
        assert (done, stop) == (rdone, rstop) and done == n
        assert list(v) == rv and list(fails) == rf and state == ref_state
        assert any(x & tp.TPF_NOT_ACTIVE for x in rf) and any(x & tp.TPF_GEN_COLD for x in rf)
    finally:
        ctx.set_overlay(None, None, 0, 1, [])


def test_tpraos_header_bytes_vs_soa_and_oracle(ctx, oracle):
    """Stored TPraos headers (BHeader = [BHBody, kesSig] in Alonzo blocks, CBOR bodies from the
    GPU generator) decoded and verified on the device (praos_verify_tpraos_header_bytes):
    every output equal to the host-SoA path on the same headers, the decoded fields equal the
    generator's, and a sample bit-exact against the oracle."""
    from praos_hip import abi, fixed
    from praos_hip.chunk import pack_chunk
    p, c_raw = _params(Fraction(1, 2))
    eta0 = b2b(b"tpraos-bytes-epoch")
    n = 2048
    H, pools, corrupted = ctx.synthesize(n, 6, p, eta0, b"\x34" * 32, first_slot=9000, slot_stride=5,
                                         body_len=0, corrupt_per_10000=400, tpraos=True)
    assert (H["body_len"] > 540).all() and (H["body_len"] <= 598).all()
    sig = [fixed.from_rational(Fraction(1, 6))] * 6
    pool_list = [(h, v, s) for (h, v), s in zip(pools, sig)]
    ctx.set_epoch(eta0, pool_list, p)
    o1 = ctx.verify_tpraos_headers(H)
    arena, off, ln = pack_chunk(H, era_tag=5)
    o2, D = ctx.verify_tpraos_header_bytes(arena, off, ln, decoded=True)
    # a body corruption (kind 5: +1 at any byte of the stored BHBody) may land in any decoded
    # field, so the SoA path (which keeps the generator's fields) only matches elsewhere
    same = corrupted != 5
    assert same.sum() > n - 60
    for k in o1:
        assert np.array_equal(o1[k][same], o2[k][same]), (k, np.nonzero((o1[k] != o2[k]).reshape(n, -1).any(1))[0][:8])
    # (round 3's r03d failure: the first version of this test compared those headers bit for bit
    # too; both paths reject every one of them, with the bits of whichever field the byte hit)
    assert (o2["bits"][~same] != 0).all() and (o1["bits"][~same] != 0).all()
    assert (D["status"][same] == 0).all()
    for k in ("slot", "cold_vk", "vrf_vk", "vrf_out", "vrf_proof", "hot_vk", "ocert_n", "ocert_c0", "ocert_sig",
              "kes_sig", "leader_out", "leader_proof"):
        assert np.array_equal(D[k][same], H[k][same]), k
    for i in np.nonzero(same)[0]:
        off_i, ln_i = int(H["body_off"][i]), int(H["body_len"][i])
        assert int(D["signed_len"][i]) == ln_i
        assert bytes(D["signed_body"][i][:ln_i]) == bytes(H["body_bytes"][off_i:off_i + ln_i])
    clean = corrupted == 0
    assert int((o2["bits"][clean] & ~np.uint16(0x1000)).astype(bool).sum()) == 0
    assert int((o2["bits"][~clean] == 0).sum()) == 0
    ep = oracle.make_epoch(eta0, 129600, 62, c_raw, pool_list)
    for i in list(range(0, n, 97)) + list(np.nonzero(~clean & same)[0][:40]):
        i = int(i)
        o_, l_ = int(H["body_off"][i]), int(H["body_len"][i])
        h = {"slot": int(H["slot"][i]), "cold_vk": bytes(H["cold_vk"][i]), "vrf_vk": bytes(H["vrf_vk"][i]),
             "vrf_out": bytes(H["vrf_out"][i]), "vrf_proof": bytes(H["vrf_proof"][i]),
             "hot_vk": bytes(H["hot_vk"][i]), "n": int(H["ocert_n"][i]), "c0": int(H["ocert_c0"][i]),
             "ocert_sig": bytes(H["ocert_sig"][i]), "kes_sig": bytes(H["kes_sig"][i]),
             "body": bytes(H["body_bytes"][o_:o_ + l_]), "leader_out": bytes(H["leader_out"][i]),
             "leader_proof": bytes(H["leader_proof"][i])}
        r = oracle.tpraos_header(ep, h)
        assert int(o2["bits"][i]) & TP_BITS == r["bits"], (i, hex(o2["bits"][i]), hex(r["bits"]), corrupted[i])
        assert bytes(o2["beta_eta"][i]) == r["beta_eta"] and bytes(o2["nonce"][i]) == r["nonce"]


def test_tpraos_header_bytes_golden_and_malformed(ctx):
    """The reference's golden TPraos headers as stored bytes: decoded fields equal the golden
    ones, OCERT passes, proof_to_hash equals the stored outputs; a Praos (10-field) header and
    a truncated one are PRAOS_BIT_INPUT."""
    from praos_hip import abi
    p, c_raw = _params()
    ctx.set_epoch(None, [], p)
    H = bytes.fromhex
    praos_kat = [k for k in json.load(open(os.path.join(HERE, "golden", "reference_kats.json")))["kats"]
                 if k["kind"] != "tpraos"][0]
    hdrs = [H(k["header_cbor"]) for k in KATS] + [H(praos_kat["header_cbor"]), H(KATS[0]["header_cbor"])[:-9]]
    off = np.cumsum([0] + [len(h) for h in hdrs[:-1]]).astype(np.uint64)
    ln = np.array([len(h) for h in hdrs], np.uint32)
    o, D = ctx.verify_tpraos_header_bytes(np.frombuffer(b"".join(hdrs), np.uint8).copy(), off, ln, decoded=True)
    for i, k in enumerate(KATS):
        assert D["status"][i] == 0 and int(D["slot"][i]) == k["slot"] and int(D["block_no"][i]) == k["block_no"]
        assert bytes(D["cold_vk"][i]) == H(k["cold_vk"]) and bytes(D["leader_out"][i]) == H(k["leader_out"])
        assert bytes(D["leader_proof"][i]) == H(k["leader_proof"]) and bytes(D["body_hash"][i]) == H(k["body_hash"])
        assert int(o["bits"][i]) & 0x001F == 0, k["era"]
        assert bytes(o["beta_eta"][i]) == H(k["eta_out"]) and bytes(o["beta_leader"][i]) == H(k["leader_out"])
    for i in (len(KATS), len(KATS) + 1):
        assert D["status"][i] & abi.DEC_FAILED and o["bits"][i] & abi.BIT_INPUT


@pytest.mark.parametrize("members", [2, 3])
def test_tpraos_group_equals_single(ctx, members):
    """praos_group_verify_tpraos_headers / _header_bytes (ABI 12): a TPraos batch split into
    contiguous shards over several contexts (one GPU here; devices 0..7 on a node) gives every
    output -- and with decoded=True every decoded field -- bit for bit as one context."""
    from praos_hip import abi, fixed
    from praos_hip.chunk import pack_chunk
    p, c_raw = _params(Fraction(1, 2))
    eta0 = b2b(b"tpraos-group")
    n = 1537
    H, pools, corrupted = ctx.synthesize(n, 40, p, eta0, b"\x36" * 32, first_slot=7000, slot_stride=3,
                                         body_len=0, corrupt_per_10000=300, tpraos=True)
    pool_list = [(h, v, fixed.from_rational(Fraction(1, 40))) for (h, v) in pools]
    ctx.set_epoch(eta0, pool_list, p)
    o1 = ctx.verify_tpraos_headers(H)
    arena, off, ln = pack_chunk(H, era_tag=5)
    b1, D1 = ctx.verify_tpraos_header_bytes(arena, off, ln, decoded=True)
    with abi.Group([0] * members) as g:
        g.set_epoch(eta0, pool_list, p)
        og = g.verify_tpraos_headers(H)
        bg, Dg = g.verify_tpraos_header_bytes(arena, off, ln, decoded=True)
    for k in o1:
        assert np.array_equal(o1[k], og[k]), k
        assert np.array_equal(b1[k], bg[k]), k
    for k in D1:
        assert np.array_equal(D1[k], Dg[k]), k
    assert np.count_nonzero(corrupted) and all(int(og["bits"][i]) for i in np.nonzero(corrupted)[0])


def test_tpraos_gpu_equals_cpu_twin(ctx):
    """The GPU TPraos path (staged VRF, key caches, 2^512 leader test) against the CPU twin's
    independent implementation (libpraos_cpu.so praos_verify_tpraos_headers: radix 2^51,
    sliding-window Straus) on a corrupted synthetic TPraos batch (pools by hash, ~4 headers per
    key: VRF / cold / KES-leaf cache hits and misses): every output bit for bit."""
    from praos_hip import cpu as C
    from praos_hip import fixed
    p, c_raw = _params(Fraction(1, 2))
    eta0 = b2b(b"tpraos-twin")
    n, npools = 3000, 700
    H, pools, corrupted = ctx.synthesize(n, npools, p, eta0, b"\x37" * 32, first_slot=20000, slot_stride=3,
                                         corrupt_per_10000=700, tpraos=True)
    pool_list = [(h, v, fixed.from_rational(Fraction(1, npools))) for (h, v) in pools]
    ctx.set_epoch(eta0, pool_list, p)
    o = ctx.verify_tpraos_headers(H)
    twin = C.CpuContext(16)
    try:
        twin.set_epoch(eta0, pool_list, p)
        t = twin.verify_tpraos_headers(H)
    finally:
        twin.close()
    for k in o:
        assert np.array_equal(np.asarray(o[k]), np.asarray(t[k])), k
    assert np.count_nonzero(corrupted) > 100 and int((o["bits"][corrupted != 0] == 0).sum()) == 0
