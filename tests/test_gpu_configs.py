"""BASELINE.json configs[1..3] at their stated size: 1,000,000 items each, built exactly as
bench.py builds them (praos_hip/configs.py) and run with the bench's context options, through
the C ABI (praos_batch_upload / praos_batch_run / praos_batch_download).

  c2: OCert Ed25519 (Praos.hs:574-580 -> Ed25519DSIGN verify over hot vk || n || c0), 1M
      distinct cold keys;
  c3: ECVRF-draft03 verify + certified output + checkLeaderNatValue (Praos.hs:528-556), the
      (slot, pool) pairs of a first-leader-wins schedule, so every clean item is a leader;
  c4: Sum6KES verify (Praos.hs:582, KES.Sum verifyKES: Merkle path + leaf Ed25519) over
      397-byte messages.

Each asserts: every clean item accepted, every corruption in a field the config checks
rejected, a ~1,000-item sample (evenly spaced + corrupted ones) bit-exact against the
oracle (bits; for c3 also beta and the leader value), and all 1,000,000 items bit-exact
against the CPU twin (libpraos_cpu.so: an independent restatement, radix 2^51 and
sliding-window Straus, itself gated bit for bit against the oracle in test_cpu_twin.py)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

OCERT_BAD, KES_MERKLE, KES_LEAF = 0x0004, 0x0008, 0x0010
VRF_MASK = 0x1F00          # pool unknown, VRF key wrong, proof, output, leader


def _hdr(H, i):
    off, ln = int(H["body_off"][i]), int(H["body_len"][i])
    return {"slot": int(H["slot"][i]), "cold_vk": bytes(H["cold_vk"][i]), "vrf_vk": bytes(H["vrf_vk"][i]),
            "vrf_out": bytes(H["vrf_out"][i]), "vrf_proof": bytes(H["vrf_proof"][i]),
            "hot_vk": bytes(H["hot_vk"][i]), "n": int(H["ocert_n"][i]), "c0": int(H["ocert_c0"][i]),
            "ocert_sig": bytes(H["ocert_sig"][i]), "kes_sig": bytes(H["kes_sig"][i]),
            "body": bytes(H["body_bytes"][off:off + ln])}


@pytest.mark.parametrize("name", ["c2", "c3", "c4"])
def test_config_full_size(ctx, oracle, name):
    from praos_hip import configs
    n = configs.ITEMS[name]
    H, pool_list, corrupted, p, eta0, c_raw, spkp, maxevo = configs.build(ctx, name)
    assert len(H["slot"]) == n == 1_000_000
    try:
        configs.options(ctx, name)
        ctx.set_epoch(eta0, pool_list, p)
        b = ctx.upload(H)
        try:
            ctx.run(b)
            ctx.sync()
            out = ctx.download(b, n)
        finally:
            ctx.free(b)
    finally:
        configs.options(ctx, "c5")                 # the session context's defaults
    bits = out["bits"]
    kernels = configs.KERNELS[name]
    clean = corrupted == 0
    # the leader test runs only with the VRF (c3); c2 / c4 carry no leader verdict
    crypto = bits if name == "c3" else bits & ~np.uint16(0x1000)
    assert int((crypto[clean] != 0).sum()) == 0, np.nonzero(crypto[clean])[0][:8]
    rel = np.isin(corrupted, configs.CHECKED_KINDS[kernels])
    assert rel.sum() == (~clean).sum() > 8_000            # corruptions only in checked fields
    assert int((crypto[rel] == 0).sum()) == 0, np.nonzero(rel & (crypto == 0))[0][:8]
    if name == "c3":
        assert int(((bits & 0x1000) == 0)[clean].sum()) == int(clean.sum())   # every clean item a leader
    # the oracle on ~1,000 items (750 evenly spaced, 250 corrupted)
    sample = sorted(set(np.linspace(0, n - 1, 750).astype(int).tolist() +
                        np.nonzero(~clean)[0][::max(1, int((~clean).sum()) // 250)][:250].tolist()))
    if name == "c3":
        ep = oracle.make_epoch(eta0, spkp, maxevo, c_raw, pool_list)
    for i in sample:
        h = _hdr(H, i)
        if name == "c2":
            m = h["hot_vk"] + h["n"].to_bytes(8, "big") + h["c0"].to_bytes(8, "big")
            want = 0 if oracle.ed25519_verify(h["cold_vk"], m, h["ocert_sig"]) else OCERT_BAD
            assert int(bits[i]) & OCERT_BAD == want, (i, corrupted[i])
        elif name == "c4":
            r = oracle.kes_verify(h["hot_vk"], max(h["slot"] // spkp - h["c0"], 0), h["body"], h["kes_sig"])
            want = {0: 0, 1: KES_MERKLE, 2: KES_LEAF}[r]
            assert int(bits[i]) & (KES_MERKLE | KES_LEAF) == want, (i, corrupted[i])
        else:
            r = oracle.praos_header(ep, h)
            assert int(bits[i]) & VRF_MASK == r["bits"] & VRF_MASK, (i, hex(int(bits[i])), hex(r["bits"]))
            assert bytes(out["beta"][i]) == r["beta"] and bytes(out["leader"][i]) == r["leader"], i
    _twin_equal(name, H, out, pool_list, p, eta0, spkp)


def _twin_equal(name, H, out, pool_list, p, eta0, spkp):
    """Every item's verdict (and for c3 beta and the leader value) against the CPU twin on the
    box's 16-thread share."""
    from praos_hip import abi
    from praos_hip import cpu as C
    bits = out["bits"]
    n = len(bits)
    twin = C.CpuContext(threads=16)
    try:
        if name == "c2":
            ok = twin.verify_ocert(H["cold_vk"], H["hot_vk"], H["ocert_n"], H["ocert_c0"], H["ocert_sig"])
            want = np.where(ok != 0, 0, OCERT_BAD).astype(np.uint16)
            got = bits & np.uint16(OCERT_BAD)
        elif name == "c4":
            kp = H["slot"] // np.uint64(spkp)
            period = np.where(kp >= H["ocert_c0"], kp - H["ocert_c0"], 0).astype(np.uint32)
            res = np.zeros(n, np.uint8)
            twin.check(twin.L.praos_verify_kes(twin.h, n, abi.ptr(H["hot_vk"]), abi.ptr(period, abi.u32p),
                                               abi.ptr(H["kes_sig"]), abi.ptr(H["body_off"], abi.u64p),
                                               abi.ptr(H["body_len"], abi.u32p), abi.ptr(H["body_bytes"]),
                                               len(H["body_bytes"]), abi.ptr(res)))
            want = np.array([0, KES_MERKLE, KES_LEAF], np.uint16)[res]
            got = bits & np.uint16(KES_MERKLE | KES_LEAF)
        else:
            twin.set_epoch(eta0, pool_list, p)
            t = twin.verify_headers(H)
            want = t["bits"] & np.uint16(VRF_MASK)
            got = bits & np.uint16(VRF_MASK)
            assert np.array_equal(out["beta"], t["beta"]) and np.array_equal(out["leader"], t["leader"])
            assert np.array_equal(out["pool_idx"], t["pool_idx"])
    finally:
        twin.close()
    diff = np.nonzero(got != want)[0]
    assert diff.size == 0, (name, diff[:8], got[diff[:8]], want[diff[:8]])


def _first(H, m):
    n = len(H["slot"])
    return {k: (v[:m] if k != "body_bytes" and hasattr(v, "shape") and v.ndim and v.shape[0] == n else v)
            for k, v in H.items()}


def test_kes_pair_equals_single(ctx):
    """k_kes_ck with two headers per lane (PRAOS_OPT_KES_PAIR, one inversion for both R'
    encodings) gives the per-header verdicts of the one-header-per-lane form: C4-shaped
    batches with 1 % corrupted KES signatures / messages, paired from 2 hits on against never
    paired, down to a prefix with an odd number of cache hits (the last lane then has no
    second header)."""
    from praos_hip import abi, configs
    H0, pool_list, corrupted0, p, eta0, c_raw, spkp, maxevo = configs.build(ctx, "c4", n=40_016)
    odd = False
    try:
        configs.options(ctx, "c4")
        ctx.set_option(abi.OPT_KES_NOCACHE, 0)        # the leaf-key cache at this size too
        ctx.set_epoch(eta0, pool_list, p)
        for m in range(40_016, 40_000, -1):
            H, corrupted = _first(H0, m), corrupted0[:m]
            outs, hits = [], []
            for pair in (0, 2):
                ctx.set_option(abi.OPT_KES_PAIR, pair)
                b = ctx.upload(H)
                try:
                    ctx.run(b)
                    ctx.sync()
                    hits.append(ctx.batch_stats(b)["kes_hits"])
                    outs.append(ctx.download(b, m)["bits"].copy())
                finally:
                    ctx.free(b)
            assert hits[0] == hits[1] and hits[0] > 1000
            np.testing.assert_array_equal(outs[0], outs[1])
            bad = np.isin(corrupted, (2, 5))
            assert bad.sum() > 100 and int((outs[1][bad] == 0).sum()) == 0
            assert int((outs[1][corrupted == 0] & np.uint16(0x0018)).sum()) == 0
            if hits[0] % 2:
                odd = True
                break
    finally:
        ctx.set_option(abi.OPT_KES_PAIR, -1)
        ctx.set_option(abi.OPT_KES_NOCACHE, -1)
        configs.options(ctx, "c5")
    assert odd, "no prefix with an odd hit count"
