"""praos_group: one process, several contexts (here all on the one GPU of the box; on
an 8-GPU node the members are devices 0..7), a batch split into contiguous shards run
concurrently, outputs gathered in place -- bit-exact against one context, and the
shard -> gather -> fold path (updateChainDepState on member 0 over the gathered
outputs) equal to the single-context fold."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def c5_batch(ctx):
    from praos_hip import chains
    from praos_hip.chunk import pack_chunk
    cfg = chains.CONFIGS["c5"]
    sched = chains.load_schedule("c5")
    H, pool_list, corrupted, p = chains.make_chain(ctx, cfg, sched, n=20_011, corrupt_per_10000=100)
    arena, off, ln = pack_chunk(H)
    return cfg, H, pool_list, corrupted, p, arena, off, ln


@pytest.mark.parametrize("members", [1, 3, 4])
def test_group_bytes_equals_single(ctx, c5_batch, members):
    from praos_hip import abi
    cfg, H, pool_list, corrupted, p, arena, off, ln = c5_batch
    ctx.set_epoch(cfg["eta0"], pool_list, p)
    o1, D1 = ctx.verify_header_bytes(arena, off, ln, decoded=True)
    with abi.Group([0] * members) as g:
        assert g.size == members
        g.set_epoch(cfg["eta0"], pool_list, p)
        og, Dg = g.verify_header_bytes(arena, off, ln, decoded=True)
    for k in o1:
        assert np.array_equal(o1[k], og[k]), k
    for k in D1:
        assert np.array_equal(D1[k], Dg[k]), k
    clean = corrupted == 0
    assert int((og["bits"][clean] != 0).sum()) == 0 and int((og["bits"][~clean] == 0).sum()) == 0


def test_group_soa_and_tiny_batches(ctx, c5_batch):
    """The SoA entry point, and batches smaller than the group (empty shards)."""
    from praos_hip import abi
    cfg, H, pool_list, corrupted, p, arena, off, ln = c5_batch
    ctx.set_epoch(cfg["eta0"], pool_list, p)
    o1 = ctx.verify_headers(H)
    with abi.Group([0, 0, 0]) as g:
        g.set_epoch(cfg["eta0"], pool_list, p)
        og = g.verify_headers(H)
        for k in o1:
            assert np.array_equal(o1[k], og[k]), k
        for n in (1, 2, 5):
            ot = g.verify_header_bytes(arena, off[:n], ln[:n])
            assert np.array_equal(ot["bits"], o1["bits"][:n]) and np.array_equal(ot["nonce"], o1["nonce"][:n])


def test_group_without_epoch_fails_loudly(ctx):
    from praos_hip import abi
    with abi.Group([0, 0]) as g:
        with pytest.raises(abi.PraosError, match="member"):
            g.verify_header_bytes(np.zeros(64, np.uint8), np.zeros(2, np.uint64), np.full(2, 10, np.uint32))


def test_shard_gather_fold(ctx, c5_batch):
    """Shard -> gather -> fold: the gathered group outputs folded (updateChainDepState on
    member 0) give the same verdicts, chain stop and state as one context's."""
    from praos_hip import abi
    cfg, H, pool_list, corrupted, p, arena, off, ln = c5_batch
    ei = (0, 0, cfg["epoch_length"], 129_600)

    def fold(c, o, D):
        st = {"last_slot": None, "counters": {}, "evolving": cfg["eta0"], "candidate": cfg["eta0"],
              "epoch_nonce": cfg["eta0"], "lab": None, "leb": None}
        Hs = dict(H, slot=D["slot"], ocert_n=D["ocert_n"])
        v, stop, done = c.update_chain_dep_state(Hs, o, D["prev_hash"], st, ei, prev_is_genesis=D["prev_is_genesis"])
        return v, stop, done, st
    ctx.set_epoch(cfg["eta0"], pool_list, p)
    r1 = fold(ctx, *ctx.verify_header_bytes(arena, off, ln, decoded=True))
    with abi.Group([0, 0, 0, 0]) as g:
        g.set_epoch(cfg["eta0"], pool_list, p)
        og, Dg = g.verify_header_bytes(arena, off, ln, decoded=True)
        rg = fold(g.member(0), og, Dg)
    assert np.array_equal(r1[0], rg[0]) and r1[1:] == rg[1:]
    first_bad = int(np.nonzero(corrupted)[0][0])
    # the chain stops at the first corrupted header; the fold carries on (would-be verdicts)
    # until a corrupted slot lands in a later epoch (another nonce: processed < n)
    assert r1[1] == first_bad and r1[2] > first_bad and r1[0][first_bad] != 0


def test_c5_full_epoch_single_and_group8(ctx, oracle):
    """configs[4] as stated: the whole 432,000-header epoch (3000 pools, 1 % corrupted) in
    ONE batch, and the same epoch split over an 8-member praos_group (the 8-GPU layout:
    contiguous slot-range shards of 54,000 headers; here all members on device 0).
    Gathered == single context on every output, clean headers all valid, corrupted ones
    all rejected, and an oracle sample bit-exact (as test_gpu_chain.test_c5_shaped_batch)."""
    from praos_hip import abi, chains, fixed
    from test_gpu_chain import _oracle_header
    cfg = chains.CONFIGS["c5"]
    sched = chains.load_schedule("c5")
    n = 432_000
    H, pool_list, corrupted, p = chains.make_chain(ctx, cfg, sched, n=n, corrupt_per_10000=100)
    ctx.set_epoch(cfg["eta0"], pool_list, p)
    o1 = ctx.verify_headers(H)
    clean = corrupted == 0
    assert int((~clean).sum()) > 4000
    assert int((o1["bits"][clean] != 0).sum()) == 0
    assert int((o1["bits"][~clean] == 0).sum()) == 0
    assert list(o1["pool_idx"][clean]) == list(sched[1][:n][clean])
    with abi.Group([0] * 8) as g:
        g.set_epoch(cfg["eta0"], pool_list, p)
        og = g.verify_headers(H)
    for k in o1:
        assert np.array_equal(o1[k], og[k]), k
    c_raw = fixed.active_slot_log(cfg["f"])
    ep = oracle.make_epoch(cfg["eta0"], cfg["slots_per_kes_period"], cfg["max_kes_evo"], c_raw, pool_list)
    # samples in every shard, the shard edges, and corrupted headers
    edges = [k * n // 8 + d for k in range(1, 8) for d in (-1, 0)]
    sample = sorted(set(np.linspace(0, n - 1, 160).astype(int).tolist()) | set(edges) |
                    set(np.nonzero(~clean)[0][::60].tolist()))
    for i in sample:
        r = _oracle_header(oracle, ep, H, i)
        assert int(og["bits"][i]) & 0x1F1F == r["bits"], (i, hex(og["bits"][i]), hex(r["bits"]), corrupted[i])
        assert bytes(og["beta"][i]) == r["beta"] and bytes(og["leader"][i]) == r["leader"]
        assert bytes(og["nonce"][i]) == r["nonce"]
    _leader_decisions_invariant(o1, pool_list, c_raw)


def _leader_decisions_invariant(o, pool_list, c_raw, band=1e-12):
    """activeSlotLog's last digits are unpinned (cardano-ledger-core ln' is not vendored,
    praos_hip/fixed.py).  Every header's leader decision is shown to hold for ANY c within
    `band` (relative) of c_raw: the exact real-number test p < 1 - (1 - f)^sigma flips at
    c* = log1p(-p) / sigma (c = ln(1 - f) < 0; leader iff c < c*), and |c* - c| / |c| >
    band for every header -- ten orders of magnitude above the 10^-24 convergence bound
    of any Fixed E34 evaluation of ln'.  The GPU's Fixed E34 decision equals the
    real-number one on every header (the Taylor comparison is exact away from c*)."""
    from praos_hip import abi
    sig = np.array([float(s) / 1e34 for _, _, s in pool_list])
    pi = o["pool_idx"]
    known = pi >= 0
    lead = o["leader"][known]
    # leading 64 bits of the 256-bit leader value: p = l / 2^256 to float64 precision
    hi = lead[:, :8].astype(np.uint64)
    top = np.zeros(len(lead), np.float64)
    for k in range(8):
        top = top * 256.0 + hi[:, k]
    p = top / 2.0 ** 64
    c = c_raw / 1e34
    cstar = np.log1p(-p) / sig[pi[known]]
    rel = (cstar - c) / abs(c)                      # > 0: leader
    gpu_leader = (o["bits"][known] & abi.BIT_LEADER) == 0
    checked = (o["bits"][known] & 0x0F1F) == 0       # crypto-valid headers reach the leader test
    assert np.array_equal(gpu_leader[checked], rel[checked] > 0)
    assert float(np.min(np.abs(rel[checked]))) > band, float(np.min(np.abs(rel[checked])))


@pytest.mark.parametrize("chunks", [2, 3, 8])
def test_pipelined_bytes_equals_single_batch(ctx, c5_batch, chunks):
    """praos_verify_header_bytes in K chunks (PRAOS_OPT_PIPELINE: H2D of chunk k+1 on the copy
    stream beside the kernels of chunk k) gives every output and decoded field of the
    one-batch path, including a header whose span lies outside the arena (DEC_RANGE)."""
    from praos_hip import abi
    cfg, H, pool_list, corrupted, p, arena, off, ln = c5_batch
    off = off.copy()
    off[5000] = len(arena) + 100                     # out of range
    ctx.set_epoch(cfg["eta0"], pool_list, p)
    try:
        ctx.set_option(abi.OPT_PIPELINE, 1)
        o1, D1 = ctx.verify_header_bytes(arena, off, ln, decoded=True)
        ctx.set_option(abi.OPT_PIPELINE, chunks)
        for _ in range(2):                            # the second call reuses the chunk batches
            o2, D2 = ctx.verify_header_bytes(arena, off, ln, decoded=True)
            for k in o1:
                assert np.array_equal(o1[k], o2[k]), k
            for k in D1:
                assert np.array_equal(D1[k], D2[k]), k
        # the cold / VRF pool-key stores kept across calls (PRAOS_OPT_POOL_KEYS; 2 empties them first):
        # the second call finds every pool key already stored -- the same outputs
        ctx.set_option(abi.OPT_POOL_KEYS, 2)
        for _ in range(2):
            o3 = ctx.verify_header_bytes(arena, off, ln)
            for k in o1:
                assert np.array_equal(o1[k], o3[k]), k
    finally:
        ctx.set_option(abi.OPT_PIPELINE, 0)
        ctx.set_option(abi.OPT_POOL_KEYS, -1)
    assert D1["status"][5000] & abi.DEC_RANGE and o1["bits"][5000] & abi.BIT_INPUT


@pytest.mark.parametrize("chunk_v", [None, "0"])
def test_submitted_bytes_equal_blocking(ctx, c5_batch, chunk_v, monkeypatch):
    """The streaming form (praos_verify_header_bytes_submit, three calls in flight, outputs written by
    the third submit after or by praos_verify_drain) gives each call the blocking call's outputs and
    decoded fields bit for bit: different inputs back to back (a damaged copy of the arena, the
    headers in another order), a blocking call that drains the calls in flight, and a page-locked
    arena and outputs (direct DMA from the caller's memory); with stage V chunk by chunk under the
    upload (default) and in the run (PRAOS_STREAM_CHUNK_V=0, a context of its own)."""
    import praos_hip
    from praos_hip import abi
    cfg, H, pool_list, corrupted, p, arena, off, ln = c5_batch
    if chunk_v is not None:
        monkeypatch.setenv("PRAOS_STREAM_CHUNK_V", chunk_v)
        ctx = praos_hip.Context(0)
    n = len(off)
    rng = np.random.default_rng(7)
    arena_b = arena.copy()
    for i in rng.choice(n, 40, replace=False):        # damaged headers (bytes inside the header body)
        arena_b[int(off[i]) + 40 + int(rng.integers(0, 200))] ^= 0x10
    perm = rng.permutation(n)
    inputs = [(arena, off, ln), (arena_b, off, ln), (arena, off[perm].copy(), ln[perm].copy())]
    ctx.set_epoch(cfg["eta0"], pool_list, p)
    try:
        ctx.set_option(abi.OPT_PIPELINE, 8)
        ref = [ctx.verify_header_bytes(a, o, l, decoded=True) for a, o, l in inputs]
        assert not np.array_equal(ref[0][0]["bits"], ref[1][0]["bits"])
        order = [0, 1, 2, 0, 2]
        outs = [(ctx.alloc_out(n), ctx.alloc_decoded(n)) for _ in order]
        for j, (o, d) in zip(order, outs):
            ctx.submit_header_bytes(*inputs[j], out=o, decoded=d)
        ctx.drain()
        for j, (o, d) in zip(order, outs):
            for k in o:
                assert np.array_equal(o[k], ref[j][0][k]), (j, k)
            for k in d[0]:
                assert np.array_equal(d[0][k], ref[j][1][k]), (j, k)
        # a blocking call with two calls in flight finishes them first
        outs = [ctx.alloc_out(n) for _ in range(2)]
        ctx.submit_header_bytes(*inputs[1], out=outs[0])
        ctx.submit_header_bytes(*inputs[2], out=outs[1])
        o4 = ctx.verify_header_bytes(*inputs[0])
        for j, o in zip((1, 2, 0), outs + [o4]):
            for k in o:
                assert np.array_equal(o[k], ref[j][0][k]), (j, k)
        # page-locked arena and outputs
        outs = [ctx.alloc_out(n) for _ in range(3)]
        bufs = [arena] + [v for o in outs for v in o.values() if v.nbytes >= (1 << 20)]
        for b_ in bufs:
            ctx.host_register(b_)
        try:
            for o in outs:
                ctx.submit_header_bytes(arena, off, ln, out=o)
            ctx.drain()
        finally:
            for b_ in bufs:
                ctx.host_unregister(b_)
        for o in outs:
            for k in o:
                assert np.array_equal(o[k], ref[0][0][k]), k
        # a new epoch nonce while calls are in flight: praos_set_epoch finishes them first (under the
        # nonce they were queued with); a call after it runs under the new one
        eta1 = bytes(32 - len(b"other")) + b"other"
        ctx.set_epoch(eta1, pool_list, p)
        ref1 = ctx.verify_header_bytes(arena, off, ln)
        assert not np.array_equal(ref1["bits"], ref[0][0]["bits"])
        ctx.set_epoch(cfg["eta0"], pool_list, p)
        outs = [ctx.alloc_out(n) for _ in range(3)]
        ctx.submit_header_bytes(arena, off, ln, out=outs[0])
        ctx.submit_header_bytes(arena, off, ln, out=outs[1])
        ctx.set_epoch(eta1, pool_list, p)
        ctx.submit_header_bytes(arena, off, ln, out=outs[2])
        ctx.drain()
        for o, want in zip(outs, (ref[0][0], ref[0][0], ref1)):
            for k in o:
                assert np.array_equal(o[k], want[k]), k
    finally:
        ctx.drain()
        ctx.set_epoch(cfg["eta0"], pool_list, p)
        ctx.set_option(abi.OPT_PIPELINE, 0)
        if chunk_v is not None:
            ctx.close()


@pytest.mark.parametrize("env,concurrent", [({"PRAOS_PRE_JOIN": "0"}, 1), ({"PRAOS_PRE_JOIN": "1"}, 1),
                                            ({"PRAOS_PRE_JOIN": "1"}, 0), ({"PRAOS_V_MAIN": "1"}, 1), ({"PRAOS_V_MAIN": "2"}, 1), ({"PRAOS_V_MAIN": "0"}, 1),
                                            ({"PRAOS_V_MAIN": "1", "PRAOS_PRE_JOIN": "0"}, 1),
                                            ({"PRAOS_V_MAIN": "3", "PRAOS_MISS_PRIO": "1"}, 1)])
def test_schedule_variants_equal_single_batch(ctx, c5_batch, env, concurrent):
    """Schedule options that move work between kernels and streams give the default context's
    one-batch outputs bit for bit: the join's pool part ahead of it as k_vrf_pool (PRAOS_PRE_JOIN,
    default on below SMALL_BATCH headers) or in the join, stage V and the join on the main stream
    (PRAOS_V_MAIN; at this batch size the default is mode 2, so mode 3 with the uncached verifies
    at raised priority, the default from SHARD_SMALL headers, is a variant here), on concurrent
    streams and on one -- in one
    batch and pipelined (8 chunks, twice)."""
    import praos_hip
    from praos_hip import abi
    cfg, H, pool_list, corrupted, p, arena, off, ln = c5_batch
    ctx.set_epoch(cfg["eta0"], pool_list, p)
    ctx.set_option(abi.OPT_PIPELINE, 1)
    try:
        o1, D1 = ctx.verify_header_bytes(arena, off, ln, decoded=True)
    finally:
        ctx.set_option(abi.OPT_PIPELINE, 0)
    os.environ.update(env)
    try:
        c2 = praos_hip.Context(0)
    finally:
        for k in env:
            del os.environ[k]
    try:
        c2.set_option(abi.OPT_CONCURRENT, concurrent)
        c2.set_epoch(cfg["eta0"], pool_list, p)
        for chunks in (1, 8, 8):                      # the second 8-chunk call reuses the batch
            c2.set_option(abi.OPT_PIPELINE, chunks)
            o2, D2 = c2.verify_header_bytes(arena, off, ln, decoded=True)
            for k in o1:
                assert np.array_equal(o1[k], o2[k]), (chunks, k)
            for k in D1:
                assert np.array_equal(D1[k], D2[k]), (chunks, k)
    finally:
        c2.close()
