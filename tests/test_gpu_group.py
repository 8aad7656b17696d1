"""praos_group: one process, several contexts (here all on the one GPU of the box; on
an 8-GPU node the members are devices 0..7), a batch split into contiguous shards run
concurrently, outputs gathered in place -- bit-exact against one context, and the
shard -> gather -> fold path (updateChainDepState on member 0 over the gathered
outputs) equal to the single-context fold."""
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
