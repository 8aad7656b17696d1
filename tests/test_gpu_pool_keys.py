"""The pool-key store (PRAOS_OPT_POOL_KEYS, k_keys.hip k_pkey_publish): cold-key and VRF-key
cache entries kept across runs of a context give the verdicts of the per-batch caches.

  - consecutive batches of a C5-shaped chain (3000 pools, f = 1/20, 1 % corrupted): bits,
    VRF outputs and nonces equal with the store on and off; with it on, no cold or VRF key is
    a miss and a later batch builds no new entry for a key an earlier one stored;
  - more distinct cold keys than the store holds (configs[1]-shaped OCerts, 20,000 keys
    against 16,384 entries): the overflow stays uncached (full verifies), the next run
    empties the full store first, and every verdict matches the store-off run."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _first(H, a, b):
    n = len(H["slot"])
    return {k: (v[a:b] if k != "body_bytes" and hasattr(v, "shape") and v.ndim and v.shape[0] == n else v)
            for k, v in H.items()}


def _run(ctx, H):
    b = ctx.upload(H)
    try:
        ctx.run(b)
        ctx.sync()
        out = ctx.download(b, len(H["slot"]))
        st = ctx.batch_stats(b)
    finally:
        ctx.free(b)
    return out, st


def test_pool_keys_equal_per_batch(ctx):
    from praos_hip import abi, configs
    H0, pool_list, corrupted, p, eta0, c_raw, spkp, maxevo = configs.build(ctx, "c5", n=24_000)
    try:
        configs.options(ctx, "c5")
        ctx.set_epoch(eta0, pool_list, p)
        ref, got, stats = [], [], []
        for mode in (0, 2):                       # store off; then on, emptied before the first batch
            ctx.set_option(abi.OPT_POOL_KEYS, mode)
            for a in range(0, 24_000, 6_000):
                out, st = _run(ctx, _first(H0, a, a + 6_000))
                (ref if mode == 0 else got).append(out)
                if mode:
                    stats.append(st)
                    ctx.set_option(abi.OPT_POOL_KEYS, 1)
    finally:
        ctx.set_option(abi.OPT_POOL_KEYS, -1)
        configs.options(ctx, "c5")
    for r, g in zip(ref, got):
        for f in ("bits", "pool_idx", "beta", "leader", "nonce"):
            np.testing.assert_array_equal(r[f], g[f])
    assert all(s["cold_misses"] == 0 and s["vrf_misses"] == 0 for s in stats), stats
    # the store only grows by keys not seen before: entries after the last batch <= pools
    assert stats[0]["vrf_keys"] <= stats[-1]["vrf_keys"] <= len(pool_list)
    assert stats[-1]["vrf_hits"] == 6_000
    clean = corrupted[:24_000] == 0
    assert int((np.concatenate([g["bits"] for g in got])[clean] != 0).sum()) == 0


def test_pool_keys_overflow(ctx):
    from praos_hip import abi, configs
    H, pool_list, corrupted, p, eta0, c_raw, spkp, maxevo = configs.build(ctx, "c2", n=20_000)
    try:
        configs.options(ctx, "c2")
        ctx.set_epoch(eta0, pool_list, p)
        ctx.set_option(abi.OPT_POOL_KEYS, 0)
        ref, _ = _run(ctx, H)
        ctx.set_option(abi.OPT_POOL_KEYS, 2)
        outs = []
        for _ in range(3):
            out, st = _run(ctx, H)
            outs.append((out, st))
            ctx.set_option(abi.OPT_POOL_KEYS, 1)
    finally:
        ctx.set_option(abi.OPT_POOL_KEYS, -1)
        configs.options(ctx, "c5")
    for out, st in outs:
        np.testing.assert_array_equal(ref["bits"], out["bits"])
        # 16,384 keys fit; the rest are misses (the second run finds the store full and empties it)
        assert st["cold_hits"] + st["cold_misses"] == 20_000 and st["cold_misses"] >= 20_000 - 16_384, st
    bad = corrupted[:20_000] != 0
    assert bad.sum() > 100 and int((ref["bits"][bad] == 0).sum()) == 0
