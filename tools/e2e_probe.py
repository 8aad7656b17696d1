#!/usr/bin/env python3
"""Breakdown of the end-to-end (PCIe-inclusive) path of the C5 bench input:
praos_batch_upload (repack + staged H2D), praos_batch_run + sync, praos_batch_download
(staged D2H), each timed separately over a few repetitions."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ouroboros-consensus_amd"))


def main():
    import praos_hip
    from praos_hip import chains
    ctx = praos_hip.Context(0)
    cfg = chains.CONFIGS["c5"]
    H, pool_list, corrupted, p = chains.make_chain(ctx, cfg, chains.load_schedule("c5"), corrupt_per_10000=100)
    n = len(H["slot"])
    nbytes = sum(v.nbytes for v in H.values())
    ctx.set_epoch(cfg["eta0"], pool_list, p)
    rows = []
    for rep in range(4):
        t0 = time.perf_counter()
        b = ctx.upload(H)
        t1 = time.perf_counter()
        ctx.run(b)
        ctx.sync()
        t2 = time.perf_counter()
        ctx.download(b, n)
        t3 = time.perf_counter()
        ctx.free(b)
        t4 = time.perf_counter()
        if rep:
            rows.append((t1 - t0, t2 - t1, t3 - t2, t4 - t3))
    best = [min(r[k] for r in rows) * 1e3 for k in range(4)]
    print(json.dumps({"headers": n, "input_bytes": nbytes, "upload_ms": round(best[0], 2), "run_ms": round(best[1], 2),
                      "download_ms": round(best[2], 2), "free_ms": round(best[3], 2),
                      "upload_GBps": round(nbytes / best[0] / 1e6, 1)}))


if __name__ == "__main__":
    main()
