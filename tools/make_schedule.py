#!/usr/bin/env python3
"""Run the first-leader-wins search (praos_leader_schedule) for a chain config and
save its schedule, e.g. the C5 chain shipped as praos_hip/data/c5_schedule.npz:

    python tools/make_schedule.py c5 [--blocks N] [--out PATH]
    python tools/make_schedule.py c5 --blocks 1000000 --resume PATH --out PATH --max-seconds S

--resume continues a saved schedule of the same config from the slot after its last block
(the C3 schedule, data/c3_schedule.npz, is the C5 schedule continued to 1M blocks); with
--max-seconds the search stops after that long and saves what it has (run again to go on).

Output: slot deltas (u32) and forging pool (u16) per block, in chain order.  The
schedule depends on the config's seed (pool keys), stake, f and eta0
(praos_hip/chains.py CONFIGS); re-run this when any of them changes."""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ouroboros-consensus_amd"))

import praos_hip  # noqa: E402
from praos_hip import chains  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("config", choices=sorted(chains.CONFIGS))
    ap.add_argument("--blocks", type=int, default=None)
    ap.add_argument("--window", type=int, default=200_000)
    ap.add_argument("--out", default=None)
    ap.add_argument("--resume", default=None, help="schedule (.npz) to continue")
    ap.add_argument("--max-seconds", type=float, default=None)
    a = ap.parse_args()
    cfg = chains.CONFIGS[a.config]
    blocks = a.blocks or cfg["blocks"]
    out = a.out or os.path.join(chains.DATA, f"{a.config}_schedule.npz")
    ctx = praos_hip.Context(0)
    t0 = time.time()

    def progress(s, found):
        dt = time.time() - t0
        print(f"slots [0, {s}): {found} blocks, {dt:.0f}s, {s * cfg['npools'] / max(dt, 1e-9) / 1e6:.1f}M evals/s "
              "(upper bound)", flush=True)
    import numpy as np
    s_pre = np.zeros(0, np.uint64)
    p_pre = np.zeros(0, np.uint32)
    first = 0
    if a.resume and os.path.exists(a.resume):
        z = np.load(a.resume, allow_pickle=False)
        s_pre = np.cumsum(z["slot_delta"].astype(np.uint64))
        p_pre = z["pool"].astype(np.uint32)
        first = int(s_pre[-1]) + 1 if len(s_pre) else 0
        print(f"resuming after {len(s_pre)} blocks (slot {first})", flush=True)
    slots, pools = chains.search_schedule(ctx, cfg, max(blocks - len(s_pre), 0), first_slot=first, window=a.window,
                                          progress=progress, max_seconds=a.max_seconds)
    slots, pools = np.concatenate([s_pre, slots]), np.concatenate([p_pre, pools])
    chains.save_schedule(out, slots, pools, a.config)
    print(f"saved {len(slots)} blocks, last slot {int(slots[-1])}, {time.time() - t0:.0f}s -> {out}", flush=True)


if __name__ == "__main__":
    main()
