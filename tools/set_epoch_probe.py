import sys, time, os
sys.path.insert(0, "/root/repo/ouroboros-consensus_amd")
import praos_hip
from praos_hip import chains
ctx = praos_hip.Context(0)
cfg = chains.CONFIGS["c5"]
H, pool_list, corrupted, p = chains.make_chain(ctx, cfg, chains.load_schedule("c5"), n=20000, corrupt_per_10000=100)
for rep in range(6):
    t = time.perf_counter(); ctx.set_epoch(cfg["eta0"], pool_list, p); t1 = time.perf_counter()
    print("set_epoch ms", round((t1 - t) * 1e3, 3), flush=True)
o = ctx.verify_headers(H)
for rep in range(4):
    t = time.perf_counter(); ctx.set_epoch(cfg["eta0"], pool_list, p); t1 = time.perf_counter()
    print("after run: set_epoch ms", round((t1 - t) * 1e3, 3), flush=True)
