#!/usr/bin/env python3
"""Wall time of praos_verify_header_bytes (the chunked stored-bytes pipeline) on the C5
bench input for several chunk counts, each call timed after one warm-up call.
usage: e2e_pipe_probe.py [--register] K [K ...]
--register: the arena and the output arrays page-locked once (praos_host_register), as bench.py's e2e"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ouroboros-consensus_amd"))


def main():
    import praos_hip
    from praos_hip import abi, chains
    from praos_hip.chunk import pack_chunk
    ctx = praos_hip.Context(0)
    cfg = chains.CONFIGS["c5"]
    H, pool_list, corrupted, p = chains.make_chain(ctx, cfg, chains.load_schedule("c5"), corrupt_per_10000=100)
    ctx.set_epoch(cfg["eta0"], pool_list, p)
    arena, off, ln = pack_chunk(H)
    args = [a for a in sys.argv[1:] if a != "--register"]
    ob = ctx.alloc_out(len(off))
    if "--register" in sys.argv:
        for a in [arena] + [v for v in ob.values() if v.nbytes >= (4 << 20)]:
            ctx.host_register(a)
    for k in [int(a) for a in args] or [6]:
        ctx.set_option(abi.OPT_PIPELINE, k)
        ctx.verify_header_bytes(arena, off, ln, out=ob)
        ts = []
        for _ in range(3):
            t0 = time.perf_counter()
            ctx.verify_header_bytes(arena, off, ln, out=ob)
            ts.append(time.perf_counter() - t0)
        print(json.dumps({"chunks": k, "ms": [round(t * 1e3, 2) for t in ts],
                          "headers_per_s": round(len(off) / min(ts), 1)}), flush=True)


if __name__ == "__main__":
    main()
