#!/usr/bin/env python3
"""Streaming form of the stored-bytes path on the C5 bench input (432k headers): CALLS calls
back to back through praos_verify_header_bytes_submit (three in flight), then praos_verify_drain,
the arena and outputs page-locked; prints the wall per call of each run and of single blocking
calls.  Run under rocprofv3 --kernel-trace --memory-copy-trace, then tools/e2e_timeline.py.
    python tools/e2e_stream_probe.py [calls] [runs] [chunks]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ouroboros-consensus_amd"))


def main():
    calls = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    runs = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    chunks = int(sys.argv[3]) if len(sys.argv) > 3 else 0       # PRAOS_OPT_PIPELINE (0: auto)
    import praos_hip
    from praos_hip import chains
    from praos_hip.chunk import pack_chunk
    ctx = praos_hip.Context(0)
    cfg = chains.CONFIGS["c5"]
    H, pool_list, corrupted, p = chains.make_chain(ctx, cfg, chains.load_schedule("c5"), corrupt_per_10000=100)
    n = len(H["slot"])
    ctx.set_epoch(cfg["eta0"], pool_list, p)
    from praos_hip import abi
    ctx.set_option(abi.OPT_PIPELINE, chunks)
    arena, off, ln = pack_chunk(H)
    obs = [ctx.alloc_out(n) for _ in range(3)]
    bufs = [arena] + [v for o in obs for v in o.values() if v.nbytes >= (4 << 20)]
    for a in bufs:
        ctx.host_register(a)
    single = []
    for _ in range(3):
        t = time.perf_counter()
        ctx.verify_header_bytes(arena, off, ln, out=obs[0])
        single.append((time.perf_counter() - t) * 1e3)
    ref = {k: v.copy() for k, v in obs[0].items()}
    stream, submit_ms = [], []
    for _ in range(runs):
        t = time.perf_counter()
        ts = []
        for j in range(calls):
            t1 = time.perf_counter()
            ctx.submit_header_bytes(arena, off, ln, out=obs[j % len(obs)])
            ts.append(round((time.perf_counter() - t1) * 1e3, 2))
        t1 = time.perf_counter()
        ctx.drain()
        ts.append(round((time.perf_counter() - t1) * 1e3, 2))
        stream.append((time.perf_counter() - t) * 1e3 / calls)
        submit_ms.append(ts)
    exact = all((o[k] == ref[k]).all() for o in obs for k in ref)
    for a in bufs:
        ctx.host_unregister(a)
    print(json.dumps({"headers": n, "single_ms": [round(x, 2) for x in single],
                      "stream_ms_per_call": [round(x, 2) for x in stream], "calls": calls, "chunks": chunks,
                      "host_ms_per_submit_then_drain": submit_ms, "exact": bool(exact)}))
    ctx.close()


if __name__ == "__main__":
    main()
