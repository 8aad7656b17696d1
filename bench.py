#!/usr/bin/env python3
"""bench.py -- Praos header-crypto validation throughput on MI355X.

Metric (BASELINE.json): Praos headers validated/sec (VRF + KES + OCert + leader).
Workload: configs[4], a mainnet-shaped epoch replay: 432,000 Praos (Babbage)
headers per GPU, 3000-pool stake distribution (sigma_i ~ 1/(i+10)), one epoch
nonce, f = 1/20, slotsPerKESPeriod 129600, maxKESEvo 62, 397-byte signed
bodies, 1% of headers corrupted with the consensus-testlib +1-byte model.  The
chain is synthesised on the GPU by the library's generator (real Ed25519 /
Sum6KES / ECVRF-draft03 signatures; db-synthesizer analogue) and is resident in
HBM before the timed region.  One step = one full validation pass (all four
kernels) over the GPU's shard.  Multi-GPU: one process per GPU; each rank owns
a contiguous slot range of its own 432k headers (weak scaling, no collective on
the data path; only the timing max-reduce).

CPU baseline: the C oracle (oracle/, a port of the reference semantics; the
Haskell reference cannot run here) timed on the host over a bounded sample of
the same headers with a process pool, cores stated; it also cross-checks the
GPU bits on that sample.
"""
import argparse
import json
import math
import multiprocessing as mp
import os
import sys
import time
from fractions import Fraction

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "ouroboros-consensus_amd"))

# Algorithmic work per header (int32 lane-ops), counted from the kernel schedule
# (DESIGN.md "Work model"): field mul 154, square 130, add/sub 17, SHA-512 block
# 5000, BLAKE2b block 2700 int32 ops.
W_OCERT = 529_000
W_KES = 555_000
W_VRF = 1_150_000
W_LEADER = 3_000
W_HEADER = W_OCERT + W_KES + W_VRF + W_LEADER
PEAK_INT32 = 256 * 64 * 2.4e9      # VOP3 integer issue: 64 lane-ops/clk/CU (measured: tools/microbench)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def epoch_setup(npools, f=Fraction(1, 20)):
    import hashlib
    from praos_hip import abi, fixed
    c_raw = fixed.active_slot_log(f)
    p = abi.params(slots_per_kes_period=129600, max_kes_evo=62, c_raw=c_raw, vrf_check_output=True)
    eta0 = hashlib.blake2b(b"bench-epoch-nonce", digest_size=32).digest()
    w = [Fraction(1, i + 10) for i in range(npools)]
    tot = sum(w)
    sig = [fixed.from_rational(x / tot) for x in w]
    return p, eta0, c_raw, sig


def _oracle_worker(payload):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    eta0, c_raw, pools, headers = payload
    ep = oracle.make_epoch(eta0, 129600, 62, c_raw, pools)
    t0 = time.perf_counter()
    bits = [oracle.praos_header(ep, h)["bits"] for h in headers]
    return bits, time.perf_counter() - t0


def cpu_baseline(H, out_bits, eta0, c_raw, pool_list, seconds, workers):
    """Times the oracle (port of the reference path) on a bounded sample."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    oracle.lib()
    per_hdr = 1.4e-3
    n_total = len(H["slot"])
    n_sample = int(min(n_total, max(workers * 8, seconds * workers / per_hdr)))
    idx = np.linspace(0, n_total - 1, n_sample).astype(np.int64)
    hs = []
    for i in idx:
        off, ln = int(H["body_off"][i]), int(H["body_len"][i])
        hs.append({"slot": int(H["slot"][i]), "cold_vk": bytes(H["cold_vk"][i]), "vrf_vk": bytes(H["vrf_vk"][i]),
                   "vrf_out": bytes(H["vrf_out"][i]), "vrf_proof": bytes(H["vrf_proof"][i]),
                   "hot_vk": bytes(H["hot_vk"][i]), "n": int(H["ocert_n"][i]), "c0": int(H["ocert_c0"][i]),
                   "ocert_sig": bytes(H["ocert_sig"][i]), "kes_sig": bytes(H["kes_sig"][i]),
                   "body": bytes(H["body_bytes"][off:off + ln])})
    chunks = [hs[k::workers] for k in range(workers)]
    t0 = time.perf_counter()
    with mp.get_context("spawn").Pool(workers) as pool:
        res = pool.map(_oracle_worker, [(eta0, c_raw, pool_list, c) for c in chunks])
    wall = time.perf_counter() - t0
    busy = max(r[1] for r in res)
    bits = [None] * n_sample
    for k, (b, _) in enumerate(res):
        for j, v in enumerate(b):
            bits[k + j * workers] = v
    mask = 0x1F1F
    agree = sum(1 for j, i in enumerate(idx) if (int(out_bits[i]) & mask) == bits[j])
    return {"value": n_sample / busy, "unit": "headers/s", "cores": workers, "kind": "port",
            "sample": f"{n_sample} headers evenly spaced over the benchmark chain, C oracle (oracle/praos.c) "
                      f"in {workers} processes; busy {busy:.1f}s, wall {wall:.1f}s",
            "parity_sample": {"n": n_sample, "bit_exact": agree}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--headers", type=int, default=432_000, help="headers per GPU")
    ap.add_argument("--pools", type=int, default=3000)
    ap.add_argument("--corrupt-per-10000", type=int, default=100)
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--cpu-workers", type=int, default=16)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--concurrent", type=int, default=1, help="run OCert/KES/VRF kernels on 3 streams")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl")
    import torch

    import praos_hip
    ctx = praos_hip.Context(local)
    ctx.set_option(1, args.concurrent)
    n = args.headers
    stride = 20                                    # 432k headers ~ 8.64M slots at f = 1/20
    p, eta0, c_raw, sig = epoch_setup(args.pools)
    t0 = time.perf_counter()
    H, pools, corrupted = ctx.synthesize(n, args.pools, p, eta0, (b"\x5a" * 28) + rank.to_bytes(4, "little"),
                                         first_slot=rank * n * stride, slot_stride=stride, body_len=397,
                                         corrupt_per_10000=args.corrupt_per_10000)
    pool_list = [(h, v, s) for (h, v), s in zip(pools, sig)]
    ctx.set_epoch(eta0, pool_list, p)
    b = ctx.upload(H)
    log(f"[rank {rank}] synthesised + uploaded {n} headers in {time.perf_counter() - t0:.1f}s")

    for _ in range(args.warmup):
        ctx.run(b)
        ctx.sync()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    kms = np.zeros(5)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        ctx.run(b)
        ctx.sync()                                 # per-step HIP-event kernel times
        kms += [ctx.kernel_ms(k) for k in range(5)]
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    dt = time.perf_counter() - t0
    if dist:
        t = torch.tensor([dt], device="cuda", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    # per-kernel durations for the roofline: serial launches (HIP events on the
    # launch stream), untimed, after the timed region
    ctx.set_option(1, 0)
    kser = np.zeros(5)
    for _ in range(3):
        ctx.run(b)
        ctx.sync()
        kser += [ctx.kernel_ms(k) for k in range(5)]
    kser /= 3
    ctx.set_option(1, args.concurrent)
    out = ctx.download(b, n)
    ctx.free(b)

    # self-check on the whole shard: clean headers must pass all crypto checks
    clean = corrupted == 0
    crypto_bits = out["bits"] & ~np.uint16(0x1000)
    clean_ok = int((crypto_bits[clean] == 0).sum())
    corrupt_caught = int((crypto_bits[~clean] != 0).sum())

    if rank != 0:
        return
    steps = args.steps
    ms_step = dt * 1e3 / steps
    value = world * n * steps / dt
    kms /= steps
    k_total = kms[4]                               # whole pipeline per step (HIP events)
    achieved = n * W_HEADER / (k_total * 1e-3)
    per_kernel = {"ocert": kser[0], "kes": kser[1], "vrf": kser[2], "leader": kser[3]}
    dominant = max(("ocert", "kes", "vrf"), key=lambda k: per_kernel[k])
    wk = {"ocert": W_OCERT, "kes": W_KES, "vrf": W_VRF}[dominant]
    dom_achieved = n * wk / (per_kernel[dominant] * 1e-3)
    line = {
        "metric": "Praos headers validated/sec (VRF+KES+OCert+leader)",
        "value": round(value, 1), "unit": "headers/s", "n_gpus": world, "steps": steps, "warmup": args.warmup,
        "ms_per_step": round(ms_step, 3), "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "u32 (GF(2^255-19) radix-2^32 limbs; Fixed E34 bignum)", "data": "synthetic",
        "config": {"workload": "configs[4]: mainnet-shaped epoch replay, 432k Praos headers per GPU, "
                               "3000-pool stake distribution, single eta0, 1% corrupted",
                   "headers_per_gpu": n, "pools": args.pools, "active_slot_coeff": "1/20",
                   "body_bytes": 397, "parallelism": f"shard-by-slot-range x{world}"},
        "roofline": {"bound": "valu-int32", "kernel": f"k_{dominant}",
                     "achieved": round(dom_achieved / 1e12, 3), "peak": round(PEAK_INT32 / 1e12, 2),
                     "unit": "T int32-ops/s", "frac": round(dom_achieved / PEAK_INT32, 4), "traffic": None,
                     "pipeline_achieved": round(achieved / 1e12, 3),
                     "pipeline_frac": round(achieved / PEAK_INT32, 4),
                     "work_per_header": W_HEADER,
                     "kernel_ms_serial": {k: round(v, 3) for k, v in per_kernel.items()},
                     "pipeline_ms": round(k_total, 3), "concurrent_streams": bool(args.concurrent)},
        "self_check": {"clean_headers": int(clean.sum()), "clean_crypto_ok": clean_ok,
                       "corrupted": int((~clean).sum()), "corrupted_rejected": corrupt_caught,
                       "leader_pass": int(((out["bits"] & 0x1000) == 0).sum())},
    }
    if world == 1 and not args.no_cpu:
        workers = max(1, min(args.cpu_workers, os.cpu_count() or 1))
        line["cpu_baseline"] = cpu_baseline(H, out["bits"], eta0, c_raw, pool_list, args.cpu_seconds, workers)
        line["gpu_vs_cpu"] = round(value / line["cpu_baseline"]["value"], 1)
    print(json.dumps(line), flush=True)
    ctx.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
