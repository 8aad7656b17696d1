#!/usr/bin/env python3
"""Throughput of the ImmutableDB block-integrity batch on one GPU.

    python tools/bench_blocks.py [--blocks 65536] [--payload 16384] [--steps 10] [--warmup 2]

Workload: `--blocks` stored Babbage blocks [6, [header, [payload], [], {}, []]] in one
resident arena (an ImmutableDB chunk analogue).  Headers come from the GPU generator
(praos_synthesize, genuine Sum6KES signatures over canonical CBOR bodies) with hbBodyHash
set to the hashTxSeq of each block's segments (hashlib on the host), so every block is
intact; 1 % of blocks get one payload byte incremented (Corruption.hs model) and must
come back PRAOS_BLK_BODY_HASH.  A step = praos_block_batch_run over the whole arena
(split + header decode + KES + segment hashes + join).  Reports blocks/s and the block
bytes/s; per-kernel durations come from rocprofv3 (profiles/).
"""
import argparse
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ouroboros-consensus_amd"))
import praos_hip  # noqa: E402
from praos_hip import abi, chunk  # noqa: E402

SPKP = 129600


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--blocks", type=int, default=262144)
    ap.add_argument("--payload", type=int, default=16384, help="tx-segment payload bytes per block")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    args = ap.parse_args()
    n, pl = args.blocks, args.payload
    rng = np.random.default_rng(0xB10C)
    pay = rng.integers(0, 256, size=(n, pl), dtype=np.uint8)
    payloads = [pay[i].tobytes() for i in range(n)]
    bh = np.frombuffer(b"".join(chunk.hash_tx_seq((chunk.tx_segment(p),) + chunk.SEG_FIXED) for p in payloads),
                       np.uint8).reshape(n, 32)
    ctx = praos_hip.Context(0)
    p = abi.params(slots_per_kes_period=SPKP, max_kes_evo=62)
    eta0 = hashlib.blake2b(b"bench-blocks", digest_size=32).digest()
    H, _, _ = ctx.synthesize(n, 3000, p, eta0, b"\xb1" * 32, slot_stride=20, body_len=0, body_hash=bh)
    bad = set(int(i) for i in rng.choice(n, size=max(1, n // 100), replace=False))
    for i in bad:   # +1 at one payload byte (Corruption.hs:29-35)
        b = bytearray(payloads[i])
        k = int(rng.integers(pl))
        b[k] = (b[k] + 1) & 0xFF
        payloads[i] = bytes(b)
    arena, off, ln = chunk.pack_blocks(H, payloads)
    b = ctx.upload_blocks(arena, off, ln)
    try:
        for _ in range(args.warmup):
            ctx.run_blocks(b, SPKP)
        ctx.sync()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            ctx.run_blocks(b, SPKP)
        ctx.sync()
        dt = (time.perf_counter() - t0) / args.steps
        res, calc = ctx.download_blocks(b, n)
    finally:
        ctx.free(b)
    want = np.zeros(n, np.uint8)
    want[list(bad)] = abi.BLK_BODY_HASH
    exact = int((res == want).sum())
    sample = range(0, n, max(1, n // 257))
    hash_ok = all(bytes(calc[i]) == chunk.hash_tx_seq((chunk.tx_segment(payloads[i]),) + chunk.SEG_FIXED)
                  for i in sample)
    total = int(ln.astype(np.int64).sum())
    print(json.dumps({
        "metric": "stored blocks integrity-checked/sec (verifyBlockIntegrity: KES + hashTxSeq)",
        "value": round(n / dt, 1), "unit": "blocks/s", "ms_per_step": round(1e3 * dt, 3),
        "block_bytes_per_s_GB": round(total / dt / 1e9, 2), "blocks": n, "avg_block_bytes": total // n,
        "steps": args.steps, "warmup": args.warmup, "data": "synthetic (GPU-signed headers, random payloads)",
        "self_check": {"exact": exact, "n": n, "body_hash_rejected": len(bad), "hash_sample_ok": hash_ok}}))
    if exact != n or not hash_ok:
        sys.exit(1)


if __name__ == "__main__":
    main()
