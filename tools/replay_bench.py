#!/usr/bin/env python3
"""End-to-end replay throughput (praos_replay_immutable): a
mainnet-shaped multi-epoch chain (f = 1/20, 432,000-slot epochs, so ~21.6k blocks per
epoch, first-leader-wins under each epoch's own nonce, linked prev hashes) is written
as an ImmutableDB (21,600-slot chunks, as mainnet) and replayed from disk: read the
chunk + secondary files, batches (spanning epochs, per-header nonces) decoded and
verified on the GPU, envelope + updateChainDepState folded on the host while the next
batch is on the device.  Prints one JSON line per batch size with the per-stage times
of the driver (ms_io / ms_device / ms_nonce / ms_fold) and headers/s from stored bytes.

    python tools/replay_bench.py [--epochs 5] [--pools 200] [--reps 3] [--batch-sizes 32768,1048576]
"""
import argparse
import json
import os
import sys
import tempfile
import time
from fractions import Fraction

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ouroboros-consensus_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--epochs", type=int, default=5)
    ap.add_argument("--pools", type=int, default=200)
    ap.add_argument("--epoch-length", type=int, default=432_000)
    ap.add_argument("--chunk-slots", type=int, default=21_600)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--batch-sizes", default="16384,32768,65536,1048576")
    ap.add_argument("--round-robin", action="store_true",
                    help="f = 1 and a block in every slot, pools in turn (the C5 shape: 432k headers per "
                         "432k-slot epoch, 3000 pools, without the leader-schedule search)")
    ap.add_argument("--window", type=int, default=None, help="stability window in slots (default 4k/f, k = 2160)")
    ap.add_argument("--chain", choices=("c5", "tp"), default=None,
                    help="the bench chain's configuration (praos_hip.chains.CONFIGS: 3000 pools, f = 1/20, 8.64M-slot "
                         "epochs); epoch 0 takes the shipped first-leader-wins schedule, later epochs are searched")
    ap.add_argument("--pool-keys", default="cold",
                    help="comma list of pool-key store modes (PRAOS_OPT_POOL_KEYS) to time: off (per-batch key "
                         "caches only), cold (the store emptied before each replay call: a fresh replay job), warm "
                         "(the store kept across calls)")
    ap.add_argument("--members", default="1",
                    help="comma list: 1 = one context, m > 1 = a praos_group of m contexts on device 0 "
                         "(praos_group_replay_immutable: batches dealt to the members in turn, one fold)")
    ap.add_argument("--schedule-out", default=None,
                    help="directory: save each searched epoch's first-leader-wins schedule (e >= 1) as "
                         "<chain>_epoch<e>_schedule.npz, so a later run can skip the search")
    ap.add_argument("--schedule-in", default=None,
                    help="comma list of epoch=file.npz schedules to use instead of searching (e.g. the c5 chain's "
                         "epoch 1: 1=ouroboros-consensus_amd/praos_hip/data/c5_epoch1_schedule.npz)")
    ap.add_argument("--env-variants", default="",
                    help="';'-separated host settings to time, each a comma list of VAR=VALUE set before a fresh "
                         "context is opened (e.g. 'PRAOS_REPLAY_PIN=0;PRAOS_REPLAY_PIN=1,PRAOS_COPY_THREADS=8'); "
                         "empty: the environment as it is")
    ap.add_argument("--tpraos", action="store_true",
                    help="a Shelley..Alonzo (TPraos) chain replayed by praos_replay_immutable_tpraos (TICKN with extra entropy)")
    args = ap.parse_args()
    import hashlib
    import praos_hip
    from praos_hip import immutable
    ctx = praos_hip.Context(0)
    f = Fraction(1) if args.round_robin else Fraction(1, 20)
    cfg = dict(npools=args.pools, stake_offset=10, f=f, slots_per_kes_period=129600, max_kes_evo=62,
               eta0=hashlib.blake2b(b"replay-bench", digest_size=32).digest(), seed=b"RB" + b"\x5b" * 30,
               round_robin=args.round_robin)
    schedules = None
    if args.chain:
        from praos_hip import chains
        assert args.tpraos == (args.chain == "tp") and not args.round_robin
        cfg = dict(chains.CONFIGS[args.chain])
        assert args.epoch_length == cfg["epoch_length"] and args.pools == cfg["npools"]
        f = cfg["f"]
        schedules = {0: chains.load_schedule(args.chain)}
    if args.schedule_in:
        import numpy as np
        schedules = dict(schedules or {})
        for item in args.schedule_in.split(","):
            e, fn = item.split("=")
            z = np.load(fn)
            schedules[int(e)] = (z["slots"], z["pools"])
    window = args.window or int(4 * 2160 / f)   # 4k/f with k = 2160: the Babbage stability window
    t0 = time.perf_counter()
    # heartbeat while the chain is generated (the linked re-signing is sequential: minutes
    # for 432k-block epochs)
    import threading
    gen_done = threading.Event()

    def beat():
        while not gen_done.wait(30):
            print(f"generating... {time.perf_counter() - t0:.0f}s", file=sys.stderr, flush=True)
    threading.Thread(target=beat, daemon=True).start()
    xe = hashlib.blake2b(b"replay-bench-extra-entropy", digest_size=32).digest() if args.tpraos else None
    data = immutable.make_multi_epoch_chain(
        ctx, cfg, args.epochs, args.epoch_length, window, tpraos=args.tpraos, extra_entropy=xe,
        progress=lambda e, n: print(f"epoch {e}: {n} blocks signed and linked ({time.perf_counter() - t0:.0f}s)",
                                    file=sys.stderr, flush=True),
        schedules=schedules)
    gen_done.set()
    t_gen = time.perf_counter() - t0
    if args.schedule_out:
        import numpy as np
        os.makedirs(args.schedule_out, exist_ok=True)
        for e in range(1, args.epochs):
            if schedules and e in schedules:
                continue
            sl, pl = data["schedules"][e]
            np.savez_compressed(os.path.join(args.schedule_out, f"{args.chain or 'replay'}_epoch{e}_schedule.npz"),
                                slots=np.asarray(sl, np.uint64), pools=np.asarray(pl, np.uint32))
    n = len(data["off"])
    env_limits = {"max_major_pv": 9, "lv_prot_major": 8, "max_header_size": 1100, "max_body_size": 90_112}
    with tempfile.TemporaryDirectory() as tmp:
        path = os.path.join(tmp, "immutable")
        nch = immutable.write_immutable(path, data["arena"], data["off"], data["len"], data["slots"],
                                        data["header_hash"], args.chunk_slots)
        from praos_hip import abi
        variants = [v for v in args.env_variants.split(";")] if args.env_variants else [""]
        env0 = dict(os.environ)
        for variant in variants:
         os.environ.clear()                                                       # each variant on its own
         os.environ.update(env0)
         for item in filter(None, variant.split(",")):
             k, v = item.split("=")
             os.environ[k] = v
         for members in [int(x) for x in args.members.split(",")]:
          # a fresh context (or group) per variant: settings read when a context starts are seen
          runner = praos_hip.Context(0) if members == 1 else abi.Group([0] * members)
          for mode in args.pool_keys.split(","):
              for batch_max in [int(x) for x in args.batch_sizes.split(",")]:
                  runs = []
                  for rep in range(args.reps + 1):                              # rep 0 warms caches / allocator
                      runner.set_option(abi.OPT_POOL_KEYS, {"off": 0, "cold": 2, "warm": 1}[mode])
                      st = {"last_slot": None, "counters": {}, "evolving": cfg["eta0"], "candidate": cfg["eta0"],
                            "epoch_nonce": cfg["eta0"], "lab": None, "leb": None}
                      env = dict(env_limits, tip=None)
                      t = time.perf_counter()
                      stats = runner.replay_immutable(path, data["pools"], data["params"], data["epoch_info"], st, env,
                                                      batch_max=batch_max, tpraos=args.tpraos, extra_entropy=xe)[0]
                      wall = time.perf_counter() - t
                      assert stats["validated"] == n and st == data["state"], stats
                      if rep:
                          runs.append(dict(stats, wall_ms=wall * 1e3))
                  best = min(runs, key=lambda r: r["wall_ms"])
                  line = {"metric": f"replayed {'TPraos' if args.tpraos else 'Praos'} headers/s from an ImmutableDB "
                                    "(read + GPU decode/crypto + host fold)",
                          "value": round(n / (best["wall_ms"] * 1e-3), 1), "unit": "headers/s", "headers": n,
                          "epochs": args.epochs, "blocks_per_epoch": round(n / args.epochs), "chunks": nch,
                          "pools": args.pools, "wall_ms": round(best["wall_ms"], 2),
                          "walls_ms": [round(r["wall_ms"], 2) for r in runs],
                          "schedule": "round-robin, f = 1" if args.round_robin else "first-leader-wins, f = 1/20",
                          "chain": args.chain or "replay-bench", "pool_keys": mode, "members": members,
                          "stages_ms": {k: round(best[k], 2) for k in ("ms_io", "ms_device", "ms_nonce", "ms_fold")},
                          "batch_max": batch_max, "batches": best["batches"], "epoch_nonces": best["epochs"],
                          "generate_s": round(t_gen, 1), "reps": args.reps, "host_settings": variant or None,
                          "data": "synthetic linked first-leader-wins chain, GPU-signed; written to a temp dir"}
                  print(json.dumps(line), flush=True)
          runner.set_option(abi.OPT_POOL_KEYS, -1)
          runner.close()
    os.environ.clear()
    os.environ.update(env0)
    ctx.close()


if __name__ == "__main__":
    main()
