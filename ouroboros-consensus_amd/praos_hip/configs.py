"""The benchmark workloads of BASELINE.json's configs, built the same way for bench.py and for
the -m gpu tests that run them at their stated sizes (host-side plumbing).

  c1  configs[0]: the first 10,000 blocks of a first-leader-wins chain, 100 pools (chains.py)
  c2  configs[1]: 1M OCert Ed25519 signatures, distinct cold keys, 1 % corrupted in OCert fields
  c3  configs[2]: 1M ECVRF verifies + leader checks under one eta0: the (slot, pool) pairs of the
      first 1,000,000 blocks of the C5 chain's first-leader-wins schedule (3000 pools, f = 1/20,
      data/c3_schedule.npz), so every clean item is a real leader and the leader test runs its
      Taylor comparison as on a chain; 1 % corrupted in the VRF proof / output
  c4  configs[3]: 1M Sum6KES signatures over 397-byte messages, 3000 pools x 64 KES periods,
      1 % corrupted in the KES signature / message
  c5  configs[4]: the first 432,000 blocks of the C5 chain (chains.py, data/c5_schedule.npz)
  tp  TPraos headers from stored bytes: the first 432,000 blocks of a first-leader-wins TPraos
      chain (3000 pools, f = 1/20, data/tp_schedule.npz)

Each returns (H, pool_list, corrupted, params, eta0, c_raw, slots_per_kes_period, max_kes_evo);
`corrupted[i]` is the synthesizer's corruption kind (0 clean, 1 OCert, 2 KES signature,
3 VRF proof, 4 VRF output, 5 signed body)."""
import hashlib
from fractions import Fraction

import numpy as np

from . import abi, chains, fixed

# crypto kernels each config runs (PRAOS_OPT_KERNELS: 1 OCert, 2 KES, 4 VRF + leader)
KERNELS = {"c1": 7, "c2": 1, "c3": 4, "c4": 2, "c5": 7, "tp": 7}
ITEMS = {"c1": 10_000, "c2": 1_000_000, "c3": 1_000_000, "c4": 1_000_000, "c5": 432_000, "tp": 432_000}
# corruption kinds a config's checks can see (the others land in fields it does not read)
CHECKED_KINDS = {1: (1,), 2: (2, 5), 4: (3, 4), 7: (1, 2, 3, 4, 5)}


def build(ctx, name, n=None, corrupt_per_10000=100, rank=0, world=1, scaling="weak"):
    """Signs config `name`'s input on the GPU (rank's shard; strong scaling splits c1/c5)."""
    n = n or ITEMS[name]
    if name in ("c1", "c5"):
        ccfg = chains.CONFIGS[name]
        sched = chains.load_schedule("c5") if name == "c5" else chains.search_schedule(ctx, ccfg, ccfg["blocks"])
        assert n <= len(sched[0]), "the shipped schedule has fewer blocks"
        if scaling == "strong":
            a, b = n * rank // world, n * (rank + 1) // world
            sched, n = (sched[0][a:b], sched[1][a:b]), b - a
        H, pool_list, corrupted, p = chains.make_chain(ctx, ccfg, sched, n=n, corrupt_per_10000=corrupt_per_10000)
        return (H, pool_list, corrupted, p, ccfg["eta0"], fixed.active_slot_log(ccfg["f"]),
                ccfg["slots_per_kes_period"], ccfg["max_kes_evo"])
    if name == "tp":
        # TPraos: the first 432,000 blocks of a first-leader-wins TPraos chain (chains.py "tp":
        # 3000 pools, f = 1/20, the leader certificate against 2^512; data/tp_schedule.npz),
        # two VRF certificates per header, BHeader bytes stored and decoded by the caller
        ccfg = chains.CONFIGS["tp"]
        sched = chains.load_schedule("tp")
        assert n <= len(sched[0]), "the shipped TPraos schedule has fewer blocks"
        H, pool_list, corrupted, p = chains.make_chain(ctx, ccfg, sched, n=n, corrupt_per_10000=corrupt_per_10000)
        return (H, pool_list, corrupted, p, ccfg["eta0"], fixed.active_slot_log(ccfg["f"]),
                ccfg["slots_per_kes_period"], ccfg["max_kes_evo"])
    if name == "c3":
        # the C5 chain's keys, stake, f and eta0; the (slot, pool) pairs of its schedule's first
        # 1M blocks (a rank > 0 of a weak-scaling run takes the next 1M-block window when the
        # schedule holds it, else the same blocks)
        ccfg = chains.CONFIGS["c5"]
        slots, pools = chains.load_schedule("c3")
        a = rank * n if (rank + 1) * n <= len(slots) else 0
        assert a + n <= len(slots), "the shipped C3 schedule has fewer blocks"
        p = chains.params(ccfg)
        H, keys, corrupted = ctx.synthesize(n, ccfg["npools"], p, ccfg["eta0"], ccfg["seed"], body_len=397,
                                            corrupt_per_10000=corrupt_per_10000,
                                            schedule=(slots[a:a + n], pools[a:a + n]),
                                            corrupt_fields=abi.CORRUPT_VRF_PROOF | abi.CORRUPT_VRF_OUT)
        pool_list = [(h, v, s) for (h, v), s in zip(keys, chains.stake(ccfg["npools"], ccfg["stake_offset"]))]
        return (H, pool_list, corrupted, p, ccfg["eta0"], fixed.active_slot_log(ccfg["f"]),
                ccfg["slots_per_kes_period"], ccfg["max_kes_evo"])
    # c2 / c4: evenly spaced slots, pools by hash (single primitives: no leader test runs)
    npools = n if name == "c2" else 3000
    c_raw = fixed.active_slot_log(Fraction(1, 20))
    p = abi.params(slots_per_kes_period=129600, max_kes_evo=62, c_raw=c_raw, vrf_check_output=True)
    eta0 = hashlib.blake2b(b"bench-epoch-nonce", digest_size=32).digest()
    fields = {"c2": abi.CORRUPT_OCERT, "c4": abi.CORRUPT_KES_SIG | abi.CORRUPT_BODY}[name]
    H, pools, corrupted = ctx.synthesize(n, npools, p, eta0, (b"\x5a" * 27) + bytes([int(name[1])]) +
                                         rank.to_bytes(4, "little"), first_slot=rank * n * 20, slot_stride=20,
                                         body_len=397, corrupt_per_10000=corrupt_per_10000,
                                         nkes=64 if name == "c2" else 0, corrupt_fields=fields)
    pool_list = [] if name == "c2" else [(h, v, s) for (h, v), s in zip(pools, chains.stake(npools, 10))]
    return H, pool_list, corrupted, p, eta0, c_raw, 129600, 62


def options(ctx, name, concurrent=1, keycache=2, dedup=1, pipeline=0):
    """The context options the bench runs a config with: the OCert dedup belongs to the header
    pipeline (a chain repeats each pool's OCert); single-primitive configs verify every item."""
    k = KERNELS[name]
    if k != 7:
        dedup = 0
    ctx.set_option(abi.OPT_CONCURRENT, concurrent)
    ctx.set_option(abi.OPT_KERNELS, k)
    ctx.set_option(abi.OPT_KEYCACHE, keycache)
    ctx.set_option(abi.OPT_DEDUP, dedup)
    ctx.set_option(abi.OPT_PIPELINE, pipeline)
    return dedup
