"""Synthetic Praos chains for the benchmark configs (db-synthesizer analogue).

The reference forges a chain slot by slot: in every slot the forgers are tried in
order and the first whose checkShouldForge says ShouldForge (checkIsLeader,
Praos.hs:375-397) forges (Forging.hs:139-148).  Here that search runs on the GPU
(praos_leader_schedule) and gives per slot the forging pool; the generator
(praos_synthesize with a schedule) then signs exactly those headers.  Every clean
header of such a chain passes meetsLeaderThreshold by construction.

  C1 (configs[0]): the tools-test genesis (f = 1/20, slotsPerKESPeriod 129600,
      maxKESEvolutions 60), 100 pools with sigma_i ~ 1/(i+1), eta0 = Blake2b-256 of
      that genesis file, the first 10,000 blocks from slot 0.
  C5 (configs[4]): 3000 pools with sigma_i ~ 1/(i+10), f = 1/20, the first 432,000
      blocks from slot 0 of one epoch.  Its first-leader-wins search costs ~26e9 VRF
      evaluations (3000 pools x ~8.6M slots), so it was run once
      (tools/make_schedule.py) and the resulting schedule (slot, pool) per block is
      shipped in data/c5_schedule.npz; headers are re-signed from it in seconds.
"""
import hashlib
import os
from fractions import Fraction

import numpy as np

from . import abi, fixed

DATA = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data")

# test/tools-test/disk/config/genesis-shelley.json: Blake2b-256 of the file bytes
C1_ETA0 = bytes.fromhex("f6bb6e9d9b217681180754232470aa936716d62f8e11e944520b97490b100b7c")

CONFIGS = {
    "c1": dict(npools=100, stake_offset=1, f=Fraction(1, 20), slots_per_kes_period=129600, max_kes_evo=60,
               blocks=10_000, eta0=C1_ETA0, seed=b"C1" + b"\xc1" * 30, epoch_length=432_000),
    "c5": dict(npools=3000, stake_offset=10, f=Fraction(1, 20), slots_per_kes_period=129600, max_kes_evo=62,
               blocks=432_000, eta0=hashlib.blake2b(b"bench-epoch-nonce", digest_size=32).digest(),
               seed=b"C5" + b"\xc5" * 30, epoch_length=8_640_000),
    # TPraos (Shelley..Alonzo) analogue of C5: the same stake distribution and f, the TPraos
    # leader certificate (mkSeed seedL, 64-byte output, bound 2^512) decides the forger
    "tp": dict(npools=3000, stake_offset=10, f=Fraction(1, 20), slots_per_kes_period=129600, max_kes_evo=62,
               blocks=432_000, eta0=hashlib.blake2b(b"bench-tpraos-nonce", digest_size=32).digest(),
               seed=b"TP" + b"\x7c" * 30, epoch_length=8_640_000, tpraos=True),
}


def stake(npools, offset):
    """sigma_i ~ 1/(i + offset), exact rationals normalised, as Fixed E34 raw values."""
    w = [Fraction(1, i + offset) for i in range(npools)]
    tot = sum(w)
    return [fixed.from_rational(x / tot) for x in w]


def params(cfg, vrf_check_output=True):
    return abi.params(slots_per_kes_period=cfg["slots_per_kes_period"], max_kes_evo=cfg["max_kes_evo"],
                      c_raw=fixed.active_slot_log(cfg["f"]), f_is_one=cfg["f"] == 1,
                      vrf_check_output=vrf_check_output)


def search_schedule(ctx, cfg, blocks, first_slot=0, window=200_000, progress=None, max_seconds=None):
    """First-leader-wins forgers from first_slot until `blocks` blocks exist (or, with
    max_seconds, the whole windows searched by then).  Returns (slots u64[], pools u32[])."""
    import time
    t0 = time.time()
    sig = stake(cfg["npools"], cfg["stake_offset"])
    p = params(cfg)
    slots, pools = [], []
    s0, found = first_slot, 0
    if blocks <= 0:
        return np.zeros(0, np.uint64), np.zeros(0, np.uint32)
    while found < blocks and (max_seconds is None or time.time() - t0 < max_seconds):
        lead = ctx.leader_schedule(cfg["seed"], sig, p, cfg["eta0"], s0, window, tpraos=cfg.get("tpraos", False))
        idx = np.nonzero(lead >= 0)[0]
        slots.append((s0 + idx).astype(np.uint64))
        pools.append(lead[idx].astype(np.uint32))
        found += len(idx)
        s0 += window
        if progress:
            progress(s0, found)
    return np.concatenate(slots)[:blocks], np.concatenate(pools)[:blocks]


def save_schedule(path, slots, pools, cfg_name):
    d = np.diff(np.concatenate([[0], slots.astype(np.int64)]))
    assert d.min() >= 0 and d.max() < 2 ** 32
    np.savez_compressed(path, slot_delta=d.astype(np.uint32), pool=pools.astype(np.uint16),
                        config=np.frombuffer(cfg_name.encode(), np.uint8))


def load_schedule(name="c5"):
    z = np.load(os.path.join(DATA, f"{name}_schedule.npz"), allow_pickle=False)
    slots = np.cumsum(z["slot_delta"].astype(np.uint64))
    return slots, z["pool"].astype(np.uint32)


def make_chain(ctx, cfg, schedule, n=None, corrupt_per_10000=0, cbor_bodies=True, body_len=397, nkes=0, link=False,
               prev0=None):
    """Sign the first n blocks of a schedule.  Returns (H, pool_list, corrupted, params)
    with pool_list = [(hash28, vrf_hash32, sigma_fp)] in forger order.  link=True: a real
    chain, hbPrev = headerHash of the previous block (block 0: prev0, None = GenesisHash),
    H["header_hash"] holds the header hashes (sequential re-signing, ~0.1 ms per block).
    TPraos configs (cfg["tpraos"]) sign BHeaders: both certificates, the 15-field BHBody as
    the KES message."""
    slots, pools = schedule
    n = len(slots) if n is None else n
    p = params(cfg)
    H, keys, corrupted = ctx.synthesize(n, cfg["npools"], p, cfg["eta0"], cfg["seed"],
                                        body_len=0 if cbor_bodies else body_len,
                                        corrupt_per_10000=corrupt_per_10000, nkes=nkes,
                                        schedule=(slots[:n], pools[:n]), link=link, prev0=prev0,
                                        tpraos=cfg.get("tpraos", False))
    sig = stake(cfg["npools"], cfg["stake_offset"])
    pool_list = [(h, v, s) for (h, v), s in zip(keys, sig)]
    return H, pool_list, corrupted, p
