"""CPU, world_size 2 (gloo): the multi-GPU data path shards by contiguous slot
range with no collective; only the verdict gather and the timing max-reduce
cross ranks (praos_hip.dist).  test_gather_library_outputs runs the real library
per shard (the CPU twin libpraos_cpu.so, same C ABI as libpraos_hip) on oracle-signed
headers and compares the gathered outputs with one process over the whole batch."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n_total, q):
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "ouroboros-consensus_amd"))
    import torch.distributed as dist
    from praos_hip import dist as pd
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = pd.shard_range(rank, world, n_total)
    # stand-in for the per-shard GPU verdicts: deterministic function of the header index
    idx = np.arange(lo, hi)
    bits = ((idx * 2654435761) % 97 == 0).astype(np.uint16) * 0x0004
    allbits = pd.gather_verdicts(bits)
    t = pd.max_over_ranks(float(rank + 1))
    if rank == 0:
        q.put((allbits.tolist(), t))
    dist.destroy_process_group()


@pytest.mark.parametrize("n_total", [1000, 1001])
def test_gather_two_ranks(n_total):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_total, q)) for r in range(world)]
    for p in procs:
        p.start()
    allbits, t = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    idx = np.arange(n_total)
    want = ((idx * 2654435761) % 97 == 0).astype(np.uint16) * 0x0004
    assert allbits == want.tolist()
    assert t == 2.0


def test_shard_ranges_cover_contiguously():
    import sys
    from praos_hip import dist as pd
    for world in (1, 2, 3, 8):
        for n in (0, 7, 432000, 432001):
            rs = [pd.shard_range(r, world, n) for r in range(world)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(rs[i][1] == rs[i + 1][0] for i in range(world - 1))
            sizes = [b - a for a, b in rs]
            assert max(sizes) - min(sizes) <= 1


def test_bitmap_pack():
    from praos_hip import dist as pd
    b = np.array([0, 4, 0, 0, 0x1000, 0, 0, 0, 0], np.uint16)
    bm = pd.pack_bitmap(b)
    assert list(np.unpackbits(bm, bitorder="little")[:9]) == [1, 0, 1, 1, 0, 1, 1, 1, 1]


def _oracle_headers(n):
    """n oracle-signed Praos headers (test_cpu_twin._oracle_chain: corruptions of every
    kind, an unknown issuer, KESBeforeStart) as the SoA the C ABI takes."""
    from fractions import Fraction
    import oracle
    from helpers import arr, b2b, rng
    from praos_hip import abi, fixed
    from test_cpu_twin import _oracle_chain
    oracle.lib()
    eta0 = b2b(b"gather-epoch")
    c_raw = fixed.active_slot_log(Fraction(9, 10))
    H, pool_list = _oracle_chain(oracle, rng(77), n, 4, eta0, c_raw)
    bodies = H["body"]
    S = {"slot": np.array(H["slot"], np.uint64), "cold_vk": arr(H["cold_vk"], 32), "vrf_vk": arr(H["vrf_vk"], 32),
         "vrf_out": arr(H["vrf_out"], 64), "vrf_proof": arr(H["vrf_proof"], 80), "hot_vk": arr(H["hot_vk"], 32),
         "ocert_n": np.array(H["ocert_n"], np.uint64), "ocert_c0": np.array(H["ocert_c0"], np.uint64),
         "ocert_sig": arr(H["ocert_sig"], 64), "kes_sig": arr(H["kes_sig"], 448),
         "body_off": np.cumsum([0] + [len(b) for b in bodies[:-1]]).astype(np.uint64),
         "body_len": np.array([len(b) for b in bodies], np.uint32),
         "body_bytes": np.frombuffer(b"".join(bodies) + bytes(8), np.uint8).copy()}
    return S, eta0, pool_list, abi.params(c_raw=c_raw)


def _slice(S, lo, hi):
    T = {k: np.ascontiguousarray(v[lo:hi]) for k, v in S.items() if k not in ("body_off", "body_len", "body_bytes")}
    off, ln = S["body_off"][lo:hi], S["body_len"][lo:hi]
    T["body_len"] = np.ascontiguousarray(ln)
    T["body_off"] = np.concatenate([[0], np.cumsum(ln.astype(np.uint64))[:-1]]).astype(np.uint64)
    T["body_bytes"] = np.concatenate([S["body_bytes"][int(o):int(o) + int(m)] for o, m in zip(off, ln)] +
                                     [np.zeros(8, np.uint8)])
    return T


def _lib_worker(rank, world, port, n_total, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "ouroboros-consensus_amd"), os.path.join(root, "oracle"),
                    os.path.join(root, "tests")]
    import torch.distributed as dist
    from praos_hip import cpu as C
    from praos_hip import dist as pd
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    S, eta0, pool_list, p = _oracle_headers(n_total)      # every rank holds the same stream
    lo, hi = pd.shard_range(rank, world, n_total)
    twin = C.CpuContext(threads=2)
    twin.set_epoch(eta0, pool_list, p)
    o = twin.verify_headers(_slice(S, lo, hi))
    twin.close()
    got = {"bits": pd.gather_verdicts(o["bits"]), "pool_idx": pd.gather_rows(o["pool_idx"]),
           "beta": pd.gather_rows(o["beta"]), "leader": pd.gather_rows(o["leader"]),
           "nonce": pd.gather_rows(o["nonce"])}
    if rank == 0:
        q.put({k: v.tolist() for k, v in got.items()})
    dist.destroy_process_group()


@pytest.mark.parametrize("n_total", [27])
def test_gather_library_outputs(n_total):
    """Each rank verifies its contiguous shard with the library; the gathered bits,
    pool indices, beta, leader and nonce values equal one process over the whole batch."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_lib_worker, args=(r, world, port, n_total, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    from praos_hip import cpu as C
    S, eta0, pool_list, p = _oracle_headers(n_total)
    twin = C.CpuContext(threads=2)
    twin.set_epoch(eta0, pool_list, p)
    want = twin.verify_headers(S)
    twin.close()
    for k in ("bits", "pool_idx", "beta", "leader", "nonce"):
        assert got[k] == want[k].tolist(), k
    assert len(set(got["bits"])) >= 5          # valid and several failure kinds, across both shards
