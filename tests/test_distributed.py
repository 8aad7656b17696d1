"""CPU, world_size 2 (gloo): the multi-GPU data path shards by contiguous slot
range with no collective; only the verdict gather and the timing max-reduce
cross ranks (praos_hip.dist)."""
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
