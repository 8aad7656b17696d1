"""Multi-GPU sharding of a header stream (one process per GPU).

Headers of an epoch are independent given (eta0, PoolDistr, params), so the
batch shards by contiguous slot range with no collective on the data path
(SURVEY.md sec. 8e).  The only exchange is the verdict gather at the end:
each rank packs its per-header verdicts into a bitmap (1 bit: header passes
every crypto check) plus the u16 check bits, and `gather_verdicts` concatenates
them in slot order on every rank (torch.distributed all_gather: RCCL over xGMI
with the "nccl" backend, or gloo on CPU).  Cross-shard fix-ups (OCert counter
continuity, nonce fold, prev-hash links) stay host-side and sequential
(praos_apply_batch).
"""
import numpy as np


def shard_range(rank: int, world: int, n_total: int):
    """Contiguous [lo, hi) header indices of `rank` (ragged tail goes to the last ranks)."""
    base, extra = divmod(n_total, world)
    lo = rank * base + min(rank, extra)
    hi = lo + base + (1 if rank < extra else 0)
    return lo, hi


def pack_bitmap(bits_u16: np.ndarray) -> np.ndarray:
    """1 bit per header: 1 = no crypto failure bit set (leader bit ignored if mask says so)."""
    ok = (bits_u16 == 0).astype(np.uint8)
    return np.packbits(ok, bitorder="little")


def gather_verdicts(bits_u16: np.ndarray, device=None):
    """All-gather of per-rank check bits in rank (= slot) order.  Returns the
    concatenated u16 array on every rank.  Ragged shards are supported."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size()
    n = torch.tensor([len(bits_u16)], dtype=torch.int64, device=device)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n)
    m = int(max(int(s.item()) for s in sizes))
    buf = torch.zeros(m, dtype=torch.int32, device=device)
    buf[:len(bits_u16)] = torch.from_numpy(bits_u16.astype(np.int32)).to(buf.device)
    parts = [torch.zeros_like(buf) for _ in range(world)]
    dist.all_gather(parts, buf)
    return np.concatenate([p[:int(s.item())].cpu().numpy().astype(np.uint16) for p, s in zip(parts, sizes)])


def gather_rows(a: np.ndarray, device=None) -> np.ndarray:
    """All-gather of per-rank row arrays (e.g. beta n x 64 bytes, pool_idx i32[n]) in rank
    (= slot) order; any fixed-width dtype, ragged row counts.  Returns the concatenation
    on every rank."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size()
    a = np.ascontiguousarray(a)
    width = int(a.dtype.itemsize * (int(np.prod(a.shape[1:])) if a.ndim > 1 else 1))
    raw = a.view(np.uint8).reshape(len(a), width)
    n = torch.tensor([len(a)], dtype=torch.int64, device=device)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n)
    m = int(max(int(s.item()) for s in sizes))
    buf = torch.zeros((m, width), dtype=torch.uint8, device=device)
    buf[:len(a)] = torch.from_numpy(raw).to(buf.device)
    parts = [torch.zeros_like(buf) for _ in range(world)]
    dist.all_gather(parts, buf)
    out = np.concatenate([p[:int(s.item())].cpu().numpy() for p, s in zip(parts, sizes)])
    return out.view(a.dtype).reshape((-1,) + a.shape[1:])


def max_over_ranks(seconds: float, device=None) -> float:
    import torch
    import torch.distributed as dist
    t = torch.tensor([seconds], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
