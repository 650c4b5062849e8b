"""Multi-GPU plumbing for the batch path: one process per GPU (torch.distributed, RCCL on the
GPU box, gloo on CPU).  Stereo pairs are independent, so the hot path shards them with no
data-path collective; only the timing barrier and the max/sum reductions of bench.py cross
ranks ("replicas only")."""
from __future__ import annotations


def shard_range(total: int, rank: int, world: int):
    """Contiguous [lo, hi) slice of `total` units owned by `rank` (balanced to within 1)."""
    base, rem = divmod(total, world)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


def pair_seed_base(rank: int) -> int:
    """Synthetic frame index offset of a rank's shard (ranks never share frames)."""
    return rank * 100000


def reduce_scalar(dist, x: float, op: str = "max") -> float:
    if dist is None:
        return x
    import torch
    dev = "cuda" if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX if op == "max" else dist.ReduceOp.SUM)
    return float(t.item())
