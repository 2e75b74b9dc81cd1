"""Env sharding across GPUs: envs are independent, so rank r owns the
contiguous global env ids [r * n_per_rank, (r + 1) * n_per_rank); every env's RNG stream
is seeded from its global id (gm_create env_offset), so results do not depend on the
number of GPUs.  The only collective is the all-gather of per-env episode returns."""
from __future__ import annotations


def shard_range(rank: int, world: int, n_per_rank: int) -> tuple[int, int]:
    """Global env ids owned by `rank` (weak scaling: fixed envs per rank)."""
    if not (0 <= rank < world):
        raise ValueError(f"rank {rank} outside world of {world}")
    return rank * n_per_rank, (rank + 1) * n_per_rank


def gather_returns(returns, world: int):
    """All-gather a rank's per-env returns tensor [n_per_rank] into [world * n_per_rank]
    (global env order).  NaN marks envs whose episode did not end this step.  Uses the
    default process group (RCCL on GPUs, gloo in the CPU tests)."""
    import torch
    import torch.distributed as dist
    if world == 1:
        return returns
    out = torch.empty((world * returns.numel(),), dtype=returns.dtype, device=returns.device)
    dist.all_gather_into_tensor(out, returns.contiguous())
    return out


def max_over_ranks(seconds: float, device=None) -> float:
    """Wall time of the slowest rank (the bench contract's MAX over ranks)."""
    import torch
    import torch.distributed as dist
    if not dist.is_available() or not dist.is_initialized():
        return seconds
    t = torch.tensor([seconds], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
