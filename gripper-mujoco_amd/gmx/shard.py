"""Env sharding across GPUs: envs are independent, so rank r owns the
contiguous global env ids [r * n_per_rank, (r + 1) * n_per_rank); every env's RNG stream
is seeded from its global id (gm_create env_offset), so results do not depend on the
number of GPUs.  The only collective is the all-gather of the per-env episode-end record
(return, length, success: gm_episode_end, include/gripper_mi355x.h), 12 bytes per env."""
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


def gather_episodes(episodes, world: int):
    """All-gather a rank's episode-end records into global env order.  `episodes` is the
    [n_per_rank, 3] int32 view of gm_episode_end (float32 bits of the return, the length
    in env-steps, the success byte + padding) that gm_autoreset_episodes writes on the
    device; the result is [world * n_per_rank, 3].  One collective per env-step (RCCL over
    xGMI on GPUs, gloo in the CPU tests), ~48 KB per 4096-env rank."""
    import torch
    import torch.distributed as dist
    if world == 1:
        return episodes
    out = torch.empty((world * episodes.shape[0], 3), dtype=episodes.dtype, device=episodes.device)
    dist.all_gather_into_tensor(out, episodes.contiguous())
    return out


def new_episode_records(n: int, device=None):
    """A [n, 3] int32 buffer for gm_autoreset_episodes (= n gm_episode_end records)."""
    import torch
    return torch.zeros((n, 3), dtype=torch.int32, device=device)


def unpack_episodes(rec):
    """(returns float32 [n] with NaN where no episode ended, lengths int32 [n] (0 there),
    success bool [n]) from gathered episode-end records."""
    import torch
    r = rec.contiguous()
    ret = r[:, 0].view(torch.float32)
    return ret, r[:, 1], (r[:, 2] & 0xFF) != 0


def pack_episodes(ret, length, success):
    """The inverse of unpack_episodes (host-side producers such as the oracle rollout)."""
    import torch
    n = ret.shape[0]
    out = torch.zeros((n, 3), dtype=torch.int32)
    out[:, 0] = ret.to(torch.float32).contiguous().view(torch.int32)
    out[:, 1] = length.to(torch.int32)
    out[:, 2] = success.to(torch.int32)
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
