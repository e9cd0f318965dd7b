"""Multi-GPU sharding for the point codec: one process per GPU (torch.distributed over RCCL).

The τ^i arrays shard trivially (every point is independent). Each rank decodes one contiguous,
equal-sized shard of every section; the only exchange is the final all-gather that assembles one
contiguous arkworks buffer on every rank (the north_star's "final RCCL all-gather over xGMI"),
plus an 8-byte all-reduce(min) of the first-bad key. No other communication.

These helpers are backend-agnostic so the same code is exercised with `gloo` on CPU tensors in
tests/test_dist.py and with `nccl` (= RCCL on ROCm) on HBM tensors in bench.py.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

NO_BAD = (1 << 64) - 1


def shard_bounds(n: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous shard [lo, hi) of n points for `rank`; equal sizes when world divides n."""
    per = (n + world - 1) // world
    lo = min(n, rank * per)
    return lo, min(n, lo + per)


def gather_shards(local: torch.Tensor, world: int, group=None) -> torch.Tensor:
    """All-gather equal-sized 1-D byte shards into one contiguous buffer (rank order)."""
    if world == 1:
        return local
    out = torch.empty(local.numel() * world, dtype=local.dtype, device=local.device)
    if dist.get_backend(group) == "gloo":  # gloo has no all_gather_into_tensor
        dist.all_gather(list(out.chunk(world)), local, group=group)  # chunks are views of out
        return out
    dist.all_gather_into_tensor(out, local, group=group)
    return out


def key_with_offset(key: int, offset: int) -> int:
    """Shift a shard-local bad key ((index << 8) | status) to global indices."""
    if key == NO_BAD:
        return NO_BAD
    return (((key >> 8) + offset) << 8) | (key & 0xFF)


def allreduce_min_key(key: int, device, group=None) -> int:
    """Global first bad point across ranks (keys are unsigned; carried as signed int64)."""
    signed = key - (1 << 64) if key >= (1 << 63) else key
    # NO_BAD (all ones) is -1 as int64: map it above every real key for the min
    t = torch.tensor([signed if key != NO_BAD else (1 << 63) - 1], dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    v = int(t.item())
    return NO_BAD if v == (1 << 63) - 1 else v & NO_BAD
