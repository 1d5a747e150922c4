"""Multi-GPU data parallelism for the GLL path.

Independent minibatch graphs shard one per rank (one process per GPU, no cross-GPU graph
edges); the only collective is an all_gather of the per-rank predictions U (m x C) over
RCCL/xGMI ("nccl" backend on ROCm) -- or gloo on CPU for tests.  The gather is issued
asynchronously so it overlaps the backward of the same step.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def shard_rank_seed(base_seed: int, rank: int) -> int:
    """Seed of the minibatch graph a rank owns (config 4 of BASELINE.json: seed = rank)."""
    return int(base_seed) + int(rank)


def gather_predictions(U: torch.Tensor, group=None, async_op: bool = True):
    """All-gather every rank's predictions into one (world * m) x C tensor.

    Returns (out, work): `out` is filled once `work.wait()` returns (work is None when
    async_op is False or the world has one rank)."""
    if not dist.is_available() or not dist.is_initialized():
        return U, None
    world = dist.get_world_size(group)
    if world == 1:
        return U, None
    U = U.contiguous()
    out = torch.empty((world * U.shape[0],) + tuple(U.shape[1:]), dtype=U.dtype, device=U.device)
    work = dist.all_gather_into_tensor(out, U, group=group, async_op=async_op)
    return out, work
