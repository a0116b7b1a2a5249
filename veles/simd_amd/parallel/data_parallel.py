"""Data parallelism over the batch dimension.

Batched primitives (conv1d over many signals, SWT over 65536 signals, batched
SGEMM) are embarrassingly parallel over the batch: each rank processes its
contiguous shard with the native kernels of its own GPU and, if the caller
needs the whole result on every rank, the shards are concatenated with one
all-gather.  Inputs can be given globally (every rank holds the full batch;
each takes its slice) or already sharded.
"""
from __future__ import annotations

from typing import Callable

import torch

from . import comm


def local_shard(x: torch.Tensor, dim: int = 0) -> torch.Tensor:
    """This rank's contiguous shard of a globally replicated tensor."""
    w, r = comm.world_size(), comm.rank()
    a, b = comm.shard_range(x.shape[dim], w, r)
    return x.narrow(dim, a, b - a)


def dp_apply(fn: Callable[..., torch.Tensor], x: torch.Tensor, *args,
             sharded_input: bool = False, gather: bool = True, **kwargs):
    """Run fn(shard, *args, **kwargs) on this rank's batch shard.

    sharded_input: x is already this rank's shard (no slicing).
    gather: all-gather the per-rank results (dim 0) so every rank gets the
    full batch; otherwise return the local result.
    """
    shard = x if sharded_input else local_shard(x)
    y = fn(shard, *args, **kwargs)
    if not gather or comm.world_size() == 1:
        return y
    if sharded_input:
        return comm.all_gather_rows(y)
    w = comm.world_size()
    counts = [b - a for a, b in (comm.shard_range(x.shape[0], w, r) for r in range(w))]
    return comm.all_gather_rows(y, counts)
