"""Process-group plumbing for the one-process-per-GPU execution model.

Every multi-GPU feature of veles.simd_amd runs as N processes (one per GPU,
launched by ``torch.distributed.run``) talking over RCCL -- the "nccl"
backend of PyTorch-ROCm -- which routes collectives over the xGMI links of an
MI355X node.  CPU tensors use "gloo" so the same code paths are testable
without GPUs.  The reference library has no distributed layer at all;
this module is new.
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass

import torch
import torch.distributed as dist


@dataclass
class DistContext:
    rank: int
    world: int
    local_rank: int
    device: torch.device
    backend: str

    @property
    def is_main(self) -> bool:
        return self.rank == 0


def init(backend: str | None = None, timeout_s: float = 600.0) -> DistContext:
    """Initialise (or reuse) the default process group from the standard
    torchrun environment (RANK, WORLD_SIZE, LOCAL_RANK, MASTER_ADDR/PORT).

    A single process without that environment gets a world of 1 and no
    process group.  GPU runs bind rank -> cuda:LOCAL_RANK and use RCCL.
    """
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    use_gpu = torch.cuda.is_available() and (backend in (None, "nccl"))
    if use_gpu:
        torch.cuda.set_device(local)
        device = torch.device("cuda", local)
    else:
        device = torch.device("cpu")
    backend = backend or ("nccl" if use_gpu else "gloo")
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        kwargs = {"timeout": datetime.timedelta(seconds=timeout_s)}
        if backend == "nccl":
            kwargs["device_id"] = device
        dist.init_process_group(backend, rank=rank, world_size=world, **kwargs)
    return DistContext(rank, world, local, device, backend)


def world_size() -> int:
    return dist.get_world_size() if dist.is_initialized() else 1


def rank() -> int:
    return dist.get_rank() if dist.is_initialized() else 0


def barrier() -> None:
    if dist.is_initialized():
        dist.barrier()


def shard_range(n: int, world: int, r: int) -> tuple[int, int]:
    """[start, stop) of shard r when n items are split as evenly as possible
    (the first n % world shards get one extra item)."""
    base, extra = divmod(n, world)
    start = r * base + min(r, extra)
    return start, start + base + (1 if r < extra else 0)


def all_gather_rows(local: torch.Tensor, counts: list[int] | None = None,
                    group=None) -> torch.Tensor:
    """Concatenate every rank's `local` along dim 0.  Uneven shards are
    padded to the largest shard for one all_gather_into_tensor (a single
    RCCL collective) and trimmed afterwards."""
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    if world == 1:
        return local
    if counts is None:
        n = torch.tensor([local.shape[0]], device=local.device)
        ns = [torch.zeros_like(n) for _ in range(world)]
        dist.all_gather(ns, n, group=group)
        counts = [int(v.item()) for v in ns]
    mx = max(counts)
    buf = local
    if local.shape[0] < mx:
        pad = local.new_zeros((mx - local.shape[0], *local.shape[1:]))
        buf = torch.cat([local, pad])
    out = local.new_empty((world * mx, *local.shape[1:]))
    dist.all_gather_into_tensor(out, buf.contiguous(), group=group)
    if all(c == mx for c in counts):
        return out
    return torch.cat([out[i * mx: i * mx + c] for i, c in enumerate(counts)])
