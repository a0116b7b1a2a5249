#!/usr/bin/env python3
"""Row-split batched SGEMM over the ranks of one node, one process per GPU:

    python -m torch.distributed.run --standalone --local-addr 127.0.0.1 \\
        --nproc-per-node 8 examples/rowsplit_torchrun.py

Every rank holds its rows of A and all of B; each C row block is all-gathered
over RCCL (xGMI) while the next matrix multiplies.  Without GPUs the same code
runs over gloo on CPU tensors (`--nproc-per-node 2` works on a laptop)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from veles.simd_amd import parallel  # noqa: E402
from veles.simd_amd.parallel import comm  # noqa: E402


def main():
    ctx = comm.init()                 # nccl (= RCCL) with GPUs, gloo without
    rank, world, dev = ctx.rank, ctx.world, ctx.device
    n, batch = (2048, 4) if dev.type == "cuda" else (128, 2)
    m_loc = n // world
    g = torch.Generator(device=dev).manual_seed(7)
    b = torch.rand(batch, n, n, device=dev, generator=g) - 0.5          # same seed: replicated
    a_full = torch.rand(batch, m_loc * world, n, device=dev, generator=g) - 0.5
    a_loc = a_full[:, rank * m_loc:(rank + 1) * m_loc].contiguous()
    c = parallel.rowsplit_bmm(a_loc, b)                                   # [batch, m, n] everywhere
    ref = a_full.double() @ b.double()
    err = (c.double() - ref).abs().max().item()
    if rank == 0:
        print(f"world {world}: C {tuple(c.shape)}, max |err| {err:.3e}")
    if torch.distributed.is_initialized():
        torch.distributed.destroy_process_group()
    return 0 if err < 2e-6 * n else 1


if __name__ == "__main__":
    sys.exit(main())
