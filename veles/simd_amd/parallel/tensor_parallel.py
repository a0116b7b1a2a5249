"""1-D row-split batched SGEMM over ranks (benchmark
config 5: batched SGEMM 8192^2 x 64 row-split across 8 GPUs with an RCCL
all-gather over xGMI).

C_i = A_i @ B_i for a batch of matrices.  Every rank owns a contiguous block
of rows of every A_i and the whole B_i (replicated, or streamed from `src` by
per-matrix broadcasts); it computes its rows of C_i with the MFMA SGEMM and
the full C_i is assembled by one all-gather per matrix.  Collectives are
issued asynchronously (RCCL runs them on its own stream, ordered after the
producing kernel), so the all-gather of C_i overlaps the SGEMM of C_{i+1} and
the broadcast of B_{i+1} is in flight while C_i is computed.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from .. import _lib, ops
from ..ops._util import on_device, ptr, stream_of
from . import comm


def _sgemm_into(a: torch.Tensor, b: torch.Tensor, c: torch.Tensor) -> None:
    """c = a @ b (2-D, contiguous, c possibly a row block of a larger
    tensor) straight into c: no temporary, no copy."""
    if not a.is_cuda:  # CPU / gloo test path: fp64-accumulated reference
        c.copy_(ops.sgemm(a, b))
        return
    m, k = a.shape
    n = b.shape[1]
    # vs_sgemm reads and writes raw pointers: everything it assumes is
    # checked here (a wrong dtype or shape would read or write past the tensors)
    for name, t in (("a", a), ("b", b), ("c", c)):
        if t.dtype != torch.float32 or t.device != a.device:
            raise TypeError(f"rowsplit_bmm: {name} must be float32 on {a.device}, "
                            f"got {t.dtype} on {t.device}")
    if b.dim() != 2 or b.shape[0] != k:
        raise ValueError(f"rowsplit_bmm: b has shape {tuple(b.shape)}, expected ({k}, n)")
    if tuple(c.shape) != (m, n) or not c.is_contiguous():
        raise ValueError(f"rowsplit_bmm: out block must be contiguous ({m}, {n}), "
                         f"got {tuple(c.shape)} contiguous={c.is_contiguous()}")
    if not (a.is_contiguous() and b.is_contiguous()):
        raise ValueError("rowsplit_bmm: operands must be contiguous")
    with on_device(a):
        _lib.call("vs_sgemm", 0, 0, m, n, k, 1.0, ptr(a), k, ptr(b), n, 0.0, ptr(c), n,
                  stream_of(a))


def rowsplit_bmm(a_local: torch.Tensor, b: torch.Tensor | None, *,
                 n: int | None = None, gather: bool = True,
                 broadcast_src: int | None = None,
                 out: torch.Tensor | None = None) -> torch.Tensor:
    """Row-split batched matmul.

    a_local: [batch, m_local, k] -- this rank's rows (equal on every rank).
    b:       [batch, k, n] replicated on every rank, or (broadcast_src set)
             only meaningful on rank broadcast_src; other ranks may pass None
             together with `n`.
    gather:  return the full C [batch, m_local * world, n] on every rank
             (else this rank's rows [batch, m_local, n]).
    """
    world = comm.world_size()
    batch, m_loc, k = a_local.shape
    if b is not None:
        n = b.shape[-1]
    if n is None:
        raise ValueError("rowsplit_bmm: pass b or n")
    if broadcast_src is not None and world > 1 and comm.rank() != broadcast_src:
        b = torch.empty((batch, k, n), dtype=a_local.dtype, device=a_local.device)
    if not gather or world == 1:
        if broadcast_src is not None and world > 1:
            dist.broadcast(b, broadcast_src)
        if out is None:
            out = torch.empty((batch, m_loc, n), dtype=a_local.dtype, device=a_local.device)
        for i in range(batch):
            _sgemm_into(a_local[i].contiguous(), b[i].contiguous(), out[i])
        return out
    if out is None:
        out = torch.empty((batch, m_loc * world, n), dtype=a_local.dtype,
                          device=a_local.device)
    me = comm.rank()
    pending = []
    bcast = {}

    def issue_bcast(i):
        if broadcast_src is not None and i < batch:
            bcast[i] = dist.broadcast(b[i], broadcast_src, async_op=True)

    issue_bcast(0)
    for i in range(batch):
        issue_bcast(i + 1)  # prefetch the next B while computing this one
        if i in bcast:
            bcast.pop(i).wait()
        # this rank's rows written in place into its slot of out[i], then the
        # in-place all-gather fills the other ranks' slots
        c_loc = out[i, me * m_loc:(me + 1) * m_loc]
        _sgemm_into(a_local[i].contiguous(), b[i].contiguous(), c_loc)
        pending.append((dist.all_gather_into_tensor(out[i], c_loc, async_op=True), c_loc))
        if len(pending) > 2:  # bound the number of in-flight result shards
            w, _ = pending.pop(0)
            w.wait()
    for w, _ in pending:
        w.wait()
    return out
