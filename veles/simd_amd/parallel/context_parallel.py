"""Sequence ("context") parallelism for very long 1-D signals .

A signal too long for one GPU (or just long enough that 8 GPUs finish it 8x
faster) is split into contiguous chunks, one per rank.  The only coupling is
a halo:
  * linear convolution: output n needs x[n - h + 1 .. n], so every rank
    receives the last h-1 samples of its left neighbour (one point-to-point
    message over xGMI; rank 0 uses zeros) and the last rank also emits the
    h-1 tail outputs.  This generalises the overlap-save block decomposition
    of the reference (src/convolve.c:181-228) across GPUs.
  * stationary wavelet level l: output i needs the level input at
    i .. i + (order-1) 2^(l-1), i.e. a right halo from the next rank; the
    last rank wraps to rank 0 for periodic extension and otherwise applies
    the reference's extension rule (src/wavelet.c:248-269) to its own tail.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from .. import ops
from . import comm


def _exchange(send_to: int | None, send: torch.Tensor | None,
              recv_from: int | None, shape, like: torch.Tensor) -> torch.Tensor | None:
    reqs = []
    buf = None
    if recv_from is not None:
        buf = like.new_empty(shape)
        reqs.append(dist.P2POp(dist.irecv, buf, recv_from))
    if send_to is not None:
        reqs.append(dist.P2POp(dist.isend, send.contiguous(), send_to))
    if reqs:
        for r in dist.batch_isend_irecv(reqs):
            r.wait()
    return buf


def cp_conv1d(x_local: torch.Tensor, h: torch.Tensor, correlate: bool = False,
              algorithm="auto") -> torch.Tensor:
    """This rank's part of the full linear convolution of a signal split
    over ranks along the last dim (x_local: [..., len_r], every chunk at least
    h - 1 long).  Rank r returns outputs [start_r, start_r + len_r); the last
    rank additionally returns the h - 1 tail outputs, so concatenating the
    ranks' results gives the full x + h - 1 outputs."""
    world, r = comm.world_size(), comm.rank()
    hk = h.flip(-1) if correlate else h
    H = hk.shape[-1]
    L = x_local.shape[-1]
    if world == 1 or H == 1:
        return ops.conv1d(x_local, hk, algorithm)
    if L < H - 1:
        raise ValueError(f"cp_conv1d: chunk ({L}) shorter than the halo ({H - 1})")
    lead = x_local.shape[:-1]
    halo = _exchange(r + 1 if r + 1 < world else None, x_local[..., L - (H - 1):],
                     r - 1 if r > 0 else None, (*lead, H - 1), x_local)
    if halo is None:
        halo = x_local.new_zeros((*lead, H - 1))
    y = ops.conv1d(torch.cat([halo, x_local], -1), hk, algorithm)
    stop = y.shape[-1] if r == world - 1 else H - 1 + L
    return y[..., H - 1: stop]


def cp_swt(x_local: torch.Tensor, family="daubechies", order: int = 8,
           levels: int = 1, ext="periodic"):
    """Multi-level stationary DWT of a signal split over ranks (last dim).
    Returns this rank's (hi [..., levels, len_r], lo [..., len_r]); each
    level exchanges one right halo of (order-1) 2^(l-1) samples."""
    world, r = comm.world_size(), comm.rank()
    fam = ops.signal._fam(family)
    e = ops.signal._ext(ext)
    if world == 1:
        return ops.swt(x_local, family, order, levels, ext)
    L = x_local.shape[-1]
    lead = x_local.shape[:-1]
    cur = x_local
    his = []
    for lvl in range(1, levels + 1):
        halo_n = (order - 1) << (lvl - 1)
        if L < halo_n:
            raise ValueError(f"cp_swt: chunk ({L}) shorter than the level-{lvl} halo")
        last = r == world - 1
        wrap = e == ops.signal.PERIODIC
        send_to = r - 1 if r > 0 else (world - 1 if wrap else None)
        recv_from = r + 1 if not last else (0 if wrap else None)
        halo = _exchange(send_to, cur[..., :halo_n], recv_from, (*lead, halo_n), cur)
        if halo is None:  # last rank, non-periodic: extension of the global end
            t = torch.arange(halo_n, device=cur.device)
            if e == ops.signal.MIRROR:
                halo = cur[..., L - 1 - t]
            elif e == ops.signal.CONSTANT:
                halo = cur[..., -1:].expand(*lead, halo_n)
            else:
                halo = cur.new_zeros((*lead, halo_n))
        xin = torch.cat([cur, halo], -1)
        hi, lo = ops.swt_level(xin, fam, order, lvl, ops.signal.ZERO)
        his.append(hi[..., :L])
        cur = lo[..., :L].contiguous()
    return torch.stack(his, -2), cur
