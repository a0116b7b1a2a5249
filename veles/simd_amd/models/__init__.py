"""Composed DSP modules (``torch.nn.Module``) built on the native ops.

The reference is a primitive library used as the signal front-end of the
Veles ML framework; these modules package its primitives the way that
front-end consumed them -- FIR filtering, wavelet feature extraction,
matched filtering with peak picking, image normalisation -- with autograd
where the op is differentiable, and batch-parallel execution on MI355X.
"""
from __future__ import annotations

import torch
from torch import nn

from .. import ops


def _cached_plan(mod: nn.Module, taps: torch.Tensor, x: torch.Tensor, algorithm,
                 correlate: bool):
    """Inference with fixed taps on the GPU: a Conv1dPlan (filter spectra
    computed once) cached on `mod`, keyed by signal length, device and the
    taps' storage and version counter; None on the CPU path, for trainable
    taps (their version changes every step) and while torch.compile traces
    (plan creation reads data pointers, which fake tensors do not have).
    The plan is run through Conv1dPlan.apply, a custom op with a backward,
    so gradients still reach x."""
    if (not x.is_cuda or x.dtype != torch.float32 or torch.compiler.is_compiling()
            or taps.requires_grad and torch.is_grad_enabled()):
        return None
    key = (x.shape[-1], x.device, taps._version, taps.data_ptr(), correlate)
    if getattr(mod, "_plan_key", None) != key:
        mod._plan = ops.Conv1dPlan(taps.detach().to(x.device), x.shape[-1], algorithm,
                                   correlate=correlate)
        mod._plan_key = key
    return mod._plan


class FIRFilter(nn.Module):
    """y = x (*) h along the last dim.  mode: "full" (x+h-1 samples, the
    reference convolve.h contract), "same" (len x, centred) or "valid".
    learnable=True makes h a Parameter (gradients via the conv1d op)."""

    def __init__(self, taps: torch.Tensor, mode: str = "full",
                 learnable: bool = False, algorithm="auto"):
        super().__init__()
        taps = taps.detach().float().clone()
        if learnable:
            self.taps = nn.Parameter(taps)
        else:
            self.register_buffer("taps", taps)
        if mode not in ("full", "same", "valid"):
            raise ValueError(mode)
        self.mode = mode
        self.algorithm = algorithm

    def _planned(self, x: torch.Tensor):
        return _cached_plan(self, self.taps, x, self.algorithm, False)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        plan = self._planned(x)
        y = (plan.apply(x, self.taps) if plan is not None
             else ops.conv1d(x, self.taps, self.algorithm))
        H = self.taps.shape[-1]
        X = x.shape[-1]
        if self.mode == "same":
            s = (H - 1) // 2
            return y[..., s: s + X]
        if self.mode == "valid":
            return y[..., H - 1: X]
        return y


class MatchedFilter(nn.Module):
    """Cross-correlates signals with a template and reports the strict local
    maxima of the response above `threshold` (correlate.h + detect_peaks.h)."""

    def __init__(self, template: torch.Tensor, threshold: float = 0.0):
        super().__init__()
        self.register_buffer("template", template.detach().float().clone())
        self.threshold = threshold

    def forward(self, x: torch.Tensor):
        plan = _cached_plan(self, self.template, x, "auto", True)
        resp = (plan.apply(x, self.template) if plan is not None
                else ops.correlate(x, self.template))
        # all rows in one launch sequence; one host read (the per-row counts)
        pos, val, row_start = ops.detect_peaks_batched(resp.detach(), ops.signal.MAXIMUM)
        keep = val > self.threshold
        kept = torch.cat([keep.new_zeros(1, dtype=torch.int64), keep.cumsum(0)])
        bounds = kept[row_start].tolist()
        pos, val = pos[keep], val[keep]
        out = [(pos[a:b], val[a:b]) for a, b in zip(bounds[:-1], bounds[1:])]
        return resp, out


class WaveletDecomposition(nn.Module):
    """Fused multi-level decimated DWT (Mallat pyramid); returns the list
    [hi_1, ..., hi_L, lo_L] (wavelet.h, applied level by level)."""

    def __init__(self, family="daubechies", order: int = 8, levels: int = 3,
                 ext="periodic"):
        super().__init__()
        self.family, self.order, self.levels, self.ext = family, order, levels, ext

    def forward(self, x: torch.Tensor):
        flat = ops.wavedec(x, self.family, self.order, self.levels, self.ext)
        n = x.shape[-1]
        out, off = [], 0
        for _ in range(self.levels):
            n //= 2
            out.append(flat[..., off: off + n])
            off += n
        out.append(flat[..., off:])
        return out


class StationaryWavelet(nn.Module):
    """Fused multi-level stationary (undecimated) DWT: (hi [.., L, n], lo)."""

    def __init__(self, family="daubechies", order: int = 8, levels: int = 8,
                 ext="periodic"):
        super().__init__()
        self.family, self.order, self.levels, self.ext = family, order, levels, ext

    def forward(self, x: torch.Tensor):
        return ops.swt(x, self.family, self.order, self.levels, self.ext)


class WaveletEnergyFeatures(nn.Module):
    """Per-band log-energy features from a stationary wavelet transform --
    a typical signal front-end: [..., levels + 1] features per signal."""

    def __init__(self, family="daubechies", order: int = 8, levels: int = 6,
                 ext="periodic", eps: float = 1e-12):
        super().__init__()
        self.swt = StationaryWavelet(family, order, levels, ext)
        self.eps = eps

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        hi, lo = self.swt(x)
        e_hi = hi.square().mean(-1)
        e_lo = lo.square().mean(-1, keepdim=True)
        return torch.log(torch.cat([e_hi, e_lo], -1) + self.eps)


class ImageNormalizer(nn.Module):
    """uint8 planes -> float32 in [-1, 1] (normalize.h normalize2D)."""

    def forward(self, img: torch.Tensor) -> torch.Tensor:
        return ops.normalize2d(img)   # every plane of the stack in one launch


class Linear(nn.Module):
    """Fully connected layer on the exact-fp32 MFMA SGEMM (matrix.h)."""

    def __init__(self, in_features: int, out_features: int, bias: bool = True):
        super().__init__()
        self.weight = nn.Parameter(torch.empty(out_features, in_features))
        nn.init.kaiming_uniform_(self.weight, a=5 ** 0.5)
        self.bias = nn.Parameter(torch.zeros(out_features)) if bias else None

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        y = ops.matmul_transposed(x.reshape(-1, x.shape[-1]), self.weight)
        if self.bias is not None:
            y = y + self.bias
        return y.reshape(*x.shape[:-1], -1)


__all__ = ["FIRFilter", "MatchedFilter", "WaveletDecomposition", "StationaryWavelet",
           "WaveletEnergyFeatures", "ImageNormalizer", "Linear"]
