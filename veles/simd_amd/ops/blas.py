"""BLAS subset as torch custom ops backed by the MFMA fp32 SGEMM.

Reference: src/matrix.c (matrix_add/sub/multiply/multiply_transposed).
"""
from __future__ import annotations

import torch

from .. import _lib
from ._util import on_device, ptr, require_gpu_tensor, stream_of


@torch.library.custom_op("veles::sgemm", mutates_args=())
def sgemm(a: torch.Tensor, b: torch.Tensor, trans_a: bool = False,
          trans_b: bool = False, alpha: float = 1.0) -> torch.Tensor:
    """alpha * op(a) @ op(b) in exact fp32 (2-D, or 3-D batched)."""
    if a.dtype != torch.float32 or b.dtype != torch.float32:
        raise TypeError("veles::sgemm expects float32 operands")
    batched = a.dim() == 3
    if not a.is_cuda:
        aa = a.transpose(-1, -2) if trans_a else a
        bb = b.transpose(-1, -2) if trans_b else b
        return alpha * torch.matmul(aa, bb)
    require_gpu_tensor(a, "veles::sgemm")
    a = a.contiguous()
    b = b.contiguous()
    m = a.shape[-1] if trans_a else a.shape[-2]
    k = a.shape[-2] if trans_a else a.shape[-1]
    kb = b.shape[-1] if trans_b else b.shape[-2]
    n = b.shape[-2] if trans_b else b.shape[-1]
    if k != kb:
        raise ValueError(f"veles::sgemm: inner dimensions differ ({k} vs {kb})")
    batch = a.shape[0] if batched else 1
    out_shape = (batch, m, n) if batched else (m, n)
    c = torch.empty(out_shape, dtype=torch.float32, device=a.device)
    lda, ldb = a.shape[-1], b.shape[-1]
    with on_device(a):
        _lib.call("vs_sgemm_strided_batched", int(trans_a), int(trans_b), m, n,
                  k, float(alpha), ptr(a), lda, m * k if batched else 0, ptr(b),
                  ldb, (k * n if b.dim() == 3 else 0), 0.0, ptr(c), n,
                  m * n if batched else 0, batch, stream_of(a))
    return c


@sgemm.register_fake
def _(a, b, trans_a=False, trans_b=False, alpha=1.0):
    m = a.shape[-1] if trans_a else a.shape[-2]
    n = b.shape[-2] if trans_b else b.shape[-1]
    shape = (a.shape[0], m, n) if a.dim() == 3 else (m, n)
    return a.new_empty(shape)


def _sgemm_setup(ctx, inputs, output):
    a, b, trans_a, trans_b, alpha = inputs
    ctx.save_for_backward(a, b)
    ctx.cfg = (trans_a, trans_b, alpha)


def _sgemm_backward(ctx, grad):
    a, b = ctx.saved_tensors
    trans_a, trans_b, alpha = ctx.cfg
    ga = gb = None
    # C = alpha op(A) op(B):  dop(A) = alpha dC op(B)^T, dop(B) = alpha op(A)^T dC
    if ctx.needs_input_grad[0]:
        if trans_a:  # dA = alpha op(B) dC^T
            ga = sgemm(b, grad, trans_b, True, alpha)
        else:
            ga = sgemm(grad, b, False, not trans_b, alpha)
    if ctx.needs_input_grad[1]:
        if trans_b:  # dB = alpha dC^T op(A)
            gb = sgemm(grad, a, True, trans_a, alpha)
        else:
            gb = sgemm(a, grad, not trans_a, False, alpha)
    return ga, gb, None, None, None


sgemm.register_autograd(_sgemm_backward, setup_context=_sgemm_setup)


def _gemm_shapes(a, b, trans_a, trans_b, name):
    m = a.shape[-1] if trans_a else a.shape[-2]
    k = a.shape[-2] if trans_a else a.shape[-1]
    kb = b.shape[-1] if trans_b else b.shape[-2]
    n = b.shape[-2] if trans_b else b.shape[-1]
    if k != kb:
        raise ValueError(f"{name}: inner dimensions differ ({k} vs {kb})")
    return m, n, k


@torch.library.custom_op("veles::sgemm_bf16x3", mutates_args=())
def sgemm_bf16x3(a: torch.Tensor, b: torch.Tensor, trans_a: bool = False,
                 trans_b: bool = False, alpha: float = 1.0) -> torch.Tensor:
    """Fast fp32 GEMM: fp32 operands split into bf16 hi + lo and multiplied
    as hi*hi + hi*lo + lo*hi on the bf16 matrix cores (~1e-5 relative)."""
    if a.dtype != torch.float32 or b.dtype != torch.float32:
        raise TypeError("veles::sgemm_bf16x3 expects float32 operands")
    if not a.is_cuda:
        aa = a.transpose(-1, -2) if trans_a else a
        bb = b.transpose(-1, -2) if trans_b else b
        return alpha * torch.matmul(aa, bb)
    require_gpu_tensor(a, "veles::sgemm_bf16x3")
    a, b = a.contiguous(), b.contiguous()
    m, n, k = _gemm_shapes(a, b, trans_a, trans_b, "veles::sgemm_bf16x3")
    batched = a.dim() == 3
    batch = a.shape[0] if batched else 1
    c = torch.empty((batch, m, n) if batched else (m, n), dtype=torch.float32,
                    device=a.device)
    with on_device(a):
        _lib.call("vs_sgemm_bf16x3_strided_batched", int(trans_a), int(trans_b), m, n, k,
                  float(alpha), ptr(a), a.shape[-1], m * k if batched else 0, ptr(b),
                  b.shape[-1], k * n if b.dim() == 3 else 0, 0.0, ptr(c), n,
                  m * n if batched else 0, batch, stream_of(a))
    return c


@sgemm_bf16x3.register_fake
def _(a, b, trans_a=False, trans_b=False, alpha=1.0):
    m = a.shape[-1] if trans_a else a.shape[-2]
    n = b.shape[-2] if trans_b else b.shape[-1]
    return a.new_empty((a.shape[0], m, n) if a.dim() == 3 else (m, n))


@torch.library.custom_op("veles::gemm_bf16", mutates_args=())
def gemm_bf16(a: torch.Tensor, b: torch.Tensor, trans_a: bool = False,
              trans_b: bool = False, alpha: float = 1.0) -> torch.Tensor:
    """alpha * op(a) @ op(b) for bf16 operands, fp32 accumulation and output."""
    if a.dtype != torch.bfloat16 or b.dtype != torch.bfloat16:
        raise TypeError("veles::gemm_bf16 expects bfloat16 operands")
    if not a.is_cuda:
        aa = a.transpose(-1, -2) if trans_a else a
        bb = b.transpose(-1, -2) if trans_b else b
        return alpha * torch.matmul(aa.float(), bb.float())
    require_gpu_tensor(a, "veles::gemm_bf16")
    a, b = a.contiguous(), b.contiguous()
    m, n, k = _gemm_shapes(a, b, trans_a, trans_b, "veles::gemm_bf16")
    batched = a.dim() == 3
    batch = a.shape[0] if batched else 1
    c = torch.empty((batch, m, n) if batched else (m, n), dtype=torch.float32,
                    device=a.device)
    with on_device(a):
        _lib.call("vs_gemm_bf16_strided_batched", int(trans_a), int(trans_b), m, n, k,
                  float(alpha), ptr(a), a.shape[-1], m * k if batched else 0, ptr(b),
                  b.shape[-1], k * n if b.dim() == 3 else 0, 0.0, ptr(c), n,
                  m * n if batched else 0, batch, stream_of(a))
    return c


@gemm_bf16.register_fake
def _(a, b, trans_a=False, trans_b=False, alpha=1.0):
    m = a.shape[-1] if trans_a else a.shape[-2]
    n = b.shape[-2] if trans_b else b.shape[-1]
    return a.new_empty((a.shape[0], m, n) if a.dim() == 3 else (m, n), dtype=torch.float32)


def matmul(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """a @ b (reference matrix_multiply)."""
    return sgemm(a, b, False, False, 1.0)


def matmul_transposed(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """a @ b.T (reference matrix_multiply_transposed)."""
    return sgemm(a, b, False, True, 1.0)
