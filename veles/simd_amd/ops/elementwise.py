"""Elementwise / reduction ops (torch custom ops over the HIP kernels).

Reference: inc/simd/arithmetic.h (conversions, real/complex arithmetic,
sum_elements, add_to_all), inc/simd/mathfun.h (sin/cos/log/exp),
src/normalize.c (minmax, normalize2D), src/memory.c (memsetf, rmemcpyf).
CPU tensors run the same math with torch (the host reference semantics);
GPU tensors always run the native kernels.
"""
from __future__ import annotations

import torch

from .. import _lib
from ._util import on_device, ptr, require_gpu_tensor, stream_of

VS_F32, VS_F16, VS_I16, VS_I32, VS_U8 = 0, 1, 2, 3, 4
_DT = {torch.float32: VS_F32, torch.int16: VS_I16, torch.int32: VS_I32,
       torch.uint8: VS_U8, torch.float16: VS_F16}
_FN = {"sin": 0, "cos": 1, "log": 2, "exp": 3, "sqrt": 4}
_OP = {"add": 0, "sub": 1, "mul": 2}


def _gpu(x: torch.Tensor, name: str) -> bool:
    if x.is_cuda:
        require_gpu_tensor(x, name)
        return True
    return False


# ------------------------------------------------------------------ convert
@torch.library.custom_op("veles::convert", mutates_args=())
def convert(x: torch.Tensor, dtype: torch.dtype) -> torch.Tensor:
    """Numeric conversion with the library semantics: float -> int truncates
    toward zero and saturates; int32 -> int16 saturates; float16 inputs may
    be given as torch.float16 (raw IEEE binary16)."""
    if not _gpu(x, "veles::convert"):
        if dtype in (torch.int16, torch.int32) and x.dtype.is_floating_point:
            info = torch.iinfo(dtype)
            t = torch.nan_to_num(x.float(), nan=0.0).trunc()
            return t.clamp(info.min, info.max).to(dtype)
        if dtype == torch.int16 and x.dtype == torch.int32:
            return x.clamp(-32768, 32767).to(torch.int16)
        return x.to(dtype)
    x = x.contiguous()
    out = torch.empty(x.shape, dtype=dtype, device=x.device)
    with on_device(x):
        _lib.call("vs_convert", ptr(x), _DT[x.dtype], ptr(out), _DT[dtype],
                  x.numel(), stream_of(x))
    return out


@convert.register_fake
def _(x, dtype):
    return torch.empty(x.shape, dtype=dtype, device=x.device)


# ------------------------------------------------------------------- binary
@torch.library.custom_op("veles::binary", mutates_args=())
def binary(a: torch.Tensor, b: torch.Tensor, op: str) -> torch.Tensor:
    """a (+|-|*) b elementwise, float32, same shape (matrix_add/sub,
    real_multiply_array)."""
    if a.shape != b.shape:
        raise ValueError("veles::binary: shape mismatch")
    if not _gpu(a, "veles::binary"):
        return {"add": torch.add, "sub": torch.sub, "mul": torch.mul}[op](a, b)
    a, b = a.contiguous(), b.contiguous()
    out = torch.empty_like(a)
    with on_device(a):
        _lib.call("vs_binary", _OP[op], ptr(a), ptr(b), ptr(out), a.numel(),
                  stream_of(a))
    return out


@binary.register_fake
def _(a, b, op):
    return torch.empty_like(a)


def add(a, b):
    return binary(a, b, "add")


def sub(a, b):
    return binary(a, b, "sub")


def mul(a, b):
    return binary(a, b, "mul")


# ------------------------------------------------------------------ complex
@torch.library.custom_op("veles::complex_multiply", mutates_args=())
def complex_multiply(a: torch.Tensor, b: torch.Tensor,
                     conjugate_b: bool = False) -> torch.Tensor:
    """Interleaved complex product over float32 tensors (last dim even)."""
    if a.shape != b.shape or a.shape[-1] % 2:
        raise ValueError("veles::complex_multiply: bad shapes")
    if not _gpu(a, "veles::complex_multiply"):
        ca = torch.view_as_complex(a.contiguous().view(*a.shape[:-1], -1, 2))
        cb = torch.view_as_complex(b.contiguous().view(*b.shape[:-1], -1, 2))
        r = ca * (cb.conj() if conjugate_b else cb)
        return torch.view_as_real(r).reshape(a.shape)
    a, b = a.contiguous(), b.contiguous()
    out = torch.empty_like(a)
    with on_device(a):
        _lib.call("vs_complex_multiply", ptr(a), ptr(b), ptr(out),
                  a.numel() // 2, int(conjugate_b), stream_of(a))
    return out


@complex_multiply.register_fake
def _(a, b, conjugate_b=False):
    return torch.empty_like(a)


@torch.library.custom_op("veles::complex_conjugate", mutates_args=())
def complex_conjugate(a: torch.Tensor) -> torch.Tensor:
    if not _gpu(a, "veles::complex_conjugate"):
        r = a.clone()
        r.view(-1)[1::2] *= -1
        return r
    a = a.contiguous()
    out = a.clone()
    with on_device(a):
        _lib.call("vs_complex_conjugate", ptr(a), ptr(out), a.numel(),
                  stream_of(a))
    return out


@complex_conjugate.register_fake
def _(a):
    return torch.empty_like(a)


# ------------------------------------------------------------------- affine
@torch.library.custom_op("veles::affine", mutates_args=())
def affine(x: torch.Tensor, scale: float = 1.0, shift: float = 0.0) -> torch.Tensor:
    """x * scale + shift (real_multiply_scalar / add_to_all)."""
    if not _gpu(x, "veles::affine"):
        if shift == 0.0:
            return x * scale
        if scale == 1.0:
            return x + shift
        return x * scale + shift
    x = x.contiguous()
    out = torch.empty_like(x)
    with on_device(x):
        _lib.call("vs_affine", ptr(x), float(scale), float(shift), ptr(out),
                  x.numel(), stream_of(x))
    return out


@affine.register_fake
def _(x, scale=1.0, shift=0.0):
    return torch.empty_like(x)


@torch.library.custom_op("veles::saxpy", mutates_args=())
def saxpy(a: float, x: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
    """a * x + y (fused multiply-add), returned as a new tensor."""
    if not _gpu(x, "veles::saxpy"):
        return torch.addcmul(y, x, torch.tensor(a, dtype=x.dtype))
    x = x.contiguous()
    out = y.contiguous().clone()
    with on_device(x):
        _lib.call("vs_saxpy", float(a), ptr(x), ptr(out), x.numel(), stream_of(x))
    return out


@saxpy.register_fake
def _(a, x, y):
    return torch.empty_like(y)


# --------------------------------------------------------------------- math
@torch.library.custom_op("veles::math", mutates_args=())
def math(x: torch.Tensor, fn: str) -> torch.Tensor:
    """sin / cos / log / exp (mathfun.h *_psv)."""
    if not _gpu(x, "veles::math"):
        return getattr(torch, fn)(x)
    x = x.contiguous()
    out = torch.empty_like(x)
    with on_device(x):
        _lib.call("vs_math", _FN[fn], ptr(x), ptr(out), x.numel(), stream_of(x))
    return out


@math.register_fake
def _(x, fn):
    return torch.empty_like(x)


def sin(x):
    return math(x, "sin")


def cos(x):
    return math(x, "cos")


def log(x):
    return math(x, "log")


def exp(x):
    return math(x, "exp")


def sqrt(x):
    return math(x, "sqrt")


@torch.library.custom_op("veles::pow", mutates_args=())
def pow(x: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
    """x ** y elementwise (avx_mathfun.h pow256_ps over arrays)."""
    if not _gpu(x, "veles::pow"):
        return torch.pow(x, y)
    x, y = torch.broadcast_tensors(x, y)
    x, y = x.contiguous(), y.contiguous()
    out = torch.empty_like(x)
    with on_device(x):
        _lib.call("vs_pow", ptr(x), ptr(y), ptr(out), x.numel(), stream_of(x))
    return out


@pow.register_fake
def _(x, y):
    return torch.empty(torch.broadcast_shapes(x.shape, y.shape), dtype=x.dtype,
                       device=x.device)


@torch.library.custom_op("veles::sincos", mutates_args=())
def sincos(x: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
    """(sin x, cos x) in one pass (sincos256_ps / sincos_ps over arrays)."""
    if not _gpu(x, "veles::sincos"):
        return torch.sin(x), torch.cos(x)
    x = x.contiguous()
    s, c = torch.empty_like(x), torch.empty_like(x)
    with on_device(x):
        _lib.call("vs_sincos", ptr(x), ptr(s), ptr(c), x.numel(), stream_of(x))
    return s, c


@sincos.register_fake
def _(x):
    return torch.empty_like(x), torch.empty_like(x)


# --------------------------------------------------------------- reductions
@torch.library.custom_op("veles::sum", mutates_args=())
def sum_all(x: torch.Tensor) -> torch.Tensor:
    """Sum of all elements as a 0-d tensor (sum_elements)."""
    if not _gpu(x, "veles::sum"):
        return x.sum()
    x = x.contiguous()
    out = torch.empty((), dtype=torch.float32, device=x.device)
    with on_device(x):
        _lib.call("vs_sum", ptr(x), x.numel(), ptr(out), stream_of(x))
    return out


@sum_all.register_fake
def _(x):
    return x.new_empty(())


@torch.library.custom_op("veles::minmax", mutates_args=())
def minmax(x: torch.Tensor) -> torch.Tensor:
    """[min, max] of a float32 tensor (minmax1D), or of a uint8 plane
    (minmax2D) -- for a stack of planes [..., h, w] one pair per plane,
    shape [..., 2], all planes in one launch sequence."""
    if x.dtype == torch.uint8:
        if x.dim() < 2:
            raise ValueError("veles::minmax: uint8 input must be [..., h, w]")
        lead = x.shape[:-2]
        if not _gpu(x, "veles::minmax"):
            flat = x.reshape(*lead, -1)
            return torch.stack([flat.min(-1).values, flat.max(-1).values], -1)
        h, w = x.shape[-2:]
        xp = x.reshape(-1, h, w)
        if xp.stride(2) != 1 or (xp.shape[0] > 1 and xp.stride(0) < (h - 1) * xp.stride(1) + w):
            xp = xp.contiguous()
        planes = xp.shape[0]
        out = torch.empty((planes, 2), dtype=torch.uint8, device=x.device)
        with on_device(x):
            _lib.call("vs_minmax2d_u8_batched", ptr(xp), xp.stride(1), xp.stride(0), w, h,
                      planes, ptr(out), stream_of(x))
        return out.reshape(*lead, 2)
    if not _gpu(x, "veles::minmax"):
        return torch.stack([x.min(), x.max()])
    x = x.contiguous()
    out = torch.empty(2, dtype=torch.float32, device=x.device)
    with on_device(x):
        _lib.call("vs_minmax", ptr(x), x.numel(), ptr(out), stream_of(x))
    return out


@minmax.register_fake
def _(x):
    if x.dtype == torch.uint8:
        return x.new_empty((*x.shape[:-2], 2))
    return x.new_empty((2,))


@torch.library.custom_op("veles::normalize2d", mutates_args=())
def normalize2d(x: torch.Tensor) -> torch.Tensor:
    """uint8 plane(s) [..., h, w] -> float32 in [-1, 1] (normalize2D), each
    plane with its own min / max, found and applied on the device without a
    host round trip; a stack of planes takes one launch sequence."""
    if x.dtype != torch.uint8 or x.dim() < 2:
        raise ValueError("veles::normalize2d expects a uint8 tensor [..., h, w]")
    h, w = x.shape[-2:]
    if not _gpu(x, "veles::normalize2d"):
        flat = x.reshape(-1, h * w).float()
        mn = flat.min(-1, keepdim=True).values
        mx = flat.max(-1, keepdim=True).values
        span = (mx - mn) / 2.0
        res = torch.where(span > 0, (flat - mn) / span.clamp_min(1e-30) - 1.0,
                          torch.zeros_like(flat))
        return res.reshape(x.shape)
    xp = x.reshape(-1, h, w)
    if xp.stride(2) != 1 or (xp.shape[0] > 1 and xp.stride(0) < (h - 1) * xp.stride(1) + w):
        xp = xp.contiguous()
    planes = xp.shape[0]
    out = torch.empty((planes, h, w), dtype=torch.float32, device=x.device)
    mm = torch.empty((planes, 2), dtype=torch.uint8, device=x.device)
    with on_device(x):
        s = stream_of(x)
        _lib.call("vs_minmax2d_u8_batched", ptr(xp), xp.stride(1), xp.stride(0), w, h, planes,
                  ptr(mm), s)
        _lib.call("vs_normalize2d_u8_batched", ptr(xp), xp.stride(1), xp.stride(0), w, h,
                  planes, ptr(mm), 0, 0, ptr(out), w, h * w, s)
    return out.reshape(x.shape)


@normalize2d.register_fake
def _(x):
    return torch.empty(x.shape, dtype=torch.float32, device=x.device)


# ------------------------------------------------------------- gradients
# Backward formulas of the differentiable elementwise ops, written with the
# ops themselves so a GPU backward runs the same kernels.
def _save(*idx):
    def setup(ctx, inputs, output):
        ctx.save_for_backward(*[inputs[i] for i in idx if isinstance(inputs[i], torch.Tensor)])
        ctx.args = inputs
    return setup


def _binary_backward(ctx, g):
    a, b, op = ctx.args
    g = g.contiguous()
    if op == "add":
        return g, g, None
    if op == "sub":
        return g, affine(g, -1.0, 0.0), None
    return binary(g, b, "mul"), binary(g, a, "mul"), None


def _complex_multiply_backward(ctx, g):
    # r = a b (or a conj(b)):  grad_a = g conj(b')  with b' the factor used,
    # grad_b = g conj(a)  (conjugated once more when b entered conjugated)
    a, b, conj_b = ctx.args
    g = g.contiguous()
    ga = complex_multiply(g, b, not conj_b)
    gb = complex_multiply(g, a, True)
    if conj_b:
        gb = complex_conjugate(gb)
    return ga, gb, None


def _math_backward(ctx, g):
    x, fn = ctx.args
    g = g.contiguous()
    if fn == "sin":
        return binary(g, math(x, "cos"), "mul"), None
    if fn == "cos":
        return affine(binary(g, math(x, "sin"), "mul"), -1.0, 0.0), None
    if fn == "exp":
        return binary(g, math(x, "exp"), "mul"), None
    if fn == "log":
        return g / x, None
    return g / affine(math(x, "sqrt"), 2.0, 0.0), None   # sqrt


def _pow_backward(ctx, g):
    x, y = ctx.args
    r = pow(x, y)
    gx = g * y * r / x
    gy = g * r * math(x.expand_as(r).contiguous(), "log")
    return gx.sum_to_size(x.shape), gy.sum_to_size(y.shape)


def _sincos_backward(ctx, gs, gc):
    x, = ctx.args
    s, c = sincos(x)
    return gs * c - gc * s


binary.register_autograd(_binary_backward, setup_context=_save(0, 1))
complex_multiply.register_autograd(_complex_multiply_backward, setup_context=_save(0, 1))
complex_conjugate.register_autograd(lambda ctx, g: complex_conjugate(g.contiguous()),
                                    setup_context=_save())
affine.register_autograd(lambda ctx, g: (affine(g.contiguous(), ctx.args[1], 0.0), None, None),
                         setup_context=_save())
saxpy.register_autograd(lambda ctx, g: (None, affine(g.contiguous(), ctx.args[0], 0.0), g),
                        setup_context=_save())
math.register_autograd(_math_backward, setup_context=_save(0))
pow.register_autograd(_pow_backward, setup_context=_save(0, 1))
sincos.register_autograd(_sincos_backward, setup_context=_save(0))
sum_all.register_autograd(lambda ctx, g: g.expand(ctx.args[0].shape),
                          setup_context=_save())
