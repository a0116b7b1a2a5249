"""Signal-processing ops: FFT, convolution / correlation, wavelets, peaks.

References: src/convolve.c + src/correlate.c (conv1d), FFTF usage in
src/convolve.c (fft / rfft / irfft), src/wavelet.c (dwt / swt / wavedec),
src/detect_peaks.c (detect_peaks).  GPU tensors run the native HIP kernels;
CPU tensors run an fp64-accumulated torch reference of the same math.
"""
from __future__ import annotations

import ctypes
import weakref

import torch

from .. import _lib
from ._util import on_device, ptr, require_gpu_tensor, stream_of

ALGORITHMS = {"auto": 0, "direct": 1, "fft": 2, "overlap_save": 3}


def _algo(a) -> int:
    return ALGORITHMS[a] if isinstance(a, str) else int(a)


def _rows(t: torch.Tensor):
    """(2-D contiguous view, original leading shape)."""
    lead = t.shape[:-1]
    return t.reshape(-1, t.shape[-1]).contiguous(), lead


# ---------------------------------------------------------------- conv1d
@torch.library.custom_op("veles::conv1d", mutates_args=())
def _conv1d(x: torch.Tensor, h: torch.Tensor, algorithm: int,
            correlate: bool) -> torch.Tensor:
    if x.dtype != torch.float32 or h.dtype != torch.float32:
        raise TypeError("veles::conv1d expects float32")
    xr, lead = _rows(x)
    batch, xlen = xr.shape
    hr = h.reshape(-1, h.shape[-1]).contiguous()
    hlen = hr.shape[1]
    if hr.shape[0] not in (1, batch):
        raise ValueError("veles::conv1d: filters must be 1 or one per signal")
    ylen = xlen + hlen - 1
    if not x.is_cuda:
        # torch conv1d is a correlation: weight = h for correlation,
        # flip(h) for convolution (reference definitions, see module doc).
        w = hr.double() if correlate else hr.double().flip(-1)
        if hr.shape[0] == 1:
            out = torch.nn.functional.conv1d(xr.double()[:, None], w[None],
                                             padding=hlen - 1)[:, 0]
        else:
            out = torch.nn.functional.conv1d(xr.double()[None], w[:, None],
                                             padding=hlen - 1, groups=batch)[0]
        return out.float().reshape(*lead, ylen)
    require_gpu_tensor(x, "veles::conv1d")
    y = torch.empty((batch, ylen), dtype=torch.float32, device=x.device)
    with on_device(x):
        _lib.call("vs_conv1d", algorithm, int(correlate), ptr(xr), xlen, xlen,
                  ptr(hr), hlen, hlen if hr.shape[0] > 1 else 0, ptr(y), ylen,
                  batch, stream_of(x))
    return y.reshape(*lead, ylen)


@_conv1d.register_fake
def _(x, h, algorithm, correlate):
    return x.new_empty((*x.shape[:-1], x.shape[-1] + h.shape[-1] - 1))


class Conv1dPlan:
    """Fixed filter(s) and signal length, many executions on the GPU
    (vs_conv1d_plan_*): the algorithm is resolved and, on the real-block
    FFT / overlap-save paths, the filter spectra are computed once at
    creation instead of at every call.  The taps are copied / transformed at
    creation, so later changes to `h` do not affect the plan.

    plan = Conv1dPlan(h, x_len); y = plan(x)   # x: [..., x_len] float32 cuda
    h: [h_len] (shared) or [batch, h_len] (one filter per signal).
    """

    def __init__(self, h: torch.Tensor, x_len: int, algorithm="auto",
                 correlate: bool = False):
        if not h.is_cuda or h.dtype != torch.float32:
            raise TypeError("Conv1dPlan: float32 cuda filter expected")
        hr = h.reshape(-1, h.shape[-1]).contiguous()
        self.x_len, self.h_len, self.n_filters = int(x_len), hr.shape[1], hr.shape[0]
        self.correlate = bool(correlate)
        self.device = h.device
        self._plan = ctypes.c_void_p()
        with on_device(h):
            _lib.call("vs_conv1d_plan_create", _algo(algorithm), int(correlate), self.x_len,
                      ptr(hr), self.h_len, self.h_len, self.n_filters,
                      ctypes.byref(self._plan), stream_of(h))
        algo, pre = ctypes.c_int(), ctypes.c_int()
        _lib.call("vs_conv1d_plan_info", self._plan, ctypes.byref(algo), ctypes.byref(pre))
        self.algorithm = {v: k for k, v in ALGORITHMS.items()}.get(algo.value, algo.value)
        self.precomputed = bool(pre.value)
        self._stream_used = torch.cuda.current_stream(h.device)
        _PLANS[id(self)] = self

    def apply(self, x: torch.Tensor, h: torch.Tensor) -> torch.Tensor:
        """Differentiable, torch.compile-traceable execution: the plan runs
        the forward; gradients to x and to h (the taps the plan was built
        from) come from the conv1d op's backward."""
        return _conv1d_planned(x, h, id(self), _algo(self.algorithm), self.correlate)

    def __call__(self, x: torch.Tensor) -> torch.Tensor:
        if x.shape[-1] != self.x_len or x.dtype != torch.float32 or x.device != self.device:
            raise ValueError("Conv1dPlan: x must be float32 [..., x_len] on the plan's device")
        xr, lead = _rows(x)
        batch = xr.shape[0]
        ylen = self.x_len + self.h_len - 1
        y = torch.empty((batch, ylen), dtype=torch.float32, device=x.device)
        self._stream_used = torch.cuda.current_stream(x.device)
        with on_device(x):
            _lib.call("vs_conv1d_plan_execute", self._plan, ptr(xr), self.x_len, ptr(y), ylen,
                      batch, stream_of(x))
        return y.reshape(*lead, ylen)

    def __del__(self):
        plan = getattr(self, "_plan", None)
        if plan is not None and plan.value:
            try:
                self._stream_used.synchronize()   # executions queued on it still read the plan
                _lib.lib().vs_conv1d_plan_destroy(plan)
            except Exception:  # noqa: BLE001 - interpreter shutdown
                pass
            self._plan = ctypes.c_void_p()


# Live plans by id(): the planned op takes the id (custom-op schemas have no
# object arguments) and falls back to the plain op when the plan is gone.
_PLANS: "weakref.WeakValueDictionary[int, Conv1dPlan]" = weakref.WeakValueDictionary()


@torch.library.custom_op("veles::conv1d_planned", mutates_args=())
def _conv1d_planned(x: torch.Tensor, h: torch.Tensor, plan_id: int, algorithm: int,
                    correlate: bool) -> torch.Tensor:
    plan = _PLANS.get(plan_id)
    if (plan is None or not x.is_cuda or x.dtype != torch.float32
            or x.shape[-1] != plan.x_len or x.device != plan.device):
        return _conv1d(x, h, algorithm, correlate)
    return plan(x)


@_conv1d_planned.register_fake
def _(x, h, plan_id, algorithm, correlate):
    return x.new_empty((*x.shape[:-1], x.shape[-1] + h.shape[-1] - 1))


def _conv_setup(ctx, inputs, output):
    x, h, algorithm, corr = inputs[0], inputs[1], inputs[-2], inputs[-1]
    ctx.save_for_backward(x, h)
    ctx.algorithm = algorithm
    ctx.corr = corr


def _conv_backward(ctx, g):
    """y = x (*) k with k = h (convolution) or flip(h) (correlation).
    dx = valid correlation of g with k; dk = valid correlation of g with x."""
    x, h = ctx.saved_tensors
    k = h.flip(-1) if ctx.corr else h
    X, H = x.shape[-1], k.shape[-1]
    gx = gh = None
    if ctx.needs_input_grad[0]:
        r = _conv1d(g.contiguous(), k.contiguous(), ctx.algorithm, True)
        gx = r[..., H - 1: H - 1 + X]
    if ctx.needs_input_grad[1]:
        gr = g.reshape(-1, g.shape[-1]).contiguous()
        xr = x.reshape(-1, X).contiguous()
        r = _conv1d(gr, xr, 0, True)[..., X - 1: X - 1 + H]
        dk = r.sum(0) if h.dim() == 1 else r.reshape(h.shape)
        gh = dk.flip(-1) if ctx.corr else dk
    return gx, gh, None, None


_conv1d.register_autograd(_conv_backward, setup_context=_conv_setup)
_conv1d_planned.register_autograd(lambda ctx, g: _conv_backward(ctx, g)[:2] + (None, None, None),
                                  setup_context=_conv_setup)


def conv1d(x: torch.Tensor, h: torch.Tensor, algorithm="auto",
           correlate: bool = False) -> torch.Tensor:
    """Full linear convolution (or cross-correlation) of every row of x with
    h (one shared filter, or one per row).  Output length x + h - 1."""
    return _conv1d(x, h, _algo(algorithm), bool(correlate))


def correlate(x, h, algorithm="auto"):
    return _conv1d(x, h, _algo(algorithm), True)


def conv1d_algorithm(xlen: int, hlen: int, batch: int = 1) -> str:
    """The algorithm "auto" resolves to on the GPU for this shape."""
    a = _lib.lib().vs_conv1d_select(xlen, hlen, batch)
    return {1: "direct", 2: "fft", 3: "overlap_save"}[a]


# ------------------------------------------------------------------- FFT
@torch.library.custom_op("veles::fft", mutates_args=())
def fft(z: torch.Tensor, inverse: bool = False) -> torch.Tensor:
    """Unnormalised complex FFT over the second-to-last dim of a float32
    tensor [..., n, 2] (interleaved re/im); n a power of two <= 2^24."""
    if z.shape[-1] != 2:
        raise ValueError("veles::fft expects [..., n, 2] interleaved complex")
    n = z.shape[-2]
    if not z.is_cuda:
        c = torch.view_as_complex(z.contiguous().double())
        r = torch.fft.ifft(c, dim=-1) * n if inverse else torch.fft.fft(c, dim=-1)
        return torch.view_as_real(r).float()
    require_gpu_tensor(z, "veles::fft")
    zc = z.contiguous()
    out = torch.empty_like(zc)
    batch = zc.numel() // (2 * n)
    with on_device(z):
        _lib.call("vs_fft_c2c", ptr(zc), ptr(out), n, batch, int(inverse),
                  stream_of(z))
    return out


@fft.register_fake
def _(z, inverse=False):
    return torch.empty_like(z)


@torch.library.custom_op("veles::rfft", mutates_args=())
def rfft(x: torch.Tensor) -> torch.Tensor:
    """Real FFT of the last dim (n a power of two): [..., n/2+1, 2]."""
    n = x.shape[-1]
    if not x.is_cuda:
        return torch.view_as_real(torch.fft.rfft(x.double(), dim=-1)).float()
    require_gpu_tensor(x, "veles::rfft")
    xc = x.contiguous()
    out = torch.empty((*x.shape[:-1], n // 2 + 1, 2), dtype=torch.float32,
                      device=x.device)
    with on_device(x):
        _lib.call("vs_fft_r2c", ptr(xc), ptr(out), n, xc.numel() // n, stream_of(x))
    return out


@rfft.register_fake
def _(x):
    return x.new_empty((*x.shape[:-1], x.shape[-1] // 2 + 1, 2))


@torch.library.custom_op("veles::irfft", mutates_args=())
def irfft(X: torch.Tensor, n: int) -> torch.Tensor:
    """Unnormalised inverse of rfft (returns n * x, the FFTF convention)."""
    if not X.is_cuda:
        c = torch.view_as_complex(X.contiguous().double())
        return (torch.fft.irfft(c, n=n, dim=-1) * n).float()
    require_gpu_tensor(X, "veles::irfft")
    Xc = X.contiguous()
    out = torch.empty((*X.shape[:-2], n), dtype=torch.float32, device=X.device)
    with on_device(X):
        _lib.call("vs_fft_c2r", ptr(Xc), ptr(out), n, out.numel() // n, stream_of(X))
    return out


@irfft.register_fake
def _(X, n):
    return X.new_empty((*X.shape[:-2], n))


# Gradients of the transforms (real pairs (re, im) as the variables): the
# adjoint of the unnormalised DFT is the unnormalised DFT of the other sign;
# the half spectra of rfft / irfft count their interior bins twice.
def _half_weights(g: torch.Tensor, interior: float) -> torch.Tensor:
    w = g.new_full((g.shape[-2], 1), interior)
    w[0] = w[-1] = 1.0
    out = g * w
    out[..., 0, 1] = 0.0    # the DC and Nyquist bins of a real signal are real
    out[..., -1, 1] = 0.0
    return out


fft.register_autograd(lambda ctx, g: (fft(g.contiguous(), not ctx.inverse), None),
                      setup_context=lambda ctx, inputs, output: setattr(ctx, "inverse", inputs[1]))
rfft.register_autograd(
    lambda ctx, g: irfft(_half_weights(g, 0.5), ctx.n),
    setup_context=lambda ctx, inputs, output: setattr(ctx, "n", inputs[0].shape[-1]))
irfft.register_autograd(lambda ctx, g: (_half_weights(rfft(g.contiguous()), 2.0), None),
                        setup_context=lambda ctx, inputs, output: None)


# -------------------------------------------------------------- wavelets
DAUBECHIES, COIFLET, SYMLET = 0, 1, 2
PERIODIC, MIRROR, CONSTANT, ZERO = 0, 1, 2, 3
_FAMILY = {"daubechies": 0, "db": 0, "coiflet": 1, "coiflets": 1, "coif": 1,
           "symlet": 2, "symlets": 2, "sym": 2}
_EXT = {"periodic": 0, "mirror": 1, "constant": 2, "zero": 3}


def _fam(t):
    return _FAMILY[t] if isinstance(t, str) else int(t)


def _ext(e):
    return _EXT[e] if isinstance(e, str) else int(e)


def wavelet_filter(family, order: int) -> torch.Tensor:
    """The library's float32 low-pass taps (reference normalisation)."""
    import ctypes
    out = torch.empty(order, dtype=torch.float32)
    _lib.check(_lib.lib().vs_wavelet_filter(_fam(family), order,
                                            ctypes.c_void_p(out.data_ptr())),
               "vs_wavelet_filter")
    return out


def _extend_host(x: torch.Tensor, size: int, ext: int) -> torch.Tensor:
    n = x.shape[-1]
    t = torch.arange(size)
    if ext == PERIODIC:
        e = x[..., t % n]
    elif ext == MIRROR:
        e = x[..., n - 1 - (t % n)]
    elif ext == CONSTANT:
        e = x[..., -1:].expand(*x.shape[:-1], size)
    else:
        e = torch.zeros(*x.shape[:-1], size, dtype=x.dtype)
    return torch.cat([x, e], dim=-1)


def _qmf(lp: torch.Tensor) -> torch.Tensor:
    o = lp.shape[0]
    sign = torch.tensor([1.0 if (i & 1) else -1.0 for i in range(o)], dtype=lp.dtype)
    return (lp * sign).flip(0)


@torch.library.custom_op("veles::dwt", mutates_args=())
def _dwt(x: torch.Tensor, family: int, order: int, ext: int) -> torch.Tensor:
    xr, lead = _rows(x)
    batch, n = xr.shape
    if not x.is_cuda:
        lp = wavelet_filter(family, order).double()
        hp = _qmf(lp)
        xe = _extend_host(xr.double(), order, ext)
        win = xe.unfold(-1, order, 2)[:, : n // 2]
        return torch.stack([win @ hp, win @ lp]).float().reshape(2, *lead, n // 2)
    require_gpu_tensor(x, "veles::dwt")
    out = torch.empty((2, batch, n // 2), dtype=torch.float32, device=x.device)
    with on_device(x):
        _lib.call("vs_dwt", family, order, ext, ptr(xr), n, n, ptr(out[0]),
                  ptr(out[1]), n // 2, batch, stream_of(x))
    return out.reshape(2, *lead, n // 2)


@_dwt.register_fake
def _(x, family, order, ext):
    return x.new_empty((2, *x.shape[:-1], x.shape[-1] // 2))


def dwt(x, family="daubechies", order=8, ext="periodic"):
    """One decimated level over the last dim: (hi, lo), each length n/2."""
    r = _dwt(x, _fam(family), order, _ext(ext))
    return r[0], r[1]


@torch.library.custom_op("veles::swt", mutates_args=())
def _swt(x: torch.Tensor, family: int, order: int, levels: int,
         ext: int) -> torch.Tensor:
    xr, lead = _rows(x)
    batch, n = xr.shape
    if not x.is_cuda:
        lp = wavelet_filter(family, order).double()
        hp = _qmf(lp)
        cur = xr.double()
        his = []
        for lvl in range(levels):
            dil = 1 << lvl
            xe = _extend_host(cur, order * dil, ext)
            idx = torch.arange(n)[:, None] + dil * torch.arange(order)[None, :]
            win = xe[:, idx]
            his.append(win @ hp)
            cur = win @ lp
        out = torch.cat([torch.stack(his, 1), cur[:, None]], 1).float()
        return out.reshape(*lead, levels + 1, n)
    require_gpu_tensor(x, "veles::swt")
    # one allocation, rows 0..levels-1 = hi, row levels = lo: the kernels
    # write both straight into it (a signal's rows are contiguous)
    out = torch.empty((batch, levels + 1, n), dtype=torch.float32, device=x.device)
    with on_device(x):
        _lib.call("vs_swt_multilevel_packed", family, order, levels, ext, ptr(xr), n,
                  ptr(out), batch, stream_of(x))
    return out.reshape(*lead, levels + 1, n)


@_swt.register_fake
def _(x, family, order, levels, ext):
    return x.new_empty((*x.shape[:-1], levels + 1, x.shape[-1]))


def swt(x, family="daubechies", order=8, levels=1, ext="periodic"):
    """Fused multi-level stationary DWT over the last dim.  Returns
    (hi [..., levels, n], lo [..., n])."""
    r = _swt(x, _fam(family), order, levels, _ext(ext))
    return r[..., :levels, :], r[..., levels, :]


@torch.library.custom_op("veles::swt_level", mutates_args=())
def _swt_level(x: torch.Tensor, family: int, order: int, level: int,
               ext: int) -> torch.Tensor:
    xr, lead = _rows(x)
    batch, n = xr.shape
    if not x.is_cuda:
        lp = wavelet_filter(family, order).double()
        hp = _qmf(lp)
        dil = 1 << (level - 1)
        xe = _extend_host(xr.double(), order * dil, ext)
        idx = torch.arange(n)[:, None] + dil * torch.arange(order)[None, :]
        win = xe[:, idx]
        return torch.stack([win @ hp, win @ lp]).float().reshape(2, *lead, n)
    require_gpu_tensor(x, "veles::swt_level")
    out = torch.empty((2, batch, n), dtype=torch.float32, device=x.device)
    with on_device(x):
        _lib.call("vs_swt", family, order, level, ext, ptr(xr), n, n, ptr(out[0]),
                  ptr(out[1]), n, batch, stream_of(x))
    return out.reshape(2, *lead, n)


@_swt_level.register_fake
def _(x, family, order, level, ext):
    return x.new_empty((2, *x.shape))


def swt_level(x, family="daubechies", order=8, level=1, ext="periodic"):
    """One stationary level (filters dilated by 2^(level-1)): (hi, lo)."""
    r = _swt_level(x, _fam(family), order, level, _ext(ext))
    return r[0], r[1]


@torch.library.custom_op("veles::wavedec", mutates_args=())
def _wavedec(x: torch.Tensor, family: int, order: int, levels: int,
             ext: int) -> torch.Tensor:
    xr, lead = _rows(x)
    batch, n = xr.shape
    if not x.is_cuda:
        parts, cur = [], xr
        for _ in range(levels):
            r = _dwt(cur, family, order, ext)
            parts.append(r[0])
            cur = r[1]
        return torch.cat(parts + [cur], -1).reshape(*lead, n)
    require_gpu_tensor(x, "veles::wavedec")
    out = torch.empty((batch, n), dtype=torch.float32, device=x.device)
    with on_device(x):
        _lib.call("vs_dwt_multilevel", family, order, levels, ext, ptr(xr), n,
                  ptr(out), batch, stream_of(x))
    return out.reshape(*lead, n)


@_wavedec.register_fake
def _(x, family, order, levels, ext):
    return torch.empty_like(x)


def wavedec(x, family="daubechies", order=8, levels=1, ext="periodic"):
    """Fused Mallat pyramid: rows [hi_1 | hi_2 | ... | hi_L | lo_L]."""
    return _wavedec(x, _fam(family), order, levels, _ext(ext))


# ---------------------------------------------------- wavelet gradients
# The transforms are linear in x: out = A x with A built from the filter taps
# and the boundary extension, so grad_x = A^T grad_out.  A^T of one level is a
# full convolution of the band gradients with the (dilated / upsampled) taps
# -- the conv1d op, HIP kernels on the GPU -- followed by folding the part that
# fell on the extension back onto the samples it was copied from.
def _fold_extension(ge: torch.Tensor, n: int, ext: int) -> torch.Tensor:
    gx = ge[..., :n].clone()
    tail = ge[..., n:]
    m = tail.shape[-1]
    if m == 0 or ext == ZERO:
        return gx
    t = torch.arange(m, device=ge.device)
    if ext == PERIODIC:
        idx = t % n
    elif ext == MIRROR:
        idx = n - 1 - (t % n)
    else:
        idx = torch.full((m,), n - 1, device=ge.device)
    return gx.index_add_(-1, idx, tail)


def _bank(family: int, order: int, device):
    lp = wavelet_filter(family, order)
    return _qmf(lp).to(device), lp.to(device)


def _dilate(f: torch.Tensor, dil: int) -> torch.Tensor:
    if dil == 1:
        return f
    fd = f.new_zeros((f.shape[0] - 1) * dil + 1)
    fd[::dil] = f
    return fd


def _swt_level_adjoint(g_hi, g_lo, hp, lp, dil: int, ext: int):
    """Gradient of one stationary level (taps dilated by `dil`) to its input."""
    n = g_hi.shape[-1]
    ge = (_conv1d(g_hi.contiguous(), _dilate(hp, dil), 0, False) +
          _conv1d(g_lo.contiguous(), _dilate(lp, dil), 0, False))
    return _fold_extension(ge, n, ext)


def _dwt_level_adjoint(g_hi, g_lo, hp, lp, ext: int, n: int):
    """Gradient of one decimated level (bands of length n // 2) to its input
    of length n."""
    half = g_hi.shape[-1]
    up = g_hi.new_zeros((2, *g_hi.shape[:-1], max(2 * half - 1, 1)))
    up[0][..., ::2] = g_hi
    up[1][..., ::2] = g_lo
    ge = _conv1d(up[0], hp, 0, False) + _conv1d(up[1], lp, 0, False)
    if ge.shape[-1] < n:
        ge = torch.nn.functional.pad(ge, (0, n - ge.shape[-1]))
    return _fold_extension(ge, n, ext)


def _wavelet_setup(ctx, inputs, output):
    ctx.params = tuple(inputs[1:])
    ctx.lead = inputs[0].shape[:-1]
    ctx.n = inputs[0].shape[-1]


def _dwt_backward(ctx, g):
    family, order, ext = ctx.params
    hp, lp = _bank(family, order, g.device)
    gr = g.reshape(2, -1, ctx.n // 2).float()
    gx = _dwt_level_adjoint(gr[0], gr[1], hp, lp, ext, ctx.n)
    return gx.reshape(*ctx.lead, ctx.n), None, None, None


def _swt_level_backward(ctx, g):
    family, order, level, ext = ctx.params
    hp, lp = _bank(family, order, g.device)
    gr = g.reshape(2, -1, ctx.n).float()
    gx = _swt_level_adjoint(gr[0], gr[1], hp, lp, 1 << (level - 1), ext)
    return gx.reshape(*ctx.lead, ctx.n), None, None, None, None


def _swt_backward(ctx, g):
    family, order, levels, ext = ctx.params
    hp, lp = _bank(family, order, g.device)
    gr = g.reshape(-1, levels + 1, ctx.n).float()
    cur = gr[:, levels]
    for lvl in range(levels - 1, -1, -1):   # the low band of level l feeds level l + 1
        cur = _swt_level_adjoint(gr[:, lvl], cur, hp, lp, 1 << lvl, ext)
    return cur.reshape(*ctx.lead, ctx.n), None, None, None, None


def _wavedec_backward(ctx, g):
    family, order, levels, ext = ctx.params
    hp, lp = _bank(family, order, g.device)
    gr = g.reshape(-1, ctx.n).float()
    # rows are [hi_1 | hi_2 | ... | hi_L | lo_L]
    starts, off, length = [], 0, ctx.n
    for _ in range(levels):
        length //= 2
        starts.append((off, length))
        off += length
    cur = gr[:, off:off + length]
    for off_l, len_l in reversed(starts):
        cur = _dwt_level_adjoint(gr[:, off_l:off_l + len_l], cur, hp, lp, ext, 2 * len_l)
    return cur.reshape(*ctx.lead, ctx.n), None, None, None, None


_dwt.register_autograd(_dwt_backward, setup_context=_wavelet_setup)
_swt_level.register_autograd(_swt_level_backward, setup_context=_wavelet_setup)
_swt.register_autograd(_swt_backward, setup_context=_wavelet_setup)
_wavedec.register_autograd(_wavedec_backward, setup_context=_wavelet_setup)


# ----------------------------------------------------------------- peaks
MAXIMUM, MINIMUM, BOTH = 1, 2, 3


def _peaks_host(xr: torch.Tensor, kind: int, pos_dtype):
    """Scalar definition (src/detect_peaks.c:123-125) row by row."""
    pos, val, starts = [], [], [0]
    for row in xr.float():
        d1 = row[1:-1] - row[:-2]
        d2 = row[1:-1] - row[2:]
        m = (d1 * d2) > 0
        m &= ((d1 > 0) & bool(kind & 1)) | ((d1 < 0) & bool(kind & 2))
        p = torch.nonzero(m).flatten() + 1
        pos.append(p.to(pos_dtype))
        val.append(row[p])
        starts.append(starts[-1] + p.numel())
    return torch.cat(pos), torch.cat(val), torch.tensor(starts, dtype=torch.int64)


@torch.library.custom_op("veles::detect_peaks", mutates_args=())
def _detect_peaks(x: torch.Tensor, kind: int) -> tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """Strict extrema of every row of x [rows, n] (float32): positions inside
    the row (int32; int64 for n >= 2^31), values, and row_start [rows + 1]
    (row r's results are [row_start[r], row_start[r + 1])).  One launch
    sequence and one host read (the total) for all rows."""
    if x.dim() != 2 or x.dtype != torch.float32:
        raise ValueError("veles::detect_peaks expects a float32 [rows, n] tensor")
    rows, n = x.shape
    pos_dtype = torch.int64 if n >= (1 << 31) else torch.int32
    if not x.is_cuda:
        return _peaks_host(x, kind, pos_dtype)
    require_gpu_tensor(x, "veles::detect_peaks")
    xc = x if x.stride(1) == 1 and (rows == 1 or x.stride(0) >= n) else x.contiguous()
    row_start = torch.empty(rows + 1, dtype=torch.int64, device=x.device)
    p64 = int(pos_dtype == torch.int64)
    with on_device(x):
        s = stream_of(x)
        _lib.call("vs_detect_peaks_batched", ptr(xc), n, xc.stride(0), rows, kind, None, p64,
                  None, 0, ptr(row_start), s)
        total = int(row_start[-1].item())
        pos = torch.empty(total, dtype=pos_dtype, device=x.device)
        val = torch.empty(total, dtype=torch.float32, device=x.device)
        if total:
            _lib.call("vs_detect_peaks_batched", ptr(xc), n, xc.stride(0), rows, kind, ptr(pos),
                      p64, ptr(val), total, ptr(row_start), s)
    return pos, val, row_start


@_detect_peaks.register_fake
def _(x, kind):
    nnz = torch.library.get_ctx().new_dynamic_size()
    pos_dtype = torch.int64 if x.shape[1] >= (1 << 31) else torch.int32
    return (x.new_empty(nnz, dtype=pos_dtype), x.new_empty(nnz),
            x.new_empty(x.shape[0] + 1, dtype=torch.int64))


def _kind(kind) -> int:
    return {"max": 1, "min": 2, "both": 3}.get(kind, kind)


def detect_peaks(x: torch.Tensor, kind=BOTH):
    """Strict extrema of a 1-D float32 tensor: (positions, values)."""
    pos, val, _ = _detect_peaks(x.reshape(1, -1), _kind(kind))
    return pos, val


def detect_peaks_batched(x: torch.Tensor, kind=BOTH):
    """Strict extrema of every row of x [..., n]: (positions, values,
    row_start); row r's results are [row_start[r], row_start[r + 1])."""
    return _detect_peaks(x.reshape(-1, x.shape[-1]), _kind(kind))
