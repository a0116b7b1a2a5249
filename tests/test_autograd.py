"""Gradients of the custom ops: the registered backward of the wavelet ops
(adjoint filter bank: conv1d op + extension fold), the transforms and the
elementwise ops against torch autograd through a plain float64 formulation
(reference definitions: /root/reference/src/wavelet.c:271-382)."""
import pytest
import torch

from veles.simd_amd import ops
from veles.simd_amd.ops import signal as sig


def _level_ref(x, lp, hp, dil, step, nout, ext):
    """out[i] = sum_r f[r] xe[step * i + r * dil] in float64, differentiable."""
    n, order = x.shape[-1], lp.shape[0]
    t = torch.arange(order * dil)
    if ext == 0:
        e = x[..., t % n]
    elif ext == 1:
        e = x[..., n - 1 - (t % n)]
    elif ext == 2:
        e = x[..., -1:].expand(*x.shape[:-1], order * dil)
    else:
        e = x.new_zeros(*x.shape[:-1], order * dil)
    xe = torch.cat([x, e], -1)
    idx = step * torch.arange(nout)[:, None] + dil * torch.arange(order)[None, :]
    win = xe[..., idx]
    return win @ hp, win @ lp


def _filters(fam, order):
    lp = ops.wavelet_filter(fam, order).double()
    return lp, sig._qmf(lp)


CASES = [("daubechies", 8, "periodic"), ("daubechies", 4, "mirror"), ("symlet", 6, "constant"),
         ("coiflet", 12, "zero"), ("daubechies", 2, "mirror"), ("daubechies", 16, "periodic")]
DEVICES = ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)]


def _compare(op_out, ref_out, x, xr, tol):
    torch.manual_seed(1)
    outs = op_out if isinstance(op_out, (tuple, list)) else [op_out]
    refs = ref_out if isinstance(ref_out, (tuple, list)) else [ref_out]
    ws = [torch.randn(o.shape, dtype=torch.float64) for o in refs]
    loss = sum((o.double().cpu() * w).sum() for o, w in zip(outs, ws))
    loss_ref = sum((o * w).sum() for o, w in zip(refs, ws))
    g, = torch.autograd.grad(loss, x)
    g_ref, = torch.autograd.grad(loss_ref, xr)
    assert (g.double().cpu() - g_ref).abs().max() <= tol * max(1.0, g_ref.abs().max().item())


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("fam,order,ext", CASES)
def test_dwt_and_swt_level_gradients(device, fam, order, ext):
    e = sig._ext(ext)
    lp, hp = _filters(fam, order)
    for n in (64, 130, 1000):
        x0 = torch.randn(3, n)
        x = x0.to(device).requires_grad_()
        xr = x0.double().requires_grad_()
        _compare(ops.dwt(x, fam, order, ext), _level_ref(xr, lp, hp, 1, 2, n // 2, e), x, xr, 2e-5)
        for level in (1, 3):
            x = x0.to(device).requires_grad_()
            xr = x0.double().requires_grad_()
            _compare(ops.swt_level(x, fam, order, level, ext),
                     _level_ref(xr, lp, hp, 1 << (level - 1), 1, n, e), x, xr, 2e-5)


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("fam,order,ext", CASES)
def test_multilevel_gradients(device, fam, order, ext):
    e = sig._ext(ext)
    lp, hp = _filters(fam, order)
    levels, n = 4, 256
    x0 = torch.randn(2, 3, n)
    # stationary: hi [..., levels, n], lo [..., n]
    x = x0.to(device).requires_grad_()
    xr = x0.double().requires_grad_()
    his, cur = [], xr
    for lvl in range(levels):
        h, cur = _level_ref(cur, lp, hp, 1 << lvl, 1, n, e)
        his.append(h)
    hi, lo = ops.swt(x, fam, order, levels, ext)
    _compare([hi, lo], [torch.stack(his, -2), cur], x, xr, 5e-5)
    # pyramid: rows [hi_1 | ... | hi_L | lo_L]
    x = x0.to(device).requires_grad_()
    xr = x0.double().requires_grad_()
    parts, cur = [], xr
    for _ in range(levels):
        h, cur = _level_ref(cur, lp, hp, 1, 2, cur.shape[-1] // 2, e)
        parts.append(h)
    _compare(ops.wavedec(x, fam, order, levels, ext), torch.cat(parts + [cur], -1), x, xr, 5e-5)


def test_wavelet_module_passes_gradient_upstream():
    """A trainable layer in front of the wavelet front-ends receives gradients."""
    from veles.simd_amd import models
    lin = torch.nn.Linear(128, 128)
    feats = models.WaveletEnergyFeatures(levels=3)
    out = feats(lin(torch.randn(4, 128)))
    out.sum().backward()
    assert lin.weight.grad is not None and lin.weight.grad.abs().sum() > 0


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("n", [8, 256, 4096])
def test_fft_gradients(device, n):
    """veles::fft / rfft / irfft against autograd through torch.fft in float64
    (the unnormalised conventions of the library, FFTF's: reference
    src/convolve.c:253-290)."""
    torch.manual_seed(n)
    z0 = torch.randn(3, n, 2)
    for inverse in (False, True):
        z = z0.to(device).requires_grad_()
        zr = z0.double().requires_grad_()
        c = torch.view_as_complex(zr)
        ref = torch.view_as_real(torch.fft.ifft(c) * n if inverse else torch.fft.fft(c))
        _compare(ops.fft(z, inverse), ref, z, zr, 2e-5 * n ** 0.5)
    x0 = torch.randn(3, n)
    x = x0.to(device).requires_grad_()
    xr = x0.double().requires_grad_()
    _compare(ops.rfft(x), torch.view_as_real(torch.fft.rfft(xr)), x, xr, 2e-5 * n ** 0.5)
    X0 = torch.randn(3, n // 2 + 1, 2)
    X0[:, 0, 1] = 0
    X0[:, -1, 1] = 0
    X = X0.to(device).requires_grad_()
    Xr = X0.double().requires_grad_()
    ref = torch.fft.irfft(torch.view_as_complex(Xr), n=n) * n
    torch.manual_seed(2)
    w = torch.randn(3, n, dtype=torch.float64)
    g, = torch.autograd.grad((ops.irfft(X, n).double().cpu() * w).sum(), X)
    g_ref, = torch.autograd.grad((ref * w).sum(), Xr)
    # torch leaves the gradient of the ignored imaginary parts of the DC and
    # Nyquist bins unspecified; compare everything else
    g, g_ref = g.double().cpu().clone(), g_ref.clone()
    for t in (g, g_ref):
        t[:, 0, 1] = 0
        t[:, -1, 1] = 0
    assert (g - g_ref).abs().max() <= 2e-5 * n ** 0.5 * max(1.0, g_ref.abs().max().item())


@pytest.mark.parametrize("device", DEVICES)
def test_elementwise_gradients(device):
    """Every differentiable elementwise op against torch autograd of the same
    formula in float64."""
    torch.manual_seed(3)
    n = 2048
    a0, b0 = torch.rand(n) * 2 + 0.5, torch.rand(n) * 2 + 0.5

    def check(fn_op, fn_ref, *inputs0, tol=2e-5):
        ins = [t.to(device).requires_grad_() for t in inputs0]
        refs = [t.double().requires_grad_() for t in inputs0]
        out, ref = fn_op(*ins), fn_ref(*refs)
        outs = out if isinstance(out, (tuple, list)) else [out]
        rfs = ref if isinstance(ref, (tuple, list)) else [ref]
        ws = [torch.randn(r.shape, dtype=torch.float64) for r in rfs]
        loss = sum((o.double().cpu() * w).sum() for o, w in zip(outs, ws))
        loss_ref = sum((r * w).sum() for r, w in zip(rfs, ws))
        gs = torch.autograd.grad(loss, ins)
        gr = torch.autograd.grad(loss_ref, refs)
        for g, r in zip(gs, gr):
            assert (g.double().cpu() - r).abs().max() <= tol * max(1.0, r.abs().max().item())

    check(ops.add, torch.add, a0, b0)
    check(ops.sub, torch.sub, a0, b0)
    check(ops.mul, torch.mul, a0, b0)
    check(lambda x: ops.affine(x, 1.7, -0.3), lambda x: x * 1.7 - 0.3, a0)
    check(lambda x, y: ops.saxpy(0.6, x, y), lambda x, y: 0.6 * x + y, a0, b0)
    for fn in ("sin", "cos", "exp", "log", "sqrt"):
        check(lambda x: ops.math(x, fn), getattr(torch, fn), a0)
    check(ops.pow, torch.pow, a0, b0, tol=1e-4)
    check(ops.sincos, lambda x: (torch.sin(x), torch.cos(x)), a0)
    check(ops.sum_all, torch.sum, a0)

    def cmul_ref(conj):
        def f(a, b):
            ca = torch.view_as_complex(a.reshape(-1, 2))
            cb = torch.view_as_complex(b.reshape(-1, 2))
            return torch.view_as_real(ca * (cb.conj() if conj else cb)).reshape(-1)
        return f
    check(lambda a, b: ops.complex_multiply(a, b), cmul_ref(False), a0, b0)
    check(lambda a, b: ops.complex_multiply(a, b, True), cmul_ref(True), a0, b0)
    check(ops.complex_conjugate,
          lambda a: torch.view_as_real(torch.view_as_complex(a.reshape(-1, 2)).conj().resolve_conj()).reshape(-1),
          a0)
