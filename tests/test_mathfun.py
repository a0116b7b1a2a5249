"""Port of reference tests/mathfun.cc: sin/cos/log/exp vs double libm,
within 4 ulp (ASSERT_FLOAT_EQ), non-finite references skipped."""
import math

import numpy as np
import pytest

from veles.simd_amd import capi

# simd=1 is the GPU path: run it (gpu-marked) where a GPU exists.
SIMDS = [0, pytest.param(1, marks=pytest.mark.gpu)]


def _ulps(a, b):
    a = np.asarray(a, np.float32).view(np.int32).astype(np.int64)
    b = np.asarray(b, np.float32).view(np.int32).astype(np.int64)
    a = np.where(a < 0, -(a & 0x7fffffff), a)
    b = np.where(b < 0, -(b & 0x7fffffff), b)
    return np.abs(a - b)


@pytest.mark.parametrize("simd", SIMDS)
@pytest.mark.parametrize("length", [1, 3, 64, 199, 100003])
@pytest.mark.parametrize("name,ref", [("sin", math.sin), ("cos", math.cos),
                                      ("log", math.log), ("exp", math.exp)])
def test_mathfun(simd, length, name, ref):
    i = np.arange(length)
    data = ((i % 19).astype(np.float32) - (i % 6).astype(np.float32)) * np.float32(1.1)
    got = capi.psv(name + "_psv", simd, data)
    with np.errstate(all="ignore"):
        want = np.array([ref(float(v)) if (name != "log" or v > 0) else np.nan
                         for v in data], np.float64).astype(np.float32)
    ok = np.isfinite(want)
    # a finite reference needs a finite result (a NaN-producing kernel must
    # not hide behind the reference's non-finite-skip rule, mathfun.cc:59-73)
    assert np.isfinite(got[ok]).all()
    assert (_ulps(got[ok], want[ok]) <= 4).all()


@pytest.mark.gpu
def test_mathfun_gpu_wide_range():
    import torch
    from veles.simd_amd import ops
    x = torch.linspace(-100, 100, 1 << 20)
    for fn in ("sin", "cos", "exp"):
        got = getattr(ops, fn)(x.cuda()).cpu()
        want = getattr(torch, fn)(x.double()).float()
        ok = want.isfinite()
        assert (_ulps(got[ok].numpy(), want[ok].numpy()) <= 4).all(), fn
    xp = torch.linspace(1e-6, 1e6, 1 << 20)
    got = ops.log(xp.cuda()).cpu()
    assert (_ulps(got.numpy(), torch.log(xp.double()).float().numpy()) <= 4).all()


def _data(length):
    i = np.arange(length)
    return ((i % 19).astype(np.float32) - (i % 6).astype(np.float32)) * np.float32(1.1)


@pytest.mark.parametrize("simd", SIMDS)
@pytest.mark.parametrize("length", [1, 3, 64, 199, 100003])
def test_sqrt_psv(simd, length):
    """neon_mathfun.h sqrt_ps (:314-332) over arrays; correctly rounded."""
    data = np.abs(_data(length)) * np.float32(3.7)
    got = capi.psv("sqrt_psv", simd, data)
    want = np.sqrt(data.astype(np.float64)).astype(np.float32)
    assert np.isfinite(got).all()
    assert (_ulps(got, want) <= 1).all()


@pytest.mark.parametrize("simd", SIMDS)
@pytest.mark.parametrize("length", [1, 3, 64, 199, 100003])
def test_sincos_psv(simd, length):
    """avx_mathfun.h sincos256_ps (:571) over arrays: both outputs <= 4 ulp."""
    data = _data(length)
    s, c = capi.sincos_psv(simd, data)
    ws = np.array([math.sin(float(v)) for v in data], np.float64).astype(np.float32)
    wc = np.array([math.cos(float(v)) for v in data], np.float64).astype(np.float32)
    assert np.isfinite(s).all() and np.isfinite(c).all()
    assert (_ulps(s, ws) <= 4).all() and (_ulps(c, wc) <= 4).all()


@pytest.mark.parametrize("simd", SIMDS)
@pytest.mark.parametrize("length", [1, 3, 64, 199, 100003])
def test_pow_psv(simd, length):
    """avx_mathfun.h pow256_ps (:720) over arrays, <= 4 ulp vs double."""
    i = np.arange(length)
    x = (np.abs(_data(length)) + np.float32(0.25)).astype(np.float32)
    y = (((i % 13).astype(np.float32) - 6) * np.float32(0.7)).astype(np.float32)
    got = capi.pow_psv(simd, x, y)
    want = np.array([math.pow(float(a), float(b)) for a, b in zip(x, y)], np.float64)
    want = want.astype(np.float32)
    ok = np.isfinite(want)
    assert np.isfinite(got[ok]).all()
    u = _ulps(got[ok], want[ok])
    worst = int(np.argmax(u))
    assert u.max() <= 4, (int(u.max()), float(x[ok][worst]), float(y[ok][worst]),
                          float(got[ok][worst]), float(want[ok][worst]))


@pytest.mark.gpu
def test_math_ops_device_api():
    """torch custom ops on device tensors: sqrt / pow / sincos (incl. a
    16-byte-unaligned sincos view) against float64 torch."""
    import torch
    from veles.simd_amd import ops
    x = torch.linspace(-50, 50, (1 << 20) + 3, device="cuda")
    s, c = ops.sincos(x)
    assert (_ulps(s.cpu().numpy(), torch.sin(x.double()).float().cpu().numpy()) <= 4).all()
    assert (_ulps(c.cpu().numpy(), torch.cos(x.double()).float().cpu().numpy()) <= 4).all()
    s1, c1 = ops.sincos(x[1:])
    assert torch.equal(s1, s[1:]) and torch.equal(c1, c[1:])
    xp = x.abs() + 0.5
    assert (_ulps(ops.sqrt(xp).cpu().numpy(), torch.sqrt(xp.double()).float().cpu().numpy())
            <= 1).all()
    y = torch.linspace(-3, 3, x.numel(), device="cuda")
    got = ops.pow(xp, y).cpu().numpy()
    want = torch.pow(xp.double(), y.double()).float().cpu().numpy()
    assert (_ulps(got, want) <= 4).all()


@pytest.mark.gpu
def test_device_math_header_composes():
    """<simd/device_math.h> from a kernel that includes nothing else of the
    library (csrc/kernels/device_math_user.hip): a Morlet atom and a log-power
    feature against float64."""
    import ctypes
    import torch
    from veles.simd_amd import _lib
    t = torch.linspace(-6, 6, 100001, device="cuda")
    mor = torch.empty_like(t)
    feat = torch.empty_like(t)
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    _lib.call("vs_device_math_example", t.data_ptr(), 5.0, 1.5, t.numel(), mor.data_ptr(),
              feat.data_ptr(), s)
    td = t.double()
    ref_m = torch.exp(-0.5 * td * td) * torch.cos(5.0 * td)
    ref_f = torch.log(1 + torch.sqrt(td.abs() ** 1.5))
    # cos(5 t) carries the float rounding of 5 t (|5 t| <= 30: 2e-6 absolute)
    assert (mor.double() - ref_m).abs().max().item() < 4e-6
    # 1 + sqrt(.) is rounded to float before the log: 6e-8 absolute
    assert (feat.double() - ref_f).abs().max().item() < 5e-7
