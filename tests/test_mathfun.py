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
    ok = np.isfinite(want) & np.isfinite(got)
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
