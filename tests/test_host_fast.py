"""Vectorised host loops for calls too small for a GPU round trip
(csrc/ref/host_fast.cpp) against the scalar host reference (`simd = 0`, `_na`).

The calls below stay under VELES_HOST_MAX_MACS / VELES_GPU_MIN_ELEMS, so they run
the host loops on a GPU box too.  Reference counterparts: the AVX loops of
/root/reference/src/convolve.c:49-100 and src/wavelet.c:395-1555."""
import numpy as np
import pytest

from veles.simd_amd import capi

WAVELETS = [(0, o) for o in (2, 4, 6, 8, 12, 16, 20, 38, 76)] + \
           [(1, o) for o in (6, 12, 18, 24, 30)] + [(2, o) for o in (4, 8, 16, 20)]


def _rng(seed):
    return np.random.default_rng(seed)


@pytest.mark.parametrize("xlen,hlen", [
    (1, 1), (7, 3), (3, 7), (64, 23), (23, 64),          # tap-by-tap accumulation
    (200, 50), (1000, 50), (50, 1000),                    # register-blocked outputs
    (512, 512), (24, 24), (63, 65), (64, 64), (65, 63), (129, 24), (700, 700)])
@pytest.mark.parametrize("correlate", [False, True])
def test_direct_matches_scalar_reference(xlen, hlen, correlate):
    rng = _rng(xlen * 1000 + hlen)
    x = rng.standard_normal(xlen).astype(np.float32)
    h = rng.standard_normal(hlen).astype(np.float32)
    fast = capi.convolve_simd(1, x, h, correlate)
    slow = capi.convolve_simd(0, x, h, correlate)
    want = np.convolve(x.astype(np.float64), h[::-1].astype(np.float64) if correlate
                       else h.astype(np.float64))
    assert fast.shape == slow.shape == want.shape
    tol = 4e-6 * min(xlen, hlen) ** 0.5 * 8
    np.testing.assert_allclose(fast, want, atol=tol)
    np.testing.assert_allclose(fast, slow, atol=tol)


@pytest.mark.parametrize("type_,order", WAVELETS)
@pytest.mark.parametrize("ext", [0, 1, 2, 3])
def test_dwt_matches_scalar_reference(type_, order, ext):
    for n in (order + (order & 1), 64, 130, 512):
        if n < order:
            continue
        src = _rng(n + order).standard_normal(n).astype(np.float32)
        hi, lo = capi.wavelet_apply(type_, order, ext, src)
        hi0, lo0 = capi.wavelet_apply(type_, order, ext, src, na=True)
        np.testing.assert_allclose(hi, hi0, atol=2e-5)
        np.testing.assert_allclose(lo, lo0, atol=2e-5)


@pytest.mark.parametrize("type_,order", [(0, 4), (0, 8), (0, 16), (1, 12), (2, 6)])
@pytest.mark.parametrize("ext", [0, 1, 2, 3])
@pytest.mark.parametrize("level", [1, 2, 3, 5])
def test_swt_matches_scalar_reference(type_, order, ext, level):
    for n in (64, 257, 512):
        src = _rng(n + level).standard_normal(n).astype(np.float32)
        hi, lo = capi.stationary_wavelet_apply(type_, order, level, ext, src)
        hi0, lo0 = capi.stationary_wavelet_apply(type_, order, level, ext, src, na=True)
        np.testing.assert_allclose(hi, hi0, atol=2e-5)
        np.testing.assert_allclose(lo, lo0, atol=2e-5)


def _child(code, **env):
    import os
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    e = dict(os.environ, **env)
    e.pop("VELES_HOST_SMALL_SCALE", None)       # the shipped default policy
    e["PYTHONPATH"] = repo + os.pathsep + e.get("PYTHONPATH", "")   # whatever the cwd is
    e.update(env)
    r = subprocess.run([sys.executable, "-c", code], env=e, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    return r.stdout + r.stderr


_SMALL_CALLS = r"""
import numpy as np
from veles.simd_amd import capi
rng = np.random.default_rng(5)
a = rng.standard_normal((37, 53)).astype(np.float32)
b = rng.standard_normal((37, 53)).astype(np.float32)
np.testing.assert_array_equal(capi.matrix_add(1, a, b, 53, 37), (a + b).ravel())
np.testing.assert_array_equal(capi.matrix_sub(1, a, b, 53, 37), (a - b).ravel())
m1 = rng.standard_normal((19, 45)).astype(np.float32)     # h1 x w1
m2 = rng.standard_normal((45, 31)).astype(np.float32)     # w1 x w2
got = capi.matrix_multiply(1, m1, m2, 45, 19, 31, 45).reshape(19, 31)
np.testing.assert_allclose(got, m1.astype(np.float64) @ m2.astype(np.float64), atol=2e-5)
m2t = np.ascontiguousarray(m2.T)                            # h2 x w2 = 31 x 45
got = capi.matrix_multiply_transposed(1, m1, m2t, 45, 19, 45, 31).reshape(19, 31)
np.testing.assert_allclose(got, m1.astype(np.float64) @ m2.astype(np.float64), atol=2e-5)
# 4 x 16 register blocks with axpy / dot remainders: every combination of tails
for h1, w1, w2 in ((4, 7, 16), (5, 9, 17), (8, 64, 32), (3, 20, 100), (64, 64, 64), (37, 53, 29),
                   (12, 1, 48), (9, 33, 15), (16, 100, 16), (7, 5, 31), (100, 120, 110),
                   (1, 300, 1000), (130, 90, 3)):
    m1 = rng.standard_normal((h1, w1)).astype(np.float32)
    m2 = rng.standard_normal((w1, w2)).astype(np.float32)
    want = m1.astype(np.float64) @ m2.astype(np.float64)
    got = capi.matrix_multiply(1, m1, m2, w1, h1, w2, w1).reshape(h1, w2)
    np.testing.assert_allclose(got, want, atol=3e-5, err_msg=str((h1, w1, w2)))
    got = capi.matrix_multiply_transposed(1, m1, np.ascontiguousarray(m2.T), w1, h1, w1, w2)
    np.testing.assert_allclose(got.reshape(h1, w2), want, atol=3e-5, err_msg=str((h1, w1, w2)))
import ctypes
img = rng.integers(0, 256, (40, 50), dtype=np.uint8)
mn, mx = ctypes.c_uint8(), ctypes.c_uint8()
capi.fn("minmax2D")(1, capi.p(img), 50, 50, 40, ctypes.byref(mn), ctypes.byref(mx))
assert (mn.value, mx.value) == (img.min(), img.max())
n1, n0 = np.empty((40, 50), np.float32), np.empty((40, 50), np.float32)
capi.fn("normalize2D")(1, capi.p(img), 50, 50, 40, capi.p(n1), 50)
capi.fn("normalize2D")(0, capi.p(img), 50, 50, 40, capi.p(n0), 50)
np.testing.assert_array_equal(n1, n0)
sig = rng.standard_normal(5000).astype(np.float32)
p1, p0 = capi.detect_peaks(1, sig, 3), capi.detect_peaks(0, sig, 3)
assert len(p1) == len(p0) > 100 and p1 == p0
fmn, fmx = ctypes.c_float(), ctypes.c_float()
capi.fn("minmax1D")(1, capi.p(sig), sig.size, ctypes.byref(fmn), ctypes.byref(fmx))
assert (fmn.value, fmx.value) == (sig.min(), sig.max())
# glibc's vector math on the host (at most 4 ulp off libm), every tail length
for n in (1, 7, 8, 9, 300, 1001):
    x = rng.uniform(0.1, 3.0, n).astype(np.float32)
    for name in ("sin_psv", "cos_psv", "exp_psv", "log_psv", "sqrt_psv"):
        fast, libm = capi.psv(name, 1, x).astype(np.float64), capi.psv(name, 0, x).astype(np.float64)
        assert (np.abs(fast - libm) <= 5e-7 * np.abs(libm) + 5e-7).all(), (name, n)
    np.testing.assert_array_equal(capi.psv("sqrt_psv", 1, x), capi.psv("sqrt_psv", 0, x))
    y = rng.uniform(-2.0, 2.0, n).astype(np.float32)
    fast, libm = capi.pow_psv(1, x, y).astype(np.float64), capi.pow_psv(0, x, y).astype(np.float64)
    assert (np.abs(fast - libm) <= 5e-7 * np.abs(libm)).all(), n
    s1, c1 = capi.sincos_psv(1, x)
    s0, c0 = capi.sincos_psv(0, x)
    assert np.abs(s1 - s0).max() <= 3e-7 and np.abs(c1 - c0).max() <= 3e-7, n
# special values follow IEEE as libm does
sp = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, -1.0, 1e-45, 3e38, 88.8, -104.0], np.float32)
with np.errstate(all="ignore"):
    for name in ("exp_psv", "log_psv", "sqrt_psv", "sin_psv", "cos_psv"):
        fast, libm = capi.psv(name, 1, sp), capi.psv(name, 0, sp)
        assert np.array_equal(np.isnan(fast), np.isnan(libm)), (name, fast, libm)
        assert np.array_equal(np.isinf(fast), np.isinf(libm)), (name, fast, libm)
        ok = np.isfinite(libm)
        assert (np.abs(fast[ok].astype(np.float64) - libm[ok]) <= 5e-7 * np.abs(libm[ok]) + 1e-44).all(), name
    px = np.array([-2, -2, 0, 0, 2, np.inf, np.nan, 1, -0.0, 1e30, 1e-30, -8, 3, 5, 7, 9], np.float32)
    py = np.array([3, 0.5, 0, -1, 0.5, -1, 0, np.nan, -3, 5, 5, 1 / 3, 2, 2, 2, 2], np.float32)
    fast, libm = capi.pow_psv(1, px, py), capi.pow_psv(0, px, py)
    assert np.array_equal(np.isnan(fast), np.isnan(libm)) and np.array_equal(np.isinf(fast), np.isinf(libm))
    ok = np.isfinite(libm)
    np.testing.assert_allclose(fast[ok], libm[ok], rtol=1e-6)
print("small calls ok")
"""


def test_small_matrix_and_math_calls_run_host_loops():
    """Default policy: the small simd = 1 calls give the host results (vector math within
    4 ulp of libm) and never report a GPU call in the level-2 log."""
    out = _child(_SMALL_CALLS, VELES_LOG_LEVEL="2")
    assert "small calls ok" in out
    assert "done on GPU" not in out


_STREAMING_CALLS = r"""
import ctypes
import numpy as np
from veles.simd_amd import capi
rng = np.random.default_rng(9)
sz = ctypes.c_size_t
# sums and differences, conversions, products: the host at every size
n = 1500
a = rng.standard_normal((n, n)).astype(np.float32)
b = rng.standard_normal((n, n)).astype(np.float32)
np.testing.assert_array_equal(capi.matrix_add(1, a, b, n, n), (a + b).ravel())
np.testing.assert_array_equal(capi.matrix_sub(1, a, b, n, n), (a - b).ravel())
m = (1 << 21) + 7
x, y, z = a.ravel()[:m], b.ravel()[:m], np.empty(m, np.float32)
capi.fn("real_multiply_array")(capi.p(x), capi.p(y), sz(m), capi.p(z))
np.testing.assert_array_equal(z, x * y)
i16 = rng.integers(-30000, 30000, m).astype(np.int16)
capi.fn("int16_to_float")(capi.p(i16), sz(m), capi.p(z))
np.testing.assert_array_equal(z, i16.astype(np.float32))
# reductions: eight-lane partial sums / lane-wise extremes
for k in (1, 7, 15, 16, 31, 32, 33, 1000, m):
    v = x[:k]
    got = capi.fn("sum_elements")(capi.p(v), sz(k))
    want = float(v.astype(np.float64).sum())
    assert abs(got - want) <= 2e-6 * float(np.abs(v).astype(np.float64).sum()) + 1e-6, (k, got, want)
    lo, hi = ctypes.c_float(), ctypes.c_float()
    capi.fn("minmax1D")(1, capi.p(v), k, ctypes.byref(lo), ctypes.byref(hi))
    assert (lo.value, hi.value) == (v.min(), v.max()), k
w = x[:100].copy(); w[17] = np.nan                       # NaNs lose every comparison
lo, hi = ctypes.c_float(), ctypes.c_float()
capi.fn("minmax1D")(1, capi.p(w), 100, ctypes.byref(lo), ctypes.byref(hi))
l0, h0 = ctypes.c_float(), ctypes.c_float()
capi.fn("minmax1D")(0, capi.p(w), 100, ctypes.byref(l0), ctypes.byref(h0))
assert (lo.value, hi.value) == (l0.value, h0.value)
# normalisation
img = rng.integers(0, 256, (700, 900), dtype=np.uint8)
n1, n0 = np.empty((700, 900), np.float32), np.empty((700, 900), np.float32)
capi.fn("normalize2D")(1, capi.p(img), 900, 900, 700, capi.p(n1), 900)
capi.fn("normalize2D")(0, capi.p(img), 900, 900, 700, capi.p(n0), 900)
np.testing.assert_array_equal(n1, n0)
# extrema: two-pass host scan, every kind, plateaus and short arrays
for k in (3, 4, 5, 64, 1000, 100000):
    sig = np.round(rng.standard_normal(k) * 3).astype(np.float32)   # many equal neighbours
    for kind in (1, 2, 3):
        assert capi.detect_peaks(1, sig, kind) == capi.detect_peaks(0, sig, kind), (k, kind)
# eight-tap wavelets stay on the host at any length
src = rng.standard_normal(1 << 19).astype(np.float32)
hi1, lo1 = capi.wavelet_apply(0, 8, 0, src)
hi0, lo0 = capi.wavelet_apply(0, 8, 0, src, na=True)
np.testing.assert_allclose(hi1, hi0, atol=2e-5)
np.testing.assert_allclose(lo1, lo0, atol=2e-5)
print("streaming calls ok")
"""


def test_streaming_calls_on_host_arrays_stay_on_the_host():
    """Default policy: calls that move more than they compute never take the GPU round trip
    for host operands, whatever their size (on a GPU box too), and match the scalar paths."""
    out = _child(_STREAMING_CALLS, VELES_LOG_LEVEL="2")
    assert "streaming calls ok" in out
    assert "done on GPU" not in out


@pytest.mark.gpu
def test_larger_calls_still_reach_the_gpu():
    code = r"""
import numpy as np
from veles.simd_amd import capi
a = np.ones((200, 200), np.float32)
capi.matrix_multiply(1, a, a, 200, 200, 200, 200)
capi.psv("sin_psv", 1, np.ones((1 << 20) + 3, np.float32))
capi.detect_peaks(1, np.random.default_rng(0).standard_normal(400000).astype(np.float32), 3)
capi.wavelet_apply(0, 16, 0, np.ones(1 << 18, np.float32))
capi.wavelet_apply(0, 76, 0, np.ones(1 << 14, np.float32))
"""
    out = _child(code, VELES_LOG_LEVEL="2")
    for what in ("matrix_multiply", "sin_psv", "detect_peaks", "wavelet_apply"):
        assert f"{what}: done on GPU" in out
    assert out.count("wavelet_apply: done on GPU") == 2
