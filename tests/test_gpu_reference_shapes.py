"""The reference's own test sweeps and goldens, run through the DEVICE kernels.

The sweeps in test_wavelet.py / test_convolve.py use
the reference's shapes (512-sample signals, 1020 x 50 convolutions), which
are below the host-API GPU thresholds, so both sides of those comparisons
ran the host reference.  Here the same cases go straight to the device API
(vs_dwt / vs_swt / vs_conv1d on device pointers), and once more through the
host C API with the thresholds forced to zero (VELES_GPU_MIN_ELEMS=0,
VELES_HOST_MAX_MACS=0) in a child process.

Reference: /root/reference/tests/wavelet.cc:252-288 (DWT / SWT sweeps),
tests/convolve.cc:53-71 and tests/correlate.cc:53-71 (goldens),
tests/convolve.cc:96-103 (tolerances).
"""
import os
import subprocess
import sys

import numpy as np
import pytest

from veles.simd_amd import capi

pytestmark = pytest.mark.gpu

D, C, S = capi.WAVELET_TYPE_DAUBECHIES, capi.WAVELET_TYPE_COIFLET, capi.WAVELET_TYPE_SYMLET
EXTS = [0, 1, 2, 3]
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _dwt_params():
    out = [(t, o, e) for t in (D, S) for o in (2, 4, 6, 8, 12, 16) for e in EXTS]
    return out + [(C, o, e) for o in (6, 12) for e in EXTS]


def _swt_params():
    out = [(t, o, l, e) for t in (D, S) for o in (2, 4, 6, 8, 12, 16)
           for l in (1, 2, 3, 4) for e in EXTS]
    return out + [(C, o, l, e) for o in (6, 12) for l in (1, 2) for e in EXTS]


def _stream():
    import torch
    return torch.cuda.current_stream().cuda_stream


@pytest.mark.parametrize("t,o,e", _dwt_params())
def test_dwt_sweep_device(t, o, e):
    """All 56 DWT cases of the reference sweep on vs_dwt (device pointers)."""
    import torch
    from veles.simd_amd import _lib
    x = torch.arange(512, dtype=torch.float32, device="cuda")
    hi = torch.full((256,), float("nan"), device="cuda")
    lo = torch.full((256,), float("nan"), device="cuda")
    _lib.call("vs_dwt", t, o, e, x.data_ptr(), 512, 0, hi.data_ptr(), lo.data_ptr(), 0, 1,
              _stream())
    vhi, vlo = capi.wavelet_apply(t, o, e, np.arange(512, dtype=np.float32), na=True)
    np.testing.assert_allclose(hi.cpu().numpy(), vhi, atol=5e-4)
    np.testing.assert_allclose(lo.cpu().numpy(), vlo, atol=5e-4)


@pytest.mark.parametrize("t,o,l,e", _swt_params())
def test_swt_sweep_device(t, o, l, e):
    """All 208 SWT cases of the reference sweep on vs_swt (device pointers)."""
    import torch
    from veles.simd_amd import _lib
    x = torch.arange(512, dtype=torch.float32, device="cuda")
    hi = torch.full((512,), float("nan"), device="cuda")
    lo = torch.full((512,), float("nan"), device="cuda")
    _lib.call("vs_swt", t, o, l, e, x.data_ptr(), 512, 0, hi.data_ptr(), lo.data_ptr(), 0, 1,
              _stream())
    vhi, vlo = capi.stationary_wavelet_apply(t, o, l, e, np.arange(512, dtype=np.float32),
                                             na=True)
    np.testing.assert_allclose(hi.cpu().numpy(), vhi, atol=5e-4)
    np.testing.assert_allclose(lo.cpu().numpy(), vlo, atol=5e-4)


ALGOS = ["direct", "fft", "overlap_save"]


def _conv_dev(x, h, algo, corr):
    import torch
    from veles.simd_amd import ops
    y = ops.conv1d(torch.tensor(np.asarray(x, np.float32)).cuda(),
                   torch.tensor(np.asarray(h, np.float32)).cuda(), algorithm=algo,
                   correlate=corr)
    return y.cpu().double().numpy()


@pytest.mark.parametrize("algo", ALGOS)
def test_conv_goldens_device(algo):
    """reference tests/convolve.cc:53-71, correlate.cc:53-71 on every kernel."""
    x8, h4 = [1, 2, 3, 4, 5, 6, 7, 8], [10, 9, 8, 7]
    if algo == "overlap_save":   # OS needs h < x/2; pad x (the leading outputs are equal)
        x = x8 + [0] * 8
        np.testing.assert_allclose(_conv_dev(x, h4, algo, False)[:11],
                                   [10, 29, 56, 90, 124, 158, 192, 226, 170, 113, 56],
                                   atol=1e-4)
        return
    np.testing.assert_allclose(_conv_dev(x8, h4, algo, False),
                               [10, 29, 56, 90, 124, 158, 192, 226, 170, 113, 56], atol=1e-4)
    np.testing.assert_allclose(_conv_dev(x8, h4, algo, True),
                               [7, 22, 46, 80, 114, 148, 182, 216, 187, 142, 80], atol=1e-4)


@pytest.mark.parametrize("algo", ALGOS)
@pytest.mark.parametrize("xlen,hlen", [(1020, 50), (1021, 50), (1024, 50), (512, 512)])
@pytest.mark.parametrize("corr", [False, True])
def test_conv_reference_shapes_device(algo, xlen, hlen, corr):
    """The reference's handle / brute-force shapes (convolve.cc:96-103,
    :171-216) on each device kernel, against fp64 numpy."""
    if algo == "overlap_save" and not hlen < xlen // 2:
        pytest.skip("overlap-save requires h < x/2 (reference contract)")
    x = (np.sin(np.arange(xlen, dtype=np.float32)) * 100).astype(np.float32)
    h = (np.arange(hlen, dtype=np.float32) / np.float32(hlen - 1.0)).astype(np.float32)
    ref = np.convolve(x.astype(np.float64), (h[::-1] if corr else h).astype(np.float64))
    got = _conv_dev(x, h, algo, corr)
    assert np.abs(got - ref).max() <= 1e-3 * max(1.0, np.abs(ref).max() / 100)


def test_host_api_sweeps_forced_to_gpu():
    """test_wavelet.py + test_convolve.py (reference sweeps and goldens) through
    the host C API with every size threshold at zero, so each call stages its
    host operands to the GPU kernels (a child process: the thresholds are read
    once per process)."""
    env = dict(os.environ, VELES_GPU_MIN_ELEMS="0", VELES_HOST_MAX_MACS="0")
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-p", "no:cacheprovider",
                        "tests/test_wavelet.py", "tests/test_convolve.py",
                        "-k", "vs_na or golden or 1024x50 or handles_vs_brute or auto_select"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]
    assert " passed" in r.stdout


def test_int16_multiply_device():
    """K16: vs_int16_multiply on device pointers (reference arithmetic.h
    int16_multiply widens to int32), ragged length past the vector width."""
    import torch
    from veles.simd_amd import _lib
    g = torch.Generator().manual_seed(16)
    n = 100003
    a = torch.randint(-32768, 32767, (n,), generator=g, dtype=torch.int16)
    b = torch.randint(-32768, 32767, (n,), generator=g, dtype=torch.int16)
    out = torch.zeros(n, dtype=torch.int32, device="cuda")
    ad, bd = a.cuda(), b.cuda()
    _lib.call("vs_int16_multiply", ad.data_ptr(), bd.data_ptr(), out.data_ptr(), n, _stream())
    assert torch.equal(out.cpu(), a.to(torch.int32) * b.to(torch.int32))
