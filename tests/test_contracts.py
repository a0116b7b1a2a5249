"""Contract (death) tests: the host C API aborts with a message naming the
call on invalid arguments, as the reference's assert() preconditions do
(reference tests use EXPECT_DEATH(..., ".*Assertion.*"), e.g.
tests/arithmetic.cc; preconditions src/matrix.c:255-343,
src/convolve.c:105, src/wavelet.c:83-98).  Each case runs in a child
process on the host path (VELES_DISABLE_GPU=1)."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

PRE = """
import ctypes, numpy as np
from veles.simd_amd import capi
P = capi.p
a = np.ones(64, np.float32); b = np.ones(64, np.float32); r = np.zeros(256, np.float32)
"""

CASES = {
    "matrix_multiply_shape": ("capi.fn('matrix_multiply')(1, P(a), P(b), 4, 4, 4, 3, P(r))",
                              "matrix_multiply"),
    "matrix_multiply_transposed_shape": (
        "capi.fn('matrix_multiply_transposed')(1, P(a), P(b), 4, 4, 3, 4, P(r))",
        "matrix_multiply_transposed"),
    "overlap_save_long_filter": ("capi.fn('convolve_overlap_save_initialize')(100, 60)",
                                 "overlap-save requires"),
    "convolution_empty": ("capi.fn('convolve_fft_initialize')(0, 10)", "empty"),
    "wavelet_odd_length": (
        "capi.fn('wavelet_apply_na')(capi.WAVELET_TYPE_DAUBECHIES, 4, 0, P(a), 63, P(r), P(b))",
        "odd length"),
    "wavelet_bad_order": (
        "capi.fn('wavelet_apply')(capi.WAVELET_TYPE_DAUBECHIES, 7, 0, P(a), 64, P(r), P(b))",
        "unsupported wavelet"),
    "swt_level_zero": (
        "capi.fn('stationary_wavelet_apply_na')(capi.WAVELET_TYPE_DAUBECHIES, 4, 0, 0, P(a), 64,"
        " P(r), P(b))", "level 0"),
    "wavelet_bad_extension": (
        "capi.fn('wavelet_apply_na')(capi.WAVELET_TYPE_DAUBECHIES, 4, 9, P(a), 64, P(r), P(b))",
        "bad extension"),
    "convolve_null": ("capi.fn('convolve_simd')(1, None, 64, P(b), 8, P(r))", "convolve_simd"),
}


@pytest.mark.parametrize("case", sorted(CASES))
def test_precondition_aborts(case):
    call, needle = CASES[case]
    env = dict(os.environ, VELES_DISABLE_GPU="1")
    r = subprocess.run([sys.executable, "-c", PRE + call + "\nprint('returned')"], cwd=ROOT,
                       env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "returned" not in r.stdout, (case, r.stdout, r.stderr[-500:])
    assert "veles.simd: fatal:" in r.stderr and needle in r.stderr, (case, r.stderr[-800:])


def test_valid_call_does_not_abort():
    env = dict(os.environ, VELES_DISABLE_GPU="1")
    r = subprocess.run([sys.executable, "-c", PRE +
                        "capi.fn('matrix_multiply')(1, P(a), P(b), 4, 4, 4, 4, P(r))\n"
                        "print('returned')"], cwd=ROOT, env=env, capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0 and "returned" in r.stdout, r.stderr[-800:]
