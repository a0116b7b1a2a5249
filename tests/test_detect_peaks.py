"""Port of reference tests/detect_peaks.cc + large device checks."""
import numpy as np
import pytest

from veles.simd_amd import capi

SIMDS = [0, pytest.param(1, marks=pytest.mark.gpu)]


@pytest.mark.parametrize("simd", SIMDS)
def test_sin(simd):
    x = np.sin(np.arange(4000) * np.pi / 100).astype(np.float32)
    pts = capi.detect_peaks(simd, x, capi.kExtremumTypeMaximum)
    assert len(pts) == 20
    for i, (p, v) in enumerate(pts):
        assert p == i * 200 + 50 and abs(v - 1.0) < 1e-6
    pts = capi.detect_peaks(simd, x, capi.kExtremumTypeMinimum)
    assert [p for p, _ in pts] == [i * 200 + 150 for i in range(20)]
    pts = capi.detect_peaks(simd, x, capi.kExtremumTypeBoth)
    assert [p for p, _ in pts] == [(i // 2) * 200 + 50 + 100 * (i % 2) for i in range(40)]
    assert all(abs(v - (1.0 - (i % 2) * 2)) < 1e-6 for i, (_, v) in enumerate(pts))


@pytest.mark.parametrize("simd", SIMDS)
def test_nasty_peaks(simd):
    x = np.zeros(101, np.float32)
    x[[7, 16, 97, 99]] = 1
    pts = capi.detect_peaks(simd, x, capi.kExtremumTypeMaximum)
    assert [p for p, _ in pts] == [7, 16, 97, 99]
    assert all(v == 1.0 for _, v in pts)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [3, 4097, 1 << 20])
def test_random_vs_host(n):
    rng = np.random.default_rng(n)
    x = np.round(rng.standard_normal(n) * 4).astype(np.float32)  # plateaus too
    for kind in (1, 2, 3):
        assert capi.detect_peaks(1, x, kind) == capi.detect_peaks(0, x, kind)
