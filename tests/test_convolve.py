"""Port of reference tests/convolve.cc and tests/correlate.cc + GPU checks
of the batched device API against an fp64 reference."""
import numpy as np
import pytest

from veles.simd_amd import capi

SIMDS = [0, pytest.param(1, marks=pytest.mark.gpu)]
X8 = [1, 2, 3, 4, 5, 6, 7, 8]
H4 = [10, 9, 8, 7]


def _sin_x(n):
    return (np.sin(np.arange(n, dtype=np.float32)) * 100).astype(np.float32)


def _ramp_h(n):
    return (np.arange(n, dtype=np.float32) / np.float32(n - 1.0)).astype(np.float32)


def _ref(x, h, corr=False):
    x = np.asarray(x, np.float64)
    h = np.asarray(h, np.float64)
    return np.convolve(x, h[::-1] if corr else h)


@pytest.mark.parametrize("simd", SIMDS)
def test_convolve_reference_golden(simd):
    z = capi.convolve_simd(simd, X8, H4)
    np.testing.assert_allclose(z, [10, 29, 56, 90, 124, 158, 192, 226, 170, 113, 56],
                               atol=1e-4)


@pytest.mark.parametrize("simd", SIMDS)
def test_correlate_reference_golden(simd):
    z = capi.convolve_simd(simd, X8, H4, correlate=True)
    np.testing.assert_allclose(z, [7, 22, 46, 80, 114, 148, 182, 216, 187, 142, 80],
                               atol=1e-4)


@pytest.mark.parametrize("prefix,xlen,hlen,tol,corr", [
    ("convolve_fft", 1020, 50, 1e-3, False),
    ("convolve_overlap_save", 1021, 50, 1e-3, False),
    ("cross_correlate_fft", 1020, 50, 1e-3, True),
    ("cross_correlate_overlap_save", 1021, 50, 1e-3, True),
])
def test_handles_vs_brute(prefix, xlen, hlen, tol, corr):
    # reference tolerance: delta^2 <= 1e-6 (convolve.cc:96-103), 1e-3 (correlate.cc)
    x, h = _sin_x(xlen), _ramp_h(hlen)
    res, _ = capi.run_handle(prefix, x, h)
    verif = capi.convolve_simd(0, x, h, correlate=corr)
    assert np.abs(res - verif).max() <= tol


@pytest.mark.gpu
@pytest.mark.parametrize("xlen,hlen", [(16384, 64), (20000, 333)])
def test_convolve_simd_gpu_direct_host_api(xlen, hlen):
    """Above VELES_HOST_MAX_MACS the simd=1 host API stages to the GPU
    direct kernel (smaller calls stay on the host reference by design)."""
    x, h = _sin_x(xlen), _ramp_h(hlen)
    np.testing.assert_allclose(capi.convolve_simd(1, x, h), _ref(x, h), atol=5e-3)
    np.testing.assert_allclose(capi.convolve_simd(1, x, h, True), _ref(x, h, True),
                               atol=5e-3)


@pytest.mark.parametrize("simd", SIMDS)
def test_convolve_simd_1024x50(simd):
    x, h = _sin_x(1024), _ramp_h(50)
    np.testing.assert_allclose(capi.convolve_simd(simd, x, h), _ref(x, h), atol=2e-3)
    np.testing.assert_allclose(capi.convolve_simd(simd, x, h, True), _ref(x, h, True),
                               atol=2e-3)


@pytest.mark.parametrize("xlen,hlen", [(100, 10), (300, 200), (1000, 50),
                                       (2000, 950), (5000, 4000)])
@pytest.mark.parametrize("corr", [False, True])
def test_auto_select(xlen, hlen, corr):
    x, h = _sin_x(xlen), _ramp_h(hlen)
    prefix = "cross_correlate" if corr else "convolve"
    res, handle = capi.run_handle(prefix, x, h)
    ref = _ref(x, h, corr)
    assert np.abs(res - ref).max() <= 2e-6 * np.abs(ref).max() * np.log2(len(ref)) + 2e-3


@pytest.mark.gpu
@pytest.mark.parametrize("algo", [1, 2, 3])
@pytest.mark.parametrize("xlen,hlen,batch", [(4096, 64, 3), (20000, 1000, 2),
                                             (50000, 4096, 2), (777, 300, 5)])
def test_device_conv1d_algorithms(algo, xlen, hlen, batch):
    import torch
    from veles.simd_amd import ops
    if algo == 3 and hlen >= xlen // 2:
        pytest.skip("overlap-save needs h < x/2")
    g = torch.Generator().manual_seed(xlen + hlen)
    x = torch.randn(batch, xlen, generator=g)
    h = torch.randn(hlen, generator=g)
    for corr in (False, True):
        y = ops.conv1d(x.cuda(), h.cuda(), algorithm=algo, correlate=corr).cpu().double()
        ref = np.stack([_ref(x[b].numpy(), h.numpy(), corr) for b in range(batch)])
        err = np.abs(y.numpy() - ref).max()
        scale = np.abs(ref).max()
        assert err <= 1e-5 * scale + 1e-4, (algo, corr, err, scale)


@pytest.mark.gpu
def test_device_conv1d_per_signal_filters_and_large_fft():
    import torch
    from veles.simd_amd import ops
    g = torch.Generator().manual_seed(7)
    x = torch.randn(3, 30000, generator=g)
    h = torch.randn(3, 20000, generator=g)        # x <= 2h -> FFT, 2^16 (four-step)
    y = ops.conv1d(x.cuda(), h.cuda()).cpu().double().numpy()
    for b in range(3):
        ref = _ref(x[b].numpy(), h[b].numpy())
        assert np.abs(y[b] - ref).max() <= 1e-5 * np.abs(ref).max()
    hs = torch.randn(3, 500, generator=g)          # per-signal, overlap-save
    y = ops.conv1d(x.cuda(), hs.cuda(), algorithm=3).cpu().double().numpy()
    for b in range(3):
        ref = _ref(x[b].numpy(), hs[b].numpy())
        assert np.abs(y[b] - ref).max() <= 1e-5 * np.abs(ref).max()


@pytest.mark.gpu
@pytest.mark.parametrize("n", [2, 8, 16, 64, 1024, 4096, 16384, 1 << 15, 1 << 18, 1 << 21])
def test_fft_c2c_vs_numpy(n):
    import torch
    from veles.simd_amd import ops
    batch = max(1, min(4, (1 << 22) // n))
    g = torch.Generator().manual_seed(n)
    z = torch.randn(batch, n, 2, generator=g)
    zc = z[..., 0].double() + 1j * z[..., 1].double()
    f = ops.fft(z.cuda()).cpu().double()
    ref = np.fft.fft(zc.numpy(), axis=-1)
    got = f[..., 0].numpy() + 1j * f[..., 1].numpy()
    assert np.abs(got - ref).max() <= 2e-6 * np.sqrt(n) * np.log2(max(n, 2)) * 4
    inv = ops.fft(f.float().cuda(), inverse=True).cpu().double() / n
    np.testing.assert_allclose(inv.numpy(), z.double().numpy(), atol=2e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [4, 64, 2048, 1 << 16])
def test_rfft_irfft(n):
    import torch
    from veles.simd_amd import ops
    g = torch.Generator().manual_seed(n + 1)
    x = torch.randn(3, n, generator=g)
    X = ops.rfft(x.cuda()).cpu().double()
    ref = np.fft.rfft(x.double().numpy(), axis=-1)
    got = X[..., 0].numpy() + 1j * X[..., 1].numpy()
    assert np.abs(got - ref).max() <= 1e-5 * np.sqrt(n) * np.log2(n) + 1e-5
    back = ops.irfft(X.float().cuda(), n).cpu().double() / n
    np.testing.assert_allclose(back.numpy(), x.double().numpy(), atol=3e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("knobs", [{}, {"conv_buffer": 0}])
@pytest.mark.parametrize("hlen", [300, 4096])
def test_device_conv1d_many_blocks(knobs, hlen):
    """Overlap-save with more block pairs than CUs and a ragged last block,
    buffer-descriptor and flat addressing; float64 FFT reference."""
    import torch
    from veles.simd_amd import _lib, ops
    lib = _lib.lib()
    g = torch.Generator().manual_seed(hlen)
    x = torch.randn(24, 300001, generator=g)
    h = torch.randn(hlen, generator=g)
    try:
        for k, v in knobs.items():
            _lib.check(lib.vs_tune_set(k.encode(), v), k)
        y = ops.conv1d(x.cuda(), h.cuda(), algorithm=3).cpu().double().numpy()
    finally:
        _lib.check(lib.vs_tune_set(b"conv_buffer", 1))
    n = x.shape[1] + hlen - 1
    m = 1 << (n - 1).bit_length()
    ref = np.fft.irfft(np.fft.rfft(x.double().numpy(), m) * np.fft.rfft(h.double().numpy(), m), m)[:, :n]
    assert np.abs(y - ref).max() <= 1e-5 * np.abs(ref).max()
