"""Randomised differential tests: every op on a CUDA tensor (HIP kernels)
against the same op on the CPU tensor (its float64 torch definition) over
shapes drawn at random with fixed seeds -- sizes that land on and next to the
kernels' tile, block and algorithm boundaries without anyone picking them.
The reference sweeps fixed grids instead (/root/reference/tests/wavelet.cc:60-160,
tests/convolve.cc:60-130)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

FAMILIES = {"daubechies": [2, 4, 6, 8, 10, 12, 16, 20, 24, 30, 38, 76],
            "coiflets": [6, 12, 18, 24, 30], "symlets": [4, 6, 8, 12, 16, 20]}
EXTS = ["periodic", "mirror", "constant", "zero"]


def _loguniform(rng, lo, hi):
    return int(round(np.exp(rng.uniform(np.log(lo), np.log(hi)))))


def _wavelet(rng):
    fam = str(rng.choice(list(FAMILIES)))
    return fam, int(rng.choice(FAMILIES[fam])), str(rng.choice(EXTS))


@pytest.mark.parametrize("seed", range(6))
def test_conv1d_random_shapes(seed):
    import torch
    from veles.simd_amd import ops
    from scipy.signal import fftconvolve
    rng = np.random.default_rng(1000 + seed)
    for case in range(25):
        xlen = _loguniform(rng, 1, 150000)
        hlen = _loguniform(rng, 1, 12000)
        batch = int(rng.integers(1, 4))
        per_signal = bool(rng.integers(0, 2))
        corr = bool(rng.integers(0, 2))
        algo = str(rng.choice(["auto", "auto", "direct", "fft", "overlap_save"]))
        if algo == "direct" and xlen * hlen > 4e7:
            algo = "auto"
        print(f"conv case {seed}/{case}: x={xlen} h={hlen} batch={batch} per_signal={per_signal} "
              f"corr={corr} algo={algo}", flush=True)
        x = rng.standard_normal((batch, xlen)).astype(np.float32)
        h = rng.standard_normal((batch if per_signal else 1, hlen)).astype(np.float32)
        hh = torch.from_numpy(h if per_signal else h[0]).cuda()
        y = ops.conv1d(torch.from_numpy(x).cuda(), hh, algorithm=algo, correlate=corr)
        y = y.cpu().double().numpy()
        for b in range(batch):
            hb = h[b if per_signal else 0].astype(np.float64)
            ref = fftconvolve(x[b].astype(np.float64), hb[::-1] if corr else hb)
            assert y[b].shape == ref.shape
            tol = 1.5e-5 * np.sqrt(min(xlen, hlen)) * np.abs(x[b]).max() * np.abs(hb).max() + 1e-4
            assert np.abs(y[b] - ref).max() <= tol, (xlen, hlen, b, algo, corr)


@pytest.mark.parametrize("seed", range(4))
def test_wavelets_random_shapes(seed):
    import torch
    from veles.simd_amd import ops
    rng = np.random.default_rng(2000 + seed)
    for case in range(30):
        fam, order, ext = _wavelet(rng)
        batch = int(rng.integers(1, 6))
        levels = int(rng.integers(1, 7))
        n = _loguniform(rng, max(4, order // 2), 40000)
        print(f"wavelet case {seed}/{case}: {fam}{order} {ext} n={n} levels={levels} "
              f"batch={batch}", flush=True)
        # stationary: any length
        x = torch.from_numpy(rng.standard_normal((batch, n)).astype(np.float32))
        hi, lo = ops.swt(x.cuda(), fam, order, levels, ext)
        hi0, lo0 = ops.swt(x, fam, order, levels, ext)
        scale = 4e-6 * 2.0 ** levels * order
        assert (hi.cpu() - hi0).abs().max() <= scale, ("swt hi", fam, order, ext, n, levels)
        assert (lo.cpu() - lo0).abs().max() <= scale, ("swt lo", fam, order, ext, n, levels)
        lvl = int(rng.integers(1, 6))
        h1, l1 = ops.swt_level(x.cuda(), fam, order, lvl, ext)
        h0, l0 = ops.swt_level(x, fam, order, lvl, ext)
        assert (h1.cpu() - h0).abs().max() <= 1e-5 * order
        assert (l1.cpu() - l0).abs().max() <= 1e-5 * order
        # decimated: even length for one level, a multiple of 2^levels for the pyramid
        ne = max(2, n & ~1)
        xe = torch.from_numpy(rng.standard_normal((batch, ne)).astype(np.float32))
        d1, a1 = ops.dwt(xe.cuda(), fam, order, ext)
        d0, a0 = ops.dwt(xe, fam, order, ext)
        assert (d1.cpu() - d0).abs().max() <= 1e-5 * order
        assert (a1.cpu() - a0).abs().max() <= 1e-5 * order
        npyr = max(1, n >> levels) << levels
        xp = torch.from_numpy(rng.standard_normal((batch, npyr)).astype(np.float32))
        w1 = ops.wavedec(xp.cuda(), fam, order, levels, ext)
        w0 = ops.wavedec(xp, fam, order, levels, ext)
        assert (w1.cpu() - w0).abs().max() <= scale, ("wavedec", fam, order, ext, npyr, levels)


@pytest.mark.parametrize("seed", range(3))
def test_sgemm_random_shapes(seed):
    import torch
    from veles.simd_amd import ops
    rng = np.random.default_rng(3000 + seed)
    for case in range(40):
        m, n, k = (_loguniform(rng, 1, 1500) for _ in range(3))
        ta, tb = bool(rng.integers(0, 2)), bool(rng.integers(0, 2))
        print(f"sgemm case {seed}/{case}: m={m} n={n} k={k} ta={ta} tb={tb}", flush=True)
        a = torch.from_numpy(rng.uniform(-1, 1, (k, m) if ta else (m, k)).astype(np.float32))
        b = torch.from_numpy(rng.uniform(-1, 1, (n, k) if tb else (k, n)).astype(np.float32))
        c = ops.sgemm(a.cuda(), b.cuda(), ta, tb).cpu().double()
        ref = (a.double().T if ta else a.double()) @ (b.double().T if tb else b.double())
        assert c.shape == ref.shape
        assert (c - ref).abs().max() <= 2e-6 * k + 1e-6, (m, n, k, ta, tb)


@pytest.mark.parametrize("seed", range(3))
def test_elementwise_reduce_peaks_random_sizes(seed):
    import torch
    from veles.simd_amd import ops
    rng = np.random.default_rng(4000 + seed)
    for case in range(20):
        n = _loguniform(rng, 3, 3_000_000)
        print(f"elementwise case {seed}/{case}: n={n}", flush=True)
        x = torch.from_numpy(rng.uniform(0.05, 6.0, n).astype(np.float32))
        y = torch.from_numpy(rng.standard_normal(n).astype(np.float32))
        xg, yg = x.cuda(), y.cuda()
        assert torch.equal(ops.add(xg, yg).cpu(), x + y)
        assert torch.equal(ops.mul(xg, yg).cpu(), x * y)
        for fn, ref in (("sin", torch.sin), ("cos", torch.cos), ("exp", torch.exp),
                        ("log", torch.log), ("sqrt", torch.sqrt)):
            got = ops.math(xg, fn).cpu().double()
            want = ref(x.double())
            assert ((got - want).abs() <= 4e-7 * want.abs() + 5e-7).all(), (fn, n)
        s = ops.sum_all(yg).item()
        assert abs(s - y.double().sum().item()) <= 2e-5 * np.sqrt(n) + 1e-4
        mm = ops.minmax(yg).cpu()
        assert mm[0].item() == y.min().item() and mm[1].item() == y.max().item()
        for kind in (ops.signal.MAXIMUM, ops.signal.MINIMUM, ops.signal.BOTH):
            p1, v1 = ops.detect_peaks(yg, kind)
            p0, v0 = ops.detect_peaks(y, kind)
            assert torch.equal(p1.cpu().long(), p0.long()) and torch.equal(v1.cpu(), v0)
        z = torch.from_numpy(rng.standard_normal(2 * (n // 2 + 1)).astype(np.float32))
        w = torch.from_numpy(rng.standard_normal(2 * (n // 2 + 1)).astype(np.float32))
        got = ops.complex_multiply(z.cuda(), w.cuda()).cpu()
        want = torch.view_as_real(torch.view_as_complex(z.double().reshape(-1, 2)) *
                                  torch.view_as_complex(w.double().reshape(-1, 2))).reshape(-1)
        assert (got.double() - want).abs().max() <= 1e-5
        h = int(rng.integers(1, 300))
        wd = int(rng.integers(1, 300))
        img = torch.from_numpy(rng.integers(0, 256, (h, wd), dtype=np.uint8))
        assert torch.allclose(ops.normalize2d(img.cuda()).cpu(), ops.normalize2d(img), atol=1e-6)


@pytest.mark.parametrize("seed", range(3))
def test_host_c_api_random_shapes(seed):
    """The reference-compatible host API (host pointers staged through the
    runtime) against simd = 0 / numpy on random shapes: small operands in the
    pinned arena, large ones through device staging."""
    from veles.simd_amd import capi
    rng = np.random.default_rng(5000 + seed)
    for case in range(12):
        xlen, hlen = _loguniform(rng, 4, 60000), _loguniform(rng, 1, 3000)
        print(f"capi case {seed}/{case}: conv x={xlen} h={hlen}", flush=True)
        x = rng.standard_normal(xlen).astype(np.float32)
        h = rng.standard_normal(hlen).astype(np.float32)
        for corr in (False, True):
            want = np.convolve(x.astype(np.float64), (h[::-1] if corr else h).astype(np.float64))
            got = capi.convolve_simd(1, x, h, corr)
            tol = 1.5e-5 * np.sqrt(min(xlen, hlen)) * np.abs(x).max() * np.abs(h).max() + 1e-4
            assert np.abs(got - want).max() <= tol, ("convolve_simd", xlen, hlen, corr)
            res, _ = capi.run_handle("cross_correlate" if corr else "convolve", x, h)
            assert np.abs(res - want).max() <= tol, ("handle", xlen, hlen, corr)
        w1, h1, w2 = (_loguniform(rng, 1, 700) for _ in range(3))
        print(f"capi case {seed}/{case}: matmul {h1}x{w1} . {w1}x{w2}", flush=True)
        a = rng.uniform(-1, 1, (h1, w1)).astype(np.float32)
        b = rng.uniform(-1, 1, (w1, w2)).astype(np.float32)
        ref = a.astype(np.float64) @ b.astype(np.float64)
        got = capi.matrix_multiply(1, a, b, w1, h1, w2, w1).reshape(h1, w2)
        assert np.abs(got - ref).max() <= 2e-6 * w1 + 1e-6
        bt = np.ascontiguousarray(b.T)
        got = capi.matrix_multiply_transposed(1, a, bt, w1, h1, w1, w2).reshape(h1, w2)
        assert np.abs(got - ref).max() <= 2e-6 * w1 + 1e-6
        c = rng.uniform(-1, 1, (h1, w1)).astype(np.float32)
        assert np.array_equal(capi.matrix_add(1, a, c, w1, h1), (a + c).ravel())
        assert np.array_equal(capi.matrix_sub(1, a, c, w1, h1), (a - c).ravel())
        n = _loguniform(rng, 3, 400000)
        v = rng.uniform(0.05, 6.0, n).astype(np.float32)
        for name, ref_fn in (("sin_psv", np.sin), ("exp_psv", np.exp), ("log_psv", np.log)):
            got = capi.psv(name, 1, v).astype(np.float64)
            want = ref_fn(v.astype(np.float64))
            assert (np.abs(got - want) <= 4e-7 * np.abs(want) + 5e-7).all(), (name, n)
        sig = rng.standard_normal(n).astype(np.float32)
        assert capi.detect_peaks(1, sig, 3) == capi.detect_peaks(0, sig, 3)
