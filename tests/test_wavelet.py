"""Port of reference tests/wavelet.cc (goldens + parametrised sweeps) plus
batched / multi-level device checks."""
import numpy as np
import pytest

from veles.simd_amd import capi

D, C, S = capi.WAVELET_TYPE_DAUBECHIES, capi.WAVELET_TYPE_COIFLET, capi.WAVELET_TYPE_SYMLET
EXTS = [0, 1, 2, 3]

VALID_LO = [1.42184071797210, 4.25026784271829, 7.07869496746448, 9.90712209221067,
            12.7355492169569, 15.5639763417030, 18.3924034664492, 21.2208305911954,
            24.0492577159416, 26.8776848406878, 29.7061119654340, 32.5345390901802,
            35.3629662149264, 37.4782538234490, 45.3048707044478, 28.8405938767906]
VALID_HI_TAIL = [-15.5030002317990, 5.58066496329142, -1.39137323046436]


def _ulps(a, b):
    a = np.asarray(a, np.float32).view(np.int32).astype(np.int64)
    b = np.asarray(b, np.float32).view(np.int32).astype(np.int64)
    return np.abs(a - b)


def test_wavelet_apply_na_golden():
    hi, lo = capi.wavelet_apply(D, 8, 0, np.arange(32, dtype=np.float32), na=True)
    assert (_ulps(lo, np.float32(VALID_LO)) <= 4).all()
    np.testing.assert_allclose(hi[:13], 0, atol=1e-5)
    np.testing.assert_allclose(hi[13:], VALID_HI_TAIL, atol=1e-5)


def test_stationary_wavelet_apply_na_golden():
    x = np.arange(32, dtype=np.float32)
    hi1, lo1 = capi.stationary_wavelet_apply(D, 8, 1, 0, x, na=True)
    hi2, lo2 = capi.stationary_wavelet_apply(D, 8, 2, 0, lo1, na=True)
    np.testing.assert_allclose(hi1[:25], 0, atol=1e-5)
    np.testing.assert_allclose(hi1[25:], [7.37209002588238, -15.5030002317990,
                                          4.68518434194794, 5.58066496329142,
                                          -0.404449011712775, -1.39137323046436,
                                          -0.339116857120903], atol=1e-5)
    np.testing.assert_allclose(hi2[11:14], [-0.0781250000022623, 0.164291522328916,
                                            0.634073488075181], atol=1e-5)
    lo_valid = [6.03235928067132, 8.03235928067132, 10.0323592806713]
    assert (_ulps(lo2[:3], np.float32(lo_valid)) <= 4).all()
    np.testing.assert_allclose(lo2[-1], 5.73072526035035, rtol=1e-6)


def test_validate_order():
    v = capi.fn("wavelet_validate_order")
    assert v(D, 8) and v(S, 76) and v(C, 30) and v(C, 6)
    assert not v(D, 7) and not v(D, 78) and not v(C, 8) and not v(C, 36)


def _params_dwt():
    out = [(t, o, e) for t in (D, S) for o in (2, 4, 6, 8, 12, 16) for e in EXTS]
    return out + [(C, o, e) for o in (6, 12) for e in EXTS]


def _params_swt():
    out = [(t, o, l, e) for t in (D, S) for o in (2, 4, 6, 8, 12, 16)
           for l in (1, 2, 3, 4) for e in EXTS]
    return out + [(C, o, l, e) for o in (6, 12) for l in (1, 2) for e in EXTS]


@pytest.mark.parametrize("t,o,e", _params_dwt())
def test_wavelet_apply_vs_na(t, o, e):
    x = np.arange(512, dtype=np.float32)
    hi, lo = capi.wavelet_apply(t, o, e, x)
    vhi, vlo = capi.wavelet_apply(t, o, e, x, na=True)
    np.testing.assert_allclose(hi, vhi, atol=5e-4)
    np.testing.assert_allclose(lo, vlo, atol=5e-4)


@pytest.mark.parametrize("t,o,l,e", _params_swt())
def test_stationary_wavelet_apply_vs_na(t, o, l, e):
    x = np.arange(512, dtype=np.float32)
    hi, lo = capi.stationary_wavelet_apply(t, o, l, e, x)
    vhi, vlo = capi.stationary_wavelet_apply(t, o, l, e, x, na=True)
    np.testing.assert_allclose(hi, vhi, atol=5e-4)
    np.testing.assert_allclose(lo, vlo, atol=5e-4)


def test_filter_banks_orthonormal():
    """Every generated bank is an orthonormal QMF with the reference scaling."""
    import ctypes
    lib = capi._lib.lib()
    for t, orders, norm in ((D, range(2, 77, 2), np.sqrt(2)), (S, range(2, 77, 2), 1.0),
                            (C, range(6, 31, 6), 1.0)):
        for o in orders:
            f = np.zeros(o, np.float32)
            assert lib.vs_wavelet_filter(t, o, ctypes.c_void_p(f.ctypes.data)) == 0
            h = f.astype(np.float64) * (np.sqrt(2) / norm)
            assert abs(h.sum() - np.sqrt(2)) < 1e-5
            for s in range(o // 2):
                want = 1.0 if s == 0 else 0.0
                assert abs(np.dot(h[:o - 2 * s], h[2 * s:]) - want) < 5e-5, (t, o, s)


@pytest.mark.gpu
@pytest.mark.parametrize("t,o", [(D, 8), (S, 16), (C, 12), (D, 76)])
@pytest.mark.parametrize("e", EXTS)
def test_device_batched_and_multilevel(t, o, e):
    import torch
    from veles.simd_amd import ops
    g = torch.Generator().manual_seed(o * 10 + e)
    x = torch.randn(5, 2048, generator=g)
    hi, lo = ops.dwt(x.cuda(), t, o, e)
    for b in range(5):
        vhi, vlo = capi.wavelet_apply(t, o, e, x[b].numpy(), na=True)
        np.testing.assert_allclose(hi[b].cpu().numpy(), vhi, atol=1e-4)
        np.testing.assert_allclose(lo[b].cpu().numpy(), vlo, atol=1e-4)
    his, lof = ops.swt(x.cuda(), t, o, levels=4, ext=e)
    cur = x.numpy()
    for l in range(1, 5):
        for b in range(5):
            vhi, vlo = capi.stationary_wavelet_apply(t, o, l, e, cur[b], na=True)
            np.testing.assert_allclose(his[b, l - 1].cpu().numpy(), vhi, atol=2e-4)
            cur[b] = vlo
    np.testing.assert_allclose(lof.cpu().numpy(), cur, atol=2e-4)
    pyr = ops.wavedec(x.cuda(), t, o, levels=3, ext=e).cpu().numpy()
    cur = x.numpy()
    off = 0
    for l in range(3):
        n = cur.shape[1] // 2
        nxt = np.zeros((5, n), np.float32)
        for b in range(5):
            vhi, vlo = capi.wavelet_apply(t, o, e, cur[b], na=True)
            np.testing.assert_allclose(pyr[b, off:off + n], vhi, atol=2e-4)
            nxt[b] = vlo
        cur = nxt
        off += n
    np.testing.assert_allclose(pyr[:, off:], cur, atol=2e-4)


@pytest.mark.gpu
@pytest.mark.parametrize("t,o", [(D, 4), (S, 8), (C, 6), (D, 16)])
@pytest.mark.parametrize("e", EXTS)
def test_host_api_large_runs_on_gpu(t, o, e):
    """Flag-less host API: length x taps >= VELES_GPU_MIN_ELEMS goes to the GPU
    (staged through pinned bounce buffers); must equal the host reference."""
    n = 1 << 18
    x = (np.sin(np.arange(n) * 0.01) * 100).astype(np.float32)
    hi, lo = capi.wavelet_apply(t, o, e, x)
    vhi, vlo = capi.wavelet_apply(t, o, e, x, na=True)
    np.testing.assert_allclose(hi, vhi, atol=5e-3)
    np.testing.assert_allclose(lo, vlo, atol=5e-3)
    shi, slo = capi.stationary_wavelet_apply(t, o, 2, e, x)
    rhi, rlo = capi.stationary_wavelet_apply(t, o, 2, e, x, na=True)
    np.testing.assert_allclose(shi, rhi, atol=5e-3)
    np.testing.assert_allclose(slo, rlo, atol=5e-3)


def _wfn(name, res, args):
    import ctypes
    f = getattr(capi._lib.lib(), name)
    f.restype = res
    f.argtypes = args
    return f


def test_prepare_array_allocate_destination_recycle():
    """Reference tests/wavelet.cc:44-86 in its non-AVX form (the GPU needs no
    shifted copies: prepare = aligned copy), plus wavelet_recycle_source's
    quarter-buffer carving (src/wavelet.c:138-165, non-AVX branch)."""
    import ctypes
    vp = ctypes.c_void_p
    libc = ctypes.CDLL(None)
    libc.free.argtypes = [vp]
    prep = _wfn("wavelet_prepare_array", vp, [ctypes.c_int, vp, ctypes.c_size_t])
    alloc = _wfn("wavelet_allocate_destination", vp, [ctypes.c_int, ctypes.c_size_t])
    recycle = _wfn("wavelet_recycle_source", None,
                   [ctypes.c_int, vp, ctypes.c_size_t] + [ctypes.POINTER(vp)] * 4)
    x = np.arange(512, dtype=np.float32)
    for order in (8, 4):
        p = prep(order, x.ctypes.data, 512)
        assert p % 64 == 0
        got = np.ctypeslib.as_array(ctypes.cast(p, ctypes.POINTER(ctypes.c_float)), (512,))
        np.testing.assert_array_equal(got, x)
        libc.free(p)
    d = alloc(8, 512)
    assert d % 64 == 0
    libc.free(d)
    outs = [vp() for _ in range(4)]
    recycle(8, x.ctypes.data, 512, *[ctypes.byref(o) for o in outs])
    base = x.ctypes.data
    assert [o.value for o in outs] == [base + 4 * 128 * i for i in range(4)]
    recycle(8, x.ctypes.data, 510, *[ctypes.byref(o) for o in outs])
    assert all(o.value is None for o in outs)


def test_multilevel_chain_via_recycle():
    """Two decimated levels chained the reference way: level-1 lo feeds
    level 2, whose outputs land in the recycled quarters of the source."""
    x = (np.sin(np.arange(256) * 0.3) * 10).astype(np.float32)
    hi1, lo1 = capi.wavelet_apply(D, 8, 0, x)
    hi2, lo2 = capi.wavelet_apply(D, 8, 0, lo1)
    rhi2, rlo2 = capi.wavelet_apply(D, 8, 0, lo1, na=True)
    np.testing.assert_allclose(hi2, rhi2, atol=5e-4)
    np.testing.assert_allclose(lo2, rlo2, atol=5e-4)


@pytest.mark.gpu
@pytest.mark.parametrize("e", EXTS)
def test_wavedec_long_signal_level_by_level(e):
    """Signals longer than the LDS pyramid (16384) run level by level."""
    import torch
    from veles.simd_amd import ops
    n = 1 << 15
    x = torch.from_numpy((np.sin(np.arange(2 * n) * 0.001) * 10).astype(np.float32)).reshape(2, n)
    pyr = ops.wavedec(x.cuda(), D, 8, levels=2, ext=e).cpu().numpy()
    cur = x.numpy()
    off = 0
    for l in range(2):
        m = cur.shape[1] // 2
        nxt = np.zeros((2, m), np.float32)
        for b in range(2):
            vhi, vlo = capi.wavelet_apply(D, 8, e, cur[b], na=True)
            np.testing.assert_allclose(pyr[b, off:off + m], vhi, atol=2e-3)
            nxt[b] = vlo
        cur = nxt
        off += m
    np.testing.assert_allclose(pyr[:, off:], cur, atol=2e-3)


@pytest.mark.gpu
@pytest.mark.parametrize("t,o,levels,n", [(D, 8, 8, 1024), (S, 16, 6, 512), (D, 2, 10, 1024),
                                          (C, 30, 5, 512), (D, 4, 9, 256)])
@pytest.mark.parametrize("e", EXTS)
@pytest.mark.parametrize("fused", [0, 1])
def test_swt_multilevel_deep(t, o, levels, n, e, fused):
    """vs_swt_multilevel at deep levels (halo up to the signal length, fused
    extension kernel; (D, 4, 9, 256) has a halo longer than the signal and
    still runs the fused kernel, one extension image per period) against the level-by-level host reference, with
    the fused kernel on and off (vs_tune_set swt_fused)."""
    import ctypes
    import torch
    from veles.simd_amd import _lib
    lib = _lib.lib()
    g = torch.Generator().manual_seed(o + 100 * levels + e)
    b = 3
    x = torch.randn(b, n, generator=g)
    hi = torch.full((b, levels, n), float("nan"), device="cuda")
    lo = torch.full((b, n), float("nan"), device="cuda")
    xd = x.cuda()
    assert lib.vs_tune_set(b"swt_fused", fused) == 0
    try:
        st = lib.vs_swt_multilevel(t, o, levels, e, ctypes.c_void_p(xd.data_ptr()), n,
                                   ctypes.c_void_p(hi.data_ptr()), ctypes.c_void_p(lo.data_ptr()),
                                   b, ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
        assert st == 0, lib.vs_last_error()
        torch.cuda.synchronize()
    finally:
        lib.vs_tune_set(b"swt_fused", -1)
    cur = x.numpy().copy()
    for lvl in range(1, levels + 1):
        for r in range(b):
            vhi, vlo = capi.stationary_wavelet_apply(t, o, lvl, e, cur[r], na=True)
            np.testing.assert_allclose(hi[r, lvl - 1].cpu().numpy(), vhi, atol=2e-4,
                                       err_msg=f"level {lvl}")
            cur[r] = vlo
    np.testing.assert_allclose(lo.cpu().numpy(), cur, atol=2e-4)


@pytest.mark.gpu
@pytest.mark.parametrize("t,o,levels,n", [(D, 8, 8, 12000), (S, 4, 3, 40000), (C, 30, 7, 9000),
                                          (D, 2, 12, 16384)])
@pytest.mark.parametrize("e", EXTS)
def test_swt_multilevel_long_tiled(t, o, levels, n, e):
    """Signals longer than one workgroup's LDS (> 8192 samples): tiled
    all-levels-in-LDS kernel (wavelet.hip swt_tiled_kernel; the last tile is
    aligned to the end of the signal and re-extends each band) against the
    level-by-level host reference and the HBM level-by-level path."""
    import ctypes
    import torch
    from veles.simd_amd import _lib
    lib = _lib.lib()
    g = torch.Generator().manual_seed(o + levels + e + n)
    b = 2
    x = torch.randn(b, n, generator=g)
    xd = x.cuda()
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    outs = []
    for fused in (1, 0):
        hi = torch.full((b, levels, n), float("nan"), device="cuda")
        lo = torch.full((b, n), float("nan"), device="cuda")
        assert lib.vs_tune_set(b"swt_fused", fused) == 0
        try:
            st = lib.vs_swt_multilevel(t, o, levels, e, ctypes.c_void_p(xd.data_ptr()), n,
                                       ctypes.c_void_p(hi.data_ptr()),
                                       ctypes.c_void_p(lo.data_ptr()), b, s)
            assert st == 0, lib.vs_last_error()
            torch.cuda.synchronize()
        finally:
            lib.vs_tune_set(b"swt_fused", -1)
        outs.append((hi.cpu(), lo.cpu()))
    torch.testing.assert_close(outs[0][0], outs[1][0], atol=1e-4, rtol=0)
    torch.testing.assert_close(outs[0][1], outs[1][1], atol=1e-4, rtol=0)
    hi, lo = outs[0]
    cur = x.numpy().copy()
    for lvl in range(1, levels + 1):
        for r in range(b):
            vhi, vlo = capi.stationary_wavelet_apply(t, o, lvl, e, cur[r], na=True)
            np.testing.assert_allclose(hi[r, lvl - 1].numpy(), vhi, atol=3e-4,
                                       err_msg=f"level {lvl}")
            cur[r] = vlo
    np.testing.assert_allclose(lo.numpy(), cur, atol=3e-4)


@pytest.mark.gpu
@pytest.mark.parametrize("t,o,levels,n", [(D, 8, 5, 8192), (D, 2, 10, 1024), (C, 30, 4, 512),
                                          (S, 16, 3, 24), (D, 4, 4, 16384), (D, 6, 2, 100)])
@pytest.mark.parametrize("e", EXTS)
def test_dwt_multilevel_vec(t, o, levels, n, e):
    """LDS pyramid (vs_dwt_multilevel): vectorised kernel (dwt_multi4_kernel;
    (S, 16, 3, 24) and (D, 6, 2, 100) have levels whose half length is not a
    multiple of 4 and take its scalar loop) against the scalar kernel
    (vs_tune_set dwt_vec 0) and the level-by-level host reference."""
    import ctypes
    import torch
    from veles.simd_amd import _lib
    lib = _lib.lib()
    g = torch.Generator().manual_seed(o + levels + e + n)
    b = 3
    x = torch.randn(b, n, generator=g)
    xd = x.cuda()
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    outs = []
    for vec in (1, 0):
        out = torch.full((b, n), float("nan"), device="cuda")
        assert lib.vs_tune_set(b"dwt_vec", vec) == 0
        try:
            st = lib.vs_dwt_multilevel(t, o, levels, e, ctypes.c_void_p(xd.data_ptr()), n,
                                       ctypes.c_void_p(out.data_ptr()), b, s)
            assert st == 0, lib.vs_last_error()
            torch.cuda.synchronize()
        finally:
            lib.vs_tune_set(b"dwt_vec", -1)
        outs.append(out.cpu())
    torch.testing.assert_close(outs[0], outs[1], atol=1e-5, rtol=0)
    pyr = outs[0].numpy()
    cur = x.numpy()
    off = 0
    for lvl in range(levels):
        m = cur.shape[1] // 2
        nxt = np.zeros((b, m), np.float32)
        for r in range(b):
            vhi, vlo = capi.wavelet_apply(t, o, e, cur[r], na=True)
            np.testing.assert_allclose(pyr[r, off:off + m], vhi, atol=5e-4, err_msg=f"level {lvl}")
            nxt[r] = vlo
        cur = nxt
        off += m
    np.testing.assert_allclose(pyr[:, off:], cur, atol=5e-4)


def _pyramid_ref(x, t, o, levels, e):
    """Level-by-level host reference of the Mallat pyramid rows."""
    b, n = x.shape
    out = np.zeros((b, n), np.float32)
    cur = x
    off = 0
    for _ in range(levels):
        m = cur.shape[1] // 2
        nxt = np.zeros((b, m), np.float32)
        for r in range(b):
            vhi, vlo = capi.wavelet_apply(t, o, e, cur[r], na=True)
            out[r, off:off + m] = vhi
            nxt[r] = vlo
        cur = nxt
        off += m
    out[:, off:] = cur
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("t,o,levels,n", [
    (D, 8, 8, 1 << 17),        # one tiled pass of 8 levels
    (D, 8, 11, 1 << 16),       # two passes (8 + 3), second on a 256-sample band
    (C, 30, 5, 3 * (1 << 14)),  # long filter: 4 levels + 1, ragged tile count
    (S, 4, 3, 40000),          # last tile overlaps the one before
    (D, 2, 12, 1 << 15),       # Haar, 12 levels down to 8 samples
    (D, 16, 6, 20480),         # bands that stop being multiples of 4 (scalar levels)
])
@pytest.mark.parametrize("e", EXTS)
def test_dwt_multilevel_long_tiled(t, o, levels, n, e):
    """Pyramid of signals longer than the LDS kernel (vs_dwt_multilevel,
    dwt_tiled_kernel): tiles with the multi-level support in LDS, hi bands
    written straight into the pyramid row, against the level-by-level host
    reference and the level-by-level device path (dwt_vec = 0)."""
    import ctypes
    import torch
    from veles.simd_amd import _lib
    lib = _lib.lib()
    b = 2
    g = torch.Generator().manual_seed(o + levels + e)
    x = torch.randn(b, n, generator=g)
    xd = x.cuda()
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    outs = []
    for vec in (1, 0):
        out = torch.full((b, n), float("nan"), device="cuda")
        assert lib.vs_tune_set(b"dwt_vec", vec) == 0
        st = lib.vs_dwt_multilevel(t, o, levels, e, ctypes.c_void_p(xd.data_ptr()), n,
                                   ctypes.c_void_p(out.data_ptr()), b, s)
        assert st == 0, lib.vs_last_error()
        outs.append(out.cpu().numpy())
    lib.vs_tune_set(b"dwt_vec", -1)
    ref = _pyramid_ref(x.numpy(), t, o, levels, e)
    scale = max(1.0, np.abs(ref).max())
    np.testing.assert_allclose(outs[0], ref, atol=3e-5 * scale * levels)
    np.testing.assert_allclose(outs[0], outs[1], atol=3e-5 * scale * levels)


@pytest.mark.gpu
@pytest.mark.parametrize("t,o", [(D, 8), (S, 16), (C, 6), (D, 76)])
@pytest.mark.parametrize("n,off", [(512, 0), (1000, 0), (8192 + 24, 0), (40000, 0), (4098, 1)])
@pytest.mark.parametrize("e", EXTS)
def test_dwt_single_level_vectorised(t, o, n, off, e):
    """Single decimated level (vs_dwt): the tiled kernel with compile-time
    filter length and float4 loads / stores (orders without an
    instantiation -- db76 -- and offset rows take the scalar paths), against
    the host reference; rows with strides, hi / lo padded apart."""
    import ctypes
    import torch
    from veles.simd_amd import _lib
    lib = _lib.lib()
    b = 3
    ss = n + 8
    os_ = n // 2 + 4
    g = torch.Generator().manual_seed(o + n + e)
    xb = torch.randn(b * ss + off, generator=g)
    xd = xb.cuda()
    hi = torch.full((b * os_ + off,), 7.0, device="cuda")
    lo = torch.full((b * os_ + off,), 7.0, device="cuda")
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    st = lib.vs_dwt(t, o, e, ctypes.c_void_p(xd.data_ptr() + 4 * off), n, ss,
                    ctypes.c_void_p(hi.data_ptr() + 4 * off), ctypes.c_void_p(lo.data_ptr() + 4 * off),
                    os_, b, s)
    assert st == 0, lib.vs_last_error()
    hi = hi.cpu().numpy()[off:off + b * os_].reshape(b, os_)
    lo = lo.cpu().numpy()[off:off + b * os_].reshape(b, os_)
    x = xb.numpy()[off:off + b * ss].reshape(b, ss)[:, :n]
    for r in range(b):
        vhi, vlo = capi.wavelet_apply(t, o, e, x[r], na=True)
        np.testing.assert_allclose(hi[r, :n // 2], vhi, atol=2e-4)
        np.testing.assert_allclose(lo[r, :n // 2], vlo, atol=2e-4)
    assert (hi[:, n // 2:] == 7.0).all() and (lo[:, n // 2:] == 7.0).all()


def _window(x, a, b, n, e, halo):
    """Host row x[a:b] followed by `halo` samples of what the transform sees
    after it: the next samples, or the extension (e: 0 periodic, 1 mirror)
    when the window ends at the end of the row."""
    import torch
    if b < n:
        return x[a:b + halo].cpu().numpy()
    tail = x[:halo] if e == 0 else x[n - halo:].flip(0)
    return torch.cat([x[a:b], tail]).cpu().numpy()


def _spots(n, w):
    return [(0, w), ((n // 2) - w, (n // 2) + w), (n - 2 * w, n)]


@pytest.mark.gpu
@pytest.mark.slow
@pytest.mark.parametrize("e", [0, 1])
def test_swt_and_dwt_rows_of_2p32(e):
    """Rows of 2^32 samples (size_t lengths in the reference,
    inc/simd/wavelet.h:61-100): stationary levels 1 and 2 (single-level and
    fused tiled kernels, 64-bit positions) and a three-level pyramid.  Every
    band is checked at its start, middle (around 2^31 of the input) and end
    (extension) against the host reference run on windows of the band before
    it, which the same checks validated."""
    import ctypes
    import torch
    from veles.simd_amd import _lib
    lib = _lib.lib()
    n = 1 << 32
    x = torch.empty(n, device="cuda")
    g = torch.Generator(device="cuda").manual_seed(3)
    for a in range(0, n, 1 << 28):
        x[a:a + (1 << 28)].normal_(generator=g)
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    vp = lambda t_: ctypes.c_void_p(t_.data_ptr())  # noqa: E731
    W = 96

    def check_swt(band_in, level, hi, lo, tol):
        for a, b in _spots(n, W):
            w = _window(band_in, a, b, n, e, 7 * (1 << (level - 1)) + 1)
            vhi, vlo = capi.stationary_wavelet_apply(D, 8, level, 3, w, na=True)
            np.testing.assert_allclose(hi[a:b].cpu().numpy(), vhi[:b - a], atol=tol)
            np.testing.assert_allclose(lo[a:b].cpu().numpy(), vlo[:b - a], atol=tol)

    hi1 = torch.empty(n, device="cuda")
    lo1 = torch.empty(n, device="cuda")
    assert lib.vs_swt(D, 8, 1, e, vp(x), n, n, vp(hi1), vp(lo1), n, 1, s) == 0, lib.vs_last_error()
    check_swt(x, 1, hi1, lo1, 2e-5)
    hi = torch.empty(2, n, device="cuda")
    lo = torch.empty(n, device="cuda")
    assert lib.vs_swt_multilevel(D, 8, 2, e, vp(x), n, vp(hi), vp(lo), 1, s) == 0, \
        lib.vs_last_error()
    for a, b in _spots(n, W):
        np.testing.assert_allclose(hi[0, a:b].cpu().numpy(), hi1[a:b].cpu().numpy(), atol=1e-5)
    check_swt(lo1, 2, hi[1], lo, 4e-5)
    del hi, lo, hi1, lo1

    out = torch.empty(n, device="cuda")
    assert lib.vs_dwt_multilevel(D, 8, 3, e, vp(x), n, vp(out), 1, s) == 0, lib.vs_last_error()
    cur, m, off = x, n, 0
    for lvl in range(3):
        half = m // 2
        bh = torch.empty(half, device="cuda")
        bl = torch.empty(half, device="cuda")
        assert lib.vs_dwt(D, 8, e, vp(cur), m, m, vp(bh), vp(bl), half, 1, s) == 0, \
            lib.vs_last_error()
        for a, b in _spots(half, W):
            w = _window(cur, 2 * a, 2 * b, m, e, 8)
            vhi, vlo = capi.wavelet_apply(D, 8, 3, w, na=True)
            k = b - a
            np.testing.assert_allclose(bh[a:b].cpu().numpy(), vhi[:k], atol=1e-4)
            np.testing.assert_allclose(bl[a:b].cpu().numpy(), vlo[:k], atol=1e-4)
            np.testing.assert_allclose(out[off + a:off + b].cpu().numpy(), vhi[:k], atol=1e-4)
            if lvl == 2:
                np.testing.assert_allclose(out[off + half + a:off + half + b].cpu().numpy(),
                                           vlo[:k], atol=1e-4)
        cur, m, off = bl, half, off + half
        del bh
