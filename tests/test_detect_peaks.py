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


@pytest.mark.gpu
@pytest.mark.parametrize("n", [3, 5, 63, 64, 65, 255, 4095, 4096, 4097, 3 * 4096 + 1, (1 << 20) + 5])
@pytest.mark.parametrize("off", [0, 1])
def test_device_paths_vs_numpy(n, off):
    """vs_detect_peaks on the device: float4 kernels (16-byte aligned x: lane
    shuffles for neighbours, wave-edge loads) and scalar kernels (offset x),
    every extremum type, chunk / wave boundaries, and a capacity below the
    count (first `cap` in position order)."""
    import ctypes
    import torch
    from veles.simd_amd import _lib
    lib = _lib.lib()
    rng = np.random.default_rng(n + off)
    xh = np.round(rng.standard_normal(n) * 4).astype(np.float32)  # plateaus too
    buf = torch.zeros(n + off, device="cuda")
    buf[off:] = torch.from_numpy(xh).cuda()
    d1, d2 = xh[1:-1] - xh[:-2], xh[1:-1] - xh[2:]
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    for kind in (1, 2, 3):
        sel = d1 * d2 > 0
        sel &= ((d1 > 0) & bool(kind & 1)) | ((d1 < 0) & bool(kind & 2))
        want = np.nonzero(sel)[0] + 1
        for cap in (len(want), max(len(want) // 3, 1)):
            pos = torch.full((cap,), -1, dtype=torch.int32, device="cuda")
            val = torch.zeros(cap, device="cuda")
            cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
            _lib.check(lib.vs_detect_peaks(ctypes.c_void_p(buf.data_ptr() + 4 * off), n, kind,
                                           ctypes.c_void_p(pos.data_ptr()),
                                           ctypes.c_void_p(val.data_ptr()), cap,
                                           ctypes.c_void_p(cnt.data_ptr()), s),
                       "vs_detect_peaks")
            assert cnt.item() == len(want)
            k = min(cap, len(want))
            assert np.array_equal(pos.cpu().numpy()[:k], want[:k])
            assert np.array_equal(val.cpu().numpy()[:k], xh[want[:k]])


@pytest.mark.parametrize("dev", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
@pytest.mark.parametrize("rows,n,kind", [(1, 4000, 3), (7, 5000, 1), (33, 4097, 2), (5, 12289, 3)])
def test_batched_rows_match_single_rows(dev, rows, n, kind):
    """vs_detect_peaks_batched: every row's segment equals the single-row
    result (the scalar definition), row_start is the CSR index."""
    import torch
    from veles.simd_amd import ops
    g = torch.Generator().manual_seed(rows * 1000 + n)
    x = torch.randn(rows, n, generator=g).to(dev)
    pos, val, rs = ops.detect_peaks_batched(x, kind)
    assert rs.shape == (rows + 1,) and rs[0] == 0 and rs[-1] == pos.numel()
    rs = rs.tolist()
    for r in range(rows):
        row = x[r].double().cpu()
        d1 = row[1:-1] - row[:-2]
        d2 = row[1:-1] - row[2:]
        m = (d1 * d2 > 0) & (((d1 > 0) & bool(kind & 1)) | ((d1 < 0) & bool(kind & 2)))
        ref = torch.nonzero(m).flatten() + 1
        got = pos[rs[r]:rs[r + 1]].cpu().long()
        assert torch.equal(got, ref), (r, got[:5], ref[:5])
        assert torch.equal(val[rs[r]:rs[r + 1]].cpu(), x[r].cpu()[ref])


@pytest.mark.gpu
def test_batched_strided_unaligned_rows():
    """Rows with a stride that is not a multiple of 4 floats and an
    unaligned base take the scalar kernels."""
    import torch
    from veles.simd_amd import ops
    base = torch.randn(6 * 1003 + 1, device="cuda")
    x = base[1:].reshape(6, 1003)[:, :1001]          # stride 1003, base offset 4 bytes
    pos, val, rs = ops.detect_peaks_batched(x, 3)
    pos_c, val_c, rs_c = ops.detect_peaks_batched(x.cpu(), 3)
    assert torch.equal(pos.cpu(), pos_c) and torch.equal(rs.cpu(), rs_c)
    assert torch.equal(val.cpu(), val_c)


@pytest.mark.gpu
def test_matched_filter_batch_in_one_launch_sequence():
    """MatchedFilter over 4096 x 65536: correlation, batched peak search and
    thresholding with a single host read, against the per-row path."""
    import torch
    from veles.simd_amd import models, ops
    g = torch.Generator(device="cuda").manual_seed(1)
    x = torch.randn(4096, 65536, device="cuda", generator=g)
    t = torch.sin(torch.arange(64, device="cuda") * 0.3)
    mf = models.MatchedFilter(t, threshold=12.0).cuda()
    resp, peaks = mf(x)
    assert len(peaks) == 4096
    for r in (0, 1, 2047, 4095):
        p, v = ops.detect_peaks(resp[r], ops.signal.MAXIMUM)
        keep = v > 12.0
        assert torch.equal(peaks[r][0], p[keep]) and torch.equal(peaks[r][1], v[keep])
    assert sum(p.numel() for p, _ in peaks) > 0


@pytest.mark.gpu
@pytest.mark.slow
def test_row_of_2p32_samples():
    """A row of 2^32 + 3 samples (reference inc/simd/detect_peaks.h:61-62
    takes size_t): positions come back as int64; spikes placed at the start,
    around 2^31 and 2^32 and at the end are found exactly, with their values
    and in order."""
    import torch
    from veles.simd_amd import ops
    n = (1 << 32) + 3
    x = torch.zeros(n, device="cuda")
    want = [1, 4097, (1 << 31) - 1, 1 << 31, (1 << 31) + 7, (1 << 32) - 2, 1 << 32, n - 2]
    vals = [float(i + 1) * (1 if i % 2 == 0 else -1) for i in range(len(want))]
    x[torch.tensor(want, device="cuda")] = torch.tensor(vals, device="cuda")
    # neighbours (2^31 - 1, 2^31): make both strict extrema of opposite sign
    pos, val = ops.detect_peaks(x, "both")
    assert pos.dtype == torch.int64
    assert pos.cpu().tolist() == want
    assert val.cpu().tolist() == vals
    pos, val = ops.detect_peaks(x, "max")
    assert pos.cpu().tolist() == [p for p, v in zip(want, vals) if v > 0]
