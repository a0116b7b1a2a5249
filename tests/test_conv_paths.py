"""Every device convolution path against an fp64 reference.

Covers the real-block overlap-save kernel (conv.hip real_conv_kernel) and the
pair kernel it replaced (tuning knob conv_real = 0), odd signal / filter
lengths (odd block starts, half-valid 8-byte edges), per-signal filters, the
uniformly partitioned path for filters longer than one overlap-save block,
rows cut into pieces (the path of rows of 2^29 outputs or more, exercised on
short rows through the conv_piece_log knob), and padded lengths beyond the
single-workgroup transform (four-step, up to 2^24).
Reference behaviour: /root/reference/src/convolve.c:116-121 (any h < x/2 runs
overlap-save), :237-244 (FFT has no size cap).
"""
import contextlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _fft_ref(x, h, corr=False):
    from scipy.signal import fftconvolve
    x = np.asarray(x, np.float64)
    h = np.asarray(h, np.float64)
    return fftconvolve(x, h[::-1] if corr else h)


@contextlib.contextmanager
def _knob(name, value, default):
    from veles.simd_amd import _lib
    _lib.call("vs_tune_set", name.encode(), value)
    try:
        yield
    finally:
        _lib.call("vs_tune_set", name.encode(), default)


@contextlib.contextmanager
def _kernel(real):
    """real: 0 pair kernel, 1 real-block kernel at every block size."""
    with _knob("conv_real", real, 1), _knob("conv_real_all", int(real == 1), 0):
        yield


def _check(xlen, hlen, batch, algo, corr, per_signal=False, seed=0, rel=2e-6):
    import torch
    from veles.simd_amd import ops
    g = torch.Generator().manual_seed(seed + xlen + 7 * hlen)
    x = torch.randn(batch, xlen, generator=g)
    h = torch.randn(batch if per_signal else 1, hlen, generator=g)
    y = ops.conv1d(x.cuda(), h.cuda() if per_signal else h[0].cuda(), algorithm=algo,
                   correlate=corr).cpu().double().numpy()
    for b in range(batch):
        ref = _fft_ref(x[b].numpy(), h[b if per_signal else 0].numpy(), corr)
        assert y[b].shape == ref.shape
        err = np.abs(y[b] - ref).max()
        # fp32 FFT error grows ~ sqrt(h) * log2(L) times the sample scale
        tol = rel * np.sqrt(hlen) * np.abs(x[b].numpy()).max() * np.abs(h.numpy()).max() * 30
        assert err <= tol + 1e-4, (xlen, hlen, b, algo, corr, err, tol)


@pytest.mark.parametrize("real", [0, 1])
@pytest.mark.parametrize("xlen,hlen,batch", [
    (1 << 16, 4096, 3),      # L = 16384 (M = 8192), pre odd
    (100003, 4095, 2),       # odd x, pre even
    (50001, 1000, 3),        # L = 4096
    (30001, 77, 4),          # L = 2048, short filter
    (9000, 2500, 1),         # few blocks
])
@pytest.mark.parametrize("corr", [False, True])
def test_overlap_save_variants(real, xlen, hlen, batch, corr):
    with _kernel(real):
        _check(xlen, hlen, batch, "overlap_save", corr)


@pytest.mark.parametrize("real", [0, 1])
@pytest.mark.parametrize("xlen,hlen", [(100, 29), (1000, 999), (5001, 3000),
                                       (12000, 4385), (16000, 385)])
def test_single_block_fft_variants(real, xlen, hlen):
    with _kernel(real):
        _check(xlen, hlen, 3, "fft", False)
        _check(xlen, hlen, 2, "fft", True)


def test_per_signal_filters_real_block():
    _check(40000, 3000, 3, "overlap_save", False, per_signal=True)
    _check(40000, 3000, 3, "overlap_save", True, per_signal=True)
    _check(9000, 7000, 3, "fft", False, per_signal=True)   # single block, per signal


@pytest.mark.parametrize("xlen,hlen,batch", [(300000, 9000, 2), (200001, 12345, 1)])
@pytest.mark.parametrize("corr", [False, True])
def test_partitioned_long_filters(xlen, hlen, batch, corr):
    """Filters of 9000-12345 taps, explicit OS request: one L = 32768 real
    block (test_partitioned_beyond_32768_block covers the partitioned path)."""
    _check(xlen, hlen, batch, "overlap_save", corr)


def test_per_signal_filters_beyond_one_block():
    """Per-signal filters whose padded transform exceeds one workgroup go
    through partitioned overlap-save (one batched launch per partition)."""
    _check(30000, 20000, 3, "auto", False, per_signal=True)


@pytest.mark.slow
@pytest.mark.parametrize("xlen,hlen", [(1 << 25, 20000), (1 << 23, 65536)])
def test_cliff_shapes(xlen, hlen):
    """Shapes past the largest single transform (2^24 points)."""
    from veles.simd_amd import _lib
    assert _lib.lib().vs_conv1d_select(xlen, hlen, 1) in (2, 3)
    _check(xlen, hlen, 1, "auto", False)


def test_four_step_fft_conv_2p23():
    """x + h - 1 just above 2^22 -> a 2^23-point four-step transform."""
    from veles.simd_amd import _lib
    xlen, hlen = (1 << 22) + 4096 - 20000 + 1, 20000
    # auto picks overlap-save here (L = 32768 blocks, 39 % useful, under the
    # 20 % rule); the explicit FFT request below still runs the 2^23 transform
    assert _lib.lib().vs_conv1d_select(xlen, hlen, 1) == 3
    _check(xlen, hlen, 1, "fft", False)
    _check(xlen, hlen, 1, "fft", True)


@pytest.mark.parametrize("logn", [22, 23, 24])
def test_four_step_fft_large(logn):
    import torch
    from veles.simd_amd import ops
    n = 1 << logn
    g = torch.Generator().manual_seed(logn)
    z = torch.randn(1, n, 2, generator=g)
    f = ops.fft(z.cuda()).cpu().double()
    zc = z[..., 0].double().numpy() + 1j * z[..., 1].double().numpy()
    ref = np.fft.fft(zc, axis=-1)
    got = f[..., 0].numpy() + 1j * f[..., 1].numpy()
    assert np.abs(got - ref).max() <= 2e-6 * np.sqrt(n) * logn * 4
    inv = ops.fft(f.float().cuda(), inverse=True).cpu().double() / n
    np.testing.assert_allclose(inv.numpy(), z.double().numpy(), atol=5e-5)


def test_select_never_unsupported():
    """Every valid (x, h) maps to a path that runs (no 2^24 cliff)."""
    from veles.simd_amd import _lib
    for xlen, hlen in [(1 << 26, 3), (1 << 26, 5000), (1 << 26, 40000), (1 << 24, 1 << 20),
                       (1 << 20, 1 << 20), (10, 10 ** 6)]:
        assert _lib.lib().vs_conv1d_select(xlen, hlen, 1) in (1, 2, 3)


@pytest.mark.parametrize("xlen,hlen,batch", [(512, 512, 1), (1000, 33, 2), (300, 1000, 1),
                                             (5000, 4096, 1), (20000, 777, 3), (17, 40, 2)])
@pytest.mark.parametrize("corr", [False, True])
def test_direct_small_grid(xlen, hlen, batch, corr):
    """Tap-split direct kernel (conv.hip direct_split_kernel): grids smaller
    than two workgroups per CU with 32 < h <= 4096."""
    _check(xlen, hlen, batch, "direct", corr, rel=1e-6)


@pytest.mark.parametrize("hlen", [33, 600, 5000])
def test_direct_large_grid(hlen):
    """Register-blocked direct kernel (conv.hip direct_kernel): grids of at
    least two workgroups per CU, filters over one 512-tap LDS chunk too."""
    _check(300000, hlen, 4, "direct", False, rel=1e-6)
    _check(300000, hlen, 4, "direct", True, rel=1e-6)


@pytest.mark.parametrize("xlen,hlen,batch", [(1 << 17, 4096, 3), (100003, 3000, 2),
                                             (70001, 700, 2), (40000, 8191, 1)])
@pytest.mark.parametrize("corr", [False, True])
def test_overlap_save_block_extra3(xlen, hlen, batch, corr):
    """os_block_extra = 3: blocks of 2^(floor(log2 h) + 3), up to L = 32768
    real samples (real_conv_kernel<14>: a 16384-point complex transform,
    128 KiB LDS)."""
    with _knob("os_block_extra", 3, 0):
        _check(xlen, hlen, batch, "overlap_save", corr)


@pytest.mark.parametrize("xlen,hlen", [(300000, 16000), (20000, 12000)])
def test_real_block_32768_default(xlen, hlen):
    """Filters of 8192..16383 taps: one L = 32768 real block (was a 50 %-useful
    16384 block or partitions), and a single-block FFT of 2^15 points."""
    _check(xlen, hlen, 2, "overlap_save", False)
    _check(xlen, hlen, 2, "overlap_save", True)
    _check(12000, 9000, 2, "fft", False)


def test_partitioned_beyond_32768_block():
    """Filters longer than the largest real block still partition."""
    _check(200000, 40000, 1, "overlap_save", False)
    _check(200000, 40000, 1, "overlap_save", True)


@pytest.mark.parametrize("block_log", [14, 13, 15])
@pytest.mark.parametrize("xlen,hlen,batch,per_signal", [
    (1 << 18, 65536, 2, False),    # 8 partitions of 8192 taps
    (100003, 200000, 2, False),    # filter longer than the signal, ragged last partition
    (1 << 17, 70001, 3, True),     # one filter per signal
    (40000, 32769, 1, False),      # just past the largest single block
    (300001, 49153, 2, False),     # odd lengths, 6 partitions + 1 tap
])
@pytest.mark.parametrize("corr", [False, True])
def test_uniformly_partitioned_overlap_save(block_log, xlen, hlen, batch, per_signal, corr):
    """Frequency-domain delay line (conv.hip fdl_*_kernel): every x block
    transformed once, partition spectra accumulated per output block, one
    inverse per block; both block sizes (L = 16384 default, 8192)."""
    with _knob("fdl_block_log", block_log, 0):
        _check(xlen, hlen, batch, "overlap_save", corr, per_signal=per_signal)


@pytest.mark.parametrize("lds", [1, 0])
def test_partitioned_many_output_tiles(lds):
    """More output blocks than one accumulation tile (32 in the LDS-staged
    kernel, 16 in the register kernel) and more than four partitions: every
    (tile, partition group) edge of both accumulation kernels."""
    with _knob("fdl_mac_lds", lds, 1):
        _check(8192 * 37 + 5, 8192 * 5 + 77, 2, "overlap_save", False)
        with _knob("fdl_block_log", 13, 0):
            _check(4096 * 41 + 3, 4096 * 9 + 1, 1, "overlap_save", True)
            _check(4096 * 70 + 3, 4096 * 2 + 1, 2, "overlap_save", False, per_signal=True)


def test_partitioned_more_partitions_than_one_lds_chunk():
    """40 and 67 partitions of 4096 taps: the LDS-staged accumulation walks them
    in chunks of 32 (two and three chunks), against the register kernel."""
    with _knob("fdl_block_log", 13, 0):
        for hlen in (4096 * 39 + 11, 4096 * 66 + 4095):
            _check(4096 * 45 + 9, hlen, 2, "overlap_save", False)
            with _knob("fdl_mac_lds", 0, 1):
                _check(4096 * 45 + 9, hlen, 1, "overlap_save", True)


def test_partitioned_plan_matches_call():
    """A plan of a partitioned shape holds the partitions' P / Q tables and
    gives the per-call result bit for bit."""
    import torch
    from veles.simd_amd import ops
    g = torch.Generator().manual_seed(5)
    x = torch.randn(3, 150000, generator=g).cuda()
    for h in (torch.randn(50000, generator=g).cuda(), torch.randn(3, 40001, generator=g).cuda()):
        plan = ops.Conv1dPlan(h, x.shape[1], algorithm="overlap_save")
        assert plan.precomputed
        y = plan(x)
        want = ops.conv1d(x, h, algorithm="overlap_save")
        assert torch.equal(y, want)


@pytest.mark.parametrize("algo,hlen,real", [
    ("direct", 4, 1), ("direct", 29, 1), ("direct", 700, 1),
    ("overlap_save", 1000, 1), ("overlap_save", 4096, 1), ("overlap_save", 1000, 0),
    ("overlap_save", 40000, 1), ("auto", 3000, 1), ("fft", 515, 1)])
@pytest.mark.parametrize("corr", [False, True])
def test_rows_cut_into_pieces(algo, hlen, real, corr):
    """Rows of 2^29 outputs or more are cut into pieces of 2^28 outputs run
    last to first (vs_conv1d); conv_piece_log = 14 runs the same code on a
    row of ~100k samples: 7 pieces, filters shorter and longer than a piece,
    every algorithm, shared and per-signal filters."""
    with _knob("conv_piece_log", 14, 28), _kernel(real):
        _check(100003, hlen, 2, algo, corr)
        _check(65536 - hlen + 1, hlen, 1, algo, corr)   # outputs end on a piece edge
        if algo != "fft":
            _check(70001, hlen, 2, algo, corr, per_signal=True)


def _window_ref(x, h, lo, hi, corr):
    """fp64 outputs [lo, hi) of conv(x, h) from the x samples they touch."""
    from scipy.signal import fftconvolve
    m = h.numel()
    a = max(0, lo - (m - 1))
    b = min(x.numel(), hi)
    xw = x[a:b].cpu().double().numpy()
    hw = h.cpu().double().numpy()
    full = fftconvolve(xw, hw[::-1] if corr else hw)   # output n of the window = a + n
    return full[lo - a:hi - a]


@pytest.mark.slow
@pytest.mark.parametrize("n,hlen,algo", [((1 << 32) + 17, 4096, "auto"),
                                         ((1 << 31) + 5, 4, "auto"),
                                         ((1 << 29) + 1001, 40000, "overlap_save")])
def test_rows_beyond_2p31(n, hlen, algo):
    """Signals of 2^31 samples and more on one GPU (reference
    inc/simd/convolve.h:100-111 takes size_t lengths): fp64 spot checks at the
    start, around every piece edge and at the end."""
    import torch
    from veles.simd_amd import ops
    x = torch.empty(n, device="cuda")
    step = 1 << 28
    g = torch.Generator(device="cuda").manual_seed(n % 1000)
    for a in range(0, n, step):
        x[a:a + step].normal_(generator=g)
    h = torch.randn(hlen, device="cuda")
    y = ops.conv1d(x, h, algorithm=algo)
    ylen = n + hlen - 1
    assert y.shape == (ylen,)
    spots = [(0, 300), (ylen - 300, ylen)]
    for e in range(step, ylen, step):
        spots.append((e - 150, e + 150))
    tol = 2e-6 * np.sqrt(hlen) * 30 * 25
    for lo, hi in spots:
        ref = _window_ref(x, h, lo, hi, False)
        got = y[lo:hi].cpu().double().numpy()
        assert np.abs(got - ref).max() <= tol, (lo, hi, np.abs(got - ref).max())
    del y
    # correlation of the same row: only the piece edges differ in kind
    y = ops.conv1d(x, h, algorithm=algo, correlate=True)
    for lo, hi in spots[:3]:
        ref = _window_ref(x, h, lo, hi, True)
        got = y[lo:hi].cpu().double().numpy()
        assert np.abs(got - ref).max() <= tol, (lo, hi)


def test_select_long_filter_overlap_save():
    """Filters whose L = 32768 block is >= 28 % useful run single-block
    overlap-save (h = 20000: 144 vs 73 Gsamples/s for the fused four-step
    FFT); longer ones the uniformly partitioned path up to 20 partitions of
    8192 taps (h = 65536: 100 vs 70, h = 163840: 73 vs 70), then up to 14
    partitions of 16384 taps (h = 200000: 72 vs 70), then the FFT
    (profiles/r3/conv/fdl.md)."""
    from veles.simd_amd import _lib
    lib = _lib.lib()
    assert lib.vs_conv1d_select(1 << 20, 20000, 64) == 3
    assert lib.vs_conv1d_select(1 << 20, 30000, 64) == 3
    assert lib.vs_conv1d_select(1 << 20, 98304, 64) == 3
    assert lib.vs_conv1d_select(1 << 20, 163840, 64) == 3
    assert lib.vs_conv1d_select(1 << 20, 200000, 64) == 3    # 13 partitions of 16384 taps
    assert lib.vs_conv1d_select(1 << 20, 229376, 64) == 3    # 14
    assert lib.vs_conv1d_select(1 << 20, 229377, 64) == 2
    assert lib.vs_conv1d_select(1 << 20, 400000, 64) == 2
    assert lib.vs_conv1d_select(1 << 27, 200000, 1) == 3   # beyond the largest transform
    _check(200000, 20000, 2, "auto", False)
    _check(200000, 20000, 1, "auto", True)
    _check(200000, 30000, 2, "auto", False)


@pytest.mark.parametrize("xlen,hlen,batch", [(300000, 40000, 3), (100003, 60000, 2),
                                             (40000, 30000, 1)])
@pytest.mark.parametrize("corr", [False, True])
def test_fused_four_step_conv(xlen, hlen, batch, corr):
    """Whole-signal FFT convolution through the fused three-pass four-step
    kernels (fft.hip conv_four_step: pack + columns, rows x H x inverse rows,
    inverse columns + unpack) against fp64, and equal to the seven-pass
    sequence (vs_tune_set conv_fused4 = 0) up to rounding."""
    import torch
    from veles.simd_amd import ops
    _check(xlen, hlen, batch, "fft", corr)
    g = torch.Generator().manual_seed(xlen)
    x = torch.randn(batch, xlen, generator=g).cuda()
    h = torch.randn(hlen, generator=g).cuda()
    y1 = ops.conv1d(x, h, algorithm="fft", correlate=corr)
    with _knob("conv_fused4", 0, 1):
        y0 = ops.conv1d(x, h, algorithm="fft", correlate=corr)
    scale = y0.abs().max().item()
    assert (y1 - y0).abs().max().item() <= 1e-5 * scale


@pytest.mark.gpu
@pytest.mark.parametrize("hlen", [1, 4, 8, 9, 16, 31, 32])
@pytest.mark.parametrize("xlen,off", [(5000, 0), (4099, 0), (2048, 1), (7, 0)])
@pytest.mark.parametrize("correlate", [0, 1])
@pytest.mark.parametrize("packed", [False, True])
def test_direct_small_vector_and_scalar_paths(hlen, xlen, off, correlate, packed):
    """Short-filter direct kernel: float4 window / store path (x rows 16-byte
    aligned; y rows packed back to back, so each row starts at a different
    offset inside 16 bytes, or padded) and the scalar path (offset x rows),
    ragged output tails."""
    import ctypes
    import torch
    from veles.simd_amd import _lib
    lib = _lib.lib()
    batch = 3
    xs = xlen + off + (4 - (xlen + off) % 4) % 4   # row stride keeps alignment iff off == 0
    ylen = xlen + hlen - 1
    ys = ylen if packed else ylen + off + (4 - (ylen + off) % 4) % 4
    xb = torch.randn(batch * xs + off, device="cuda")
    h = torch.randn(hlen, device="cuda")
    yb = torch.full((batch * ys + off,), 3.0, device="cuda")
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    _lib.check(lib.vs_conv1d(1, correlate, ctypes.c_void_p(xb.data_ptr() + 4 * off), xlen, xs,
                             ctypes.c_void_p(h.data_ptr()), hlen, 0,
                             ctypes.c_void_p(yb.data_ptr() + 4 * off), ys, batch, s),
               "vs_conv1d")
    x = xb[off:off + batch * xs].reshape(batch, xs)[:, :xlen].double()
    taps = h.double() if correlate else h.double().flip(0)
    want = torch.nn.functional.conv1d(x[:, None], taps[None, None], padding=hlen - 1)[:, 0]
    got = yb[off:off + batch * ys].reshape(batch, ys)
    assert (got[:, :ylen].double() - want).abs().max().item() < 1e-4
    assert (got[:, ylen:] == 3.0).all()


@pytest.mark.slow
def test_fft_batch_beyond_2p31_elements():
    """Batched c2c FFT whose arrays hold 2^32 + 48 complex numbers
    (2^28 + 3 transforms of 16 points): 64-bit offsets across the batch
    chunks; spot rows against torch.fft."""
    import torch
    from veles.simd_amd import ops
    n, batch = 16, (1 << 28) + 3
    z = torch.empty(batch, n, 2, device="cuda")
    g = torch.Generator(device="cuda").manual_seed(8)
    step = 1 << 24
    for a in range(0, batch, step):
        z[a:a + step].normal_(generator=g)
    f = ops.fft(z)
    rows = torch.tensor([0, 1, 65534, 65535, 65536, (1 << 27) - 1, 1 << 27, (1 << 28) - 1, 1 << 28,
                         batch - 1], device="cuda")
    want = torch.view_as_real(torch.fft.fft(torch.view_as_complex(z[rows].double()), dim=-1))
    assert (f[rows].double() - want).abs().max().item() < 1e-4


@pytest.mark.parametrize("hlen,per_signal", [(1000, False), (4096, True), (40000, False)])
@pytest.mark.parametrize("corr", [False, True])
def test_plan_rows_cut_into_pieces(hlen, per_signal, corr):
    """vs_conv1d_plan_execute on rows longer than one launch sequence: the
    pieces of vs_conv1d with the plan's precomputed spectra (single-block
    overlap-save and partitioned plans, shared and per-signal filters)."""
    import torch
    from veles.simd_amd import ops
    batch, xlen = 2, 100003
    g = torch.Generator().manual_seed(hlen)
    x = torch.randn(batch, xlen, generator=g)
    h = torch.randn(batch if per_signal else 1, hlen, generator=g)
    hd = h.cuda() if per_signal else h[0].cuda()
    with _knob("conv_piece_log", 14, 28):
        plan = ops.Conv1dPlan(hd, xlen, algorithm="overlap_save", correlate=corr)
        assert plan.precomputed
        y = plan(x.cuda()).cpu().double().numpy()
    for b in range(batch):
        ref = _fft_ref(x[b].numpy(), h[b if per_signal else 0].numpy(), corr)
        tol = 2e-6 * np.sqrt(hlen) * np.abs(x[b].numpy()).max() * np.abs(h.numpy()).max() * 30
        assert np.abs(y[b] - ref).max() <= tol + 1e-4
