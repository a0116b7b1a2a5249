"""The SGEMM kernel family (csrc/kernels/sgemm.hip sgemm_kernel): every
transpose combination, ragged M / N / K (buffer LDS-DMA whose out-of-range
lanes read zeros), 16- and 4-byte DMA, beta, batches and every pipeline
depth, against float64.  Reference: /root/reference/src/matrix.c:255-343
(matrix_multiply / matrix_multiply_transposed), /root/reference/tests/
matrix.cc:159-204 (the 299 x 125 x 999 odd shapes)."""
import ctypes

import pytest

pytestmark = pytest.mark.gpu
# 0 / 1 / 2: 64 x 64, 128 x 128, 256 x 256 tiles with automatic k slicing
# (workspace + reduction), 3 / 4 / 5: the same, whole tiles only
VARIANTS = [0, 1, 2, 3, 4, 5]


def _run(variant, m, n, k, ta, tb, lda_pad=0, ldb_pad=0, alpha=1.0, beta=0.0, seed=0,
         offset=0):
    import torch
    from veles.simd_amd import _lib
    lib = _lib.lib()
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    g = torch.Generator(device="cuda").manual_seed(seed + m + 3 * n + 7 * k)
    ra, ca = (k, m) if ta else (m, k)
    rb, cb = (n, k) if tb else (k, n)
    lda, ldb = ca + lda_pad, cb + ldb_pad
    abuf = torch.rand(ra * lda + offset, device="cuda", generator=g) - 0.5
    bbuf = torch.rand(rb * ldb + offset, device="cuda", generator=g) - 0.5
    a = abuf[offset:].view(ra, lda)[:, :ca]
    b = bbuf[offset:].view(rb, ldb)[:, :cb]
    c = torch.rand(m, n, device="cuda", generator=g)
    ref = alpha * ((a.double().T if ta else a.double()) @ (b.double().T if tb else b.double()))
    ref += beta * c.double()
    _lib.check(lib.vs_sgemm_variant(variant, ta, tb, m, n, k, alpha, a.data_ptr(), lda,
                                    b.data_ptr(), ldb, beta, c.data_ptr(), n, s),
               "vs_sgemm_variant")
    err = (c.double() - ref).abs().max().item()
    assert err < 2e-6 * k + 1e-5, (variant, m, n, k, ta, tb, err)


@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("ta,tb", [(0, 0), (0, 1), (1, 0), (1, 1)])
@pytest.mark.parametrize("m,n,k", [(512, 512, 256), (300, 1000, 256), (299, 999, 125),
                                   (1, 1, 1), (129, 70, 33), (257, 513, 16), (64, 300, 1000)])
def test_gen6_shapes(variant, ta, tb, m, n, k):
    _run(variant, m, n, k, ta, tb)


@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("ta,tb", [(0, 0), (0, 1), (1, 0), (1, 1)])
def test_gen6_unaligned_and_beta(variant, ta, tb):
    """4-byte DMA: leading dimensions and base addresses not multiples of 4."""
    _run(variant, 200, 136, 100, ta, tb, lda_pad=1, ldb_pad=3, offset=1, alpha=0.5, beta=2.0)
    _run(variant, 256, 256, 128, ta, tb, lda_pad=4, ldb_pad=8, alpha=-1.0, beta=0.5)


@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("k", [4, 16, 32, 48, 64, 80, 100, 4096])
def test_gen6_pipeline_depths(variant, k):
    _run(variant, 512, 256, k, 0, 1, beta=1.0)
    _run(variant, 512, 256, k, 0, 0, beta=1.0)


@pytest.mark.parametrize("variant", VARIANTS)
def test_gen6_batched(variant):
    import torch
    from veles.simd_amd import _lib
    lib = _lib.lib()
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    a = torch.randn(3, 130, 70, device="cuda")
    b = torch.randn(3, 90, 70, device="cuda")      # NT
    c = torch.zeros(3, 130, 90, device="cuda")
    for i in range(3):
        _lib.check(lib.vs_sgemm_variant(variant, 0, 1, 130, 90, 70, 1.0, a[i].data_ptr(), 70,
                                        b[i].data_ptr(), 70, 0.0, c[i].data_ptr(), 90, s),
                   "vs_sgemm_variant")
    ref = torch.bmm(a.double(), b.double().transpose(1, 2))
    assert (c.double() - ref).abs().max().item() < 1e-4


@pytest.mark.parametrize("variant", [0, 1, 2])
@pytest.mark.parametrize("ta,tb", [(0, 0), (0, 1), (1, 1)])
def test_gen6_split_k(variant, ta, tb):
    """Deep K on few output tiles: split into >= 256-deep slices, reduced
    with alpha / beta applied once."""
    _run(variant, 100, 130, 8192, ta, tb, alpha=0.5, beta=-1.5)
    _run(variant, 300, 257, 3001, ta, tb, alpha=2.0, beta=0.0)


@pytest.mark.parametrize("ta,tb", [(0, 0), (1, 1)])
def test_k_zero_scales_c(ta, tb):
    """k = 0: C = beta C, and exactly 0 for beta = 0 (no product is read)."""
    import torch
    from veles.simd_amd import _lib
    lib = _lib.lib()
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    a = torch.empty(4, device="cuda")
    c = torch.full((37, 53), 3.0, device="cuda")
    c[0, 0] = float("nan")
    _lib.check(lib.vs_sgemm(ta, tb, 37, 53, 0, 1.0, a.data_ptr(), 37 if ta else 1,
                            a.data_ptr(), 1 if tb else 53, 0.5, c.data_ptr(), 53, s), "vs_sgemm")
    assert torch.isnan(c[0, 0]) and (c.flatten()[1:] == 1.5).all()
    _lib.check(lib.vs_sgemm(ta, tb, 37, 53, 0, 1.0, a.data_ptr(), 37 if ta else 1,
                            a.data_ptr(), 1 if tb else 53, 0.0, c.data_ptr(), 53, s), "vs_sgemm")
    assert (c == 0).all()


@pytest.mark.parametrize("variant", [0, 1, 2])
@pytest.mark.parametrize("ta,tb", [(0, 0), (0, 1), (1, 0)])
def test_tail_tiles_sliced(variant, ta, tb):
    """More tiles than CUs with a remainder: the whole tiles run first, the
    remainder is cut into k slices (partials in a workspace, reduced with
    alpha / beta applied once).  Ragged edges fall into sliced tiles."""
    dim = (64, 128, 256)[variant]
    # 17 x 17 = 289 tiles on 256 CUs -> 33 sliced; the last row / column ragged
    m = n = 16 * dim + dim // 2 + 4
    _run(variant, m, n, 384, ta, tb, alpha=0.75, beta=0.5, seed=variant)


@pytest.mark.parametrize("variant", [0, 1, 2, 3])
def test_batched_units(variant):
    """Strided batches: few tiles per matrix (sliced, per-batch workspace
    slabs) and many (whole tiles)."""
    import torch
    from veles.simd_amd import _lib
    lib = _lib.lib()
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    for (bt, m, n, k) in [(3, 200, 136, 1024), (5, 384, 520, 96)]:
        g = torch.Generator(device="cuda").manual_seed(bt)
        a = torch.rand(bt, m, k, device="cuda", generator=g) - 0.5
        b = torch.rand(bt, k, n, device="cuda", generator=g) - 0.5
        c = torch.rand(bt, m, n, device="cuda", generator=g)
        ref = 1.5 * torch.bmm(a.double(), b.double()) - 0.5 * c.double()
        _lib.check(lib.vs_sgemm_variant_batched(variant, 0, 0, m, n, k, 1.5, a.data_ptr(), k,
                                                m * k, b.data_ptr(), n, k * n, -0.5,
                                                c.data_ptr(), n, m * n, bt, s),
                   "vs_sgemm_variant_batched")
        assert (c.double() - ref).abs().max().item() < 2e-6 * k + 1e-5, (variant, bt, m, n, k)
