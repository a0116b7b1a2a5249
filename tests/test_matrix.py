"""Port of the reference tests/matrix.cc (goldens + MatrixTest sweep) plus
GPU-vs-fp64 checks of the MFMA SGEMM."""
import numpy as np
import pytest

from veles.simd_amd import capi

# simd=1 is the GPU path: run it (gpu-marked) where a GPU exists.
SIMDS = [0, pytest.param(1, marks=pytest.mark.gpu)]


def _fixture(w1, h1, w2, h2):
    # tests/matrix.cc:39-51: m1[i][j] = -j % 17 + i % 6, m2 = j % 15 - i % 5
    # (C semantics of -j % 17: the remainder keeps the sign of -j).
    i1, j1 = np.meshgrid(np.arange(h1), np.arange(w1), indexing="ij")
    m1 = (-(j1 % 17) + i1 % 6).astype(np.float32)
    i2, j2 = np.meshgrid(np.arange(h2), np.arange(w2), indexing="ij")
    m2 = (j2 % 15 - i2 % 5).astype(np.float32)
    return m1.ravel(), m2.ravel()


def test_add_validate():
    m1 = [1, 2, 3, -2, 0, 4]
    m2 = [0, 1, 3, 5, -1, 2]
    np.testing.assert_allclose(capi.matrix_add(0, m1, m2, 3, 2),
                               [1, 3, 6, 3, -1, 6], atol=0.01)


def test_sub_validate():
    m1 = [1, 2, 3, -2, 0, 4]
    m2 = [0, 1, 3, 5, -1, 2]
    np.testing.assert_allclose(capi.matrix_sub(0, m1, m2, 3, 2),
                               [1, 1, 0, -7, 1, 2], atol=0.01)


VALID = [1, -1, -5, 12, -12, -2, -22, 12]


@pytest.mark.parametrize("simd", SIMDS)
def test_multiply_validate(simd):
    m1 = [1, 2, 3, -2, 0, 4]
    m2 = [0, 1, 3, -2, 5, -1, 2, 4, -3, 0, -4, 2]
    np.testing.assert_allclose(capi.matrix_multiply(simd, m1, m2, 3, 2, 4, 3),
                               VALID, atol=0.01)


@pytest.mark.parametrize("simd", SIMDS)
def test_multiply_transposed_validate(simd):
    m1 = [1, 2, 3, -2, 0, 4]
    m2 = [0, 5, -3, 1, -1, 0, 3, 2, -4, -2, 4, 2]
    np.testing.assert_allclose(
        capi.matrix_multiply_transposed(simd, m1, m2, 3, 2, 3, 4), VALID,
        atol=0.01)


SWEEP = ([(d, d, d, d) for d in (1, 3, 99)] +
         [(128, 300, 1000, 128), (125, 299, 999, 125)])


@pytest.mark.gpu
@pytest.mark.parametrize("dims", SWEEP)
@pytest.mark.parametrize("kind", ["add", "sub", "mul", "mulT"])
def test_matrix_sweep(dims, kind):
    w1, h1, w2, h2 = dims
    if kind in ("add", "sub") and dims[0] == 128:
        pytest.skip("reference sweeps add/sub on the square sizes and 125x299")
    if kind == "mulT":
        w2, h2 = h2, w2
    m1, m2 = _fixture(w1, h1, w2, h2)
    if kind == "add":
        base = capi.matrix_add(0, m1, m2, w1, h1)
        simd = capi.matrix_add(1, m1, m2, w1, h1)
    elif kind == "sub":
        base = capi.matrix_sub(0, m1, m2, w1, h1)
        simd = capi.matrix_sub(1, m1, m2, w1, h1)
    elif kind == "mul":
        base = capi.matrix_multiply(0, m1, m2, w1, h1, w2, h2)
        simd = capi.matrix_multiply(1, m1, m2, w1, h1, w2, h2)
    else:
        base = capi.matrix_multiply_transposed(0, m1, m2, w1, h1, w2, h2)
        simd = capi.matrix_multiply_transposed(1, m1, m2, w1, h1, w2, h2)
    np.testing.assert_allclose(simd, base, atol=0.1)


@pytest.mark.gpu
def test_add_sub_125x299():
    m1, m2 = _fixture(125, 299, 125, 299)
    np.testing.assert_allclose(capi.matrix_add(1, m1, m2, 125, 299),
                               capi.matrix_add(0, m1, m2, 125, 299), atol=0.1)
    np.testing.assert_allclose(capi.matrix_sub(1, m1, m2, 125, 299),
                               capi.matrix_sub(0, m1, m2, 125, 299), atol=0.1)


@pytest.mark.gpu
@pytest.mark.parametrize("m,n,k", [(1, 1, 1), (33, 65, 17), (128, 128, 16),
                                   (299, 999, 125), (256, 512, 1024),
                                   (1000, 300, 256)])
@pytest.mark.parametrize("ta,tb", [(0, 0), (0, 1), (1, 0), (1, 1)])
def test_sgemm_gpu_vs_fp64(m, n, k, ta, tb):
    import torch
    from veles.simd_amd import ops
    g = torch.Generator().manual_seed(m * 7 + n * 3 + k)
    a = torch.rand((k, m) if ta else (m, k), generator=g) * 2 - 1
    b = torch.rand((n, k) if tb else (k, n), generator=g) * 2 - 1
    ref = ((a.double().T if ta else a.double()) @ (b.double().T if tb else b.double()))
    c = ops.sgemm(a.cuda(), b.cuda(), bool(ta), bool(tb)).cpu().double()
    err = (c - ref).abs().max().item()
    # exact-fp32 MFMA: error ~1e-7 * sum|a*b| <= 1e-7 * k
    assert err <= 2e-6 * k + 1e-6, err


@pytest.mark.gpu
def test_sgemm_identity_asymmetric():
    """A = I with an asymmetric B catches a transposed C/D map."""
    import torch
    from veles.simd_amd import ops
    n = 160
    b = torch.arange(n * n, dtype=torch.float32).reshape(n, n) / (n * n)
    c = ops.sgemm(torch.eye(n).cuda(), b.cuda()).cpu()
    assert torch.equal(c, b)


@pytest.mark.gpu
def test_sgemm_batched_and_alpha():
    import torch
    from veles.simd_amd import ops
    a = torch.randn(5, 70, 90)
    b = torch.randn(5, 90, 40)
    c = ops.sgemm(a.cuda(), b.cuda(), alpha=0.5).cpu()
    torch.testing.assert_close(c, 0.5 * torch.bmm(a.double(), b.double()).float(),
                               atol=1e-4, rtol=1e-4)


@pytest.mark.gpu
def test_sgemm_autograd():
    import torch
    from veles.simd_amd import ops
    a = torch.randn(37, 45, device="cuda", requires_grad=True)
    b = torch.randn(45, 29, device="cuda", requires_grad=True)
    ops.sgemm(a, b).sum().backward()
    a2 = a.detach().clone().requires_grad_()
    b2 = b.detach().clone().requires_grad_()
    (a2 @ b2).sum().backward()
    torch.testing.assert_close(a.grad, a2.grad, atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(b.grad, b2.grad, atol=1e-4, rtol=1e-4)


@pytest.mark.gpu
@pytest.mark.parametrize("variant", list(range(6)))
def test_sgemm_every_variant(variant):
    """Every SGEMM kernel variant (include/simd/gpu.h VS_SGEMM_VARIANTS) on
    an aligned NN shape (gen 5's shape) and on ragged / transposed shapes,
    against float64."""
    import ctypes
    import torch
    from veles.simd_amd import _lib
    lib = _lib.lib()
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    g = torch.Generator(device="cuda").manual_seed(variant)
    for (m, n, k, ta, tb) in [(512, 512, 256, 0, 0), (300, 257, 96, 0, 0), (256, 512, 64, 1, 1),
                              (129, 70, 33, 0, 1)]:
        a = torch.rand((k, m) if ta else (m, k), device="cuda", generator=g) - 0.5
        b = torch.rand((n, k) if tb else (k, n), device="cuda", generator=g) - 0.5
        c = torch.full((m, n), 3.0, device="cuda")
        _lib.check(lib.vs_sgemm_variant(variant, ta, tb, m, n, k, 1.0, a.data_ptr(), a.shape[1],
                                        b.data_ptr(), b.shape[1], 0.0, c.data_ptr(), n, s),
                   "vs_sgemm_variant")
        ref = (a.double().T if ta else a.double()) @ (b.double().T if tb else b.double())
        assert (c.double() - ref).abs().max().item() < 1e-5 * k + 1e-5, (variant, m, n, k)


@pytest.mark.gpu
@pytest.mark.parametrize("variant", [0, 1, 2, 3, 4, 5])
@pytest.mark.parametrize("k", [16, 32, 48, 64, 80, 96, 112, 128, 144, 4096, 5, 23, 100])
def test_sgemm_pipeline_depths(variant, k):
    """The LDS-DMA rings at every pipeline depth: 1, 2, 3 and more k tiles
    (prologue / drain paths of the counted-vmcnt schedule), beta != 0."""
    import ctypes
    import torch
    from veles.simd_amd import _lib
    lib = _lib.lib()
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    g = torch.Generator(device="cuda").manual_seed(k)
    m, n = 512, 256
    a = torch.rand(m, k, device="cuda", generator=g) - 0.5
    b = torch.rand(k, n, device="cuda", generator=g) - 0.5
    c = torch.rand(m, n, device="cuda", generator=g)
    ref = 0.5 * (a.double() @ b.double()) + 2.0 * c.double()
    _lib.check(lib.vs_sgemm_variant(variant, 0, 0, m, n, k, 0.5, a.data_ptr(), k, b.data_ptr(),
                                    n, 2.0, c.data_ptr(), n, s), "vs_sgemm_variant")
    assert (c.double() - ref).abs().max().item() < 1e-5 * k + 1e-5, (variant, k)


@pytest.mark.gpu
@pytest.mark.parametrize("m,n,k", [(2048, 2048, 512), (4096, 4096, 256)])
def test_sgemm_default_large_paths(m, n, k):
    """Default selection at sizes that pick the 128 x 128 and 256 x 256
    tiles."""
    import torch
    from veles.simd_amd import ops
    g = torch.Generator(device="cuda").manual_seed(m + k)
    a = torch.rand(m, k, device="cuda", generator=g) * 2 - 1
    b = torch.rand(k, n, device="cuda", generator=g) * 2 - 1
    c = ops.sgemm(a, b)
    ref = a.double() @ b.double()
    assert (c.double() - ref).abs().max().item() < 2e-6 * k


@pytest.mark.gpu
def test_host_api_pinned_operands_match_pageable():
    """Page-locked operands (vs_host_alloc) take the DMA / in-place staging
    path: same result as the pageable call, bit for bit (same kernel, same
    data)."""
    h1, w1, w2 = 300, 256, 1000
    rng = np.random.default_rng(11)
    a = rng.standard_normal(h1 * w1).astype(np.float32)
    b = rng.standard_normal(w1 * w2).astype(np.float32)
    bt = np.ascontiguousarray(b.reshape(w1, w2).T).ravel()
    want = capi.matrix_multiply(1, a, b, w1, h1, w2, w1)
    pins = [capi.PinnedArray(n) for n in (a.size, b.size, bt.size, h1 * w2)]
    try:
        pa, pb, pbt, got = (q.array for q in pins)
        pa[:], pb[:], pbt[:] = a, b, bt
        for _ in range(3):  # repeated calls reuse the mapping
            got[:] = np.nan
            capi.fn("matrix_multiply")(1, capi.p(pa), capi.p(pb), w1, h1, w2, w1, capi.p(got))
            np.testing.assert_array_equal(got, want)
        got[:] = np.nan
        capi.fn("matrix_multiply_transposed")(1, capi.p(pa), capi.p(pbt), w1, h1, w1, w2,
                                              capi.p(got))
        np.testing.assert_allclose(got, want, rtol=1e-5, atol=1e-4)
        # mixed: pinned inputs, pageable output
        np.testing.assert_array_equal(capi.matrix_multiply(1, pa, pb, w1, h1, w2, w1), want)
    finally:
        for q in pins:
            q.close()


@pytest.mark.gpu
def test_host_api_pinned_convolve():
    """A long pinned signal through the host convolution API."""
    n, m = 1 << 18, 257
    rng = np.random.default_rng(12)
    x = rng.standard_normal(n).astype(np.float32)
    h = rng.standard_normal(m).astype(np.float32)
    want = capi.convolve_simd(1, x, h)
    with capi.PinnedArray(n) as px:
        px[:] = x
        got = capi.convolve_simd(1, px, h)
    np.testing.assert_array_equal(got, want)


_STAGE_LIMIT_CODE = r"""
import numpy as np
from veles.simd_amd import capi
rng = np.random.default_rng(21)
h1, w1, w2 = 300, 256, 1000                      # operands of 0.3, 1.0 and 1.2 MB
a = rng.uniform(-1, 1, (h1, w1)).astype(np.float32)
b = rng.uniform(-1, 1, (w1, w2)).astype(np.float32)
ref = a.astype(np.float64) @ b.astype(np.float64)
for rep in range(3):                             # the image is reused call after call
    got = capi.matrix_multiply(1, a, b, w1, h1, w2, w1).reshape(h1, w2)
    assert np.abs(got - ref).max() <= 2e-6 * w1, rep
for n in (200, 700, 1500):                       # 0.16, 1.96 and 9 MB per operand
    x = rng.standard_normal((n, n)).astype(np.float32)
    y = rng.standard_normal((n, n)).astype(np.float32)
    assert np.array_equal(capi.matrix_add(1, x, y, n, n), (x + y).ravel()), n
    assert np.array_equal(capi.matrix_sub(1, x, y, n, n), (x - y).ravel()), n
x = rng.standard_normal(300000).astype(np.float32)
h = rng.standard_normal(500).astype(np.float32)
want = np.convolve(x.astype(np.float64), h.astype(np.float64))
assert np.abs(capi.convolve_simd(1, x, h) - want).max() <= 2e-3
v = rng.uniform(0.1, 6.0, 262144).astype(np.float32)
got = capi.psv("log_psv", 1, v).astype(np.float64)
assert (np.abs(got - np.log(v.astype(np.float64))) <= 4e-7 * np.abs(np.log(v)) + 5e-7).all()
# long maps go through the image in pieces of 262,144 elements, two in flight
for n in (2 * 262144, 3 * 262144 + 77, 5 * 262144 - 1):
    v = rng.uniform(0.1, 6.0, n).astype(np.float32)
    w = rng.uniform(-2.0, 2.0, n).astype(np.float32)
    v64, w64 = v.astype(np.float64), w.astype(np.float64)
    got = capi.psv("log_psv", 1, v).astype(np.float64)
    assert (np.abs(got - np.log(v64)) <= 4e-7 * np.abs(np.log(v64)) + 5e-7).all(), n
    s, c = capi.sincos_psv(1, v)
    assert np.abs(s - np.sin(v64)).max() <= 1e-6 and np.abs(c - np.cos(v64)).max() <= 1e-6, n
    got = capi.pow_psv(1, v, w).astype(np.float64)
    want = np.power(v64, w64)
    assert (np.abs(got - want) <= 4e-6 * np.abs(want) + 1e-6).all(), n
    inplace = v.copy()                                   # result over the input
    capi.fn("exp_psv")(1, capi.p(inplace), n, capi.p(inplace))
    assert (np.abs(inplace - np.exp(v64)) <= 4e-7 * np.exp(v64)).all(), n
# long signals are convolved in pieces with overlap-add between them
from scipy.signal import fftconvolve
for n, k in ((3 * (1 << 19) + 12345, 1000), (5 << 20, 4096)):
    x = rng.standard_normal(n).astype(np.float32)
    h = rng.standard_normal(k).astype(np.float32)
    want = fftconvolve(x.astype(np.float64), h.astype(np.float64))
    assert np.abs(capi.convolve_simd(1, x, h) - want).max() <= 4e-3, (n, k)
    res, _ = capi.run_handle("convolve", x, h)
    assert np.abs(res - want).max() <= 4e-3, (n, k)
    want = fftconvolve(x.astype(np.float64), h[::-1].astype(np.float64))
    assert np.abs(capi.convolve_simd(1, x, h, True) - want).max() <= 4e-3, (n, k)
print("stage-limit ok")
"""


@pytest.mark.gpu
@pytest.mark.parametrize("env", [
    {},                                                        # 4 MiB operands in a 16 MiB image
    {"VELES_STAGE_MAX_KB": "64"},                              # a pageable copy per large operand
    {"VELES_STAGE_MAX_KB": "4096", "VELES_STAGE_ARENA_MB": "2"},   # image full after one operand
    {"VELES_ZERO_COPY": "0"},                                  # outputs through the device image
    {"VELES_PIPELINED_MAP": "0"},                              # long maps as whole arrays
    {"VELES_STAGE_ARENA_MB": "0"},                             # no image: a copy per operand
], ids=["default", "limit64k", "image2m", "no_zero_copy", "no_pieces", "no_image"])
def test_host_api_staging_limits(env):
    """Pageable operands below and above the limit of the pinned staging image
    (VELES_STAGE_MAX_KB), with the image large, nearly full and bypassed: the
    same results on every path."""
    import os
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    e = dict(os.environ, PYTHONPATH=repo + os.pathsep + os.environ.get("PYTHONPATH", ""), **env)
    r = subprocess.run([sys.executable, "-c", _STAGE_LIMIT_CODE], env=e, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "stage-limit ok" in r.stdout
