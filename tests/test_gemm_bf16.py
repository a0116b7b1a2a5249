"""bf16 matrix-core GEMM and the bf16x3 fast-fp32 mode (csrc/kernels/gemm_bf16.hip).

Oracle: float64 torch matmul.  bf16 GEMM: inputs are exactly representable,
so only fp32 accumulation error remains.  bf16x3: the split x = hi + lo
leaves |x - hi - lo| <= 2^-17 |x| and the dropped lo*lo term is ~2^-16 of a
product, so each product carries <= ~3 * 2^-17 relative error; summed with
random signs over k that is ~3 * 2^-17 * sqrt(k) for operands in [-1, 1].
"""
import math

import pytest
import torch

from veles.simd_amd import ops

SHAPES = [(1, 1, 1), (3, 3, 3), (99, 99, 99), (300, 1000, 128), (299, 999, 125),
          (256, 256, 512), (1024, 768, 1000)]


@pytest.mark.gpu
@pytest.mark.parametrize("m,n,k", SHAPES)
@pytest.mark.parametrize("ta,tb", [(False, False), (False, True), (True, False), (True, True)])
def test_bf16x3_matches_fp64(m, n, k, ta, tb):
    g = torch.Generator(device="cuda").manual_seed(m * 7 + n + k)
    a = torch.rand((k, m) if ta else (m, k), device="cuda", generator=g) * 2 - 1
    b = torch.rand((n, k) if tb else (k, n), device="cuda", generator=g) * 2 - 1
    c = ops.sgemm_bf16x3(a, b, ta, tb)
    ref = (a.double().T if ta else a.double()) @ (b.double().T if tb else b.double())
    err = (c.double() - ref).abs().max().item()
    assert err <= 8 * 2.0 ** -17 * math.sqrt(k) + 1e-6, err


@pytest.mark.gpu
def test_bf16x3_is_much_better_than_bf16():
    g = torch.Generator(device="cuda").manual_seed(5)
    a = torch.rand(512, 2048, device="cuda", generator=g) * 2 - 1
    b = torch.rand(2048, 512, device="cuda", generator=g) * 2 - 1
    ref = a.double() @ b.double()
    e3 = (ops.sgemm_bf16x3(a, b).double() - ref).abs().max().item()
    e1 = (ops.gemm_bf16(a.bfloat16(), b.bfloat16()).double() - ref).abs().max().item()
    assert e3 * 50 < e1, (e3, e1)


@pytest.mark.gpu
def test_bf16x3_batched_and_alpha():
    g = torch.Generator(device="cuda").manual_seed(9)
    a = torch.rand(3, 130, 70, device="cuda", generator=g) - 0.5
    b = torch.rand(3, 70, 200, device="cuda", generator=g) - 0.5
    c = ops.sgemm_bf16x3(a, b, False, False, 0.5)
    ref = 0.5 * (a.double() @ b.double())
    assert (c.double() - ref).abs().max().item() < 1e-4


@pytest.mark.gpu
@pytest.mark.parametrize("m,n,k", SHAPES)
@pytest.mark.parametrize("ta,tb", [(False, False), (False, True), (True, True)])
def test_gemm_bf16_matches_fp64(m, n, k, ta, tb):
    g = torch.Generator(device="cuda").manual_seed(m + n * 3 + k)
    a = (torch.rand((k, m) if ta else (m, k), device="cuda", generator=g) * 2 - 1).bfloat16()
    b = (torch.rand((n, k) if tb else (k, n), device="cuda", generator=g) * 2 - 1).bfloat16()
    c = ops.gemm_bf16(a, b, ta, tb)
    assert c.dtype == torch.float32
    ref = (a.double().T if ta else a.double()) @ (b.double().T if tb else b.double())
    err = (c.double() - ref).abs().max().item()
    assert err <= 2e-6 * k + 1e-6, err


@pytest.mark.gpu
def test_gemm_bf16_batched_shared_b():
    g = torch.Generator(device="cuda").manual_seed(11)
    a = (torch.rand(4, 64, 96, device="cuda", generator=g) - 0.5).bfloat16()
    b = (torch.rand(96, 80, device="cuda", generator=g) - 0.5).bfloat16()
    c = ops.gemm_bf16(a, b)
    ref = a.double() @ b.double()
    assert (c.double() - ref).abs().max().item() < 1e-4


def test_cpu_fallback_semantics():
    a = torch.rand(5, 7)
    b = torch.rand(7, 3)
    torch.testing.assert_close(ops.sgemm_bf16x3(a, b), a @ b)
    torch.testing.assert_close(ops.gemm_bf16(a.bfloat16(), b.bfloat16()),
                               a.bfloat16().float() @ b.bfloat16().float())


def test_fake_tensor_shapes():
    from torch._subclasses.fake_tensor import FakeTensorMode
    with FakeTensorMode():
        a = torch.empty(4, 8, 16)
        b = torch.empty(16, 32)
        assert ops.sgemm_bf16x3(a, b).shape == (4, 8, 32)
        assert ops.gemm_bf16(a.bfloat16(), b.bfloat16(), False, False).dtype == torch.float32


@pytest.mark.gpu
@pytest.mark.parametrize("ta,tb", [(False, False), (True, True)])
def test_large_shapes_use_lds_dma_kernel(ta, tb):
    """>= 256 tiles of 256 x 128 select the global_load_lds pipelined kernel
    (ragged M / N / K exercise the zero-padded images)."""
    m, n, k = 4000, 2100, 520
    g = torch.Generator(device="cuda").manual_seed(3)
    a = torch.rand((k, m) if ta else (m, k), device="cuda", generator=g) * 2 - 1
    b = torch.rand((n, k) if tb else (k, n), device="cuda", generator=g) * 2 - 1
    ref = (a.double().T if ta else a.double()) @ (b.double().T if tb else b.double())
    c3 = ops.sgemm_bf16x3(a, b, ta, tb)
    assert (c3.double() - ref).abs().max().item() <= 8 * 2.0 ** -17 * math.sqrt(k) + 1e-6
    ah, bh = a.bfloat16(), b.bfloat16()
    c1 = ops.gemm_bf16(ah, bh, ta, tb)
    ref1 = (ah.double().T if ta else ah.double()) @ (bh.double().T if tb else bh.double())
    assert (c1.double() - ref1).abs().max().item() <= 2e-6 * k + 1e-6


@pytest.mark.gpu
@pytest.mark.parametrize("variant", [0, 1, 2, 3, 4])
def test_every_kernel_variant(variant):
    """Each bf16 / bf16x3 kernel variant on a ragged shape, NN and TT."""
    import ctypes
    from veles.simd_amd import _lib
    lib = _lib.lib()
    m, n, k = 1000, 700, 300
    g = torch.Generator(device="cuda").manual_seed(variant)
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    for ta, tb in ((0, 0), (1, 1)):
        a = torch.rand((k, m) if ta else (m, k), device="cuda", generator=g) * 2 - 1
        b = torch.rand((n, k) if tb else (k, n), device="cuda", generator=g) * 2 - 1
        c = torch.empty(m, n, device="cuda")
        _lib.check(lib.vs_sgemm_bf16x3(ta, tb, m, n, k, 1.0, a.data_ptr(), a.shape[1],
                                       b.data_ptr(), b.shape[1], 0.0, c.data_ptr(), n,
                                       variant, s), "bf16x3")
        ref = (a.double().T if ta else a.double()) @ (b.double().T if tb else b.double())
        assert (c.double() - ref).abs().max().item() <= 8 * 2.0 ** -17 * math.sqrt(k) + 1e-6
        ah, bh = a.bfloat16(), b.bfloat16()
        _lib.check(lib.vs_gemm_bf16_variant(variant, ta, tb, m, n, k, 1.0, ah.data_ptr(),
                                            ah.shape[1], bh.data_ptr(), bh.shape[1], 0.0,
                                            c.data_ptr(), n, s), "bf16")
        ref1 = (ah.double().T if ta else ah.double()) @ (bh.double().T if tb else bh.double())
        assert (c.double() - ref1).abs().max().item() <= 2e-6 * k + 1e-6


@pytest.mark.gpu
@pytest.mark.parametrize("variant", [0, 1, 2, 3, 4])
@pytest.mark.parametrize("ld_pad", [0, 8, 4])
def test_whole_tile_operands_read_in_place(variant, ld_pad):
    """bf16 operands stored K-contiguous with whole tiles skip the pack
    prepass and are read in place with their own row stride (ld_pad 0 / 8);
    a stride that is not 8-aligned (ld_pad 4) takes the packed path with
    scalar loads.  All four transpose combinations, so A and B each go
    in place and packed."""
    import ctypes
    from veles.simd_amd import _lib
    lib = _lib.lib()
    m, n, k = 512, 512, 256
    g = torch.Generator(device="cuda").manual_seed(100 + variant)
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    for ta, tb in ((0, 0), (0, 1), (1, 0), (1, 1)):
        ra, ca = (k, m) if ta else (m, k)
        rb, cb = (n, k) if tb else (k, n)
        af = (torch.rand(ra, ca + ld_pad, device="cuda", generator=g) * 2 - 1).bfloat16()
        bf = (torch.rand(rb, cb + ld_pad, device="cuda", generator=g) * 2 - 1).bfloat16()
        a, b = af[:, :ca], bf[:, :cb]
        c = torch.full((m, n), float("nan"), device="cuda")
        _lib.check(lib.vs_gemm_bf16_variant(variant, ta, tb, m, n, k, 1.0, a.data_ptr(),
                                            af.shape[1], b.data_ptr(), bf.shape[1], 0.0,
                                            c.data_ptr(), n, s), "bf16")
        ref = (a.double().T if ta else a.double()) @ (b.double().T if tb else b.double())
        assert (c.double() - ref).abs().max().item() <= 2e-6 * k + 1e-6, (ta, tb)


@pytest.mark.gpu
def test_batched_in_place_operands():
    """Strided-batched bf16 with every operand read in place (A batch
    stride, B shared with stride 0) and with B transposed per batch."""
    g = torch.Generator(device="cuda").manual_seed(21)
    a = (torch.rand(3, 256, 128, device="cuda", generator=g) - 0.5).bfloat16()
    b = (torch.rand(128, 256, device="cuda", generator=g) - 0.5).bfloat16()
    assert (ops.gemm_bf16(a, b).double() - a.double() @ b.double()).abs().max().item() < 1e-4
    bt = (torch.rand(3, 256, 128, device="cuda", generator=g) - 0.5).bfloat16()
    c = ops.gemm_bf16(a, bt, False, True)
    ref = a.double() @ bt.double().transpose(1, 2)
    assert (c.double() - ref).abs().max().item() < 1e-4
