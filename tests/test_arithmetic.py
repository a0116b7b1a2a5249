"""Port of the reference tests/arithmetic.cc + GPU checks of the
elementwise kernels against fp32/fp64 torch references."""
import ctypes

import numpy as np
import pytest

from veles.simd_amd import capi

F16_DATA = [12288, 16777, 18103, 49820, 17421, 18573, 18420, 49771, 24528, 2,
            32785, 168]
F16_REF = [0.125, 2.76757812, 6.71484375, -3.3046875, 4.05078125, 9.1015625,
           7.953125, -3.20898438, 500.066406, 0.0000001, -0.000001, 0.00001]


def _call_conv(name, src, out_dtype):
    src = np.ascontiguousarray(src)
    out = np.zeros(src.size, out_dtype)
    capi.fn(name)(capi.p(src), src.size, capi.p(out))
    return out


def test_float16_to_float_na_goldens():
    data = np.array(F16_DATA, np.uint16)
    out = _call_conv("float16_to_float_na", data, np.float32)
    for i in range(len(data) - 3):
        assert abs(out[i] - F16_REF[i]) <= abs(F16_REF[i]) / 1000
    for i in range(len(data) - 3, len(data)):
        assert abs(out[i] - F16_REF[i]) <= 0.2e-7
    special = np.array([32768, 0, 64512, 31744, 32256], np.uint16)
    out = _call_conv("float16_to_float_na", special, np.float32)
    assert out[0] == 0 and np.signbit(out[0])
    assert out[1] == 0 and not np.signbit(out[1])
    assert out[2] == -np.inf and out[3] == np.inf and np.isnan(out[4])


def test_float16_exhaustive_matches_numpy():
    data = np.arange(65536, dtype=np.uint16)
    out = _call_conv("float16_to_float", data, np.float32)
    ref = data.view(np.float16).astype(np.float32)
    same = (out.view(np.uint32) == ref.view(np.uint32)) | (np.isnan(out) & np.isnan(ref))
    assert same.all()


@pytest.mark.parametrize("name,src,out_dtype", [
    ("int16_to_int32", np.array([1, 2, 3, -150, 16000, -27000, 30], np.int16), np.int32),
    ("int32_to_int16", np.array([1, -15, -240, 25000, 30], np.int32), np.int16),
    ("int32_to_float", np.array([1, 1000000, -140, 31], np.int32), np.float32),
    ("float_to_int32", np.array([1, 24.1, 25.5, 26.8, -3.7], np.float32), np.int32),
    ("int16_to_float", np.array([1, -504, -18, -25000, 26000], np.int16), np.float32),
    ("float_to_int16", np.array([14.1, 15.5, 16.7, -2.9], np.float32), np.int16),
])
def test_conversions_match_na(name, src, out_dtype):
    # reference: memcmp(accelerated, _na) on misaligned slices (arithmetic.cc:223-333)
    for off in (0, 1):
        s = src[off:]
        np.testing.assert_array_equal(_call_conv(name, s, out_dtype),
                                      _call_conv(name + "_na", s, out_dtype))


def test_complex_and_real_multiply():
    a = np.array([1, 2, 3, 4, 5, 6, 7, 8], np.float32)
    b = np.array([-1.5, 1, 3.5, 3, -5.5, 6.5, 2, -9], np.float32)
    for name in ("complex_multiply", "complex_multiply_conjugate", "real_multiply"):
        res = np.zeros(8, np.float32)
        capi.fn(name)(capi.p(a), capi.p(b), capi.p(res))
        ca, cb = a.view(np.complex64), b.view(np.complex64)
        if name == "real_multiply":
            ref = a * b
        elif name == "complex_multiply":
            ref = (ca * cb).view(np.float32)
        else:
            ref = (ca * np.conj(cb)).view(np.float32)
        np.testing.assert_array_equal(res, ref)


def test_int16_multiply():
    a = np.arange(16, dtype=np.int16)
    b = (16 - np.arange(16)).astype(np.int16)
    res = np.zeros(16, np.int32)
    capi.fn("int16_multiply")(capi.p(a), capi.p(b), capi.p(res))
    np.testing.assert_array_equal(res, a.astype(np.int32) * b)


def test_real_multiply_scalar_and_sums():
    ar = np.arange(1, 20, dtype=np.float32)
    res = np.zeros(18, np.float32)
    capi.fn("real_multiply_scalar")(capi.p(ar[1:]), 18, 2.0, capi.p(res))
    np.testing.assert_array_equal(res, ar[1:] * 2)
    x = np.arange(100, dtype=np.float32)
    assert capi.fn("sum_elements")(capi.p(x), 100) == 4950.0
    assert capi.fn("next_highest_power_of_2")(100) == 128
    assert capi.fn("next_highest_power_of_2")(128) == 128


# --------------------------------------------------------------- GPU paths
@pytest.mark.gpu
def test_gpu_conversions_exact():
    import torch
    from veles.simd_amd import ops
    g = torch.Generator().manual_seed(0)
    i16 = torch.randint(-32768, 32767, (100003,), dtype=torch.int16, generator=g)
    i32 = torch.randint(-2**31, 2**31 - 1, (100003,), dtype=torch.int32, generator=g)
    f = (torch.rand(100003, generator=g) - 0.5) * 80000
    for x, dt in [(i16, torch.float32), (i32, torch.float32), (i16, torch.int32),
                  (i32, torch.int16), (f, torch.int32), (f, torch.int16)]:
        ref = ops.convert(x, dt)          # host semantics
        got = ops.convert(x.cuda(), dt).cpu()
        assert torch.equal(got, ref), (x.dtype, dt)
    h = torch.arange(65536, dtype=torch.int32).to(torch.int16).view(torch.float16)
    got = ops.convert(h.cuda(), torch.float32).cpu()
    ref = h.float()
    assert torch.equal(got.view(torch.int32)[~ref.isnan()],
                       ref.view(torch.int32)[~ref.isnan()])
    assert got[ref.isnan()].isnan().all()


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 7, 1000, 1 << 20, (1 << 20) + 3])
def test_gpu_elementwise(n):
    import torch
    from veles.simd_amd import ops
    a = torch.randn(n)
    b = torch.randn(n)
    ga, gb = a.cuda(), b.cuda()
    assert torch.equal(ops.add(ga, gb).cpu(), a + b)
    assert torch.equal(ops.sub(ga, gb).cpu(), a - b)
    assert torch.equal(ops.mul(ga, gb).cpu(), a * b)
    assert torch.equal(ops.affine(ga, 2.5).cpu(), a * 2.5)
    assert torch.equal(ops.affine(ga, 1.0, 0.75).cpu(), a + 0.75)
    torch.testing.assert_close(ops.saxpy(1.5, ga, gb).cpu(), 1.5 * a + b)
    s = ops.sum_all(ga).item()
    assert abs(s - a.double().sum().item()) <= 1e-5 * n ** 0.5 * 4 + 1e-5
    mm = ops.minmax(ga).cpu()
    assert mm[0] == a.min() and mm[1] == a.max()


@pytest.mark.gpu
def test_gpu_complex_and_misaligned():
    import torch
    from veles.simd_amd import ops
    a = torch.randn(2 * 4097)
    b = torch.randn(2 * 4097)
    for conj in (False, True):
        got = ops.complex_multiply(a.cuda(), b.cuda(), conj).cpu()
        torch.testing.assert_close(got, ops.complex_multiply(a, b, conj))
    # misaligned (offset 1 float) views take the scalar path
    x = torch.randn(1001).cuda()
    y = torch.randn(1001).cuda()
    torch.testing.assert_close(ops.add(x[1:], y[1:]), x[1:] + y[1:])
    conj = ops.complex_conjugate(a.cuda()).cpu()
    assert torch.equal(conj, ops.complex_conjugate(a))


@pytest.mark.gpu
def test_capi_large_array_goes_to_gpu():
    """Host arrays >= VELES_GPU_MIN_ELEMS run through the staged GPU path."""
    n = (1 << 20) + 5
    x = np.random.default_rng(1).standard_normal(n).astype(np.float32)
    res = np.zeros(n, np.float32)
    capi.fn("real_multiply_scalar")(capi.p(x), n, 3.0, capi.p(res))
    np.testing.assert_array_equal(res, x * np.float32(3.0))
    i16 = (np.arange(n) % 65536 - 32768).astype(np.int16)
    out = np.zeros(n, np.float32)
    capi.fn("int16_to_float")(capi.p(i16), n, capi.p(out))
    np.testing.assert_array_equal(out, i16.astype(np.float32))


def test_mismatched_alignment_is_accepted():
    """The reference EXPECT_DEATHs when src and dst have different 32-byte
    alignment under AVX (arithmetic.cc:234-332): an AVX-only contract.  This
    library has no alignment requirement (16-byte vector paths are chosen per
    call), so the same calls must return the _na result instead of dying."""
    src = np.arange(40, dtype=np.int16)
    for s_off in (0, 1, 3):
        for d_off in (0, 2):
            s = src[s_off:s_off + 30]
            out = np.zeros(30 + d_off, np.float32)[d_off:]
            fn = getattr(capi._lib.lib(), "int16_to_float")
            fn(capi.p(s), s.size, capi.p(out))
            np.testing.assert_array_equal(out, s.astype(np.float32))


@pytest.mark.gpu
@pytest.mark.parametrize("n,off", [(1 << 20, 0), ((1 << 20) + 3, 0), (4099, 1), (4098, 2), (1, 0)])
def test_complex_conjugate_device_paths(n, off):
    """float4 path (16-byte aligned) and scalar path (offset views), odd lengths:
    pairs conjugated, an odd trailing float left untouched."""
    import ctypes
    import torch
    from veles.simd_amd import _lib
    lib = _lib.lib()
    a = torch.randn(n + off, device="cuda")
    out = torch.full((n + off,), 9.0, device="cuda")
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    _lib.check(lib.vs_complex_conjugate(ctypes.c_void_p(a.data_ptr() + 4 * off),
                                        ctypes.c_void_p(out.data_ptr() + 4 * off), n, s),
               "vs_complex_conjugate")
    even = n & ~1
    want = a[off:off + even].clone()
    want[1::2] = -want[1::2]
    assert torch.equal(out[off:off + even], want)
    if n & 1:
        assert out[off + n - 1].item() == 9.0


@pytest.mark.gpu
@pytest.mark.parametrize("pairs", [0, 1])
@pytest.mark.parametrize("n,soff,doff", [(1 << 20, 0, 0), ((1 << 20) + 1, 3, 0),
                                         ((1 << 20) + 2, 2, 0), (4099, 1, 0), (4100, 0, 1),
                                         (7, 1, 0), (1, 0, 0)])
def test_reverse_device_paths(pairs, n, soff, doff):
    """vs_reverse: the float4 path (dst and src + n 16-byte aligned, n % 4 tail
    from the front of src), the scalar path, and complex-pair reversal."""
    import ctypes
    import torch
    from veles.simd_amd import _lib
    lib = _lib.lib()
    src = torch.randn(n + soff, device="cuda")
    dst = torch.full((n + doff,), 5.0, device="cuda")
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    _lib.check(lib.vs_reverse(ctypes.c_void_p(src.data_ptr() + 4 * soff),
                              ctypes.c_void_p(dst.data_ptr() + 4 * doff), n, pairs, s),
               "vs_reverse")
    x = src[soff:]
    if pairs:
        np_ = n // 2
        want = x[:2 * np_].reshape(np_, 2).flip(0).reshape(-1)
        assert torch.equal(dst[doff:doff + 2 * np_], want)
    else:
        assert torch.equal(dst[doff:], x.flip(0))
