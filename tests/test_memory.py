"""Port of reference tests/memory_test.cc (memory.h host helpers) through the
C library, plus the complex-reversed copy and zeropaddingex."""
import ctypes

import numpy as np
import pytest

from veles.simd_amd import _lib

pytestmark = pytest.mark.skipif(not _lib.available(), reason="native library not built")


def _fn(name, res, args):
    f = getattr(_lib.lib(), name)
    f.restype = res
    f.argtypes = args
    return f


_vp = ctypes.c_void_p
_libc = ctypes.CDLL(None)
_libc.free.argtypes = [_vp]


def _aligned(n, dtype, align=64):
    """numpy array of n elements whose data pointer is `align`-aligned."""
    itemsize = np.dtype(dtype).itemsize
    raw = np.zeros(n * itemsize + align, np.uint8)
    off = (-raw.ctypes.data) % align
    return raw[off:off + n * itemsize].view(dtype)


@pytest.mark.parametrize("name,dtype,cases", [
    ("align_complement_f32", np.float32, [(0, 0), (1, 7), (3, 5), (7, 1), (8, 0)]),
    ("align_complement_i16", np.int16, [(0, 0), (1, 15), (3, 13), (15, 1), (16, 0)]),
    ("align_complement_u16", np.uint16, [(0, 0), (1, 15), (16, 0)]),
    ("align_complement_i32", np.int32, [(0, 0), (1, 7), (3, 5), (7, 1), (8, 0)]),
    ("align_complement_u32", np.uint32, [(0, 0), (5, 3), (8, 0)]),
])
def test_align_complement(name, dtype, cases):
    """Elements to the next 32-byte boundary (reference memory_test.cc:18-45)."""
    f = _fn(name, ctypes.c_int, [_vp])
    a = _aligned(32, dtype, 32)
    for idx, want in cases:
        assert f(a.ctypes.data + idx * a.itemsize) == want


def test_malloc_aligned_and_offset():
    ma = _fn("malloc_aligned", _vp, [ctypes.c_size_t])
    mo = _fn("malloc_aligned_offset", _vp, [ctypes.c_size_t, ctypes.c_int])
    mf = _fn("mallocf", _vp, [ctypes.c_size_t])
    p = ma(100)
    assert p % 64 == 0
    _libc.free(p)
    p = mo(100, 3)
    assert p % 64 == 3
    _libc.free(p - 3)
    p = mf(100)
    assert p % 64 == 0
    _libc.free(p)


def test_memsetf():
    f = _fn("memsetf", None, [_vp, ctypes.c_float, ctypes.c_size_t])
    a = _aligned(102, np.float32, 32)
    f(a.ctypes.data + 3 * 4, 3.0, 99)
    assert np.all(a[3:102] == 3.0) and np.all(a[:3] == 0)


@pytest.mark.parametrize("n,want", [(100, 256), (128, 512), (1, 4), (1000, 2048)])
def test_zeropadding(n, want):
    """nl = 2^(floor(log2 n) + 2) (reference memory.c:131-137; test :91-108)."""
    f = _fn("zeropadding", _vp, [_vp, ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t)])
    src = np.ones(n, np.float32)
    nl = ctypes.c_size_t()
    p = f(src.ctypes.data, n, ctypes.byref(nl))
    assert nl.value == want and p % 64 == 0
    out = np.ctypeslib.as_array(ctypes.cast(p, ctypes.POINTER(ctypes.c_float)), (want,))
    assert np.all(out[:n] == 1) and np.all(out[n:] == 0)
    _libc.free(p)


def test_zeropaddingex():
    f = _fn("zeropaddingex", _vp, [_vp, ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t),
                                   ctypes.c_size_t])
    src = np.arange(100, dtype=np.float32)
    nl = ctypes.c_size_t()
    p = f(src.ctypes.data, 100, ctypes.byref(nl), 7)
    out = np.ctypeslib.as_array(ctypes.cast(p, ctypes.POINTER(ctypes.c_float)),
                                (nl.value + 7,))
    assert nl.value == 256
    np.testing.assert_array_equal(out[:100], src)
    assert np.all(out[100:256] == 0)  # the extra tail is uninitialised, as in the reference
    _libc.free(p)


def test_rmemcpyf():
    f = _fn("rmemcpyf", _vp, [_vp, _vp, ctypes.c_size_t])
    src = np.arange(25, dtype=np.float32)
    dst = np.zeros(25, np.float32)
    f(dst.ctypes.data + 4, src.ctypes.data + 4, 24)
    for i in range(1, 25):
        assert dst[i] == src[25 - i]


def test_crmemcpyf():
    """Reversed copy of interleaved complex pairs (reference memory.c:176-183)."""
    f = _fn("crmemcpyf", _vp, [_vp, _vp, ctypes.c_size_t])
    src = np.arange(20, dtype=np.float32)
    dst = np.zeros(20, np.float32)
    f(dst.ctypes.data, src.ctypes.data, 20)
    want = src.reshape(10, 2)[::-1].reshape(-1)
    np.testing.assert_array_equal(dst, want)
