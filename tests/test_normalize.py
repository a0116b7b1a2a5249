"""Port of reference tests/normalize.cc plus device checks."""
import ctypes

import numpy as np
import pytest

from veles.simd_amd import capi

# simd=1 is the GPU path: run it (gpu-marked) where a GPU exists.
SIMDS = [0, pytest.param(1, marks=pytest.mark.gpu)]


def _plane():
    a = np.ones(128 * 100, np.uint8)
    a[0], a[1], a[10], a[89], a[128 + 21] = 127, 15, 252, 31, 3
    return a


@pytest.mark.parametrize("simd", SIMDS)
def test_normalize2d(simd):
    src = _plane()
    res = np.zeros(100 * 100, np.float32)
    capi.fn("normalize2D")(simd, capi.p(src), 128, 100, 100, capi.p(res), 100)
    f = np.float32
    assert abs(res[0] - (f(2) * (127 - 1) / 251 - 1)) <= 1e-6
    np.testing.assert_allclose(res[1], f(2) * (15 - 1) / 251 - 1, rtol=1e-6)
    assert res[2] == -1.0 and res[10] == 1.0
    np.testing.assert_allclose(res[89], f(2) * (31 - 1) / 251 - 1, rtol=1e-6)
    np.testing.assert_allclose(res[121], f(2) * (3 - 1) / 251 - 1, rtol=1e-6)


@pytest.mark.parametrize("simd", SIMDS)
def test_minmax1d(simd):
    a = np.ones(100, np.float32)
    a[0], a[1], a[10], a[89], a[21] = 127, 15, 252, 31, 3
    mn, mx = ctypes.c_float(), ctypes.c_float()
    capi.fn("minmax1D")(simd, capi.p(a), 100, ctypes.byref(mn), ctypes.byref(mx))
    assert mx.value == 252 and mn.value == 1
    capi.fn("minmax1D")(simd, capi.p(a), 100, None, None)
    mx2 = ctypes.c_float()
    capi.fn("minmax1D")(simd, capi.p(a), 100, None, ctypes.byref(mx2))
    assert mx2.value == 252


@pytest.mark.parametrize("simd", SIMDS)
def test_minmax2d_and_flat(simd):
    src = _plane()
    mn, mx = ctypes.c_uint8(), ctypes.c_uint8()
    capi.fn("minmax2D")(simd, capi.p(src), 128, 100, 100, ctypes.byref(mn),
                        ctypes.byref(mx))
    assert (mn.value, mx.value) == (1, 252)
    # max == min: zeros row by row, row padding of dst untouched
    flat = np.full(64 * 10, 7, np.uint8)
    dst = np.full(40 * 10, 5.0, np.float32)
    capi.fn("normalize2D_minmax")(simd, 7, 7, capi.p(flat), 64, 30, 10,
                                  capi.p(dst), 40)
    d = dst.reshape(10, 40)
    assert (d[:, :30] == 0).all() and (d[:, 30:] == 5.0).all()


@pytest.mark.gpu
def test_normalize2d_device_large():
    import torch
    from veles.simd_amd import ops
    g = torch.Generator().manual_seed(3)
    x = torch.randint(3, 250, (1080, 1923), dtype=torch.uint8, generator=g)
    got = ops.normalize2d(x.cuda()).cpu()
    mn, mx = int(x.min()), int(x.max())
    want = (x.float() - mn) / np.float32((mx - mn) / 2.0) - 1.0
    torch.testing.assert_close(got, want, atol=0, rtol=0)
    assert torch.equal(ops.minmax(x.cuda()).cpu(), torch.tensor([mn, mx], dtype=torch.uint8))


@pytest.mark.gpu
@pytest.mark.parametrize("h,w,sstride,dstride,off", [
    (37, 1923, 1923, 1923, 0),     # odd width: rows drift in and out of alignment
    (64, 4096, 4096, 4096, 0),     # every row 16-aligned: all-vector path
    (50, 1000, 1003, 1001, 3),     # odd strides, source offset 3 bytes
    (1, 1 << 20, 1 << 20, 1 << 20, 0),  # one wide row: x blocks of the 2-D grid
    (3000, 5, 7, 6, 1),            # narrow rows: head / tail only
])
def test_normalize2d_device_strided(h, w, sstride, dstride, off):
    """vs_minmax2d_u8 / vs_normalize2d_u8 (16-byte / uchar4 -> float4 paths with
    scalar heads and tails) against the host formula on strided, offset planes."""
    import ctypes
    import torch
    from veles.simd_amd import _lib
    lib = _lib.lib()
    g = torch.Generator().manual_seed(h + w)
    buf = torch.randint(0, 256, (off + h * sstride + 16,), dtype=torch.uint8, generator=g)
    x = buf[off:off + h * sstride].reshape(h, sstride)[:, :w]
    mn, mx = int(x.min()), int(x.max())
    dbuf = torch.full((h * dstride + 4,), 7.0, device="cuda")
    src = buf.cuda()
    mm = torch.empty(2, dtype=torch.uint8, device="cuda")
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    sp = ctypes.c_void_p(src.data_ptr() + off)
    _lib.check(lib.vs_minmax2d_u8(sp, sstride, w, h, ctypes.c_void_p(mm.data_ptr()), s),
               "vs_minmax2d_u8")
    assert mm.cpu().tolist() == [mn, mx]
    # destination offset by one float: a 4-byte aligned, not 16-byte aligned start
    dp = ctypes.c_void_p(dbuf.data_ptr() + 4)
    _lib.check(lib.vs_normalize2d_u8(sp, sstride, w, h, ctypes.c_void_p(mm.data_ptr()), 0, 0,
                                     dp, dstride, s), "vs_normalize2d_u8")
    got = dbuf.cpu()[1:1 + h * dstride].reshape(h, dstride)
    want = (x.float() - mn) / np.float32((mx - mn) / 2.0) - 1.0
    torch.testing.assert_close(got[:, :w], want, atol=0, rtol=0)
    if dstride > w:
        assert (got[:, w:] == 7.0).all()


@pytest.mark.parametrize("dev", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
def test_batched_planes(dev):
    """A stack of planes in one launch: each plane normalised with its own
    min / max (one flat plane gives zeros), equal to the per-plane op."""
    import torch
    from veles.simd_amd import ops
    g = torch.Generator().manual_seed(4)
    img = torch.randint(0, 256, (5, 3, 37, 53), dtype=torch.uint8, generator=g)
    img[1, 2] = 77                                   # flat plane
    img[0, 0] = img[0, 0] // 4 + 100                 # narrow range
    x = img.to(dev)
    out = ops.normalize2d(x)
    mm = ops.minmax(x)
    assert out.shape == x.shape and mm.shape == (5, 3, 2)
    for i in range(5):
        for j in range(3):
            ref = ops.normalize2d(x[i, j])
            assert torch.equal(out[i, j], ref)
            assert mm[i, j, 0] == x[i, j].min() and mm[i, j, 1] == x[i, j].max()
    assert (out[1, 2] == 0).all()


@pytest.mark.gpu
def test_batched_planes_strided():
    """Planes cut out of a larger tensor (row stride > width, plane stride > plane)."""
    import torch
    from veles.simd_amd import ops
    big = torch.randint(0, 256, (4, 40, 64), dtype=torch.uint8, device="cuda")
    x = big[:, 3:35, 5:50]
    out = ops.normalize2d(x)
    for i in range(4):
        assert torch.equal(out[i], ops.normalize2d(x[i].contiguous()))
