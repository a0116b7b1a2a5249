"""nn.Module wrappers and autograd of the conv1d op (CPU here, GPU-marked
variants on the device)."""
import pytest
import torch

from veles.simd_amd import models, ops

DEVICES = ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)]


@pytest.mark.parametrize("dev", DEVICES)
@pytest.mark.parametrize("corr", [False, True])
@pytest.mark.parametrize("per_row", [False, True])
def test_conv1d_autograd(dev, corr, per_row):
    g = torch.Generator().manual_seed(5)
    x = torch.randn(3, 200, generator=g, dtype=torch.float64)
    h = torch.randn(3 if per_row else 1, 17, generator=g, dtype=torch.float64)
    if not per_row:
        h = h[0]
    xf = x.float().to(dev).requires_grad_()
    hf = h.float().to(dev).requires_grad_()
    y = ops.conv1d(xf, hf, correlate=corr)
    w = torch.randn(y.shape, generator=g).to(dev)
    (y * w).sum().backward()
    # fp64 reference through torch autograd
    xd = x.clone().requires_grad_()
    hd = h.clone().requires_grad_()
    k = hd if corr else hd.flip(-1)
    if per_row:
        yd = torch.nn.functional.conv1d(xd[None], k[:, None], padding=16, groups=3)[0]
    else:
        yd = torch.nn.functional.conv1d(xd[:, None], k[None, None], padding=16)[:, 0]
    (yd * w.double().cpu()).sum().backward()
    torch.testing.assert_close(xf.grad.cpu().double(), xd.grad, atol=1e-3, rtol=1e-3)
    torch.testing.assert_close(hf.grad.cpu().double(), hd.grad, atol=1e-3, rtol=1e-3)


@pytest.mark.parametrize("dev", DEVICES)
def test_modules(dev):
    g = torch.Generator().manual_seed(6)
    x = torch.randn(4, 1024, generator=g).to(dev)
    fir = models.FIRFilter(torch.ones(5) / 5, mode="same").to(dev)
    assert fir(x).shape == x.shape
    bands = models.WaveletDecomposition("db", 8, 3)(x)
    assert [b.shape[-1] for b in bands] == [512, 256, 128, 128]
    feats = models.WaveletEnergyFeatures(levels=4)(x)
    assert feats.shape == (4, 5) and torch.isfinite(feats).all()
    t = torch.sin(torch.arange(64) * 0.3).to(dev)
    resp, peaks = models.MatchedFilter(t, threshold=5.0)(x)
    assert resp.shape == (4, 1024 + 63) and len(peaks) == 4
    lin = models.Linear(1024, 10).to(dev)
    out = lin(x)
    torch.testing.assert_close(out, x @ lin.weight.T + lin.bias, atol=1e-3, rtol=1e-3)
    img = torch.randint(0, 255, (2, 31, 47), dtype=torch.uint8, generator=g).to(dev)
    nimg = models.ImageNormalizer()(img)
    assert nimg.shape == img.shape and nimg.min() >= -1 and nimg.max() <= 1


def test_torch_compile_fake_kernels():
    """Every custom op has a fake impl: FakeTensor tracing works."""
    from torch._subclasses.fake_tensor import FakeTensorMode
    with FakeTensorMode():
        x = torch.empty(4, 100)
        h = torch.empty(9)
        assert torch.ops.veles.conv1d(x, h, 0, False).shape == (4, 108)
        assert torch.ops.veles.sgemm(torch.empty(5, 7), torch.empty(7, 3)).shape == (5, 3)
        assert torch.ops.veles.swt(x, 0, 8, 3, 0).shape == (4, 4, 100)
        assert torch.ops.veles.rfft(torch.empty(2, 64)).shape == (2, 33, 2)
