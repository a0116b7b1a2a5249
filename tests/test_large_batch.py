"""Batches beyond one grid dimension (65535 blocks) are walked in chunks by
the native entry points (csrc/runtime/runtime.h batch_chunks)."""
import numpy as np
import pytest
import torch

from veles.simd_amd import ops

B = 70001  # > 65535 and not a multiple of it


@pytest.mark.gpu
def test_dwt_swt_large_batch():
    x = torch.randn(B, 32, device="cuda")
    hi, lo = ops.dwt(x, 0, 4, 0)
    hi2, lo2 = ops.dwt(x[-5:].contiguous(), 0, 4, 0)
    torch.testing.assert_close(hi[-5:], hi2)
    torch.testing.assert_close(lo[-5:], lo2)
    sh, sl = ops.swt_level(x, 0, 4, 2, 0)
    sh2, sl2 = ops.swt_level(x[-3:].contiguous(), 0, 4, 2, 0)
    torch.testing.assert_close(sh[-3:], sh2)


@pytest.mark.gpu
@pytest.mark.parametrize("algo", ["direct", "fft"])
def test_conv_large_batch(algo):
    x = torch.randn(B, 24, device="cuda")
    h = torch.randn(5, device="cuda")
    y = ops.conv1d(x, h, algorithm=algo)
    ref = torch.stack([torch.from_numpy(np.convolve(r, h.cpu().numpy()))
                       for r in x[-4:].cpu().numpy()])
    torch.testing.assert_close(y[-4:].cpu(), ref.float(), atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(y[:2].cpu(), torch.stack(
        [torch.from_numpy(np.convolve(r, h.cpu().numpy())) for r in x[:2].cpu().numpy()]
    ).float(), atol=1e-4, rtol=1e-4)


@pytest.mark.gpu
def test_fft_large_batch():
    x = torch.randn(B, 16, device="cuda")
    z = ops.rfft(x)
    ref = torch.fft.rfft(x[-7:].double().cpu())
    got = torch.view_as_complex(z[-7:].reshape(7, -1, 2).double().cpu().contiguous())
    torch.testing.assert_close(got, ref, atol=1e-4, rtol=1e-4)


@pytest.mark.gpu
def test_sgemm_large_batch():
    a = torch.randn(B, 3, 5, device="cuda")
    b = torch.randn(B, 5, 2, device="cuda")
    c = ops.sgemm(a, b)
    torch.testing.assert_close(c[-9:], torch.bmm(a[-9:], b[-9:]), atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(c[:9], torch.bmm(a[:9], b[:9]), atol=1e-4, rtol=1e-4)
