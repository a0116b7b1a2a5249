"""HIP-graph capture of veles op sequences (veles.simd_amd.utils.graphs)."""
import pytest
import torch

from veles.simd_amd import ops
from veles.simd_amd.utils import CapturedCall


@pytest.mark.gpu
def test_capture_replay_matches_eager():
    g = torch.Generator(device="cuda").manual_seed(0)
    x = torch.randn(64, 4096, device="cuda", generator=g)
    h = torch.randn(129, device="cuda", generator=g)
    a = torch.randn(256, 192, device="cuda", generator=g)
    b = torch.randn(192, 128, device="cuda", generator=g)

    def pipeline(x, a, b):
        hi, lo = ops.swt(x, "daubechies", 8, levels=3)
        y = ops.conv1d(lo, h)
        c = ops.sgemm(a, b)
        return y, c, ops.sin(c)

    cap = CapturedCall(pipeline, x, a, b)
    for seed in (1, 2):
        g2 = torch.Generator(device="cuda").manual_seed(seed)
        x2 = torch.randn(x.shape, device="cuda", generator=g2)
        a2 = torch.randn(a.shape, device="cuda", generator=g2)
        b2 = torch.randn(b.shape, device="cuda", generator=g2)
        y, c, s = cap(x2, a2, b2)
        torch.cuda.synchronize()
        ye, ce, se = pipeline(x2, a2, b2)
        torch.testing.assert_close(y, ye)
        torch.testing.assert_close(c, ce)
        torch.testing.assert_close(s, se)


def test_capture_requires_gpu():
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(RuntimeError):
        CapturedCall(lambda x: x, torch.zeros(1))
