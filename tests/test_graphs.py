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


@pytest.mark.gpu
@pytest.mark.skip(reason="replaying this capture faulted the GPU (graph-owned scratch of several "
                         "MiB: partitioned overlap-save spectra, pyramid bands); the cause is "
                         "not established, so the library now refuses scratch above 1 MiB "
                         "inside a capture (test_capture_refuses_large_scratch) and this "
                         "pipeline can no longer be captured")
def test_capture_replay_partitioned_conv_and_tiled_wavelets():
    """The multi-kernel paths that take scratch from the pool inside the
    capture: uniformly partitioned overlap-save (forward / accumulate /
    inverse kernels), the tiled DWT pyramid in two passes and the tiled
    SWT.  Three replays with eager work in between, each checked against
    the eager result."""
    g = torch.Generator(device="cuda").manual_seed(3)
    x = torch.randn(3, 1 << 16, device="cuda", generator=g)
    h = torch.randn(40000, device="cuda", generator=g)

    def pipeline(x):
        y = ops.conv1d(x, h, algorithm="overlap_save")
        pyr = ops.wavedec(x, "daubechies", 8, levels=11)
        hi, lo = ops.swt(x, "daubechies", 4, levels=3)
        d_hi, d_lo = ops.dwt(x, "symlet", 8)
        return y, pyr, hi, lo, d_hi, d_lo

    cap = CapturedCall(pipeline, x)
    for seed in (1, 2, 3):
        g2 = torch.Generator(device="cuda").manual_seed(seed)
        x2 = torch.randn(x.shape, device="cuda", generator=g2)
        got = [t.clone() for t in cap(x2)]
        torch.cuda.synchronize()
        want = pipeline(x2)
        for a, b in zip(got, want):
            torch.testing.assert_close(a, b)


@pytest.mark.gpu
def test_capture_refuses_large_scratch():
    """A call that needs more than 1 MiB of scratch in one allocation
    (partitioned overlap-save keeps every block spectrum) reports an error
    when captured instead of recording a graph-owned allocation; nothing is
    replayed.  The same call runs eagerly afterwards."""
    from veles.simd_amd import _lib
    g = torch.Generator(device="cuda").manual_seed(4)
    x = torch.randn(3, 1 << 16, device="cuda", generator=g)
    h = torch.randn(40000, device="cuda", generator=g)
    want = ops.conv1d(x, h, algorithm="overlap_save")
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with pytest.raises(_lib.VelesError, match="stream capture"):
        with torch.cuda.graph(graph):
            ops.conv1d(x, h, algorithm="overlap_save")
    del graph
    torch.cuda.synchronize()
    torch.testing.assert_close(ops.conv1d(x, h, algorithm="overlap_save"), want)


@pytest.mark.gpu
def test_capture_sgemm_with_sliced_tail_uses_whole_tiles():
    """3072^3 runs with its tail tiles cut into k slices (a workspace of
    several MiB) when called eagerly; inside a capture the planner falls
    back to whole tiles (no scratch) and the replays match."""
    g = torch.Generator(device="cuda").manual_seed(5)
    a = torch.randn(3072, 3072, device="cuda", generator=g)
    b = torch.randn(3072, 3072, device="cuda", generator=g)
    cap = CapturedCall(ops.sgemm, a, b)
    for seed in (1, 2, 3):
        g2 = torch.Generator(device="cuda").manual_seed(seed)
        a2 = torch.randn(a.shape, device="cuda", generator=g2)
        b2 = torch.randn(b.shape, device="cuda", generator=g2)
        got = cap(a2, b2).clone()
        torch.cuda.synchronize()
        torch.testing.assert_close(got, ops.sgemm(a2, b2), rtol=1e-4, atol=1e-2)


def test_capture_requires_gpu():
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(RuntimeError):
        CapturedCall(lambda x: x, torch.zeros(1))
