"""vs_conv1d_plan_* (ops.Conv1dPlan): same results as vs_conv1d on every
path, filter spectra precomputed on the real-block FFT / overlap-save paths,
taps copied at creation, per-signal filters, and FIRFilter's cached plan."""
import pytest

pytestmark = pytest.mark.gpu


def _ref(x, h, algo, corr):
    from veles.simd_amd import ops
    return ops.conv1d(x, h, algorithm=algo, correlate=corr)


@pytest.mark.parametrize("xlen,hlen,batch,per_signal,algo,precomputed", [
    (100000, 4096, 3, False, "auto", True),          # overlap-save, M = 8192 real blocks
    (40000, 3000, 3, True, "overlap_save", True),    # per-signal filters
    (9000, 3000, 2, False, "fft", True),             # one real block
    (200000, 20000, 1, False, "auto", True),         # L = 32768 blocks (15 % rule)
    (5000, 16, 4, False, "auto", False),             # direct: taps copied, vs_conv1d
    (200000, 40000, 1, False, "overlap_save", True),   # partitioned: one P / Q table per partition
])
@pytest.mark.parametrize("corr", [False, True])
def test_plan_matches_conv1d(xlen, hlen, batch, per_signal, algo, precomputed, corr):
    import torch
    from veles.simd_amd import ops
    g = torch.Generator(device="cuda").manual_seed(xlen + hlen)
    x = torch.randn(batch, xlen, device="cuda", generator=g)
    h = torch.randn(batch if per_signal else 1, hlen, device="cuda", generator=g)
    hh = h if per_signal else h[0]
    plan = ops.Conv1dPlan(hh, xlen, algorithm=algo, correlate=corr)
    assert plan.precomputed == precomputed
    y = plan(x)
    ref = _ref(x, hh, algo, corr)
    scale = ref.abs().max().item()
    assert (y - ref).abs().max().item() <= 1e-5 * scale + 1e-5
    # the plan owns its copy: changing the taps does not change its output
    hh.mul_(2.0)
    torch.testing.assert_close(plan(x), y, atol=0, rtol=0)


def test_plan_batch_checks():
    import torch
    from veles.simd_amd import ops
    from veles.simd_amd._lib import VelesError
    h = torch.randn(3, 100, device="cuda")
    plan = ops.Conv1dPlan(h, 1000)
    with pytest.raises(VelesError):
        plan(torch.randn(2, 1000, device="cuda"))   # 3 per-signal filters, batch 2
    with pytest.raises(ValueError):
        plan(torch.randn(3, 999, device="cuda"))    # wrong signal length


def test_fir_filter_uses_cached_plan():
    import torch
    from veles.simd_amd import models, ops
    taps = torch.randn(2048, device="cuda")
    fir = models.FIRFilter(taps, mode="same").cuda().eval()
    x = torch.randn(4, 50000, device="cuda")
    with torch.no_grad():
        y1 = fir(x)
        plan = fir._plan
        y2 = fir(x)
    assert fir._plan is plan and plan.precomputed
    ref = ops.conv1d(x, taps)[..., 1023: 1023 + 50000]
    torch.testing.assert_close(y1, ref, atol=1e-3, rtol=1e-4)
    torch.testing.assert_close(y2, y1, atol=0, rtol=0)
    with torch.no_grad():
        fir.taps.mul_(0.5)                            # new version -> new plan
        y3 = fir(x)
    assert fir._plan is not plan
    torch.testing.assert_close(y3, 0.5 * y1, atol=1e-3, rtol=1e-4)
