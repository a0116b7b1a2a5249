"""torch.library.opcheck over every veles:: custom op: schema, fake (meta)
kernel, autograd registration and the AOT dispatch path, on CPU tensors
here and on the device (gpu-marked).  The op list is checked against the
registered ops, so a new op without a row here fails."""
import pytest
import torch

from veles.simd_amd import ops  # noqa: F401  (registers the ops)

DEVICES = ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)]


def _samples(dev):
    g = torch.Generator().manual_seed(3)

    def r(*shape, dtype=torch.float32):
        return torch.randn(*shape, generator=g).to(dtype).to(dev)

    pos = (torch.rand(64, generator=g) + 0.5).to(dev)
    u8 = torch.randint(0, 255, (17, 23), dtype=torch.uint8, generator=g).to(dev)
    return {
        "affine": [(r(100), 2.0, -1.0)],
        "binary": [(r(33), r(33), "add"), (r(33), r(33), "mul")],
        "complex_conjugate": [(r(32),)],
        "complex_multiply": [(r(32), r(32), False), (r(32), r(32), True)],
        "conv1d": [(r(3, 200).requires_grad_(), r(17).requires_grad_(), 0, False),
                   (r(3, 200), r(3, 17), 1, True)],
        "conv1d_planned": [(r(2, 128).requires_grad_(), r(9), 0, 0, False)],
        "convert": [(r(40) * 100, torch.int16), (r(40).half(), torch.float32)],
        "detect_peaks": [(r(3, 200), 3), (r(1, 50), 1)],
        "dwt": [(r(4, 64), 0, 8, 0)],
        "fft": [(r(4, 64, 2), False), (r(4, 64, 2), True)],
        "gemm_bf16": [(r(32, 48, dtype=torch.bfloat16), r(48, 16, dtype=torch.bfloat16))],
        "irfft": [(r(2, 33, 2), 64)],
        "math": [(pos, "log"), (r(64), "sin")],
        "minmax": [(r(100),), (u8,), (u8.reshape(1, 17, 23).repeat(3, 1, 1),)],
        "normalize2d": [(u8,), (u8.reshape(1, 17, 23).repeat(2, 1, 1),)],
        "pow": [(pos, r(64))],
        "rfft": [(r(2, 64),)],
        "saxpy": [(0.5, r(50), r(50))],
        "sgemm": [(r(20, 30).requires_grad_(), r(30, 10).requires_grad_()),
                  (r(30, 20), r(10, 30), True, True)],
        "sgemm_bf16x3": [(r(20, 30), r(30, 10))],
        "sincos": [(r(64),)],
        "sum": [(r(1000),)],
        "swt": [(r(4, 64), 0, 8, 3, 0)],
        "swt_level": [(r(4, 64), 2, 4, 2, 1)],
        "wavedec": [(r(4, 64), 0, 4, 2, 0)],
    }


def _registered():
    return sorted(n.split("::")[1] for n in torch.library._defs if n.startswith("veles::")) \
        if hasattr(torch.library, "_defs") else None


def test_every_op_has_samples():
    names = sorted(k for k in dir(torch.ops.veles) if not k.startswith("_"))
    # torch.ops.veles only lists ops already touched; use the library's own registry
    import veles.simd_amd.ops as pkg
    import inspect
    found = set()
    for _, mod in inspect.getmembers(pkg, inspect.ismodule):
        src = inspect.getsource(mod)
        import re
        found |= set(re.findall(r'custom_op\("veles::([a-z0-9_]+)"', src))
    assert found == set(_samples("cpu")), (found ^ set(_samples("cpu")), names)


@pytest.mark.parametrize("dev", DEVICES)
@pytest.mark.parametrize("name", sorted(_samples("cpu")))
def test_opcheck(name, dev):
    op = getattr(torch.ops.veles, name).default
    for args in _samples(dev)[name]:
        torch.library.opcheck(op, args)


@pytest.mark.parametrize("dev", DEVICES)
def test_fixed_tap_fir_passes_gradient_to_x(dev):
    """FIRFilter / MatchedFilter with buffer taps (a cached Conv1dPlan on the
    GPU) still differentiate with respect to their input."""
    from veles.simd_amd import models
    g = torch.Generator().manual_seed(9)
    taps = torch.randn(33, generator=g)
    fir = models.FIRFilter(taps, mode="full").to(dev)
    x = torch.randn(3, 500, generator=g).to(dev).requires_grad_()
    w = torch.randn(3, 532, generator=g).to(dev)
    (fir(x) * w).sum().backward()
    xd = x.detach().double().cpu().requires_grad_()
    yd = torch.nn.functional.conv1d(xd[:, None], taps.double().flip(-1)[None, None],
                                    padding=32)[:, 0]
    (yd * w.double().cpu()).sum().backward()
    assert x.grad is not None
    torch.testing.assert_close(x.grad.double().cpu(), xd.grad, atol=1e-3, rtol=1e-3)
    if dev == "cuda":
        assert fir._plan is not None   # the planned path ran
    mf = models.MatchedFilter(taps).to(dev)
    x2 = torch.randn(2, 300, generator=g).to(dev).requires_grad_()
    resp, _ = mf(x2)
    resp.square().sum().backward()
    assert x2.grad is not None and torch.isfinite(x2.grad).all() and x2.grad.abs().sum() > 0


@pytest.mark.gpu
def test_fir_compiles_without_touching_the_plan():
    """Under torch.compile the cached-plan path is skipped (plan creation
    reads data pointers): the traced graph uses the conv1d custom op."""
    from veles.simd_amd import models
    fir = models.FIRFilter(torch.randn(65), mode="same").cuda()
    x = torch.randn(2, 4096, device="cuda")
    ref = fir(x)
    out = torch.compile(fir, backend="aot_eager")(x)
    torch.testing.assert_close(out, ref, atol=1e-4, rtol=1e-4)
