"""Grid-stride loops of the shared elementwise / helper kernels.

With the default cap (2^20 workgroups, csrc/runtime/runtime.cpp
elementwise_grid) no test input reaches a second pass of the loops shared
by map1 / map2 / cmul / fill / reverse and the conv / FFT helpers.  This
runs those paths in a child process with VS_EW_GRID_CAP=3 (the cap is read
once per process), so every launch strides, and compares against torch.
"""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import numpy as np, torch
from veles.simd_amd import ops
g = torch.Generator().manual_seed(3)
n = (1 << 20) + 13                   # ragged: vector body + scalar tail
a = torch.randn(n, generator=g).cuda(); b = torch.randn(n, generator=g).cuda()
torch.testing.assert_close(ops.add(a, b), a + b)
torch.testing.assert_close(ops.mul(a, b), a * b)
torch.testing.assert_close(ops.saxpy(1.5, a, b), 1.5 * a + b)
torch.testing.assert_close(ops.affine(a, 2.0, -1.0), 2 * a - 1)
torch.testing.assert_close(ops.sin(a), torch.sin(a), atol=1e-6, rtol=1e-6)
z = torch.randn(4, 1 << 12, 2, generator=g).cuda()
zc = torch.view_as_complex(z.contiguous())
torch.testing.assert_close(torch.view_as_complex(ops.fft(z).contiguous()),
                           torch.fft.fft(zc), atol=2e-3, rtol=1e-4)
zm = torch.randn(3, 4097, 2, generator=g).cuda()
w = torch.randn(3, 4097, 2, generator=g).cuda()
torch.testing.assert_close(torch.view_as_complex(ops.complex_multiply(zm, w).contiguous()),
                           torch.view_as_complex(zm.contiguous()) * torch.view_as_complex(w.contiguous()),
                           atol=1e-5, rtol=1e-5)
x = torch.randn(2, 300000, generator=g)
h = torch.randn(5000, generator=g)
for algo in ("fft", "overlap_save"):
    y = ops.conv1d(x.cuda(), h.cuda(), algorithm=algo).cpu().double().numpy()
    for r in range(2):
        ref = np.convolve(x[r].double().numpy(), h.double().numpy())
        assert np.abs(y[r] - ref).max() < 5e-2 * np.abs(ref).max() / 100 + 1e-2, algo
r = torch.randn(2, 1 << 22, generator=g).cuda()   # four-step r2c / c2r helpers
X = ops.rfft(r)
torch.testing.assert_close(ops.irfft(X, r.shape[-1]) / r.shape[-1], r, atol=2e-4, rtol=1e-4)
print("grid-stride ok")
'''


def test_helpers_with_tiny_grid_cap():
    env = dict(os.environ, VS_EW_GRID_CAP="3")
    r = subprocess.run([sys.executable, "-c", CHILD], cwd=ROOT, env=env, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0 and "grid-stride ok" in r.stdout, r.stdout[-2000:] + r.stderr[-3000:]
