"""Which outputs of the real-block conv are wrong (debug probe)."""
import sys
import numpy as np
import torch
sys.path.insert(0, ".")
from veles.simd_amd import ops
from scipy.signal import fftconvolve

for (xl, hl, b, per) in [(40000, 3000, 3, True), (40000, 3000, 3, False), (40000, 3000, 1, False),
                         (9000, 2500, 1, False), (40000, 3001, 3, True)]:
    g = torch.Generator().manual_seed(1)
    x = torch.randn(b, xl, generator=g)
    h = torch.randn(b if per else 1, hl, generator=g)
    y = ops.conv1d(x.cuda(), h.cuda() if per else h[0].cuda(), algorithm="overlap_save").cpu().double().numpy()
    for r in range(b):
        ref = fftconvolve(x[r].double().numpy(), h[r if per else 0].double().numpy())
        bad = np.nonzero(np.abs(y[r] - ref) > 1e-2)[0]
        print(xl, hl, b, per, "row", r, "bad", len(bad), bad[:12], flush=True)
