#!/usr/bin/env python3
"""Run each SGEMM variant (and torch.matmul) a few times at one shape, for
rocprofv3 kernel-trace / PMC collection.  VARIANTS=2,3 SHAPE=4096 REPS=5."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from veles.simd_amd import _lib  # noqa: E402

lib = _lib.lib()
n = int(os.environ.get("SHAPE", "4096"))
reps = int(os.environ.get("REPS", "5"))
variants = [int(v) for v in os.environ.get("VARIANTS", "1,2").split(",")]
torch.backends.cuda.matmul.allow_tf32 = False
a = torch.rand(n, n, device="cuda") * 2 - 1
b = torch.rand(n, n, device="cuda") * 2 - 1
c = torch.empty(n, n, device="cuda")
s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
for v in variants:
    for _ in range(reps):
        st = lib.vs_sgemm_variant(v, 0, 0, n, n, n, ctypes.c_float(1.0),
                                  ctypes.c_void_p(a.data_ptr()), ctypes.c_int64(n),
                                  ctypes.c_void_p(b.data_ptr()), ctypes.c_int64(n),
                                  ctypes.c_float(0.0), ctypes.c_void_p(c.data_ptr()),
                                  ctypes.c_int64(n), s)
        assert st == 0
    torch.cuda.synchronize()
for _ in range(reps):
    torch.matmul(a, b, out=c)
torch.cuda.synchronize()
print("done")
