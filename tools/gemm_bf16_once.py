#!/usr/bin/env python3
"""A few bf16 GEMM calls for counter collection: N^3 (env N, default 8192),
NT layout by default (both operands read in place; TB=0: NN), env VARIANT
(default 2)."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from veles.simd_amd import _lib  # noqa: E402

n = int(os.environ.get("N", "8192"))
v = int(os.environ.get("VARIANT", "2"))
tb = int(os.environ.get("TB", "1"))  # 0: NN (B stored [K][N])
lib = _lib.lib()
a = (torch.rand(n, n, device="cuda") - 0.5).bfloat16()
b = (torch.rand(n, n, device="cuda") - 0.5).bfloat16()
c = torch.empty(n, n, device="cuda")
s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
for _ in range(int(os.environ.get("REPS", "5"))):
    _lib.check(lib.vs_gemm_bf16_variant(v, 0, tb, n, n, n, 1.0, a.data_ptr(), n, b.data_ptr(),
                                        n, 0.0, c.data_ptr(), n, s), "bf16")
if os.environ.get("TORCH") == "1":   # hipBLASLt on the same operands, for the counters
    for _ in range(3):
        torch.matmul(a, b.T if tb else b)
torch.cuda.synchronize()
print("ok")
