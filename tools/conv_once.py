#!/usr/bin/env python3
"""One conv configuration a few times, for rocprofv3 kernel-trace / PMC runs.
XLEN=1048576 HLEN=4096 BATCH=64 ALGO=0 REPS=5 [OSLOG=14] [CONV_REAL=0/1/2]"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from veles.simd_amd import _lib  # noqa: E402

lib = _lib.lib()
xl = int(os.environ.get("XLEN", 1 << 20))
hl = int(os.environ.get("HLEN", 4096))
batch = int(os.environ.get("BATCH", 64))
algo = int(os.environ.get("ALGO", 0))
reps = int(os.environ.get("REPS", 5))
for knob in ("conv_real", "conv_buffer"):
    if knob.upper() in os.environ:
        lib.vs_tune_set(knob.encode(), int(os.environ[knob.upper()]))
if "OSLOG" in os.environ:
    lib.vs_tune_set(b"os_block_log_max", int(os.environ["OSLOG"]))
x = torch.randn(batch, xl, device="cuda")
h = torch.randn(hl, device="cuda")
yl = xl + hl - 1
y = torch.empty(batch, yl, device="cuda")
s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
for _ in range(reps):
    _lib.check(lib.vs_conv1d(algo, 0, ctypes.c_void_p(x.data_ptr()), xl, xl,
                             ctypes.c_void_p(h.data_ptr()), hl, 0,
                             ctypes.c_void_p(y.data_ptr()), yl, batch, s), "vs_conv1d")
torch.cuda.synchronize()
print("done")
