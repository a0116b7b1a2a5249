"""Per-call SGEMM 4096^3 time from a cold start: how many calls until the
kernel reaches its steady-state time (clock ramp / first-touch effects that a
5-warmup / 20-step bench would see).  Prints one line per bucket of calls."""
import ctypes
import json
import sys

import torch

from veles.simd_amd import _lib

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
calls = int(sys.argv[2]) if len(sys.argv) > 2 else 400
lib = _lib.lib()
s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
a = torch.rand((n, n), device="cuda") * 2 - 1
b = torch.rand((n, n), device="cuda") * 2 - 1
c = torch.empty((n, n), device="cuda")
pa, pb, pc = (ctypes.c_void_p(t.data_ptr()) for t in (a, b, c))
torch.cuda.synchronize()
ev = [torch.cuda.Event(enable_timing=True) for _ in range(calls + 1)]
ev[0].record()
for i in range(calls):
    lib.vs_sgemm(0, 0, n, n, n, 1.0, pa, n, pb, n, 0.0, pc, n, s)
    ev[i + 1].record()
torch.cuda.synchronize()
ms = [ev[i].elapsed_time(ev[i + 1]) for i in range(calls)]
buckets = [(0, 5), (5, 10), (10, 25), (25, 50), (50, 100), (100, 200), (200, calls)]
out = {}
for lo, hi in buckets:
    seg = ms[lo:hi]
    if seg:
        out[f"{lo}-{hi}"] = round(2 * n ** 3 / (sum(seg) / len(seg)) / 1e9, 1)
print(json.dumps({"n": n, "tflops_by_call_bucket_gflops": out, "first10_ms": [round(x, 4) for x in ms[:10]]}))
