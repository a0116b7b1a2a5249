#!/usr/bin/env python3
"""Time the GEMM modes at square sizes (median of interleaved rounds):
exact fp32 MFMA (vs_sgemm), bf16x3 fast fp32, bf16 matrix cores (NN through the
pack prepass, NT read in place; kernel variants: tools/bench_gemm_bf16.py), and torch.matmul fp32 / bf16 (hipBLASLt) for context.  TFLOP/s are
2 n^3 / t for every mode (the bf16x3 figure is fp32-equivalent throughput)."""
import ctypes
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from veles.simd_amd import _lib  # noqa: E402

lib = _lib.lib()


def main():
    sizes = [int(x) for x in os.environ.get("SIZES", "2048,4096,8192").split(",")]
    rounds = int(os.environ.get("ROUNDS", "5"))
    torch.backends.cuda.matmul.allow_tf32 = False
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    res = {}
    for n in sizes:
        a = torch.rand(n, n, device="cuda") * 2 - 1
        b = torch.rand(n, n, device="cuda") * 2 - 1
        ah, bh = a.bfloat16(), b.bfloat16()
        c = torch.empty(n, n, device="cuda")
        ref = (a[:128].double() @ b.double())
        modes = {
            "exact": lambda: lib.vs_sgemm(0, 0, n, n, n, 1.0, a.data_ptr(), n, b.data_ptr(), n,
                                          0.0, c.data_ptr(), n, s),
            "bf16x3": lambda: lib.vs_sgemm_bf16x3(0, 0, n, n, n, 1.0, a.data_ptr(), n,
                                                  b.data_ptr(), n, 0.0, c.data_ptr(), n, -1, s),
            "bf16": lambda: lib.vs_gemm_bf16_strided_batched(0, 0, n, n, n, 1.0, ah.data_ptr(),
                                                             n, 0, bh.data_ptr(), n, 0, 0.0,
                                                             c.data_ptr(), n, 0, 1, s),
            "bf16_nt": lambda: lib.vs_gemm_bf16_variant(-1, 0, 1, n, n, n, 1.0, ah.data_ptr(), n,
                                                        bh.data_ptr(), n, 0.0, c.data_ptr(), n,
                                                        s),
            "torch_fp32": lambda: torch.matmul(a, b, out=c),
            "torch_bf16": lambda: torch.matmul(ah, bh),
        }
        reps = max(3, int(3e11 / (2 * n ** 3)))
        times = {k: [] for k in modes}
        errs = {}
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for r in range(rounds):
            for k, fn in modes.items():
                st = fn()
                if isinstance(st, int) and st != 0:
                    raise RuntimeError(f"{k}: {lib.vs_last_error().decode()}")
                if r == 0 and not k.startswith("torch") and "_nt" not in k:
                    torch.cuda.synchronize()
                    errs[k] = (c[:128].double() - ref).abs().max().item()
                e0.record()
                for _ in range(reps):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                times[k].append(e0.elapsed_time(e1) / reps)
        out = {k: round(2 * n ** 3 / statistics.median(v) / 1e9, 1) for k, v in times.items()}
        res[n] = {"gflops": out, "max_abs_err_first128rows": errs}
        print(n, json.dumps(res[n]), flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
