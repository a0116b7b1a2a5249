#!/usr/bin/env python3
"""bf16 GEMM variants against hipBLASLt (torch.matmul bf16), NT form (both
operands K-contiguous, read in place), interleaved rounds, TFLOP/s.
SIZES=4096,8192 VARIANTS=1,2 ROUNDS=7"""
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
    sizes = [int(x) for x in os.environ.get("SIZES", "4096,8192").split(",")]
    variants = [int(x) for x in os.environ.get("VARIANTS", "1,2").split(",")]
    rounds = int(os.environ.get("ROUNDS", "7"))
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    res = {}
    for n in sizes:
        a = (torch.rand(n, n, device="cuda") * 2 - 1).bfloat16()
        bt = (torch.rand(n, n, device="cuda") * 2 - 1).bfloat16()   # [n][k]
        c = torch.empty(n, n, device="cuda")
        ref = a[:128].double() @ bt.double().T
        arms = {f"v{v}": (lambda v=v: _lib.check(lib.vs_gemm_bf16_variant(
            v, 0, 1, n, n, n, ctypes.c_float(1.0), ctypes.c_void_p(a.data_ptr()), n,
            ctypes.c_void_p(bt.data_ptr()), n, ctypes.c_float(0.0), ctypes.c_void_p(c.data_ptr()),
            n, s), "vs_gemm_bf16_variant")) for v in variants}
        arms["hipblaslt"] = lambda: torch.matmul(a, bt.T)
        if os.environ.get("X3") == "1":   # the fast-fp32 mode on the same kernels (fp32 operands)
            af, bf = a.float(), bt.float().T.contiguous()
            for v in variants:
                arms[f"x3_v{v}"] = (lambda v=v: _lib.check(lib.vs_sgemm_bf16x3(
                    0, 0, n, n, n, ctypes.c_float(1.0), ctypes.c_void_p(af.data_ptr()), n,
                    ctypes.c_void_p(bf.data_ptr()), n, ctypes.c_float(0.0),
                    ctypes.c_void_p(c.data_ptr()), n, v, s), "vs_sgemm_bf16x3"))
        for name, fn in arms.items():
            fn()
            if name.startswith("v"):
                err = (c[:128].double() - ref).abs().max().item()
                assert err < 1e-2 * n ** 0.5, (name, err)
        for _ in range(50):   # clock ramp
            arms["hipblaslt"]()
        times = {k: [] for k in arms}
        e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
        reps = max(3, int(2e13 / (2 * n ** 3)))
        for _ in range(rounds):
            for name, fn in arms.items():
                fn()
                e0.record()
                for _ in range(reps):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                times[name].append(e0.elapsed_time(e1) / reps)
        res[n] = {k: round(2 * n ** 3 / statistics.median(v) / 1e9, 1) for k, v in times.items()}
        print(n, "TFLOP/s", res[n], flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
