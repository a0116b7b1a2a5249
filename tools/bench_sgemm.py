#!/usr/bin/env python3
"""A/B the SGEMM tile variants in one process (interleaved rounds, median),
against torch.matmul (hipBLASLt) on the same random data."""
import ctypes
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from veles.simd_amd import _lib  # noqa: E402

lib = _lib.lib()
lib.vs_sgemm_variant.argtypes = [ctypes.c_int] * 6 + [ctypes.c_float, ctypes.c_void_p,
                                 ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64,
                                 ctypes.c_float, ctypes.c_void_p, ctypes.c_int64,
                                 ctypes.c_void_p]


def check_transposes(variants):
    """Every variant x (ta, tb) on ragged shapes vs float64 torch."""
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    for (m, n, k) in [(300, 1000, 256), (257, 129, 95), (128, 256, 64), (1, 7, 3)]:
        for ta in (0, 1):
            for tb in (0, 1):
                a = torch.rand((k, m) if ta else (m, k), device="cuda") - 0.5
                b = torch.rand((n, k) if tb else (k, n), device="cuda") - 0.5
                ref = (a.double().T if ta else a.double()) @ (b.double().T if tb else b.double())
                for v in variants:
                    c = torch.full((m, n), 7.0, device="cuda")
                    st = lib.vs_sgemm_variant(v, ta, tb, m, n, k, 1.0, a.data_ptr(),
                                              a.shape[1], b.data_ptr(), b.shape[1], 0.0,
                                              c.data_ptr(), n, s)
                    assert st == 0, lib.vs_last_error()
                    err = (c.double() - ref).abs().max().item()
                    assert err < 1e-5 * k + 1e-5, (v, ta, tb, m, n, k, err)
    print("transpose check ok for variants", variants, flush=True)


def main():
    shapes = [(4096, 4096, 4096), (8192, 8192, 8192), (2048, 2048, 2048),
              (300, 1000, 256)]
    variants = [int(v) for v in os.environ.get("VARIANTS", "0,1,2,3,4").split(",")]
    rounds = int(os.environ.get("ROUNDS", "5"))
    check_transposes(variants)
    torch.backends.cuda.matmul.allow_tf32 = False
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    res = {}
    for (m, n, k) in shapes:
        a = torch.rand(m, k, device="cuda") * 2 - 1
        b = torch.rand(k, n, device="cuda") * 2 - 1
        c = torch.empty(m, n, device="cuda")
        ref = a.double() @ b.double()
        reps = max(2, int(2e11 / (2 * m * n * k)))
        times = {v: [] for v in variants + ["torch"]}
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for r in range(rounds):
            for v in variants + ["torch"]:
                def run():
                    if v == "torch":
                        torch.matmul(a, b, out=c)
                    else:
                        st = lib.vs_sgemm_variant(v, 0, 0, m, n, k, 1.0, a.data_ptr(), k,
                                                  b.data_ptr(), n, 0.0, c.data_ptr(), n, s)
                        assert st == 0, lib.vs_last_error()
                run()
                ev0.record()
                for _ in range(reps):
                    run()
                ev1.record()
                torch.cuda.synchronize()
                times[v].append(ev0.elapsed_time(ev1) / reps)
                if r == 0:
                    err = (c.double() - ref).abs().max().item()
                    assert err < 1e-5 * k + 1e-4, (v, err)
        out = {str(v): round(2 * m * n * k / statistics.median(t) / 1e9, 1)
               for v, t in times.items()}
        res[f"{m}x{n}x{k}"] = out
        print(f"{m}x{n}x{k} TFLOP/s (median of {rounds}):",
              {kk: round(vv / 1e3, 1) for kk, vv in out.items()}, flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
