#!/usr/bin/env python3
"""A/B the SGEMM tile variants in one process (interleaved rounds, median),
against torch.matmul (hipBLASLt, same transposes) on the same random data.
SHAPES="MxNxK:tt,..." (tt = nn / nt / tn / tt), VARIANTS="0,1,2,3,4", ROUNDS,
CHECK=0 skips the transpose check."""
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


def parse_shapes(spec):
    """"MxNxK:tt,..." with tt in nn / nt / tn / tt (A / B stored transposed)."""
    out = []
    for item in spec.split(","):
        dims, _, tt = item.partition(":")
        m, n, k = (int(v) for v in dims.split("x"))
        tt = tt or "nn"
        out.append((m, n, k, int(tt[0] == "t"), int(tt[1] == "t")))
    return out


def main():
    shapes = parse_shapes(os.environ.get(
        "SHAPES", "4096x4096x4096:nn,4096x4096x4096:nt,8192x8192x8192:nn,2048x2048x2048:nn,"
                  "300x1000x256:nn,300x1000x256:nt,299x999x125:nn,299x999x125:nt"))
    variants = [int(v) for v in os.environ.get("VARIANTS", "0,1,2").split(",")]
    rounds = int(os.environ.get("ROUNDS", "5"))
    if os.environ.get("CHECK", "1") == "1":
        check_transposes(variants)
    torch.backends.cuda.matmul.allow_tf32 = False
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    res = {}
    for (m, n, k, ta, tb) in shapes:
        a = torch.rand((k, m) if ta else (m, k), device="cuda") * 2 - 1
        b = torch.rand((n, k) if tb else (k, n), device="cuda") * 2 - 1
        ao = a.T if ta else a   # logical operands for torch (hipBLASLt transposes)
        bo = b.T if tb else b
        c = torch.empty(m, n, device="cuda")
        ref = ao.double() @ bo.double()
        reps = max(2, int(2e11 / (2 * m * n * k)))
        times = {v: [] for v in variants + ["torch"]}
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for r in range(rounds):
            for v in variants + ["torch"]:
                def run():
                    if v == "torch":
                        torch.matmul(ao, bo, out=c)
                    else:
                        st = lib.vs_sgemm_variant(v, ta, tb, m, n, k, 1.0, a.data_ptr(),
                                                  a.shape[1], b.data_ptr(), b.shape[1], 0.0,
                                                  c.data_ptr(), n, s)
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
                    assert os.environ.get("NOCHECK") or err < 1e-5 * k + 1e-4, (v, err)
        out = {str(v): round(2 * m * n * k / statistics.median(t) / 1e9, 1)
               for v, t in times.items()}
        tag = f"{m}x{n}x{k}:{'tn'[ta == 0]}{'tn'[tb == 0]}"
        res[tag] = out
        print(f"{tag} TFLOP/s (median of {rounds}):",
              out, flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
