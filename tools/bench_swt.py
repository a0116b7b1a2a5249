#!/usr/bin/env python3
"""SWT multi-level throughput (benchmark config 4 shape: db8, 8 levels,
signals x 1024) against the HBM ceilings measured in the same process:
a write-only fill and a read+write copy of the same byte volume (torch).
Effective bytes = input + levels hi rows + final lo (each fp32).
ORDERS="8,16" LEVELS=8 SIGNALS=65536 LEN=1024 ROUNDS=5 KNOBS="name=a/b"."""
import ctypes
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from veles.simd_amd import _lib  # noqa: E402

lib = _lib.lib()
lib.vs_tune_set.argtypes = [ctypes.c_char_p, ctypes.c_int]


def timed(fn, reps):
    ev0, ev1 = torch.cuda.Event(True), torch.cuda.Event(True)
    fn()
    ev0.record()
    for _ in range(reps):
        fn()
    ev1.record()
    torch.cuda.synchronize()
    return ev0.elapsed_time(ev1) / reps * 1e-3


def main():
    orders = [int(v) for v in os.environ.get("ORDERS", "8").split(",")]
    levels = int(os.environ.get("LEVELS", 8))
    nsig = int(os.environ.get("SIGNALS", 65536))
    n = int(os.environ.get("LEN", 1024))
    rounds = int(os.environ.get("ROUNDS", 5))
    knobs = [kv.split("=") for kv in os.environ.get("KNOBS", "").split(",") if kv]
    arms = [("default", {})]
    for name, vals in knobs:
        arms += [(f"{name}={v}", {name: int(v)}) for v in vals.split("/")]
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    x = torch.randn(nsig, n, device="cuda")
    hi = torch.empty(nsig, levels, n, device="cuda")
    lo = torch.empty(nsig, n, device="cuda")
    packed = torch.empty(nsig, levels + 1, n, device="cuda") if os.environ.get("PACKED") == "1" else None
    if packed is not None:
        hi, lo = packed[:, :levels], packed[:, levels]
    nbytes = 4 * nsig * n * (levels + 2)
    res = {}
    # ceilings on the same volume (NO_CEIL=1 skips them)
    wbuf = torch.empty(nbytes // 4, device="cuda") if os.environ.get("NO_CEIL") != "1" else None
    half = torch.empty(nbytes // 8, device="cuda") if wbuf is not None else None
    half2 = torch.empty_like(half) if wbuf is not None else None
    if wbuf is not None:
        fill = statistics.median(timed(lambda: wbuf.fill_(1.0), 5) for _ in range(rounds))
        copy = statistics.median(timed(lambda: half2.copy_(half), 5) for _ in range(rounds))
        res["ceiling_fill_TBps"] = round(nbytes / fill / 1e12, 2)
        res["ceiling_copy_TBps"] = round(nbytes / copy / 1e12, 2)
    del wbuf, half, half2
    for order in orders:
        ref = None
        for name, kn in arms:
            for k, v in kn.items():
                lib.vs_tune_set(k.encode(), v)

            def run():
                if os.environ.get("PACKED") == "1":   # one [signals][levels + 1][len] array
                    st = lib.vs_swt_multilevel_packed(0, order, levels, 0,
                                                      ctypes.c_void_p(x.data_ptr()), n,
                                                      ctypes.c_void_p(packed.data_ptr()), nsig, s)
                else:
                    st = lib.vs_swt_multilevel(0, order, levels, 0, ctypes.c_void_p(x.data_ptr()),
                                               n, ctypes.c_void_p(hi.data_ptr()),
                                               ctypes.c_void_p(lo.data_ptr()), nsig, s)
                assert st == 0, lib.vs_last_error()
            run()
            torch.cuda.synchronize()
            if ref is None:
                ref = (hi[:64].clone(), lo[:64].clone())
            else:
                assert torch.allclose(hi[:64], ref[0], atol=1e-4), name
                assert torch.allclose(lo[:64], ref[1], atol=1e-4), name
            t = statistics.median(timed(run, 5) for _ in range(rounds))
            res[f"db{order}_{name}"] = {"ms": round(t * 1e3, 3),
                                        "TBps": round(nbytes / t / 1e12, 2),
                                        "Msamples_per_s": round(nsig * n / t / 1e6, 1)}
            for k in kn:
                lib.vs_tune_set(k.encode(), -1)
            print(f"db{order} {name}:", res[f"db{order}_{name}"], flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
