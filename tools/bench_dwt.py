#!/usr/bin/env python3
"""DWT pyramid throughput (vs_dwt_multilevel): signals x len, db-order,
levels; effective bytes = input + output (the pyramid is len floats per
signal), against a torch copy of the same volume in the same process.
ORDERS=8 LEVELS=5 SIGNALS=65536 LEN=1024 ROUNDS=5 VEC=1,0 (vs_tune_set dwt_vec arms)
THREADS=0 (dwt_threads arms, comma list; 0 = auto)
SINGLE=1 times one decimated level (vs_dwt: hi and lo of len / 2) instead."""
import ctypes
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from veles.simd_amd import _lib  # noqa: E402

lib = _lib.lib()


def timed(fn, reps=5):
    ev0, ev1 = torch.cuda.Event(True), torch.cuda.Event(True)
    fn()
    ev0.record()
    for _ in range(reps):
        fn()
    ev1.record()
    torch.cuda.synchronize()
    return ev0.elapsed_time(ev1) / reps * 1e-3


def main():
    orders = [int(v) for v in os.environ.get("ORDERS", "2,8,16").split(",")]
    levels = int(os.environ.get("LEVELS", 5))
    nsig = int(os.environ.get("SIGNALS", 65536))
    n = int(os.environ.get("LEN", 1024))
    rounds = int(os.environ.get("ROUNDS", 5))
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    x = torch.randn(nsig, n, device="cuda")
    out = torch.empty(nsig, n, device="cuda")
    nbytes = 8 * nsig * n
    res = {"copy_TBps": round(nbytes / statistics.median(
        timed(lambda: out.copy_(x)) for _ in range(rounds)) / 1e12, 2)}
    vecs = [int(a) for a in os.environ.get("VEC", "1,0").split(",")]
    thr = [int(a) for a in os.environ.get("THREADS", "0").split(",")]
    for k in ("dwt_tile", "dwt_halo_div"):   # DWT_TILE / DWT_HALO_DIV: tiled-pass knobs
        if os.environ.get(k.upper()):
            assert lib.vs_tune_set(k.encode(), int(os.environ[k.upper()])) == 0
    for vec, nt, order in [(v, t, o) for v in vecs for t in thr for o in orders]:
        assert lib.vs_tune_set(b"dwt_vec", vec) == 0
        assert lib.vs_tune_set(b"dwt_threads", nt) == 0

        def run():
            if os.environ.get("SINGLE") == "1":
                st = lib.vs_dwt(0, order, 0, ctypes.c_void_p(x.data_ptr()), n, n,
                                ctypes.c_void_p(out.data_ptr()),
                                ctypes.c_void_p(out.data_ptr() + 2 * n * nsig), n // 2, nsig, s)
            else:
                st = lib.vs_dwt_multilevel(0, order, levels, 0, ctypes.c_void_p(x.data_ptr()), n,
                                           ctypes.c_void_p(out.data_ptr()), nsig, s)
            assert st == 0, lib.vs_last_error()
        t = statistics.median(timed(run) for _ in range(rounds))
        key = f"db{order}_vec{vec}" + (f"_t{nt}" if nt else "")
        res[key] = {"ms": round(t * 1e3, 3), "TBps": round(nbytes / t / 1e12, 2)}
        print(key, res[key], flush=True)
    lib.vs_tune_set(b"dwt_vec", -1)
    lib.vs_tune_set(b"dwt_threads", -1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
