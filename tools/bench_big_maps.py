#!/usr/bin/env python3
"""Long element-wise host-API calls on pageable arrays (math functions over 2^20 to
2^24 floats), microseconds per call and per MiB of input: the pieces of
pipelined_map (csrc/runtime/runtime.cpp) against the whole-array path
(VELES_PIPELINED_MAP=0)."""
import ctypes
import os
import statistics
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def child():
    import numpy as np
    from veles.simd_amd import capi
    sz = ctypes.c_size_t
    rng = np.random.default_rng(0)
    for n in (1 << 20, 1 << 22, 1 << 24):
        x = rng.uniform(0.1, 4.0, n).astype(np.float32)
        y = rng.uniform(-1.0, 1.0, n).astype(np.float32)
        out, out2 = np.empty_like(x), np.empty_like(x)
        calls = {
            "sin_psv": lambda: capi.fn("sin_psv")(1, capi.p(x), sz(n), capi.p(out)),
            "pow_psv": lambda: capi.fn("pow_psv")(1, capi.p(x), capi.p(y), sz(n), capi.p(out)),
            "sincos_psv": lambda: capi.fn("sincos_psv")(1, capi.p(x), sz(n), capi.p(out),
                                                        capi.p(out2)),
        }
        for name, fn in calls.items():
            for _ in range(3):
                fn()
            ts = []
            for _ in range(9):
                t0 = time.perf_counter()
                fn()
                ts.append((time.perf_counter() - t0) * 1e6)
            med = statistics.median(ts)
            print(f"{name:12s} {n:9d}: {med:8.0f} us  {med / (n * 4 / 2 ** 20):6.1f} us per MiB",
                  flush=True)


def main():
    if os.environ.get("BIGMAP_CHILD"):
        return child()
    for label, env in (("pieces (default)", {}), ("whole array (VELES_PIPELINED_MAP=0)",
                                                  {"VELES_PIPELINED_MAP": "0"})):
        print("==", label, flush=True)
        e = dict(os.environ, BIGMAP_CHILD="1", PYTHONPATH=REPO, **env)
        r = subprocess.run([sys.executable, os.path.abspath(__file__)], env=e, timeout=600)
        if r.returncode != 0:
            return r.returncode
    return 0


if __name__ == "__main__":
    sys.exit(main())
