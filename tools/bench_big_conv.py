#!/usr/bin/env python3
"""convolve_simd on long pageable host arrays, pieces (piped_conv in
csrc/api/convolve.cpp) against the whole-signal path (VELES_PIPELINED_MAP=0)."""
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
    for n, k in ((1 << 21, 512), (1 << 22, 4096), (1 << 24, 4096), (1 << 24, 65536)):
        x = rng.standard_normal(n, dtype=np.float32)
        h = rng.standard_normal(k, dtype=np.float32)
        y = np.empty(n + k - 1, np.float32)
        for name in ("convolve_simd", "convolve"):
            if name == "convolve_simd":
                fn = lambda: capi.fn(name)(1, capi.p(x), sz(n), capi.p(h), sz(k), capi.p(y))  # noqa: E731
            else:
                handle = capi.fn("convolve_initialize")(n, k)
                fn = lambda: capi.fn("convolve")(handle, capi.p(x), capi.p(h), capi.p(y))  # noqa: E731
            for _ in range(2):
                fn()
            ts = []
            for _ in range(5):
                t0 = time.perf_counter()
                fn()
                ts.append((time.perf_counter() - t0) * 1e6)
            med = statistics.median(ts)
            print(f"{name:14s} {n:9d} x {k:6d}: {med:8.0f} us  {med / (n * 4 / 2 ** 20):6.1f} us per MiB",
                  flush=True)
            if name == "convolve":
                capi.fn("convolve_finalize")(handle)


def main():
    if os.environ.get("BIGCONV_CHILD"):
        return child()
    for label, env in (("pieces (default)", {}),
                       ("whole signal (VELES_PIPELINED_MAP=0)", {"VELES_PIPELINED_MAP": "0"})):
        print("==", label, flush=True)
        e = dict(os.environ, BIGCONV_CHILD="1", PYTHONPATH=REPO, **env)
        r = subprocess.run([sys.executable, os.path.abspath(__file__)], env=e, timeout=600)
        if r.returncode != 0:
            return r.returncode
    return 0


if __name__ == "__main__":
    sys.exit(main())
