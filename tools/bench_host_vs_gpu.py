#!/usr/bin/env python3
"""Reference-compatible host API on pageable host arrays: the staged GPU path
against the library's own host loops, per call and size.  Two child processes
(the policy knobs are read once per process): one with every small-call limit
at zero (everything that can goes to the GPU), one with every limit out of
reach (nothing does).  Shows where the shipped limits should sit."""
import ctypes
import json
import os
import statistics
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

ARMS = {
    "gpu": {"VELES_HOST_SMALL_SCALE": "0", "VELES_GPU_MIN_ELEMS": "1", "VELES_HOST_MAX_MACS": "0"},
    "host": {"VELES_HOST_SMALL_SCALE": "100000000", "VELES_GPU_MIN_ELEMS": "2000000000",
             "VELES_HOST_MAX_MACS": "2000000000"},
    "shipped": {},
}


def child():
    import numpy as np
    from veles.simd_amd import capi
    rng = np.random.default_rng(0)
    f = lambda n: rng.standard_normal(n, dtype=np.float32)  # noqa: E731
    sz = ctypes.c_size_t
    cases = {}

    def case(name, cname, keep, *args):
        fnc = capi.fn(cname)
        cases[name] = (lambda: fnc(*args), keep)

    for n in (128, 256, 512, 1024):
        x, y, z = f(n * n), f(n * n), f(n * n)
        case(f"matrix_add {n}x{n}", "matrix_add", (x, y, z), 1, capi.p(x), capi.p(y), n, n,
             capi.p(z))
    for n in (1 << 16, 1 << 20, 1 << 22):
        x, y, z = f(n), f(n), f(n)
        case(f"real_multiply_array {n}", "real_multiply_array", (x, y, z), capi.p(x), capi.p(y),
             sz(n), capi.p(z))
        i16 = rng.integers(-30000, 30000, n).astype(np.int16)
        case(f"int16_to_float {n}", "int16_to_float", (i16, z), capi.p(i16), sz(n), capi.p(z))
        case(f"sum_elements {n}", "sum_elements", (x,), capi.p(x), sz(n))
        lo, hi = ctypes.c_float(), ctypes.c_float()
        case(f"minmax1D {n}", "minmax1D", (x, lo, hi), 1, capi.p(x), n, ctypes.byref(lo),
             ctypes.byref(hi))
    for n in (256, 1024, 2048):
        img = rng.integers(0, 256, (n, n), dtype=np.uint8)
        out = np.empty((n, n), np.float32)
        case(f"normalize2D {n}x{n}", "normalize2D", (img, out), 1, capi.p(img), n, n, n,
             capi.p(out), n)
    for n in (1 << 14, 1 << 17, 1 << 20):
        x = f(n)
        hi_, lo_ = np.empty(n // 2, np.float32), np.empty(n // 2, np.float32)
        case(f"wavelet_apply db8 {n}", "wavelet_apply", (x, hi_, lo_), 0, 8, 0, capi.p(x), sz(n),
             capi.p(hi_), capi.p(lo_))
        h2, l2 = np.empty(n, np.float32), np.empty(n, np.float32)
        case(f"stationary_wavelet_apply db8 {n}", "stationary_wavelet_apply", (x, h2, l2), 0, 8, 1,
             0, capi.p(x), sz(n), capi.p(h2), capi.p(l2))

        def peaks(x=x, n=n):
            res, cnt = ctypes.c_void_p(), sz()
            capi.fn("detect_peaks")(1, capi.p(x), sz(n), 3, ctypes.byref(res), ctypes.byref(cnt))
            capi.fn("free")(res)
        cases[f"detect_peaks {n}"] = (peaks, (x,))
    for n in (1 << 10, 1 << 12, 1 << 14, 1 << 15, 1 << 16, 1 << 17):
        x, y, z = np.abs(f(n)) + 0.1, f(n), f(n)
        case(f"log_psv {n}", "log_psv", (x, y), 1, capi.p(x), sz(n), capi.p(y))
        case(f"sin_psv {n}", "sin_psv", (x, y), 1, capi.p(x), sz(n), capi.p(y))
        case(f"pow_psv {n}", "pow_psv", (x, y, z), 1, capi.p(x), capi.p(y), sz(n), capi.p(z))
    for n in (32, 48, 64, 96, 128):
        x, y, z = f(n * n), f(n * n), f(n * n)
        case(f"matrix_multiply {n}^3", "matrix_multiply", (x, y, z), 1, capi.p(x), capi.p(y), n, n,
             n, n, capi.p(z))
    for n, k in ((1024, 256), (1024, 512), (2048, 512), (4096, 512), (65536, 16), (65536, 64)):
        x, h, y = f(n), f(k), f(n + k - 1)
        case(f"convolve_simd {n}x{k}", "convolve_simd", (x, h, y), 1, capi.p(x), sz(n), capi.p(h),
             sz(k), capi.p(y))
    only = os.environ.get("ONLY")
    if only:
        cases = {k: v for k, v in cases.items() if any(o in k for o in only.split(","))}
    out = {}
    for name, (fn, _keep) in cases.items():
        for _ in range(5):
            fn()
        ts = []
        for _ in range(9):
            t0 = time.perf_counter()
            for _ in range(10):
                fn()
            ts.append((time.perf_counter() - t0) / 10 * 1e6)
        out[name] = round(statistics.median(ts), 1)
    print(json.dumps(out))


def main():
    if os.environ.get("HVG_CHILD"):
        return child()
    rows = {}
    for arm, knobs in ARMS.items():
        env = dict(os.environ, HVG_CHILD="1", PYTHONPATH=REPO)
        for k in ARMS["gpu"]:
            env.pop(k, None)
        env.update(knobs)
        r = subprocess.run([sys.executable, os.path.abspath(__file__)], env=env,
                           capture_output=True, text=True, timeout=600)
        if r.returncode != 0:
            print(r.stderr[-3000:])
            return 1
        rows[arm] = json.loads(r.stdout.strip().splitlines()[-1])
        print(arm, "done", flush=True)
    print(f"{'call (us, median)':40s}" + "".join(f"{a:>10s}" for a in ARMS))
    for n in rows["gpu"]:
        print(f"{n:40s}" + "".join(f"{rows[a][n]:10.1f}" for a in ARMS))
    return 0


if __name__ == "__main__":
    sys.exit(main())
