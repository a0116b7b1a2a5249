#!/usr/bin/env python3
"""Host-API call latency with pageable operands under different limits of the
per-call pinned staging image (VELES_STAGE_MAX_KB): runs itself once per limit
in a child process (the limit is read once per process) and prints a table."""
import ctypes
import json
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
    rng = np.random.default_rng(0)
    f = lambda *s: rng.standard_normal(s, dtype=np.float32)  # noqa: E731
    cases = {}

    def case(name, cname, *args):
        fnc = capi.fn(cname)
        cases[name] = lambda: fnc(*args)

    a, b, c = f(256, 300), f(300, 1000), f(256, 1000)
    case("matrix_multiply 300x256x1000", "matrix_multiply", 1, capi.p(a), capi.p(b), 300, 256,
         1000, 300, capi.p(c))
    for n in (256, 512, 768, 1024):
        x, y, z = f(n, n), f(n, n), f(n, n)
        case(f"matrix_add {n}x{n}", "matrix_add", 1, capi.p(x), capi.p(y), n, n, capi.p(z))
        cases[f"matrix_add {n}x{n}"].keep = (x, y, z)
    for n in (65536, 262144):
        x, y = f(n), f(n)
        case(f"sin_psv {n}", "sin_psv", 1, capi.p(x), ctypes.c_size_t(n), capi.p(y))
        cases[f"sin_psv {n}"].keep = (x, y)
    for n, k in ((100000, 2000), (300000, 500)):
        x, h, y = f(n), f(k), f(n + k - 1)
        case(f"convolve_simd {n}x{k}", "convolve_simd", 1, capi.p(x), ctypes.c_size_t(n),
             capi.p(h), ctypes.c_size_t(k), capi.p(y))
        cases[f"convolve_simd {n}x{k}"].keep = (x, h, y)
    out = {}
    for name, fn in cases.items():
        for _ in range(20):
            fn()
        ts = []
        for _ in range(15):
            t0 = time.perf_counter()
            for _ in range(20):
                fn()
            ts.append((time.perf_counter() - t0) / 20 * 1e6)
        out[name] = round(statistics.median(ts), 1)
    print(json.dumps(out))


def main():
    if os.environ.get("STAGE_CHILD"):
        return child()
    limits = [int(x) for x in os.environ.get("LIMITS", "64,512,1536,4096").split(",")]
    rows = {}
    for kb in limits:
        env = dict(os.environ, STAGE_CHILD="1", VELES_STAGE_MAX_KB=str(kb), PYTHONPATH=REPO)
        r = subprocess.run([sys.executable, os.path.abspath(__file__)], env=env,
                           capture_output=True, text=True, timeout=300)
        if r.returncode != 0:
            print(r.stderr[-2000:])
            return 1
        rows[kb] = json.loads(r.stdout.strip().splitlines()[-1])
        print(kb, rows[kb], flush=True)
    names = list(rows[limits[0]])
    print(f"{'call (us, median)':34s}" + "".join(f"{kb:>9d}K" for kb in limits))
    for n in names:
        print(f"{n:34s}" + "".join(f"{rows[kb][n]:10.1f}" for kb in limits))
    return 0


if __name__ == "__main__":
    sys.exit(main())
