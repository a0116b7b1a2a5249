#!/usr/bin/env python3
"""Bandwidth of the memory-bound kernels (elementwise, reductions, normalisation, peaks) at
2^26 elements against same-process HBM ceilings (torch fill_ = write-only,
copy_ = read + write).  Bytes are the minimum each op must move (inputs read
once, outputs written once).  Every op is timed after bench.py's clock-ramp
warm-up.  Prints one JSON line.  Usage: python tools/bench_memops.py [log2 n]"""
import ctypes
import json
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from bench import _device_warm  # noqa: E402
from veles.simd_amd import _lib  # noqa: E402

F32, F16, I16, I32, U8 = 0, 1, 2, 3, 4


def timed(fn, steps=20):
    _device_warm(fn, False)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps


def main():
    n = 1 << (int(sys.argv[1]) if len(sys.argv) > 1 else 26)
    lib = _lib.lib()
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    g = torch.Generator(device="cuda").manual_seed(0)
    x = torch.randn(n, device="cuda", generator=g)
    y = torch.randn(n, device="cuda", generator=g)
    z = torch.empty(n, device="cuda")
    w2 = torch.empty(n, device="cuda")
    xa = x.abs() + 0.1
    xi16 = (x * 1000).to(torch.int16)
    yi16 = (y * 1000).to(torch.int16)
    oi16 = torch.empty(n, dtype=torch.int16, device="cuda")
    oi32 = torch.empty(n, dtype=torch.int32, device="cuda")
    xf16 = x.half()
    img = (torch.rand(8192, n // 8192, device="cuda", generator=g) * 255).to(torch.uint8)
    mm = torch.empty(2, dtype=torch.uint8, device="cuda")
    out = torch.empty(4, device="cuda")
    pos = torch.empty(n // 2, dtype=torch.int32, device="cuda")
    val = torch.empty(n // 2, device="cuda")
    cnt = torch.empty(1, dtype=torch.int64, device="cuda")

    def chk(st):
        if st:
            raise RuntimeError(lib.vs_last_error().decode())

    ops = {
        "fill (write ceiling, torch)": (lambda: z.fill_(1.0), 4 * n),
        "copy (read+write ceiling, torch)": (lambda: z.copy_(x), 8 * n),
        "convert f32->i16": (lambda: chk(lib.vs_convert(P(x), F32, P(oi16), I16, n, s)), 6 * n),
        "convert i16->f32": (lambda: chk(lib.vs_convert(P(xi16), I16, P(z), F32, n, s)), 6 * n),
        "convert f16->f32": (lambda: chk(lib.vs_convert(P(xf16), F16, P(z), F32, n, s)), 6 * n),
        "binary mul": (lambda: chk(lib.vs_binary(2, P(x), P(y), P(z), n, s)), 12 * n),
        "complex multiply": (lambda: chk(lib.vs_complex_multiply(P(x), P(y), P(z), n // 2, 0, s)),
                             12 * n),
        "complex conjugate": (lambda: chk(lib.vs_complex_conjugate(P(x), P(z), n, s)), 8 * n),
        "reverse": (lambda: chk(lib.vs_reverse(P(x), P(z), n, 0, s)), 8 * n),
        "reverse complex pairs": (lambda: chk(lib.vs_reverse(P(x), P(z), n, 1, s)), 8 * n),
        "affine": (lambda: chk(lib.vs_affine(P(x), ctypes.c_float(2.0), ctypes.c_float(1.0),
                                             P(z), n, s)), 8 * n),
        "fill": (lambda: chk(lib.vs_fill(P(z), ctypes.c_float(1.5), n, s)), 4 * n),
        "pow": (lambda: chk(lib.vs_pow(P(xa), P(y), P(z), n, s)), 12 * n),
        "sincos": (lambda: chk(lib.vs_sincos(P(x), P(z), P(w2), n, s)), 12 * n),
        "int16 multiply": (lambda: chk(lib.vs_int16_multiply(P(xi16), P(yi16), P(oi32), n, s)),
                           8 * n),
        "sum": (lambda: chk(lib.vs_sum(P(x), n, P(out), s)), 4 * n),
        "minmax": (lambda: chk(lib.vs_minmax(P(x), n, P(out), s)), 4 * n),
        "minmax2d u8": (lambda: chk(lib.vs_minmax2d_u8(P(img), img.shape[1], img.shape[1],
                                                       img.shape[0], P(mm), s)), n),
        "normalize2d u8->f32 (fused minmax)": (
            lambda: chk(lib.vs_normalize2d_u8(P(img), img.shape[1], img.shape[1], img.shape[0],
                                              P(mm), 0, 0, P(z), img.shape[1], s)), 5 * n),
        "detect_peaks both (count + emit)": (
            lambda: chk(lib.vs_detect_peaks(P(x), ctypes.c_size_t(n), 3, P(pos), P(val),
                                            ctypes.c_size_t(n // 2), P(cnt), s)), 4 * n),
    }
    # detect_peaks moves 4 n bytes in plus 8 bytes (position + value) per
    # extremum out; count them once
    d = x[1:-1]
    npk = int(((d - x[:-2]) * (d - x[2:]) > 0).sum().item())
    fn, _ = ops["detect_peaks both (count + emit)"]
    ops["detect_peaks both (count + emit)"] = (fn, 4 * n + 8 * npk)
    res = {}
    for name, (fn, nbytes) in ops.items():
        t = timed(fn)
        res[name] = {"us": round(t * 1e6, 1), "TB_per_s": round(nbytes / t / 1e12, 2)}
    print(json.dumps({"n": n, "ops": res}))


if __name__ == "__main__":
    main()
