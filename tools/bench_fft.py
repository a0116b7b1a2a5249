#!/usr/bin/env python3
"""Batched FFT throughput: this library's Stockham LDS FFT (vs_fft_c2c /
r2c) against torch.fft (rocFFT) on the same data, interleaved rounds."""
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
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    res = {}
    for logn in (8, 10, 12, 14, 16, 20):
        n = 1 << logn
        batch = max(1, (1 << 26) // n)
        x = torch.randn(batch, n, 2, device="cuda")
        y = torch.empty_like(x)
        xc = torch.view_as_complex(x)
        xr = torch.randn(batch, n, device="cuda")
        yr = torch.empty(batch, n + 2, device="cuda")
        ref = torch.fft.fft(xc[:4].to(torch.complex128))
        _lib.check(lib.vs_fft_c2c(x.data_ptr(), y.data_ptr(), n, batch, 0, s), "c2c")
        err = (torch.view_as_complex(y[:4]).to(torch.complex128) - ref).abs().max().item() / \
            ref.abs().max().item()
        modes = {
            "veles_c2c": lambda: lib.vs_fft_c2c(x.data_ptr(), y.data_ptr(), n, batch, 0, s),
            "torch_c2c": lambda: torch.fft.fft(xc),
            "veles_r2c": lambda: lib.vs_fft_r2c(xr.data_ptr(), yr.data_ptr(), n, batch, s),
            "torch_r2c": lambda: torch.fft.rfft(xr),
        }
        times = {k: [] for k in modes}
        e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
        for _ in range(5):
            for k, fn in modes.items():
                fn()
                e0.record()
                for _ in range(5):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                times[k].append(e0.elapsed_time(e1) / 5)
        out = {k: round(batch * n / statistics.median(v) / 1e6, 1) for k, v in times.items()}
        out["c2c_rel_err"] = err
        res[n] = out
        print(n, "Gpoints/s", out, flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
