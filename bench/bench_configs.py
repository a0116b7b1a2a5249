#!/usr/bin/env python3
"""BASELINE.json secondary configurations on the local GPU(s).

  elementwise : sin/cos/log/exp + saxpy fp32 (config 1; GPU and host path)
  sgemm       : SGEMM 4096^2 fp32 (config 2)
  os_conv     : overlap-save conv, signal 2^22, filter 4096, batch 256 (config 3)
  swt         : db8 stationary DWT, 8 levels, batch 65536 x 1024 samples,
                data-parallel over the ranks (config 4)
  rowsplit    : batched SGEMM 8192^2 x 64, rows split over the ranks, C
                all-gathered over RCCL (config 5; --batch to shrink)
Run one GPU: python bench/bench_configs.py all
Run N GPUs : torchrun --nproc-per-node N bench/bench_configs.py swt rowsplit
Prints one JSON line per configuration (rank 0).
"""
import argparse
import ctypes
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from veles.simd_amd import _lib, ops, parallel  # noqa: E402
from bench import _device_warm  # noqa: E402  (repo-root bench.py: clock-ramp warm-up)


def _timeit(fn, steps, warmup, dist_on):
    _device_warm(fn, dist_on)
    for _ in range(warmup):
        fn()
    if dist_on:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    if dist_on:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if dist_on:
        t = torch.tensor([dt], device="cuda", dtype=torch.float64)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        dt = t.item()
    return dt / steps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("configs", nargs="*", default=["all"])
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=64, help="rowsplit batch")
    args = ap.parse_args()
    ctx = parallel.init()
    dist_on = torch.distributed.is_initialized()
    world, rank = ctx.world, ctx.rank
    cfgs = set(args.configs)
    run_all = "all" in cfgs
    lib = _lib.lib()
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    out = []

    if run_all or "elementwise" in cfgs:
        n = 1 << 26
        x = torch.rand(n, device="cuda") * 10 + 0.1
        y = torch.empty_like(x)
        res = {}
        for fn, code in (("sin", 0), ("cos", 1), ("log", 2), ("exp", 3)):
            t = _timeit(lambda: lib.vs_math(code, x.data_ptr(), y.data_ptr(), n, s),
                        args.steps, args.warmup, dist_on)
            res[f"{fn}_GB_per_s"] = round(8 * n / t / 1e9, 1)
        t = _timeit(lambda: lib.vs_saxpy(ctypes.c_float(2.0), x.data_ptr(), y.data_ptr(), n, s),
                    args.steps, args.warmup, dist_on)
        res["saxpy_GB_per_s"] = round(12 * n / t / 1e9, 1)
        out.append({"config": "elementwise fp32 (2^26 elements)", **res})

    if run_all or "sgemm" in cfgs:
        n = 4096
        a = torch.rand(n, n, device="cuda") * 2 - 1
        b = torch.rand(n, n, device="cuda") * 2 - 1
        c = torch.empty(n, n, device="cuda")
        t = _timeit(lambda: lib.vs_sgemm(0, 0, n, n, n, ctypes.c_float(1.0), a.data_ptr(), n,
                                         b.data_ptr(), n, ctypes.c_float(0.0), c.data_ptr(),
                                         n, s), args.steps, args.warmup, dist_on)
        out.append({"config": "SGEMM 4096^2 fp32", "tflops_aggregate":
                    round(2 * n ** 3 * world / t / 1e12, 2), "ms": round(t * 1e3, 3)})

    if run_all or "os_conv" in cfgs:
        xl, hl, batch = 1 << 22, 4096, 256
        x = torch.randn(batch, xl, device="cuda")
        h = torch.randn(hl, device="cuda")
        yl = xl + hl - 1
        y = torch.empty(batch, yl, device="cuda")
        t = _timeit(lambda: lib.vs_conv1d(3, 0, x.data_ptr(), xl, xl, h.data_ptr(), hl, 0,
                                          y.data_ptr(), yl, batch, s),
                    max(2, args.steps // 2), 1, dist_on)
        out.append({"config": "overlap-save conv 2^22 x 4096, batch 256",
                    "msamples_per_s_aggregate": round(xl * batch * world / t / 1e6, 1),
                    "ms": round(t * 1e3, 3)})
        del x, y

    if run_all or "swt" in cfgs:
        total, n, levels = 65536, 1024, 8
        a, b = parallel.shard_range(total, world, rank)
        x = torch.randn(b - a, n, device="cuda")
        hi = torch.empty(b - a, levels, n, device="cuda")
        lo = torch.empty(b - a, n, device="cuda")
        t = _timeit(lambda: lib.vs_swt_multilevel(0, 8, levels, 0, x.data_ptr(), n,
                                                  hi.data_ptr(), lo.data_ptr(), b - a, s),
                    args.steps, args.warmup, dist_on)
        out.append({"config": f"SWT db8 x {levels} levels, 65536 x {n} samples, dp{world}",
                    "msamples_per_s_aggregate": round(total * n / t / 1e6, 1),
                    "GB_per_s_per_gpu": round((b - a) * n * 4 * (levels + 2) / t / 1e9, 1),
                    "ms": round(t * 1e3, 3)})
        del x, hi, lo

    if run_all or "rowsplit" in cfgs:
        n, batch = 8192, args.batch
        m_loc = n // world
        g = torch.Generator(device="cuda").manual_seed(rank)
        a_loc = torch.rand(batch, m_loc, n, device="cuda", generator=g) - 0.5
        bm = torch.rand(batch, n, n, device="cuda", generator=torch.Generator(
            device="cuda").manual_seed(99)) - 0.5
        c = torch.empty(batch, n, n, device="cuda")
        t = _timeit(lambda: parallel.rowsplit_bmm(a_loc, bm, out=c), max(1, args.steps // 5),
                    1, dist_on)
        out.append({"config": f"row-split batched SGEMM {n}^2 x {batch}, tp{world}",
                    "tflops_aggregate": round(2 * n ** 3 * batch / t / 1e12, 2),
                    "ms": round(t * 1e3, 1)})

    if rank == 0:
        for o in out:
            print(json.dumps(o), flush=True)
    if dist_on:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
