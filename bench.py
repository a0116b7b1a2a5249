#!/usr/bin/env python3
"""Headline benchmark (driver contract, see README "Benchmark").

Metric (BASELINE.json): "GFLOP/s SGEMM 4096^2 fp32; Msamples/s 1D conv
len=2^20, at 1/2/4/8 MI355X".  One step = one 4096x4096x4096 exact-fp32
SGEMM (C = A @ B, MFMA f32 kernel) per GPU; `value` is the whole-job
aggregate GFLOP/s (weak scaling: every rank multiplies its own pair of
matrices).  The second half of the metric, 1D convolution throughput at
signal length 2^20 (filter 4096, batch 64 per GPU, auto-selected algorithm),
is timed the same way and reported in `secondary`, as are two
other benchmark configurations of BASELINE.json: overlap-save convolution 2^22 x 4096 taps,
batch 256 (config 3), row-split batched SGEMM 8192^2 x 64 (C row blocks
all-gathered over RCCL / xGMI, config 5) and the SWT db8 x 8 levels over
65536 signals sharded data-parallel (config 4).

Run: python bench.py --gpus N --steps K --warmup W   (N > 1 under
torch.distributed.run; one rank per GPU, RCCL backend).
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

from veles.simd_amd import _lib  # noqa: E402

SGEMM_N = 4096
CONV_LEN = 1 << 20
CONV_H = 4096
CONV_BATCH = 64


def _baseline():
    """Reference numbers this run is divided by (None if there are none)."""
    path = os.path.join(REPO, "bench", "reference_cpu_baseline.json")
    if os.path.exists(path):
        with open(path) as f:
            return json.load(f)
    return {}


def _sync_all(dist_on):
    if dist_on:
        torch.distributed.barrier()
    torch.cuda.synchronize()


# The GPU ramps its clock over the first ~25 ms of sustained load: measured
# per-call SGEMM 4096^3 from a cold start (tools/probes/warm_curve.py,
# profiles/r2/session6/warm_curve.md) runs 105 TF over calls 0-5, 132 over
# 5-10, 140 over 10-25 and a flat 143 from call 25 on.  A driver run of
# --warmup 5 --steps 20 would time the ramp, not the kernel, so every timed
# section first keeps the device busy for DEVICE_WARM_S of untimed calls of
# the same step, THEN runs the W warmup steps and times exactly K steps.
DEVICE_WARM_S = 0.25


def _device_warm(fn, dist_on):
    """Untimed calls of `fn` for ~DEVICE_WARM_S; every rank runs the same
    count (max over ranks) so collectives inside `fn` stay matched.  The
    first call (one-time setup: plans, twiddle tables, allocator growth) is
    not used to size the count."""
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    one = max((time.perf_counter() - t0) / 3, 1e-5)
    count = min(5000, int(DEVICE_WARM_S / one))
    if dist_on:
        t = torch.tensor([count], dtype=torch.int64, device="cuda")
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        count = int(t.item())
    for _ in range(count):
        fn()
    return count + 4


def _timed(fn, steps, warmup, dist_on):
    _device_warm(fn, dist_on)
    for _ in range(warmup):
        fn()
    _sync_all(dist_on)
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    _sync_all(dist_on)
    dt = time.perf_counter() - t0
    if dist_on:
        t = torch.tensor([dt], dtype=torch.float64, device="cuda")
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        dt = t.item()
    return dt


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--no-conv", action="store_true")
    ap.add_argument("--no-comm", action="store_true",
                    help="skip the row-split SGEMM / SWT data-parallel secondaries")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # Under torchrun (RANK set) always bring up the RCCL group, even at N=1,
    # so the timed region's barrier / max-reduction is the same code at every N.
    dist_on = "RANK" in os.environ
    torch.cuda.set_device(local)
    if dist_on:
        torch.distributed.init_process_group("nccl", device_id=torch.device("cuda", local))
    lib = _lib.lib()
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)

    # ---------------------------------------------------------------- SGEMM
    g = torch.Generator(device="cuda").manual_seed(1234 + rank)
    n = SGEMM_N
    a = torch.rand((n, n), device="cuda", generator=g) * 2 - 1
    b = torch.rand((n, n), device="cuda", generator=g) * 2 - 1
    c = torch.empty((n, n), device="cuda")
    pa, pb, pc = (ctypes.c_void_p(t.data_ptr()) for t in (a, b, c))

    def sgemm_step():
        st = lib.vs_sgemm(0, 0, n, n, n, 1.0, pa, n, pb, n, 0.0, pc, n, stream)
        if st:
            raise RuntimeError(lib.vs_last_error().decode())

    dt = _timed(sgemm_step, args.steps, args.warmup, dist_on)
    flops = 2.0 * n * n * n * args.steps * world
    gflops = flops / dt / 1e9
    ms = dt / args.steps * 1e3

    # Numerics guard: the timed kernel must be right.
    ref = torch.matmul(a[:256].double(), b.double())
    err = (c[:256].double() - ref).abs().max().item()
    if err > 2e-6 * n:
        raise RuntimeError(f"SGEMM numerics check failed: max err {err}")

    # hipBLASLt fp32 (torch.matmul, TF32 disabled) on the same data, for context.
    torch.backends.cuda.matmul.allow_tf32 = False
    dt_t = _timed(lambda: torch.matmul(a, b, out=c), max(5, args.steps // 2),
                  3, dist_on)
    torch_gflops = 2.0 * n ** 3 * max(5, args.steps // 2) * world / dt_t / 1e9

    secondary = {"torch_matmul_fp32_gflops": round(torch_gflops, 1),
                 "sgemm_max_abs_err": err}

    # Fast-fp32 mode on the bf16 matrix cores (hi/lo split, 3 products;
    # ~2^-17 relative per product): reported for context, NOT the headline.
    def _x3_section():
        def x3_step():
            st = lib.vs_sgemm_bf16x3(0, 0, n, n, n, 1.0, pa, n, pb, n, 0.0, pc, n, -1, stream)
            if st:
                raise RuntimeError(lib.vs_last_error().decode())
        dt3 = _timed(x3_step, max(5, args.steps // 2), 3, dist_on)
        err3 = (c[:256].double() - ref).abs().max().item()
        secondary["sgemm_bf16x3_gflops"] = round(
            2.0 * n ** 3 * max(5, args.steps // 2) * world / dt3 / 1e9, 1)
        secondary["sgemm_bf16x3_max_abs_err"] = err3

    # A failure in a secondary section (it would be the same on every rank: a
    # shape or API error, not a lost rank) is recorded instead of losing the
    # headline line.
    def _secondary(name, fn):
        try:
            fn()
        except Exception as e:  # noqa: BLE001
            secondary[name + "_error"] = f"{type(e).__name__}: {e}"[:300]

    # bf16 matrix-core GEMM (fp32 accumulate and fp32 C), NT form (both operands
    # K-contiguous, read in place), for context: NOT the headline.
    def _bf16_section():
        ah = a.bfloat16()
        bth = b.t().contiguous().bfloat16()    # [n][k]
        pah, pbh = ctypes.c_void_p(ah.data_ptr()), ctypes.c_void_p(bth.data_ptr())

        def bf16_step():
            st = lib.vs_gemm_bf16_variant(-1, 0, 1, n, n, n, 1.0, pah, n, pbh, n, 0.0, pc, n,
                                          stream)
            if st:
                raise RuntimeError(lib.vs_last_error().decode())
        bsteps = max(20, args.steps)
        dtb = _timed(bf16_step, bsteps, 3, dist_on)
        errb = (c[:256].double() - ah[:256].double() @ bth.double().t()).abs().max().item()
        dtbt = _timed(lambda: torch.matmul(ah, bth.t()), bsteps, 3, dist_on)
        secondary["gemm_bf16_gflops"] = round(2.0 * n ** 3 * bsteps * world / dtb / 1e9, 1)
        secondary["gemm_bf16_max_abs_err"] = errb
        secondary["torch_matmul_bf16_gflops"] = round(2.0 * n ** 3 * bsteps * world / dtbt / 1e9, 1)

    if hasattr(lib, "vs_sgemm_bf16x3"):
        _secondary("sgemm_bf16x3", _x3_section)
    if hasattr(lib, "vs_gemm_bf16_variant"):
        _secondary("gemm_bf16", _bf16_section)

    # ----------------------------------------------------------------- conv
    def _conv_section():
        x = torch.randn((CONV_BATCH, CONV_LEN), device="cuda", generator=g)
        h = torch.randn((CONV_H,), device="cuda", generator=g)
        ylen = CONV_LEN + CONV_H - 1
        y = torch.empty((CONV_BATCH, ylen), device="cuda")
        px, ph, py = (ctypes.c_void_p(t.data_ptr()) for t in (x, h, y))
        algo = lib.vs_conv1d_select(CONV_LEN, CONV_H, CONV_BATCH)

        def conv_step():
            st = lib.vs_conv1d(0, 0, px, CONV_LEN, CONV_LEN, ph, CONV_H, 0, py,
                               ylen, CONV_BATCH, stream)
            if st:
                raise RuntimeError(lib.vs_last_error().decode())

        csteps = max(50, args.steps)  # ~0.25 ms per call: time >= 12 ms
        dtc = _timed(conv_step, csteps, max(2, args.warmup // 2), dist_on)
        msamples = CONV_LEN * CONV_BATCH * csteps * world / dtc / 1e6
        # Same convolution through a vs_conv1d plan (filter spectra computed
        # once at plan creation, outside the timed loop -- the fixed-filter
        # FIR / serving use; the number above recomputes them every call).
        plan = ctypes.c_void_p()
        if lib.vs_conv1d_plan_create(0, 0, CONV_LEN, ph, CONV_H, 0, 1, ctypes.byref(plan),
                                     stream) == 0:
            def plan_step():
                st = lib.vs_conv1d_plan_execute(plan, px, CONV_LEN, py, ylen, CONV_BATCH,
                                                stream)
                if st:
                    raise RuntimeError(lib.vs_last_error().decode())
            dtp = _timed(plan_step, csteps, max(2, args.warmup // 2), dist_on)
            torch.cuda.synchronize()
            lib.vs_conv1d_plan_destroy(plan)
            secondary["conv1d_plan_msamples_per_s"] = round(
                CONV_LEN * CONV_BATCH * csteps * world / dtp / 1e6, 1)
        del x, y
        # benchmark config 3: overlap-save convolution, signal 2^22, filter
        # 4096, batch 256 (per GPU), per call and through a plan
        c3_len, c3_batch = 1 << 22, 256
        x3 = torch.randn((c3_batch, c3_len), device="cuda", generator=g)
        y3len = c3_len + CONV_H - 1
        y3 = torch.empty((c3_batch, y3len), device="cuda")
        px3, py3 = (ctypes.c_void_p(t.data_ptr()) for t in (x3, y3))

        def conv3_step():
            st = lib.vs_conv1d(3, 0, px3, c3_len, c3_len, ph, CONV_H, 0, py3, y3len, c3_batch,
                               stream)
            if st:
                raise RuntimeError(lib.vs_last_error().decode())

        c3steps = max(10, args.steps // 2)
        dt3c = _timed(conv3_step, c3steps, 2, dist_on)
        secondary["conv1d_os_2^22x4096x256_msamples_per_s"] = round(
            c3_len * c3_batch * c3steps * world / dt3c / 1e6, 1)
        secondary["conv1d_os_2^22x4096x256_ms_per_step"] = round(dt3c / c3steps * 1e3, 3)
        plan3 = ctypes.c_void_p()
        if lib.vs_conv1d_plan_create(3, 0, c3_len, ph, CONV_H, 0, 1, ctypes.byref(plan3),
                                     stream) == 0:
            def plan3_step():
                st = lib.vs_conv1d_plan_execute(plan3, px3, c3_len, py3, y3len, c3_batch, stream)
                if st:
                    raise RuntimeError(lib.vs_last_error().decode())
            dt3p = _timed(plan3_step, c3steps, 2, dist_on)
            torch.cuda.synchronize()
            lib.vs_conv1d_plan_destroy(plan3)
            secondary["conv1d_os_2^22x4096x256_plan_msamples_per_s"] = round(
                c3_len * c3_batch * c3steps * world / dt3p / 1e6, 1)
        del x3, y3
        secondary.update({
            "conv1d_msamples_per_s": round(msamples, 1),
            "conv1d_ms_per_step": round(dtc / csteps * 1e3, 3),
            "conv1d_config": {"x_len": CONV_LEN, "h_len": CONV_H,
                              "batch_per_gpu": CONV_BATCH,
                              "algorithm": ["direct", "fft", "overlap_save"][
                                  max(0, algo - 1)]},
        })

    if not args.no_conv and hasattr(lib, "vs_conv1d"):
        _secondary("conv1d", _conv_section)

    # ------------------------------------- benchmark configs with communication
    # Config 5 (row-split batched SGEMM 8192^2 x 64, RCCL all-gather of the C
    # row blocks over xGMI, overlapped with the next matrix's GEMM: every rank
    # holds its rows of the 64 A matrices, all of B and the gathered C,
    # 34-48 GiB per GPU) and config 4
    # (SWT db8 x 8 levels over 65536 x 1024 signals, batch sharded over the
    # ranks).  Both run under the same barrier / max-over-ranks clock.
    def _rowsplit_section():
        from veles.simd_amd import parallel
        rs_n, rs_batch = 8192, 64
        m_loc = rs_n // world
        ga = torch.Generator(device="cuda").manual_seed(77 + rank)
        a_loc = torch.rand(rs_batch, m_loc, rs_n, device="cuda", generator=ga) - 0.5
        bmat = torch.rand(rs_batch, rs_n, rs_n, device="cuda",
                          generator=torch.Generator(device="cuda").manual_seed(99)) - 0.5
        cfull = torch.empty(rs_batch, m_loc * world, rs_n, device="cuda")
        rsteps = max(2, args.steps // 20)
        dtr = _timed(lambda: parallel.rowsplit_bmm(a_loc, bmat, out=cfull), rsteps, 1, dist_on)
        # numerics: this rank's rows of the first matrix, 64 rows
        r0 = rank * m_loc
        got = cfull[0, r0:r0 + 64].double()
        ref = a_loc[0, :64].double() @ bmat[0].double()
        rs_err = (got - ref).abs().max().item()
        if rs_err > 2e-6 * rs_n:
            raise RuntimeError(f"row-split SGEMM numerics check failed: {rs_err}")
        secondary.update({
            "rowsplit_sgemm_gflops": round(2.0 * rs_n ** 3 * rs_batch * rsteps / dtr / 1e9, 1),
            "rowsplit_ms_per_step": round(dtr / rsteps * 1e3, 2),
            "rowsplit_ms_per_matrix": round(dtr / rsteps / rs_batch * 1e3, 3),
            "rowsplit_allgather_GB_per_rank_per_step": round(
                rs_batch * (world - 1) * m_loc * rs_n * 4 / 1e9, 3),
            "rowsplit_config": {"n": rs_n, "batch": rs_batch, "parallelism": f"tp{world}",
                                "collective": "all_gather_into_tensor (RCCL)" if world > 1
                                else "none (1 rank)"},
        })
        del a_loc, bmat, cfull

    def _swt_section():
        from veles.simd_amd import parallel
        total, sn, levels = 65536, 1024, 8
        ga = torch.Generator(device="cuda").manual_seed(78 + rank)
        s0, s1 = parallel.shard_range(total, world, rank)
        xs = torch.randn(s1 - s0, sn, device="cuda", generator=ga)
        hi = torch.empty(s1 - s0, levels, sn, device="cuda")
        lo = torch.empty(s1 - s0, sn, device="cuda")

        def swt_step():
            st = lib.vs_swt_multilevel(0, 8, levels, 0, ctypes.c_void_p(xs.data_ptr()), sn,
                                       ctypes.c_void_p(hi.data_ptr()),
                                       ctypes.c_void_p(lo.data_ptr()), s1 - s0, stream)
            if st:
                raise RuntimeError(lib.vs_last_error().decode())

        ssteps = max(20, args.steps)
        dts = _timed(swt_step, ssteps, 5, dist_on)
        secondary.update({
            "swt_dp_msamples_per_s": round(total * sn * ssteps / dts / 1e6, 1),
            "swt_dp_ms_per_step": round(dts / ssteps * 1e3, 3),
            "swt_dp_config": {"wavelet": "db8", "levels": levels, "signals": total,
                              "len": sn, "parallelism": f"dp{world}"},
        })
        del xs, hi, lo

    if not args.no_comm:
        _secondary("rowsplit", _rowsplit_section)
        _secondary("swt_dp", _swt_section)

    # The reference's own benchmark shapes through the reference-compatible host
    # C API on pageable numpy arrays, microseconds per call (rank 0 only; host
    # work, no collective).  For context: NOT the headline.
    def _hostapi_section():
        import numpy as np
        from veles.simd_amd import capi
        rng = np.random.default_rng(7)
        f = lambda *s: rng.standard_normal(s, dtype=np.float32)  # noqa: E731
        sz = ctypes.c_size_t
        ma, mb, mc = f(300, 256), f(256, 1000), f(300, 1000)
        cx, ch, cy = f(512), f(512), f(1023)
        aa, ab, ac = f(1024 * 1024), f(1024 * 1024), f(1024 * 1024)
        sx, sy = np.abs(f(1 << 16)) + 0.1, f(1 << 16)
        calls = {   # name: (calls, function, arguments converted once)
            "matrix_multiply_300x256x1000": (200, capi.fn("matrix_multiply"), (
                1, capi.p(ma), capi.p(mb), 256, 300, 1000, 256, capi.p(mc))),
            "convolve_simd_512x512": (2000, capi.fn("convolve_simd"), (
                1, capi.p(cx), sz(512), capi.p(ch), sz(512), capi.p(cy))),
            "matrix_add_1024x1024": (100, capi.fn("matrix_add"), (
                1, capi.p(aa), capi.p(ab), 1024, 1024, capi.p(ac))),
            "log_psv_65536": (500, capi.fn("log_psv"), (1, capi.p(sx), sz(1 << 16), capi.p(sy))),
        }
        out = {}
        for name, (reps, fn, fargs) in calls.items():
            for _ in range(max(3, reps // 20)):
                fn(*fargs)
            t0 = time.perf_counter()
            for _ in range(reps):
                fn(*fargs)
            out[name] = round((time.perf_counter() - t0) / reps * 1e6, 3)
        secondary["hostapi_us_per_call"] = out
        secondary["hostapi_note"] = ("through ctypes (about 1 us per call on top of the library); "
                                     "reference AVX on the same host: 4543 us (matrix_multiply), "
                                     "17.8 us (convolve_simd)")

    if rank == 0:
        _secondary("hostapi", _hostapi_section)

    base = _baseline()
    vs_base = None
    if base.get("sgemm_4096_gflops"):
        # The reference publishes no numbers; this is its own
        # AVX code measured on one host core (tools/measure_reference_cpu.py).
        vs_base = round(gflops / base["sgemm_4096_gflops"], 1)
        secondary["baseline_source"] = base.get("source")
        secondary["baseline_sgemm_gflops"] = base["sgemm_4096_gflops"]
        ref_conv = base.get("conv_direct_2^20x4096_msamples_per_s")
        if ref_conv and "conv1d_msamples_per_s" in secondary:
            secondary["conv1d_vs_baseline"] = round(
                secondary["conv1d_msamples_per_s"] / ref_conv, 1)

    if rank == 0:
        print(json.dumps({
            "metric": "GFLOP/s SGEMM 4096^2 fp32",
            "value": round(gflops, 1),
            "unit": "GFLOP/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": vs_base,
            "dtype": "fp32",
            "data": "synthetic (uniform [-1,1) fp32 matrices; gaussian signals)",
            "config": {"model": "sgemm_4096x4096x4096_fp32",
                       "global_batch": world, "seq_len": n,
                       "parallelism": f"dp{world}"},
            "device_warmup_s": DEVICE_WARM_S,
            "secondary": secondary,
        }), flush=True)
    if dist_on:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
