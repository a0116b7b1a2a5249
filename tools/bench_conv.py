#!/usr/bin/env python3
"""Conv1d throughput sweep (Msamples/s of input) over algorithms, filter
lengths and overlap-save block caps, interleaved in one process.
PLAN=1 adds a vs_conv1d_plan arm (filter spectra computed once);
SKIP_DIRECT=1 drops the direct arm (long filters); "os" is an explicit
overlap-save request (single block up to L = 32768, else partitions).
KNOBS="name=v0/v1,..." adds A/B arms of vs_tune_set knobs on the auto path
(e.g. KNOBS="conv_buffer=0/1"); every arm is checked against
the first one."""
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
DEFAULTS = {"conv_buffer": 1, "conv_real": 1, "conv_real_all": 0, "os_block_extra": 0}


def main():
    xlen = int(os.environ.get("XLEN", 1 << 20))
    batch = int(os.environ.get("BATCH", 64))
    rounds = int(os.environ.get("ROUNDS", 5))
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    x = torch.randn(batch, xlen, device="cuda")
    res = {}
    hlens = [int(v) for v in os.environ.get("HLENS", "16,64,512,4096").split(",")]
    for hlen in hlens:
        h = torch.randn(hlen, device="cuda")
        ylen = xlen + hlen - 1
        y = torch.empty(batch, ylen, device="cuda")
        knobs = [kv.split("=") for kv in os.environ.get("KNOBS", "").split(",") if kv]
        variants = [("auto", 0, 15, {})]
        for name, vals in knobs:
            variants += [(f"{name}={v}", 0, 15, {name: int(v)}) for v in vals.split("/")]
        if not knobs:
            if os.environ.get("SKIP_DIRECT") != "1":
                variants += [("direct", 1, 15, {})]
            variants += [("fft", 2, 15, {}), ("os", 3, 15, {})]
            variants += [(f"os{lg}", 3, lg, {}) for lg in (11, 12, 13, 14)
                         if (1 << lg) > 2 * hlen + 64]
        plan = None
        if os.environ.get("PLAN") == "1":   # vs_conv1d_plan: filter spectra precomputed
            plan = ctypes.c_void_p()
            assert lib.vs_conv1d_plan_create(0, 0, xlen, h.data_ptr(), hlen, 0, 1,
                                             ctypes.byref(plan), s) == 0, lib.vs_last_error()
            variants.append(("plan", 0, 15, {}))
        times = {v[0]: [] for v in variants}
        ev0, ev1 = torch.cuda.Event(True), torch.cuda.Event(True)
        ref = None
        for r in range(rounds):
            for name, algo, lg, kn in variants:
                lib.vs_tune_set(b"os_block_log_max", lg)
                for k, v in kn.items():
                    lib.vs_tune_set(k.encode(), v)
                if name == "plan":
                    run = lambda: lib.vs_conv1d_plan_execute(plan, x.data_ptr(), xlen,
                                                             y.data_ptr(), ylen, batch, s)
                else:
                    run = lambda: lib.vs_conv1d(algo, 0, x.data_ptr(), xlen, xlen,
                                                h.data_ptr(), hlen, 0, y.data_ptr(), ylen,
                                                batch, s)
                assert run() == 0, lib.vs_last_error()
                if r == 0:
                    if ref is None:
                        ref = y.clone()
                    else:
                        err = (y - ref).abs().max().item() / ref.abs().max().item()
                        assert err < 1e-4, (name, err)
                reps = 3
                ev0.record()
                for _ in range(reps):
                    run()
                ev1.record()
                torch.cuda.synchronize()
                times[name].append(ev0.elapsed_time(ev1) / reps)
                for k in kn:  # back to the library defaults
                    lib.vs_tune_set(k.encode(), DEFAULTS.get(k, 1))
        lib.vs_tune_set(b"os_block_log_max", 15)
        out = {k: round(xlen * batch / statistics.median(v) / 1e3, 1) for k, v in times.items()}
        res[hlen] = out
        print(f"h={hlen}: Msamples/s", out, flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
