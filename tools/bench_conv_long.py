#!/usr/bin/env python3
"""Long-filter convolution throughput (Msamples/s of input), x = XLEN x BATCH:
explicit overlap-save (the partitioned path past one block), the whole-signal
FFT and auto, shared and per-signal filters.  Run once per library
(VELES_SIMD_LIB) for an A/B.  HLENS=65536,200000 XLEN=1048576 BATCH=64
[TUNE=fdl_mac_lds=0,...  vs_tune_set knobs for the whole run]."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from veles.simd_amd import _lib, ops  # noqa: E402


def main():
    xlen = int(os.environ.get("XLEN", 1 << 20))
    batch = int(os.environ.get("BATCH", 64))
    rounds = int(os.environ.get("ROUNDS", 4))
    hlens = [int(v) for v in os.environ.get("HLENS", "65536,200000").split(",")]
    for kv in [kv for kv in os.environ.get("TUNE", "").split(",") if kv]:
        name, value = kv.split("=")
        _lib.call("vs_tune_set", name.encode(), int(value))
    x = torch.randn(batch, xlen, device="cuda")
    res = {}
    for hlen in hlens:
        for per in (False, True):
            h = torch.randn(batch if per else 1, hlen, device="cuda")
            hh = h if per else h[0]
            arms = ["overlap_save", "auto"] + ([] if per else ["fft"])
            ref = None
            out = {}
            for arm in arms:
                y = ops.conv1d(x, hh, algorithm=arm)
                if ref is None:
                    ref = y
                else:
                    err = (y - ref).abs().max().item() / ref.abs().max().item()
                    assert err < 1e-4, (arm, err)
                ts = []
                for _ in range(rounds):
                    e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
                    e0.record()
                    y = ops.conv1d(x, hh, algorithm=arm)
                    e1.record()
                    e1.synchronize()
                    ts.append(e0.elapsed_time(e1))
                out[arm] = round(batch * xlen / statistics.median(ts) / 1e3, 1)
                del y
            key = f"h={hlen}{' per-signal' if per else ''}"
            res[key] = out
            print(key, "Msamples/s", out, flush=True)
            del ref
    print(json.dumps({"lib": os.path.basename(_lib.LIB_PATH), "xlen": xlen, "batch": batch,
                      "res": res}))


if __name__ == "__main__":
    main()
