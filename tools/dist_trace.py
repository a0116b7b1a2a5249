#!/usr/bin/env python3
"""Issue-concurrency evidence for the sharded host-pointer entry points.

  rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace \
      --output-format csv -d OUT -o dist -- python3 tools/dist_trace.py run
  python3 tools/dist_trace.py report OUT

`run`: a 4-rank LOCAL group (four virtual ranks on one GPU, each with its own
stream and host thread) runs vs_dist_sgemm_rowsplit on pageable host arrays
(batch 4 of 4096 x 2048 . 2048 x 4096), twice to warm up and once more
between two marker kernels (a small torch fill_ before and after).
`report`: from the traces of the marked call, when each rank's SGEMM kernels
were launched by the host (hipLaunchKernel entry), when they started and
ended on the device, and when the first device-to-host copy of C completed.
"""
import csv
import glob
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def run():
    import numpy as np
    import torch
    from veles.simd_amd.parallel import native
    rng = np.random.default_rng(0)
    batch, m, k, n = 4, 4096, 2048, 4096
    a = rng.standard_normal((batch, m, k), dtype=np.float32)
    b = rng.standard_normal((batch, k, n), dtype=np.float32)
    mark = torch.zeros(7, device="cuda")
    with native.DeviceGroup(4, backend="local") as g:
        for _ in range(2):
            c = g.sgemm_rowsplit(a, b)
        torch.cuda.synchronize()
        mark.fill_(1.0)                # marker kernel
        torch.cuda.synchronize()
        c = g.sgemm_rowsplit(a, b)
        torch.cuda.synchronize()
        mark.fill_(2.0)
        torch.cuda.synchronize()
    ref = a[1, :8].astype(np.float64) @ b[1].astype(np.float64)
    print("max err", float(np.abs(c[1, :8] - ref).max()))


def _rows(d, pat):
    f = glob.glob(os.path.join(d, "**", pat), recursive=True)
    return list(csv.DictReader(open(f[0]))) if f else []


def report(d):
    kern = _rows(d, "*kernel_trace.csv")
    cop = _rows(d, "*memory_copy_trace.csv")
    api = _rows(d, "*hip_api_trace.csv") or _rows(d, "*hip_runtime_api_trace.csv")
    marks = [r for r in kern if "FillFunctor" in r["Kernel_Name"]][-2:]
    t0, t1 = int(marks[-2]["End_Timestamp"]), int(marks[-1]["Start_Timestamp"])
    gem = [r for r in kern if "sgemm" in r["Kernel_Name"] and t0 < int(r["Start_Timestamp"]) < t1]
    d2h = [r for r in cop if t0 < int(r["Start_Timestamp"]) < t1 and "DEVICE_TO_HOST" in r["Direction"].upper()]
    h2d = [r for r in cop if t0 < int(r["Start_Timestamp"]) < t1 and "HOST_TO_DEVICE" in r["Direction"].upper()]
    launches = [r for r in api if r["Function"].startswith("hipLaunchKernel") or
                r["Function"].startswith("hipModuleLaunchKernel") or r["Function"] == "hipExtLaunchKernel"]
    launches = [r for r in launches if t0 < int(r["Start_Timestamp"]) < t1 - 1000000]
    us = lambda t: (int(t) - t0) / 1e3  # noqa: E731
    print(f"marked call: {us(t1):.0f} us between the markers")
    print(f"SGEMM kernels: {len(gem)}, on {len({r['Queue_Id'] for r in gem})} queues / "
          f"{len({r.get('Stream_Id', '') for r in gem})} streams")
    print(f"  first start {us(min(r['Start_Timestamp'] for r in gem)):.0f} us, "
          f"last end {us(max(r['End_Timestamp'] for r in gem)):.0f} us")
    if h2d:
        print(f"H2D copies: {len(h2d)}, {us(min(r['Start_Timestamp'] for r in h2d)):.0f} .. "
              f"{us(max(r['End_Timestamp'] for r in h2d)):.0f} us")
    tl = sorted(int(r["Start_Timestamp"]) for r in launches)
    if not d2h and tl:
        # pageable destinations: the runtime copies through its own staging
        # kernels, no memory-copy records -- take the hipMemcpyAsync calls
        # issued after the first launch (each returns when its rows are home)
        d2h = [r for r in api if r["Function"] == "hipMemcpyAsync" and tl[0] < int(r["Start_Timestamp"]) < t1]
        print("(D2H from the hipMemcpyAsync calls after the first launch: pageable "
              "destinations leave no memory-copy records)")
    if d2h:
        first = min(int(r["End_Timestamp"]) for r in d2h)
        print(f"D2H copies: {len(d2h)}, first completes at {us(first):.0f} us, last at "
              f"{us(max(r['End_Timestamp'] for r in d2h)):.0f} us")
        if tl:
            print(f"host launch calls in the window: {len(tl)} from "
                  f"{len({r['Thread_Id'] for r in launches})} threads, first {us(tl[0]):.0f} us, "
                  f"last {us(tl[-1]):.0f} us; {sum(t < first for t in tl)} of {len(tl)} issued "
                  f"before the first D2H completed")
        started = sum(int(r["Start_Timestamp"]) < first for r in gem)
        print(f"SGEMM kernels started on the device before the first D2H completed: "
              f"{started} of {len(gem)}")
    per = {}
    for r in gem:
        per.setdefault(r.get("Stream_Id") or r["Queue_Id"], []).append(r)
    for q, rs in sorted(per.items()):
        print(f"  stream {q}: {len(rs)} kernels, {us(min(x['Start_Timestamp'] for x in rs)):.0f} .. "
              f"{us(max(x['End_Timestamp'] for x in rs)):.0f} us")


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run()
    else:
        report(sys.argv[2])
