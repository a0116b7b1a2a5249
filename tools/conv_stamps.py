#!/usr/bin/env python3
"""Phase timeline of the real-block conv kernel from the diagnostic build
(`make stamps`; run with VELES_SIMD_LIB=build-stamps/lib/libvelessimd.so).
XLEN / HLEN / BATCH as tools/conv_once.py.  Prints the median cycles per
phase (load issue, forward FFT, spectrum step, inverse FFT, store + drain)
and how many workgroups were resident per CU over the kernel."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from veles.simd_amd import _lib  # noqa: E402

lib = _lib.lib()
xl = int(os.environ.get("XLEN", 1 << 20))
hl = int(os.environ.get("HLEN", 4096))
batch = int(os.environ.get("BATCH", 64))
x = torch.randn(batch, xl, device="cuda")
h = torch.randn(hl, device="cuda")
yl = xl + hl - 1
y = torch.empty(batch, yl, device="cuda")
s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
for _ in range(4):
    _lib.check(lib.vs_conv1d(3, 0, ctypes.c_void_p(x.data_ptr()), xl, xl,
                             ctypes.c_void_p(h.data_ptr()), hl, 0,
                             ctypes.c_void_p(y.data_ptr()), yl, batch, s), "vs_conv1d")
torch.cuda.synchronize()
nblk_total = 1 << 16
buf = (ctypes.c_ulonglong * (nblk_total * 8))()
_lib.check(lib.vs_conv_stamps(buf, nblk_total), "vs_conv_stamps")
a = np.frombuffer(buf, dtype=np.uint64).reshape(nblk_total, 8).astype(np.int64)
a = a[a[:, 0] > 0]
print("workgroups", len(a))
ph = np.diff(a[:, 0:6], axis=1)
names = ["load issue", "fwd FFT (+load wait)", "spectrum", "inv FFT", "store+drain"]
for i, n in enumerate(names):
    print(f"{n:22s} median {np.median(ph[:, i]):8.0f}  p10 {np.percentile(ph[:, i], 10):8.0f}"
          f"  p90 {np.percentile(ph[:, i], 90):8.0f} cycles")
life = a[:, 5] - a[:, 0]
print(f"{'lifetime':22s} median {np.median(life):8.0f}")
t0, t1 = a[:, 0].min(), a[:, 5].max()
print("kernel span cycles", t1 - t0)
# per-CU concurrency: HW_ID bits: wave[3:0] simd[5:4] cu[11:8] sh[12] se[15:13]
hw = a[:, 6]
cu = ((hw >> 8) & 0xF) | (((hw >> 12) & 1) << 4) | (((hw >> 13) & 7) << 5) | (a[:, 7] << 8)
ucu = np.unique(cu)
print("distinct CUs", len(ucu))
busy = 0.0
conc = []
for c in ucu[:64]:
    sel = a[cu == c]
    ev = sorted([(r[0], 1) for r in sel] + [(r[5], -1) for r in sel])
    cur = 0
    last = ev[0][0]
    tot = {}
    for tt, d in ev:
        tot[cur] = tot.get(cur, 0) + (tt - last)
        cur += d
        last = tt
    conc.append(tot)
agg = {}
for tot in conc:
    for k, v in tot.items():
        agg[k] = agg.get(k, 0) + v
ssum = sum(agg.values())
print("residency (workgroups on a CU: share of time)",
      {k: round(v / ssum, 3) for k, v in sorted(agg.items())})
print("blocks per CU", np.bincount(np.searchsorted(ucu, cu)).mean())
for xcc in np.unique(a[:, 7])[:2]:
    sel = a[a[:, 7] == xcc]
    print(f"xcc {xcc}: {len(sel)} workgroups, span {sel[:, 5].max() - sel[:, 0].min()} cycles")
ev0, ev1 = torch.cuda.Event(True), torch.cuda.Event(True)
ev0.record()
for _ in range(5):
    lib.vs_conv1d(3, 0, ctypes.c_void_p(x.data_ptr()), xl, xl, ctypes.c_void_p(h.data_ptr()),
                  hl, 0, ctypes.c_void_p(y.data_ptr()), yl, batch, s)
ev1.record()
torch.cuda.synchronize()
print("call ms", ev0.elapsed_time(ev1) / 5)
# raw HW_ID fields of a few workgroups of one CU id
c0 = cu[0]
sel = a[cu == c0][:6]
for r in sel:
    print("start", r[0] - sel[0, 0], "end", r[5] - sel[0, 0], "hw", hex(r[6]))
for w in range(3):
    print("runtime occupancy (blocks/CU) of variant", w, lib.vs_conv_occupancy(w))
for kb in (8, 16, 24, 32, 40, 48, 64, 80, 96, 128, 160):
    print("256-thread kernel, LDS", kb, "KiB: runtime blocks/CU", lib.vs_lds_occupancy(kb * 1024))
