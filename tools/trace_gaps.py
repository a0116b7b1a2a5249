#!/usr/bin/env python3
"""Gaps between consecutive kernels in a rocprofv3 kernel trace:
tools/trace_gaps.py <run_kernel_trace.csv> [name-substring ...]"""
import csv
import statistics
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
keys = sys.argv[2:]
if keys:
    ev = [e for e in ev if any(k in e[2] for k in keys)]
gaps = {}
for a, b in zip(ev, ev[1:]):
    name = b[2].replace("(anonymous namespace)::", "").split("(")[0][:60]
    gaps.setdefault(name, []).append((b[0] - a[1]) / 1e3)
for name, g in gaps.items():
    print(f"{name:60s} n={len(g):4d} gap before: median {statistics.median(g):7.2f} us  "
          f"max {max(g):8.2f} us")
