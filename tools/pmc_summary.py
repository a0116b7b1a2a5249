#!/usr/bin/env python3
"""Condense rocprofv3 counter CSVs (``*_counter_collection.csv``) into one
row per kernel: short name, dispatch count, mean duration and the mean of
every counter per dispatch, plus derived ratios when their inputs exist:

  mfma_busy  = SQ_VALU_MFMA_BUSY_CYCLES / (4 * SQ_BUSY_CU_CYCLES)
               (the MFMA counter sums the four SIMDs of a CU)
  wait_frac  = SQ_WAIT_ANY / SQ_WAVE_CYCLES

Usage: pmc_summary.py OUT.md CSV [CSV ...]   (prints the table as well)
"""
from __future__ import annotations

import collections
import csv
import re
import sys


def short(name: str) -> str:
    name = name.replace("(anonymous namespace)::", "")
    name = re.sub(r"\(.*", "", name)           # drop the argument list
    name = re.sub(r"^void ", "", name)
    if len(name) > 70:
        name = name[:67] + "..."
    return name


def main(argv):
    out, paths = argv[1], argv[2:]
    # (kernel, dispatch) -> counter -> value ; plus duration per dispatch
    per = collections.defaultdict(dict)
    dur = {}
    for p in paths:
        for r in csv.DictReader(open(p)):
            key = (short(r["Kernel_Name"]), p, r["Dispatch_Id"])
            per[key][r["Counter_Name"]] = float(r["Counter_Value"])
            dur[key] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for (k, _, _), cs in per.items():
        for c, v in cs.items():
            agg[k][c].append(v)
    for key, d in dur.items():
        agg[key[0]]["_dur"].append(d)
    counters = sorted({c for cs in agg.values() for c in cs if c != "_dur"})
    lines = ["| kernel | n | us | " + " | ".join(counters) + " | mfma_busy | wait_frac |",
             "|---" * (len(counters) + 5) + "|"]
    for k, cs in sorted(agg.items(), key=lambda kv: -sum(kv[1]["_dur"])):
        mean = {c: sum(v) / len(v) for c, v in cs.items()}
        us = mean["_dur"] * 1e6
        busy = wait = ""
        if "SQ_VALU_MFMA_BUSY_CYCLES" in mean and "SQ_BUSY_CU_CYCLES" in mean:
            busy = f"{mean['SQ_VALU_MFMA_BUSY_CYCLES'] / max(4 * mean['SQ_BUSY_CU_CYCLES'], 1):.3f}"
        if "SQ_WAIT_ANY" in mean and "SQ_WAVE_CYCLES" in mean:
            wait = f"{mean['SQ_WAIT_ANY'] / max(mean['SQ_WAVE_CYCLES'], 1):.3f}"
        vals = " | ".join(f"{mean[c]:.4g}" if c in mean else "" for c in counters)
        lines.append(f"| {k} | {len(cs['_dur'])} | {us:.1f} | {vals} | {busy} | {wait} |")
    text = "\n".join(lines) + "\n"
    with open(out, "w") as f:
        f.write(text)
    print(text)


if __name__ == "__main__":
    main(sys.argv)
