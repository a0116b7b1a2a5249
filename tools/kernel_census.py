#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace --stats run of `pytest -m gpu` into a
markdown census of the library's kernels (which of our kernels the GPU suite
launched, how often, total time), grouped by kernel family (rows K1-K16 of docs/ARCHITECTURE.md).

Usage: tools/kernel_census.py <dir with *_kernel_stats.csv> > out.md"""
import csv
import glob
import os
import re
import sys

# kernel family rows -> name patterns of our kernels
ROWS = [
    ("K1 conversions", r"Convert<"),
    ("K2 fp16->fp32", r"Convert<unsigned short, float>"),
    ("K3 complex mul/conj", r"cmul_kernel|conj_kernel"),
    ("K4 elementwise family", r"map1_kernel|map2_kernel"),
    ("K5 reductions", r"sum_pass|minmax_pass"),
    ("K6 normalize2D", r"normalize2d|minmax2d"),
    ("K7 mathfun", r"MathOp|sincos|PowOp"),
    ("K8 SGEMM / GEMM", r"sgemm|gemm_glds|scale_c|pack_kernel|slices_reduce"),
    ("K9 direct conv", r"direct"),
    ("K10 FFT", r"fft::"),
    ("K11 fused overlap-save / block conv", r"block_conv|real_conv|real_filter|fdl_"),
    ("K12 fused pointwise", r"spectrum_mul|pack_pairs|unpack_pairs|pad_filter"),
    ("K13 DWT", r"dwt"),
    ("K14 SWT", r"swt"),
    ("K15 detect_peaks", r"peaks::"),
    ("K16 int16 multiply", r"Int16Mul"),
]


def short(name):
    """Kernel name without 'void', anonymous namespaces and the argument list."""
    n = name.replace("(anonymous namespace)::", "")
    if n.startswith("void "):
        n = n[5:]
    depth = 0
    for i, ch in enumerate(n):
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0:
            return n[:i]
    return n


def main():
    paths = glob.glob(os.path.join(sys.argv[1], "**", "*kernel_stats.csv"), recursive=True)
    if not paths:
        sys.exit("no kernel_stats.csv under " + sys.argv[1])
    rows = []
    for p in paths:
        with open(p) as f:
            for r in csv.DictReader(f):
                rows.append((r["Name"], int(r["Calls"]), float(r["TotalDurationNs"])))
    ours = [(short(n), c, t) for n, c, t in rows if short(n).startswith("vs::")]
    print("# Kernels launched by `pytest -m gpu` (rocprofv3 --kernel-trace --stats)\n")
    print(f"{len(ours)} distinct kernels of this library, {sum(r[1] for r in ours)} launches; "
          f"{len(rows) - len(ours)} other kernels (PyTorch / runtime).\n")
    print("| kernel row | kernels hit | launches |\n|---|---|---|")
    for label, pat in ROWS:
        hit = [r for r in ours if re.search(pat, r[0])]
        print(f"| {label} | {len(hit)} | {sum(r[1] for r in hit)} |")
    print("\n## Every kernel of this library that ran\n")
    print("| kernel | calls | total ms |\n|---|---|---|")
    for name, calls, ns in sorted(ours, key=lambda r: r[0]):
        print(f"| `{name}` | {calls} | {ns / 1e6:.2f} |")


if __name__ == "__main__":
    main()
