#!/usr/bin/env python3
"""Per-kernel register / scratch / LDS usage of HIP sources, from hipcc's
-Rpass-analysis=kernel-resource-usage remarks (device code for gfx950).

Usage: tools/resource_usage.py [--filter REGEX] [--spills] file.hip [...]
  --spills   print only kernels with scratch (exit 1 if any)
"""
import argparse
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def usage(path):
    cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", f"-I{REPO}", f"-I{REPO}/include",
           "-DVELES_SIMD_IMPLEMENTATION", "-x", "hip", "--offload-arch=gfx950",
           "-ffp-contract=fast", "-Xclang", "-target-feature", "-Xclang", "-packed-fp32-ops", "--cuda-device-only", "-c", path, "-o", os.devnull,
           "-Rpass-analysis=kernel-resource-usage"]
    out = subprocess.run(cmd, capture_output=True, text=True).stderr
    rows, cur = [], None
    for line in out.splitlines():
        m = re.search(r"remark: Function Name: (\S+)", line)
        if m:
            cur = {"kernel": m.group(1)}
            rows.append(cur)
            continue
        m = re.search(r"remark: +([A-Za-z ]+?)(?: \[[^\]]*\])?: (\S+) \[", line)
        if m and cur is not None:
            cur[m.group(1).strip()] = m.group(2)
    return rows


def demangle(names):
    try:
        r = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-cxxfilt"], input="\n".join(names),
                           capture_output=True, text=True)
        return r.stdout.splitlines()
    except OSError:
        return names


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("files", nargs="+")
    ap.add_argument("--filter", default="")
    ap.add_argument("--spills", action="store_true")
    a = ap.parse_args()
    bad = 0
    for f in a.files:
        rows = [r for r in usage(f) if re.search(a.filter, r["kernel"])]
        names = demangle([r["kernel"] for r in rows])
        for r, n in zip(rows, names):
            scratch = int(r.get("ScratchSize", "0"))
            if a.spills and scratch == 0:
                continue
            bad += scratch > 0
            n = re.sub(r"\(.*", "", n).replace("(anonymous namespace)::", "")
            print(f"{os.path.basename(f):16s} {n[:90]:90s} VGPR {r.get('VGPRs', '?'):>3s} "
                  f"AGPR {r.get('AGPRs', '?'):>3s} scratch {scratch:4d} "
                  f"occ {r.get('Occupancy', '?')} LDS {r.get('LDS Size', '?')}")
    return 1 if (a.spills and bad) else 0


if __name__ == "__main__":
    sys.exit(main())
