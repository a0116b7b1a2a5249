#!/usr/bin/env python3
"""Per-file host line coverage of a `make coverage` build: runs gcov on every
.gcda under BUILD (clang's gcov-format notes are read by GNU gcov) and prints
one row per source of this repo, then the total.
Usage: tools/coverage_report.py build-cov"""
import os
import re
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    build = os.path.abspath(sys.argv[1] if len(sys.argv) > 1 else "build-cov")
    rows = {}
    with tempfile.TemporaryDirectory() as tmp:
        for root, _, files in os.walk(build):
            for f in files:
                if not f.endswith(".gcda"):
                    continue
                out = subprocess.run(["gcov", "-n", "-o", root, os.path.join(root, f)],
                                     cwd=tmp, capture_output=True, text=True).stdout
                cur = None
                for line in out.splitlines():
                    m = re.match(r"File '(.+)'", line)
                    if m:
                        cur = os.path.normpath(os.path.join(REPO, m.group(1)))
                        continue
                    m = re.match(r"Lines executed:([\d.]+)% of (\d+)", line)
                    if m and cur:
                        if cur.startswith(REPO + os.sep) and "/build" not in cur[len(REPO):]:
                            total = int(m.group(2))
                            hit = round(float(m.group(1)) * total / 100)
                            old = rows.get(cur, (0, 0))
                            # a header seen from several objects: keep the best
                            if total > old[1] or hit > old[0]:
                                rows[cur] = (max(hit, old[0]), max(total, old[1]))
                        cur = None
    th = tt = 0
    print(f"{'file':60s} {'lines':>7s} {'hit':>7s} {'cover':>7s}")
    for path in sorted(rows):
        hit, total = rows[path]
        th += hit
        tt += total
        print(f"{os.path.relpath(path, REPO):60s} {total:7d} {hit:7d} {100 * hit / max(total, 1):6.1f}%")
    print(f"{'TOTAL':60s} {tt:7d} {th:7d} {100 * th / max(tt, 1):6.1f}%")


if __name__ == "__main__":
    main()
