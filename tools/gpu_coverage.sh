#!/usr/bin/env bash
# Host line coverage of the library under the whole test suite: the `make
# coverage` build (build-cov, made beforehand on the CPU host) runs the native
# C test, `pytest -m gpu` and the CPU suite on the GPU box, counts
# accumulating in one set of .gcda files; per-file report to
# gpurun_out/coverage_gpu.txt.  build-cov is in .gpurunignore (23 MiB that no
# other GPU run reads): drop that line for the call.
# Usage (from gpurun): bash tools/gpu_coverage.sh
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"
COV="$ROOT/build-cov"
mkdir -p "$OUT"
cd "$ROOT"
[ -f "$COV/lib/libvelessimd.so" ] || { echo "build-cov missing: run make coverage first"; exit 2; }
find "$COV" -name '*.gcda' -delete
timeout -k 10 120 "$COV/tests/capi_test" > "$OUT/cov_capi.log" 2>&1
rc=$?
echo "capi_test rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
VELES_SIMD_LIB="$COV/lib/libvelessimd.so" timeout -k 10 900 \
  python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > "$OUT/cov_pytest.log" 2>&1
rc=$?
echo "pytest rc=$rc"; tail -n 3 "$OUT/cov_pytest.log"
if grep -q '+++ Timeout +++' "$OUT/cov_pytest.log"; then exit 124; fi
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
VELES_SIMD_LIB="$COV/lib/libvelessimd.so" timeout -k 10 600 \
  python -u -m pytest tests -m "not gpu" -q -p no:cacheprovider > "$OUT/cov_pytest_cpu.log" 2>&1
rc=$?
echo "pytest (not gpu) rc=$rc"; tail -n 3 "$OUT/cov_pytest_cpu.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
python tools/coverage_report.py "$COV" > "$OUT/coverage_gpu.txt"
tail -n 30 "$OUT/coverage_gpu.txt"
