#!/usr/bin/env bash
# Kernel census of the GPU test suite: first the
# reference-shape device tests alone, then `pytest -m gpu` under
# rocprofv3 --kernel-trace --stats; tools/kernel_census.py turns the stats
# into a markdown table (profiles/*/gpu_suite_kernels.md).
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_reference_shapes.py -q -x --timeout 120 \
    --timeout-method thread > "$OUT/refshape_tests.log" 2>&1
rc=$?
tail -3 "$OUT/refshape_tests.log"
if [ $rc -ne 0 ] || grep -q '+++ Timeout +++' "$OUT/refshape_tests.log"; then
  echo "reference-shape tests rc=$rc: stop"; exit 1
fi
export TMPDIR=/tmp
cd /tmp
timeout -k 10 1000 rocprofv3 --kernel-trace --stats -d "$OUT/census" -o suite \
    --output-format csv -- python3 -u -m pytest "$ROOT/tests" -m gpu -q -p no:cacheprovider \
    --rootdir "$ROOT" --timeout 120 --timeout-method thread > "$OUT/census_pytest.log" 2>&1
rc=$?
tail -3 "$OUT/census_pytest.log"
echo "census rc=$rc"
exit $rc
