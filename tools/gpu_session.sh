#!/usr/bin/env bash
# One GPU-box session: build check, GPU tests, bench, rocprofv3 kernel stats.
# Every GPU step has its own time limit; a crash / hang / abort ends the
# session (no further GPU work), plain test failures (exit 1) do not.
# Usage (from gpurun): bash tools/gpu_session.sh [tests|bench|prof|all] [pytest -k expr]
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
cd "$ROOT"
MODE="${1:-all}"
KEXPR="${2:-}"

step() {  # step <name> <timeout> <cmd...>
  local name=$1 limit=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$limit" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 25 "$OUT/$name.log"
  # pytest-timeout's thread method ends a hung test with os._exit(1): rc 1
  # then means "GPU possibly stuck", not "tests failed".
  if grep -q '+++ Timeout +++' "$OUT/$name.log"; then
    echo "!!! $name hit a per-test timeout (possible GPU hang): stopping the session"
    exit 124
  fi
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "!!! $name ended with rc=$rc: stopping the session"
    exit $rc
  fi
  return 0
}

rocm-smi --showproductname > "$OUT/device.txt" 2>&1 || true
if [ "$MODE" = "tests" ] || [ "$MODE" = "all" ]; then
  if [ -n "$KEXPR" ]; then
    step pytest_gpu 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -k "$KEXPR"
  else
    step pytest_gpu 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread
  fi
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
if [ "$MODE" = "bench" ] || [ "$MODE" = "all" ]; then
  step bench 600 python bench.py --steps 20 --warmup 5
fi
if [ "$MODE" = "prof" ] || [ "$MODE" = "all" ]; then
  export TMPDIR=/tmp
  (cd /tmp && step rocprof 600 rocprofv3 --kernel-trace --stats \
      -d "$OUT/prof" -o run --output-format csv -- \
      python3 "$ROOT/bench.py" --steps 10 --warmup 2)
fi
echo "session done"
