# Conv tests + kernel-time profile of the bench conv configuration (gpurun).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_conv_paths.py tests/test_convolve.py -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/pytest_conv.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_conv.log
if [ $rc -gt 1 ] || grep -q '+++ Timeout +++' gpurun_out/pytest_conv.log; then echo "hung/crashed: stop"; exit 1; fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/convprof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/tools/conv_once.py" > "$GRAFT_REPO_ROOT/gpurun_out/convprof.log" 2>&1 || exit 1
cut -d, -f1-8 "$GRAFT_REPO_ROOT"/gpurun_out/convprof/run_kernel_stats.csv | head -8
