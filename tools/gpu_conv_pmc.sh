set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_conv_paths.py -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/pytest_conv.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_conv.log
if [ $rc -gt 1 ] || grep -q '+++ Timeout +++' gpurun_out/pytest_conv.log; then echo "hung/crashed: stop"; exit 1; fi
CONV_REAL=1 bash tools/pmc_kernel.sh pmc_real all tools/conv_once.py > gpurun_out/pmc_real.log 2>&1 || exit 1
CONV_REAL=0 bash tools/pmc_kernel.sh pmc_pair all tools/conv_once.py > gpurun_out/pmc_pair.log 2>&1 || exit 1
cat gpurun_out/pmc_real/summary.md gpurun_out/pmc_pair/summary.md
