# Conv path tests + A/B of the real-block vs pair kernels (gpurun).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_conv_paths.py tests/test_convolve.py -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/pytest_conv.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_conv.log
if [ $rc -gt 1 ] || grep -q '+++ Timeout +++' gpurun_out/pytest_conv.log; then echo "hung/crashed: stop"; exit 1; fi
timeout -k 10 300 env KNOBS="conv_real=0/1" HLENS=64,1500,3000,4096 python -u tools/bench_conv.py > gpurun_out/conv_ab.log 2>&1; tail -6 gpurun_out/conv_ab.log
timeout -k 10 300 env KNOBS="conv_real=0/1" HLENS=4096 XLEN=4194304 BATCH=256 ROUNDS=3 python -u tools/bench_conv.py > gpurun_out/conv_ab_cfg3.log 2>&1; tail -2 gpurun_out/conv_ab_cfg3.log
