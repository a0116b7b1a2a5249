# Conv block-size A/B (os_block_extra 2 vs 3) after the conv path tests.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_conv_paths.py tests/test_convolve.py tests/test_gpu_reference_shapes.py -q -x -m gpu --timeout 120 --timeout-method thread > gpurun_out/conv_tests.log 2>&1; rc=$?; tail -3 gpurun_out/conv_tests.log
if [ $rc -ne 0 ] || grep -q '+++ Timeout +++' gpurun_out/conv_tests.log; then echo "tests failed/hung: stop"; exit 1; fi
HLENS=1000,2000,3000,4096 KNOBS="os_block_extra=2/3" ROUNDS=5 timeout -k 10 300 python -u tools/bench_conv.py > gpurun_out/conv_extra_ab.log 2>&1 || exit 1
tail -5 gpurun_out/conv_extra_ab.log
XLEN=4194304 BATCH=256 HLENS=4096 KNOBS="os_block_extra=2/3" ROUNDS=3 timeout -k 10 300 python -u tools/bench_conv.py > gpurun_out/conv_extra_cfg3.log 2>&1 || exit 1
tail -2 gpurun_out/conv_extra_cfg3.log
