set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
# rc 1 with pytest-timeout's banner is a hang (os._exit(1)), not a test failure.
if [ $rc -gt 1 ] || grep -q '+++ Timeout +++' gpurun_out/pytest_gpu.log; then echo "pytest hung or crashed: stopping"; exit 1; fi
timeout -k 10 300 env KNOBS="conv_buffer=0/1" HLENS=16,64,512,4096 python -u tools/bench_conv.py > gpurun_out/conv_ab.log 2>&1 && tail -6 gpurun_out/conv_ab.log &&
timeout -k 10 300 env VARIANTS=15,16,19,21,22 ROUNDS=5 python -u tools/bench_sgemm.py > gpurun_out/sgemm_ab.log 2>&1 && tail -2 gpurun_out/sgemm_ab.log &&
timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 > gpurun_out/bench.log 2>&1 && tail -1 gpurun_out/bench.log
