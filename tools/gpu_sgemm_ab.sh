# SGEMM gen-6 tests + interleaved A/B against hipBLASLt (gpurun).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_sgemm_gen6.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_sgemm.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_sgemm.log
if [ $rc -ne 0 ] || grep -q '+++ Timeout +++' gpurun_out/pytest_sgemm.log; then echo "failed/hung: stop"; exit 1; fi
timeout -k 10 400 env VARIANTS=${VARIANTS:-0,1,2,3,4} CHECK=0 ROUNDS=5 python -u tools/bench_sgemm.py > gpurun_out/sgemm_ab.log 2>&1; tail -12 gpurun_out/sgemm_ab.log
