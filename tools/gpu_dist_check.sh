# dist / parallel GPU tests + bench.py standalone and under torchrun N=1 (gpurun).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_dist.py tests/test_parallel.py -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_dist.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_dist.log
if [ $rc -ne 0 ] || grep -q '+++ Timeout +++' gpurun_out/pytest_dist.log; then echo "failed/hung: stop"; exit 1; fi
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_torchrun.log 2>&1 || { tail -20 gpurun_out/bench_torchrun.log; exit 1; }
grep metric gpurun_out/bench_torchrun.log | tail -1
