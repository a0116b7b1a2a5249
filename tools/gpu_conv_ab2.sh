# Conv A/B: plan of the M = 8192 real block (conv_real 1 = 32 points/thread,
# 2 = 16 points/thread) and the block-size rule at small h.
set -o pipefail
mkdir -p gpurun_out
HLENS=3000,4096 KNOBS="conv_real=1/2" ROUNDS=5 timeout -k 10 300 python -u tools/bench_conv.py > gpurun_out/conv_plan_ab.log 2>&1 || exit 1
tail -3 gpurun_out/conv_plan_ab.log
HLENS=64,300,512,700 KNOBS="os_block_extra=2/3" ROUNDS=5 timeout -k 10 300 python -u tools/bench_conv.py > gpurun_out/conv_small_ab.log 2>&1 || exit 1
tail -5 gpurun_out/conv_small_ab.log
XLEN=4194304 BATCH=256 HLENS=4096 KNOBS="conv_real=1/2" ROUNDS=3 timeout -k 10 300 python -u tools/bench_conv.py > gpurun_out/conv_plan_cfg3.log 2>&1 || exit 1
tail -2 gpurun_out/conv_plan_cfg3.log
