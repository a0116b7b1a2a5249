# A/B of two library builds (VELES_SIMD_LIB) over a benchmark script, in
# alternating processes: bash tools/gpu_lib_ab.sh <lib_a> <lib_b> <rounds> <script> [args]
set -o pipefail
A=$1; B=$2; N=$3; shift 3
mkdir -p gpurun_out
for i in $(seq 1 "$N"); do
  for tag in A B; do
    lib=$A; [ $tag = B ] && lib=$B
    echo "== $tag round $i ($lib)"
    VELES_SIMD_LIB=$lib timeout -k 10 300 python -u "$@" 2>&1 | grep -v amdgpu.ids | tail -4 || exit 1
  done
done
