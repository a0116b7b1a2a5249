#!/usr/bin/env bash
# PMC counter passes over tools/sgemm_once.py (our variants + torch.matmul),
# one rocprofv3 run per counter set (counters only, no trace domains).
# Usage (from gpurun): bash tools/pmc_sgemm.sh VARIANTS SHAPE TAG
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
VARIANTS="${1:-3}"; SHAPE="${2:-4096}"; TAG="${3:-pmc}"
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
SETS=(
  "GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY"
  "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU"
  "SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_LDS"
  "SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM"
)
i=0
for s in "${SETS[@]}"; do
  i=$((i + 1))
  VARIANTS="$VARIANTS" SHAPE="$SHAPE" REPS=3 timeout -k 10 300 \
    rocprofv3 --pmc $s -d "$OUT/set$i" -o run --output-format csv \
    -- python3 "$ROOT/tools/sgemm_once.py" > "$OUT/set$i.log" 2>&1
  rc=$?
  echo "set$i rc=$rc"
  if [ $rc -ne 0 ]; then tail -20 "$OUT/set$i.log"; exit $rc; fi
done
python3 "$ROOT/tools/pmc_summary.py" "$OUT/summary.md" $(find "$OUT" -name '*counter_collection.csv')
