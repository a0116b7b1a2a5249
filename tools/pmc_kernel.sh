#!/usr/bin/env bash
# PMC counter passes over any python script (one rocprofv3 run per counter
# set, counters only, no trace domains), then a kernel-trace pass for the
# per-kernel resource usage (VGPRs, LDS, scratch), summarised by
# tools/pmc_summary.py.  Environment variables reach the script unchanged.
# Usage (from gpurun): bash tools/pmc_kernel.sh TAG SETS script.py [args...]
#   SETS: "core" (wave / VALU / LDS), "mem" (HBM bytes + L2), "all"
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="$1"; WHICH="$2"; shift 2
SCRIPT="$1"; shift
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
CORE=(
  "GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY"
  "SQ_ACTIVE_INST_VALU SQ_BUSY_CU_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU"
  "SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_LDS"
  "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS"
)
MEM=(
  "FETCH_SIZE"
  "WRITE_SIZE TCC_HIT_sum"
  "TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum"
)
case "$WHICH" in
  core) SETS=("${CORE[@]}") ;;
  mem) SETS=("${MEM[@]}") ;;
  *) SETS=("${CORE[@]}" "${MEM[@]}") ;;
esac
i=0
for s in "${SETS[@]}"; do
  i=$((i + 1))
  timeout -s KILL 120 rocprofv3 --pmc $s -d "$OUT/set$i" -o run --output-format csv \
    -- python3 "$ROOT/$SCRIPT" "$@" > "$OUT/set$i.log" 2>&1
  rc=$?
  echo "set$i rc=$rc"
  if [ $rc -ne 0 ]; then tail -20 "$OUT/set$i.log"; exit $rc; fi
done
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run \
  --output-format csv -- python3 "$ROOT/$SCRIPT" "$@" > "$OUT/trace.log" 2>&1 || exit $?
python3 "$ROOT/tools/pmc_summary.py" "$OUT/summary.md" \
  $(find "$OUT" -name '*counter_collection.csv')
python3 - "$OUT" <<'EOF'
import csv, glob, sys
out = sys.argv[1]
seen = {}
for p in glob.glob(f"{out}/trace/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(p)):
        k = r["Kernel_Name"][:100]
        if k not in seen:
            seen[k] = {c: r.get(c) for c in ("Arch_VGPR_Count", "Accum_VGPR_Count", "SGPR_Count",
                                              "LDS_Block_Size", "Scratch_Size", "Workgroup_Size",
                                              "Grid_Size")}
with open(f"{out}/resources.md", "w") as f:
    for k, v in seen.items():
        f.write(f"{k}: {v}\n")
        print(k, v)
EOF
