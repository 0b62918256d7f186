#!/bin/bash
# dev: rocprofv3 PMC passes (one counter group per run, each run its own time limit) over a command; per-kernel means
# usage: gpu_pmc.sh TAG "python3 script.py args" ["PASS1 counters" "PASS2 counters" ...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
TAG=$1; CMD=$2; shift 2
PASSES=("$@")
[ ${#PASSES[@]} -eq 0 ] && PASSES=("FETCH_SIZE" "WRITE_SIZE" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS" "SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE GRBM_COUNT")
cd /tmp && export TMPDIR=/tmp
P="$R/gpurun_out/pmc_$TAG"
rm -rf "$P"
i=0
for C in "${PASSES[@]}"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --pmc $C --output-format csv -d "$P/p$i" -o p -- $CMD > "$R/gpurun_out/pmc_${TAG}_p$i.log" 2>&1 || { echo "pmc pass $i ($C) failed"; tail -5 "$R/gpurun_out/pmc_${TAG}_p$i.log"; exit 1; }
done
python3 "$R/tools/dev/pmc_table.py" "$P" > "$R/gpurun_out/pmc_${TAG}_summary.txt"
cat "$R/gpurun_out/pmc_${TAG}_summary.txt"
rm -rf "$P"
