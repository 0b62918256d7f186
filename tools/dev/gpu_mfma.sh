#!/bin/bash
# MFMA-utilisation + HBM evidence for one command: a kernel trace (durations) and three PMC passes (MFMA instruction
# count and busy cycles; FETCH_SIZE; WRITE_SIZE), joined per kernel by tools/dev/mfma_table.py.
# usage: gpu_mfma.sh TAG "python3 /abs/script.py args"      output: gpurun_out/mfma_TAG.txt
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
TAG=$1; CMD=$2
cd /tmp && export TMPDIR=/tmp
P="$R/gpurun_out/mfma_$TAG"
rm -rf "$P"
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d "$P/trace" -o t -- $CMD > "$R/gpurun_out/mfma_${TAG}_trace.log" 2>&1 || { echo "trace failed"; tail -5 "$R/gpurun_out/mfma_${TAG}_trace.log"; exit 1; }
i=0
for C in "SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --pmc $C --output-format csv -d "$P/p$i" -o p -- $CMD > "$R/gpurun_out/mfma_${TAG}_p$i.log" 2>&1 || { echo "pmc pass $i ($C) failed"; tail -5 "$R/gpurun_out/mfma_${TAG}_p$i.log"; exit 1; }
done
python3 "$R/tools/dev/mfma_table.py" "$P" > "$R/gpurun_out/mfma_${TAG}.txt"
cat "$R/gpurun_out/mfma_${TAG}.txt"
rm -rf "$P"
