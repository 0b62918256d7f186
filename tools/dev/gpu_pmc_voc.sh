#!/bin/bash
# dev: PMC counters of the vocoder convs (separate passes per counter group) over a FULL decode of ${F:-512} frames
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
P="$R/gpurun_out/pmc_voc"
rm -rf "$P"
i=0
for G in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_SALU" \
         "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_VMEM" \
         "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $G --output-format csv -d "$P/p$i" -o p -- python3 "$R/tools/dev/voc_only.py" ${F:-512} > "$R/gpurun_out/pmc_voc_$i.log" 2>&1 || { echo "pmc pass $i failed"; tail -5 "$R/gpurun_out/pmc_voc_$i.log"; exit 1; }
done
python3 "$R/tools/dev/pmc_table.py" "$P" 30 > "$R/gpurun_out/pmc_voc_table.txt"
cat "$R/gpurun_out/pmc_voc_table.txt"
rm -rf "$P"
