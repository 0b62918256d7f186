#!/bin/bash
# dev: ordered kernel sequence (with durations) of the last FULL vocoder decode of voc_only.py
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
TAG=${1:-vseq}
cd /tmp && export TMPDIR=/tmp
P="$R/gpurun_out/prof_$TAG"
rm -rf "$P"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$P" -o run -- python3 "$R/tools/dev/voc_only.py" ${F:-512} > "$R/gpurun_out/prof_$TAG.log" 2>&1 || { echo "rocprof failed"; tail -20 "$R/gpurun_out/prof_$TAG.log"; exit 1; }
T=$(find "$P" -name '*kernel_trace.csv' | head -1)
python3 "$R/tools/dev/prof_stats.py" "$T" --seq ${N:-260} > "$R/gpurun_out/prof_${TAG}_seq.txt"
rm -rf "$P"
grep vocoder "$R/gpurun_out/prof_$TAG.log"
