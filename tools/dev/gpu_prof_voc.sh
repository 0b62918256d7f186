#!/bin/bash
# dev: kernel trace of the FULL vocoder over 512 frames, summarised per kernel
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
TAG=${1:-voc}
cd /tmp && export TMPDIR=/tmp
P="$R/gpurun_out/prof_$TAG"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$P" -o run -- python3 "$R/tools/dev/voc_only.py" ${F:-512} > "$R/gpurun_out/prof_$TAG.log" 2>&1 || { echo "rocprof failed"; tail -20 "$R/gpurun_out/prof_$TAG.log"; exit 1; }
T=$(find "$P" -name '*kernel_trace.csv' | head -1)
python3 "$R/tools/dev/prof_stats.py" "$T" --by-grid > "$R/gpurun_out/prof_${TAG}_summary.txt"
grep vocoder "$R/gpurun_out/prof_$TAG.log"
head -40 "$R/gpurun_out/prof_${TAG}_summary.txt"
rm -rf "$P"
