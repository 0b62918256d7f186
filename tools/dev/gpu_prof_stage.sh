#!/bin/bash
# dev: kernel trace of the captured talker-step graph replayed at one position (stage_only.py), per-kernel summary.
# usage: gpu_prof_stage.sh TAG SLOTS [POS] [STAGE]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
TAG=${1:-stage64}
B=${2:-64}
POS=${3:-266}
STAGE=${4:-0}
cd /tmp && export TMPDIR=/tmp
P="$R/gpurun_out/prof_$TAG"
rm -rf "$P"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$P" -o run -- python3 "$R/tools/dev/stage_only.py" $STAGE $B $POS 10 > "$R/gpurun_out/prof_$TAG.log" 2>&1 || { echo "rocprof failed"; tail -20 "$R/gpurun_out/prof_$TAG.log"; exit 1; }
T=$(find "$P" -name '*kernel_trace.csv' | head -1)
python3 "$R/tools/dev/prof_stats.py" "$T" --by-grid > "$R/gpurun_out/prof_${TAG}_summary.txt"
rm -rf "$P"
grep stage "$R/gpurun_out/prof_$TAG.log"
head -40 "$R/gpurun_out/prof_${TAG}_summary.txt"
