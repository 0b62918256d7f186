#!/bin/bash
# dev: kernel trace of the batched (B=64) frame loop, summarised per kernel and split into talker/CP phases
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
TAG=${1:-b64}
B=${B:-64}
cd /tmp && export TMPDIR=/tmp
P="$R/gpurun_out/prof_$TAG"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$P" -o run -- python3 "$R/bench.py" --batch $B --vocoder none --steps 1 --warmup 0 --frames 6 --cpu-baseline off --stage-iters 2 > "$R/gpurun_out/prof_$TAG.log" 2>&1 || { echo "rocprof failed"; tail -20 "$R/gpurun_out/prof_$TAG.log"; exit 1; }
T=$(find "$P" -name '*kernel_trace.csv' | head -1)
python3 "$R/tools/dev/prof_stats.py" "$T" > "$R/gpurun_out/prof_${TAG}_summary.txt"
python3 "$R/tools/dev/trace_phases.py" "$T" > "$R/gpurun_out/phases_$TAG.txt" || true
cat "$R/gpurun_out/prof_${TAG}_summary.txt" | head -30
cat "$R/gpurun_out/phases_$TAG.txt" | head -40
rm -rf "$P"
