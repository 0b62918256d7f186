#!/bin/bash
# dev: bench line + rocprof kernel stats (csv) for the default bench command
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
TAG=${1:-r01}
timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo bench failed; tail -30 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_$TAG" -o run -- python "$R/bench.py" --steps 1 --warmup 1 --cpu-baseline off > "$R/gpurun_out/prof_$TAG.log" 2>&1
echo "rocprof rc=$?"
find "$R/gpurun_out/prof_$TAG" -type f | head -20
