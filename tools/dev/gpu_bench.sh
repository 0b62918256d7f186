#!/bin/bash
# dev: bench line + rocprof kernel stats (csv, summarised on the box) + FETCH_SIZE pass on the talker step
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
TAG=${1:-r01}
BENCH_ARGS=${BENCH_ARGS:-}
if [ -z "$SKIP_BENCH" ]; then
timeout -k 10 600 python bench.py $BENCH_ARGS > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo bench failed; tail -30 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
fi
cd /tmp && export TMPDIR=/tmp
P="$R/gpurun_out/prof_$TAG"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$P" -o run -- python3 "$R/bench.py" --steps 1 --warmup 0 --frames 12 --cpu-baseline off > "$R/gpurun_out/prof_$TAG.log" 2>&1 || { echo "rocprof failed"; tail -20 "$R/gpurun_out/prof_$TAG.log"; exit 1; }
T=$(find "$P" -name '*kernel_trace.csv' | head -1)
S=$(find "$P" -name '*kernel_stats.csv' | head -1)
python3 "$R/tools/dev/prof_stats.py" "$T" > "$R/gpurun_out/prof_${TAG}_summary.txt"
cp "$S" "$R/gpurun_out/prof_${TAG}_kernel_stats.csv"
gzip -f "$T"
cat "$R/gpurun_out/prof_${TAG}_summary.txt" | head -30
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$P/pmc" -o pmc -- python3 "$R/tools/dev/stage_only.py" 0 1 266 10 > "$R/gpurun_out/pmc_$TAG.log" 2>&1 || { echo "pmc failed"; tail -20 "$R/gpurun_out/pmc_$TAG.log"; exit 1; }
C=$(find "$P/pmc" -name '*counter_collection.csv' | head -1)
python3 "$R/tools/dev/pmc_sum.py" "$C" 11 > "$R/gpurun_out/pmc_${TAG}_summary.txt"
cat "$R/gpurun_out/pmc_${TAG}_summary.txt"
gzip -f "$C"
