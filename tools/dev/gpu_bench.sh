#!/bin/bash
# bench line + rocprof kernel stats (csv, summarised on the box) + FETCH_SIZE passes on the talker step (B=1, B=64)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
TAG=${1:-r01}
BENCH_ARGS=${BENCH_ARGS:-}
if [ -z "$SKIP_BENCH" ]; then
timeout -k 10 900 python bench.py $BENCH_ARGS > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo bench failed; tail -30 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
fi
cd /tmp && export TMPDIR=/tmp
P="$R/gpurun_out/prof_$TAG"
rm -rf "$P"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$P" -o run -- python3 "$R/bench.py" --steps 1 --warmup 0 --frames 12 --cpu-baseline off --batched 0 --serve 0 > "$R/gpurun_out/prof_$TAG.log" 2>&1 || { echo "rocprof failed"; tail -20 "$R/gpurun_out/prof_$TAG.log"; exit 1; }
T=$(find "$P" -name '*kernel_trace.csv' | head -1)
S=$(find "$P" -name '*kernel_stats.csv' | head -1)
python3 "$R/tools/dev/prof_stats.py" "$T" > "$R/gpurun_out/prof_${TAG}_summary.txt"
python3 "$R/tools/dev/trace_phases.py" "$T" > "$R/gpurun_out/phases_${TAG}.txt"
cp "$S" "$R/gpurun_out/prof_${TAG}_kernel_stats.csv"
rm -rf "$P"
head -30 "$R/gpurun_out/prof_${TAG}_summary.txt"
for B in 1 64; do
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$P/pmc$B" -o pmc -- python3 "$R/tools/dev/stage_only.py" 0 $B 266 10 > "$R/gpurun_out/pmc_${TAG}_b$B.log" 2>&1 || { echo "pmc failed"; tail -20 "$R/gpurun_out/pmc_${TAG}_b$B.log"; exit 1; }
  C=$(find "$P/pmc$B" -name '*counter_collection.csv' | head -1)
  python3 "$R/tools/dev/pmc_sum.py" "$C" 11 > "$R/gpurun_out/pmc_${TAG}_b${B}_summary.txt"
  cat "$R/gpurun_out/pmc_${TAG}_b${B}_summary.txt" | head -8
done
rm -rf "$P"
