#!/bin/bash
# dev iteration: GPU parity tests -> quick bench (no CPU baseline) -> kernel trace split into talker/CP phases.
# Every GPU step is time-limited; the script stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
TAG=${1:-it}
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 700 python -m pytest tests -q -m gpu -x --timeout 600 -rf > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_$TAG.log
[ $rc -ne 0 ] && exit 1
fi
timeout -k 10 300 python bench.py --vocoder ${VOC:-none} --steps 2 --warmup 1 --cpu-baseline off --batched 0 $BENCH_ARGS > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo bench failed; tail -20 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
cd /tmp && export TMPDIR=/tmp
P="$R/gpurun_out/prof_$TAG"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$P" -o run -- python3 "$R/bench.py" --vocoder none --steps 1 --warmup 0 --frames 12 --cpu-baseline off --batched 0 --serve 0 > "$R/gpurun_out/prof_$TAG.log" 2>&1 || { echo "rocprof failed"; tail -20 "$R/gpurun_out/prof_$TAG.log"; exit 1; }
T=$(find "$P" -name '*kernel_trace.csv' | head -1)
python3 "$R/tools/dev/trace_phases.py" "$T" > "$R/gpurun_out/phases_$TAG.txt"
cat "$R/gpurun_out/phases_$TAG.txt"
rm -rf "$P"
