#!/bin/bash
# dev: parity tests, bench line, rocprof kernel stats (each GPU step time-limited; stop at first failure)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -m gpu --timeout 500 -rf > gpurun_out/gpu3.log 2>&1
echo "pytest rc=$?"; tail -3 gpurun_out/gpu3.log
timeout -k 10 400 python bench.py --vocoder none --steps 2 --warmup 1 > gpurun_out/bench1.json 2> gpurun_out/bench1.err || { echo bench failed; tail -20 gpurun_out/bench1.err; exit 1; }
cat gpurun_out/bench1.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof1" -o run -- python "$R/bench.py" --vocoder none --steps 1 --warmup 0 --cpu-baseline off > "$R/gpurun_out/prof1.log" 2>&1
echo "rocprof rc=$?"
find "$R/gpurun_out/prof1" -name "*stats*" | head
