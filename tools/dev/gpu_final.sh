#!/bin/bash
# dev (round 4): end-of-round check on one box: the GPU test suite, smoke(), the default bench line, and the
# kernel-trace summaries (gpu.sh phases: the shortened bench; the 64-slot talker stage).  Stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/final_tests.log 2>&1 || { tail -30 gpurun_out/final_tests.log; exit 1; }
tail -2 gpurun_out/final_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final_smoke.log 2>&1 || { tail -20 gpurun_out/final_smoke.log; exit 1; }
tail -1 gpurun_out/final_smoke.log
timeout -k 10 600 python bench.py > gpurun_out/final_bench.json 2> gpurun_out/final_bench.err || { tail -20 gpurun_out/final_bench.err; exit 1; }
cat gpurun_out/final_bench.json
bash tools/dev/gpu.sh phases final > gpurun_out/final_prof.log 2>&1 || { tail -20 gpurun_out/final_prof.log; exit 1; }
bash tools/dev/gpu.sh trace final_stage64_talker "python3 $R/tools/dev/stage_only.py 0 64 266 20" >> gpurun_out/final_prof.log 2>&1 || exit 1
echo done
