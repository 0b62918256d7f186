#!/bin/bash
# GPU test suite + smoke on the box (one pytest process; per-test and whole-run time limits); logs under gpurun_out/
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
SEL=${1:-tests}
EXTRA=${2:-}
timeout -k 10 1000 python -u -m pytest $SEL -m gpu -v --maxfail=5 --timeout 300 --timeout-method thread -s $EXTRA \
    > gpurun_out/gpu_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed|frames|exact|max\|d\|" gpurun_out/gpu_tests.log | tail -60
[ $rc -ne 0 ] && { tail -80 gpurun_out/gpu_tests.log; exit $rc; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -30 gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
