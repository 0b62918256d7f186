#!/bin/bash
# dev (round 4): the persistent-kernel measurement batch, one GPU step per line, each under its own time limit; stops at
# the first failure.  usage: gpu_r4.sh [VARIANT...]   (VARIANT: experiment libraries libq3t_<name>.so to time A/B)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
T="timeout -k 10"
[ -x tools/dev/_build/selbench ] && { $T 60 tools/dev/_build/selbench || exit 1; }
$T 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_persist.py tests/test_gpu_select.py 2>&1 | tail -3 || exit 1
for v in "" "$@"; do
    echo "== lib ${v:-release}"
    for a in "0 1 266 50 544" "0 1 500 50 544" "0 1 40 50 544" "0 1 1500 30 2048" "1 1 266 50"; do
        Q3T_DEV_LIB=$v $T 60 python3 tools/dev/stage_only.py $a || exit 1
    done
done
Q3T_DEV_LIB=1 $T 120 python3 tools/dev/persist_dump.py 0 tk544 266 544 || exit 1
Q3T_DEV_LIB=1 $T 120 python3 tools/dev/persist_dump.py 1 cpr || exit 1
