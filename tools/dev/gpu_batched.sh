#!/bin/bash
# dev: batched-path parity tests, 64-slot stage timings, concurrent-context probe
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 600 python -u -m pytest tests/test_gpu_long.py tests/test_gpu_mfma.py tests/test_gpu_queue.py -x -v -s --timeout 300 --timeout-method thread -m gpu > gpurun_out/batched.log 2>&1
rc=$?
grep -E "PASS|FAIL|passed|failed|Error" gpurun_out/batched.log | head -40
[ $rc -eq 0 ] || { tail -40 gpurun_out/batched.log; exit $rc; }
fi
timeout -k 10 120 python3 tools/dev/stage_only.py 0 64 266 20 || exit 1
timeout -k 10 120 python3 tools/dev/stage_only.py 1 64 266 4 || exit 1
timeout -k 10 240 python3 tools/dev/replica_probe.py 64 128
