# dev (round 6): batched talker attention A/B: stage replays at 16-64 slots, then the batched-family GPU tests
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for B in 64 32; do timeout -k 10 120 python3 tools/dev/stage_only.py 0 $B 266 20 || exit 1; done
timeout -k 10 120 python3 tools/dev/stage_only.py 0 64 500 20 564 || exit 1
timeout -k 10 120 python3 tools/dev/stage_only.py 0 64 60 20 || exit 1
timeout -k 10 900 python -u -m pytest tests/test_gpu_tkb.py tests/test_gpu_depth.py tests/test_gpu_mfma.py tests/test_gpu_queue.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/g3_tests.log 2>&1; rc=$?; tail -5 gpurun_out/g3_tests.log; exit $rc
