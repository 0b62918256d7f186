# dev (round 6): pipelined 7-tap conv (k_conv_pd) A/B: bit-exactness tests, vocoder timing and kernel traces with
# Q3T_CONV_PD=0 / 1 (per grid size)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_vocoder.py -m gpu -x -q -k "pipelined or fused or full_matches" --timeout 200 --timeout-method thread > gpurun_out/g4_tests.log 2>&1; rc=$?; tail -1 gpurun_out/g4_tests.log; [ $rc -eq 0 ] || exit $rc
for V in 2 3; do Q3T_CONV_PD=$V timeout -k 10 120 python3 tools/dev/voc_only.py 512 0 16 | tail -3 || exit 1; done
for V in 2 3; do Q3T_CONV_PD=$V bash tools/dev/gpu.sh trace voc_pd$V "python3 $R/tools/dev/voc_only.py 512" --by-grid > /dev/null || exit 1; grep -E "conv_pd|conv_mt<2, 96, 2, 7|total" gpurun_out/prof_voc_pd${V}_summary.txt; done
