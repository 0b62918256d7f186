# dev (round 6): pipelined residual unit (k_resunit96_pd): bit-exactness tests, then per-grid kernel traces with
# Q3T_RESUNIT_PD=0 / 1
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_vocoder.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/g6_tests.log 2>&1; rc=$?; tail -1 gpurun_out/g6_tests.log; [ $rc -eq 0 ] || { tail -30 gpurun_out/g6_tests.log; exit $rc; }
for V in 0 1; do
  Q3T_RESUNIT_PD=$V timeout -k 10 120 python3 tools/dev/voc_only.py 512 0 16 | tail -3 || exit 1
  Q3T_RESUNIT_PD=$V bash tools/dev/gpu.sh trace voc_ru$V "python3 $R/tools/dev/voc_only.py 512" --by-grid > /dev/null || exit 1
  grep -E "resunit|total" gpurun_out/prof_voc_ru${V}_summary.txt
done
