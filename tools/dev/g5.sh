# dev (round 6): vocoder A/B against the previous build (libq3t_head.so): bit-exact PCM, then kernel traces per grid
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
Q3T_DEV_LIB=head timeout -k 10 120 python3 tools/dev/voc_dump.py gpurun_out/voc_head.npz || exit 1
timeout -k 10 120 python3 tools/dev/voc_dump.py gpurun_out/voc_new.npz || exit 1
python3 tools/dev/voc_dump.py --cmp gpurun_out/voc_head.npz gpurun_out/voc_new.npz || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_vocoder.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/g5_tests.log 2>&1; rc=$?; tail -1 gpurun_out/g5_tests.log; [ $rc -eq 0 ] || exit $rc
for V in head new; do
  if [ $V = head ]; then export Q3T_DEV_LIB=head; else unset Q3T_DEV_LIB; fi
  timeout -k 10 120 python3 tools/dev/voc_only.py 512 0 16 | tail -4 || exit 1
  bash tools/dev/gpu.sh trace voc_$V "python3 $R/tools/dev/voc_only.py 512" --by-grid > /dev/null || exit 1
  grep -E "attn_prefill|total" gpurun_out/prof_voc_${V}_summary.txt
done
