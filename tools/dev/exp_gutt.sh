# dev experiment: 64-token tiles for the batched gate/up projection only (Q3T_MM_GU_TT=2) vs the default 32
set -o pipefail
T="timeout -k 10 120"
for tt in 1 2 1 2; do
  echo "== Q3T_MM_GU_TT=$tt"
  Q3T_MM_GU_TT=$tt $T python3 tools/dev/stage_only.py 0 64 266 20 || exit 1
  Q3T_MM_GU_TT=$tt $T python3 tools/dev/stage_only.py 1 64 266 20 || exit 1
done
Q3T_MM_GU_TT=2 $T python3 -u -m pytest -x -q --timeout 100 --timeout-method thread tests/test_gpu_mfma.py 2>&1 | tail -3 || exit 1
