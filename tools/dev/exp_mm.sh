# dev experiment: 64-slot talker step / code-predictor frame with 32- vs 64-token GEMM tiles (Q3T_MFMA_TT, dev build)
set -o pipefail
T="timeout -k 10 120"
for tt in 1 2 1 2; do
  echo "== Q3T_MFMA_TT=$tt"
  Q3T_DEV_LIB=1 Q3T_MFMA_TT=$tt $T python3 tools/dev/stage_only.py 0 64 266 20 || exit 1
  Q3T_DEV_LIB=1 Q3T_MFMA_TT=$tt $T python3 tools/dev/stage_only.py 1 64 266 20 || exit 1
done
