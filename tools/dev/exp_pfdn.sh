# dev experiment: the gate/up GEMM's spare CUs prefetch the down projection (Q3T_MM_PREFETCH=2) vs norms only (=1)
set -o pipefail
T="timeout -k 10 120"
$T python3 -u -m pytest -x -q --timeout 100 --timeout-method thread tests/test_gpu_mfma.py 2>&1 | tail -3 || exit 1
for pf in 1 2 1 2 1 2; do
  echo "== Q3T_MM_PREFETCH=$pf"
  Q3T_MM_PREFETCH=$pf $T python3 tools/dev/stage_only.py 0 64 266 20 || exit 1
done
