# dev experiment: talker step / code-predictor frame replay times of experiment builds, alternating on one box
# (usage: exp_cp.sh VARIANT_A VARIANT_B [VARIANT_C ...])
set -o pipefail
T="timeout -k 10 120"
VS=${*:-prev cur}
for i in 1 2; do
  for v in $VS; do
    echo "== $v"
    Q3T_DEV_LIB=$v $T python3 tools/dev/stage_only.py 0 1 266 50 || exit 1
    Q3T_DEV_LIB=$v $T python3 tools/dev/stage_only.py 1 1 266 50 || exit 1
  done
done
