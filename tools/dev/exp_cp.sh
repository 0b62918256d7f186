# dev experiment: talker step / code-predictor frame replay times of two experiment builds, alternating on one box
# (usage: exp_cp.sh VARIANT_A VARIANT_B)
set -o pipefail
T="timeout -k 10 120"
A=${1:-prev}; B=${2:-cur}
for i in 1 2; do
  for v in $A $B; do
    echo "== $v"
    Q3T_DEV_LIB=$v $T python3 tools/dev/stage_only.py 0 1 266 50 || exit 1
    Q3T_DEV_LIB=$v $T python3 tools/dev/stage_only.py 1 1 266 50 || exit 1
  done
done
