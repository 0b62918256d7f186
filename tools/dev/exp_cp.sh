# dev experiment: talker step / code-predictor frame replay times, release library vs experiment variants
set -o pipefail
T="timeout -k 10 120"
for i in 1 2; do
$T python3 tools/dev/stage_only.py 0 1 266 50 || exit 1
Q3T_DEV_LIB=h0 $T python3 tools/dev/stage_only.py 0 1 266 50 || exit 1
$T python3 tools/dev/stage_only.py 1 1 266 50 || exit 1
Q3T_DEV_LIB=h1 $T python3 tools/dev/stage_only.py 1 1 266 50 || exit 1
done
