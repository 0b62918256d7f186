# dev experiment: vocoder FULL decode time, fused residual units vs the two-conv form, then the vocoder tests
set -o pipefail
T="timeout -k 10 120"
$T python3 tools/dev/voc_only.py 512 0 8 || exit 1
Q3T_VOC_FUSE=0 $T python3 tools/dev/voc_only.py 512 0 8 || exit 1
