#!/bin/bash
# dev: FULL 512-frame vocoder time per conv tile variant (development library, Q3T_CONV_VARIANT)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
for v in 0 1 2 3 4; do
  echo "variant $v"
  Q3T_DEV_LIB=1 Q3T_CONV_VARIANT=$v timeout -k 10 100 python3 tools/dev/voc_only.py 512 0 0 | tail -1 || exit 1
done
