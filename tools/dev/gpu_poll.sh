#!/bin/bash
# dev: B=1 talker step / CP frame per persistent-kernel poll sleep (experiment builds libq3t_<v>.so)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
for v in 1 s0 s4; do
  lib=$v; [ "$v" = 1 ] && lib=""
  for st in 0 1; do
    Q3T_DEV_LIB=$lib timeout -k 10 100 python3 tools/dev/stage_only.py $st 1 266 40 | sed "s/^/$v: /" || exit 1
  done
done
