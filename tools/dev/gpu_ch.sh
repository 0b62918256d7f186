#!/bin/bash
# dev: B=1 talker step time at several KV positions per persistent attention chunk (Q3T_PERSIST_CH, dev library)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
for ch in 64 128 256; do
  for pos in 60 266 500; do
    Q3T_DEV_LIB=1 Q3T_PERSIST_CH=$ch timeout -k 10 100 python3 tools/dev/stage_only.py 0 1 $pos 40 | sed "s/^/ch $ch: /" || exit 1
  done
done
