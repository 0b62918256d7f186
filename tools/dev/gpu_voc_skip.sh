#!/bin/bash
# dev: FULL 512-frame vocoder time with parts of the multi-tap convs skipped (Q3T_CONV_SKIP, development library):
# 1 weight loads, 2 window loads, 4 epilogue; the per-launch sequence of each run under rocprof
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
for v in ${SKIPS:-0 1 2 4 7}; do
  P="$R/gpurun_out/prof_skip$v"; rm -rf "$P"
  Q3T_DEV_LIB=1 Q3T_CONV_SKIP=$v timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d "$P" -o run -- python3 "$R/tools/dev/voc_only.py" 512 > "$R/gpurun_out/skip$v.log" 2>&1 || exit 1
  T=$(find "$P" -name '*kernel_trace.csv' | head -1)
  python3 "$R/tools/dev/prof_stats.py" "$T" --seq 260 > "$R/gpurun_out/skip${v}_seq.txt"
  rm -rf "$P"
  echo "skip $v: $(grep vocoder "$R/gpurun_out/skip$v.log" | tail -1)"
  grep "g982528x1\|g327680x2\|g81920x4\|g16384x8" "$R/gpurun_out/skip${v}_seq.txt" | grep ", 7, " | tail -4
done
