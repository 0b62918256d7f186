#!/bin/bash
# dev: kernel microbenchmarks then the iteration script
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
TAG=${1:-kb}
timeout -k 10 300 ./tools/dev/_build/kbench > gpurun_out/kbench_$TAG.txt 2>&1 || { echo kbench failed; tail -20 gpurun_out/kbench_$TAG.txt; exit 1; }
grep -v "min_blocks 1024" gpurun_out/kbench_$TAG.txt
./tools/dev/gpu_iter.sh $TAG
