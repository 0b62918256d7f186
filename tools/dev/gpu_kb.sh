#!/bin/bash
# dev: GPU parity tests first (the library), then kernel microbenchmarks (rebuilt here against the current headers),
# then the bench/trace iteration.  Stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
TAG=${1:-kb}
timeout -k 10 700 python -m pytest tests -q -m gpu -x --timeout 600 -rf > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_$TAG.log
[ $rc -ne 0 ] && exit 1
rm -f tools/dev/_build/kbench && make -s -C tools/dev kbench > gpurun_out/kbench_build_$TAG.log 2>&1 || { echo "kbench build failed"; tail gpurun_out/kbench_build_$TAG.log; exit 1; }
timeout -k 10 300 ./tools/dev/_build/kbench > gpurun_out/kbench_$TAG.txt 2>&1 || { echo kbench failed; tail -20 gpurun_out/kbench_$TAG.txt; exit 1; }
grep -v "min_blocks 1024" gpurun_out/kbench_$TAG.txt
SKIP_TESTS=1 ./tools/dev/gpu_iter.sh $TAG
