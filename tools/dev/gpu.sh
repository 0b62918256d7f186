#!/bin/bash
# tools/dev/gpu.sh — the GPU-box steps of development, one parameterised script (run through gpurun from the repo
# root).  Every GPU step runs under its own time limit and the script stops at the first failure (no retries).
#
#   gpu.sh tests [SELECTION] [PYTEST_ARGS]   GPU tests in one pytest process + smoke()       -> gpurun_out/gpu_tests.log
#   gpu.sh bench TAG [BENCH_ARGS]            bench line                                       -> gpurun_out/bench_TAG.json
#   gpu.sh trace TAG "CMD" [--by-grid|--seq N]  kernel trace + per-kernel summary of CMD      -> gpurun_out/prof_TAG_summary.txt
#   gpu.sh phases TAG                        kernel trace of a short B=1 bench, split into talker / CP / vocoder phases
#   gpu.sh fetch TAG [SLOTS...]              FETCH_SIZE pass over the talker-step replay at KV position 266 (x2 gfx950
#                                            correction in pmc_sum.py)                        -> gpurun_out/pmc_TAG_bN_summary.txt
#   gpu.sh pmc TAG "CMD" ["COUNTERS" ...]    PMC passes, one counter group per run            -> gpurun_out/pmc_TAG_summary.txt
#   gpu.sh mfma TAG "CMD"                    kernel trace + SQ_INSTS_MFMA / FETCH / WRITE passes joined per kernel
#   gpu.sh stage STAGE SLOTS [POS] [ITERS]   replay time of the talker step (0) / code-predictor frame (1)
#
# CMD examples: "python3 $R/tools/dev/stage_only.py 0 64 266 5", "python3 $R/tools/dev/voc_only.py 512".
# Development-library knobs (Q3T_DEV_LIB=1 with make DEV=1, or Q3T_DEV_LIB=<variant>) pass through the environment.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
task=$1
shift

prof_dir() { cd /tmp && export TMPDIR=/tmp; P="$R/gpurun_out/prof_$1"; rm -rf "$P"; }

case "$task" in
tests)
    SEL=${1:-tests}; EXTRA=${2:-}
    timeout -k 10 1000 python -u -m pytest $SEL -m gpu -v --maxfail=5 --timeout 300 --timeout-method thread -s $EXTRA \
        > gpurun_out/gpu_tests.log 2>&1
    rc=$?
    grep -E "PASSED|FAILED|ERROR|passed|failed|exact|max\|d\|" gpurun_out/gpu_tests.log | tail -80
    [ $rc -ne 0 ] && { tail -80 gpurun_out/gpu_tests.log; exit $rc; }
    timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -30 gpurun_out/smoke.log; exit 1; }
    tail -2 gpurun_out/smoke.log ;;
bench)
    TAG=$1; shift
    timeout -k 10 900 python bench.py "$@" > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo bench failed; tail -30 gpurun_out/bench_$TAG.err; exit 1; }
    cat gpurun_out/bench_$TAG.json ;;
trace)
    TAG=$1; CMD=$2; MODE=${3:-}; N=${4:-}
    prof_dir "$TAG"
    timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$P" -o run -- $CMD > "$R/gpurun_out/prof_$TAG.log" 2>&1 || { echo "rocprof failed"; tail -20 "$R/gpurun_out/prof_$TAG.log"; exit 1; }
    T=$(find "$P" -name '*kernel_trace.csv' | head -1)
    S=$(find "$P" -name '*kernel_stats.csv' | head -1)
    python3 "$R/tools/dev/prof_stats.py" "$T" $MODE $N > "$R/gpurun_out/prof_${TAG}_summary.txt"
    [ -n "$S" ] && cp "$S" "$R/gpurun_out/prof_${TAG}_kernel_stats.csv"
    rm -rf "$P"
    grep -E "stage|vocoder" "$R/gpurun_out/prof_$TAG.log"
    head -40 "$R/gpurun_out/prof_${TAG}_summary.txt" ;;
phases)
    TAG=$1
    prof_dir "$TAG"
    timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$P" -o run -- python3 "$R/bench.py" --steps 1 --warmup 0 --frames 12 --cpu-baseline off --batched 0 --serve 0 > "$R/gpurun_out/prof_$TAG.log" 2>&1 || { echo "rocprof failed"; tail -20 "$R/gpurun_out/prof_$TAG.log"; exit 1; }
    T=$(find "$P" -name '*kernel_trace.csv' | head -1)
    S=$(find "$P" -name '*kernel_stats.csv' | head -1)
    python3 "$R/tools/dev/prof_stats.py" "$T" > "$R/gpurun_out/prof_${TAG}_summary.txt"
    python3 "$R/tools/dev/trace_phases.py" "$T" > "$R/gpurun_out/phases_${TAG}.txt"
    cp "$T" "$R/gpurun_out/trace_${TAG}.csv"
    cp "$S" "$R/gpurun_out/prof_${TAG}_kernel_stats.csv"
    rm -rf "$P"
    head -30 "$R/gpurun_out/prof_${TAG}_summary.txt" ;;
fetch)
    TAG=$1; shift
    SLOTS=${*:-1 64}
    prof_dir "fetch_$TAG"
    for B in $SLOTS; do
        Q3T_CP_QKV_TABLE=0 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$P/pmc$B" -o pmc -- python3 "$R/tools/dev/stage_only.py" 0 $B 266 10 > "$R/gpurun_out/pmc_${TAG}_b$B.log" 2>&1 || { echo "pmc failed"; tail -20 "$R/gpurun_out/pmc_${TAG}_b$B.log"; exit 1; }
        C=$(find "$P/pmc$B" -name '*counter_collection.csv' | head -1)
        python3 "$R/tools/dev/pmc_sum.py" "$C" 11 > "$R/gpurun_out/pmc_${TAG}_b${B}_summary.txt"
        head -8 "$R/gpurun_out/pmc_${TAG}_b${B}_summary.txt"
    done
    rm -rf "$P" ;;
pmc)
    TAG=$1; CMD=$2; shift 2
    PASSES=("$@")
    [ ${#PASSES[@]} -eq 0 ] && PASSES=("FETCH_SIZE" "WRITE_SIZE" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS" "SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE GRBM_COUNT")
    prof_dir "pmc_$TAG"
    i=0
    for C in "${PASSES[@]}"; do
        i=$((i+1))
        timeout -s KILL 180 rocprofv3 --pmc $C --output-format csv -d "$P/p$i" -o p -- $CMD > "$R/gpurun_out/pmc_${TAG}_p$i.log" 2>&1 || { echo "pmc pass $i ($C) failed"; tail -5 "$R/gpurun_out/pmc_${TAG}_p$i.log"; exit 1; }
    done
    python3 "$R/tools/dev/pmc_table.py" "$P" > "$R/gpurun_out/pmc_${TAG}_summary.txt"
    cat "$R/gpurun_out/pmc_${TAG}_summary.txt"
    rm -rf "$P" ;;
mfma)
    TAG=$1; CMD=$2
    prof_dir "mfma_$TAG"
    timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d "$P/trace" -o t -- $CMD > "$R/gpurun_out/mfma_${TAG}_trace.log" 2>&1 || { echo "trace failed"; tail -5 "$R/gpurun_out/mfma_${TAG}_trace.log"; exit 1; }
    i=0
    for C in "SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" "FETCH_SIZE" "WRITE_SIZE"; do
        i=$((i+1))
        timeout -s KILL 180 rocprofv3 --pmc $C --output-format csv -d "$P/p$i" -o p -- $CMD > "$R/gpurun_out/mfma_${TAG}_p$i.log" 2>&1 || { echo "pmc pass $i ($C) failed"; tail -5 "$R/gpurun_out/mfma_${TAG}_p$i.log"; exit 1; }
    done
    python3 "$R/tools/dev/mfma_table.py" "$P" > "$R/gpurun_out/mfma_${TAG}.txt"
    cat "$R/gpurun_out/mfma_${TAG}.txt"
    rm -rf "$P" ;;
stage)
    timeout -k 10 120 python3 tools/dev/stage_only.py "$1" "$2" "${3:-266}" "${4:-20}" ;;
*)
    sed -n '2,20p' "$0"; exit 2 ;;
esac
