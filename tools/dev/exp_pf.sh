# dev experiment: batched residual-norm rewrite (straight-line slab loads), weight prefetch workgroups
# (Q3T_MM_PREFETCH), k_attn_seq three-buffer pipeline
set -o pipefail
T="timeout -k 10 120"
$T python3 -u -m pytest -x -q --timeout 100 --timeout-method thread tests/test_gpu_mfma.py 2>&1 | tail -5 || exit 1
for pf in 0 1 0 1; do
  echo "== Q3T_MM_PREFETCH=$pf"
  Q3T_DEV_LIB=1 Q3T_MM_PREFETCH=$pf $T python3 tools/dev/stage_only.py 0 64 266 20 || exit 1
  Q3T_DEV_LIB=1 Q3T_MM_PREFETCH=$pf $T python3 tools/dev/stage_only.py 1 64 266 20 || exit 1
done
export TMPDIR=/tmp
Q3T_DEV_LIB=1 timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/pf_prof -o pf -- python3 tools/dev/stage_only.py 0 64 266 20 > gpurun_out/pf_prof.log 2>&1 || exit 1
