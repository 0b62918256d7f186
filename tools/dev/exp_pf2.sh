# dev experiment: kernel times of the 64-slot talker step with and without weight prefetch (Q3T_MM_PREFETCH)
set -o pipefail
export TMPDIR=/tmp
for pf in 0 1; do
  Q3T_DEV_LIB=1 Q3T_MM_PREFETCH=$pf timeout -k 10 180 rocprofv3 --kernel-trace -d gpurun_out/pf$pf -o pf -- python3 tools/dev/stage_only.py 0 64 266 20 > gpurun_out/pf$pf.log 2>&1 || exit 1
done
for pf in 0 1 0 1; do
  Q3T_DEV_LIB=1 Q3T_MM_PREFETCH=$pf timeout -k 10 120 python3 tools/dev/stage_only.py 0 64 266 20 || exit 1
done
