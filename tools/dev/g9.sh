# dev (round 6): vocoder A/B against the previous build (libq3t_head.so): bit-exact PCM, per-grid traces of both
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
Q3T_DEV_LIB=head timeout -k 10 120 python3 tools/dev/voc_dump.py gpurun_out/voc_head.npz || exit 1
timeout -k 10 120 python3 tools/dev/voc_dump.py gpurun_out/voc_new.npz || exit 1
python3 tools/dev/voc_dump.py --cmp gpurun_out/voc_head.npz gpurun_out/voc_new.npz || exit 1
for V in head new; do
  if [ $V = head ]; then export Q3T_DEV_LIB=head; else unset Q3T_DEV_LIB; fi
  bash tools/dev/gpu.sh trace voc_$V "python3 $R/tools/dev/voc_only.py 512" --by-grid > /dev/null || exit 1
  grep -E "attn_prefill|total" gpurun_out/prof_voc_${V}_summary.txt
done
