# dev (round 6): XCD-aware tile order of the 1-tap narrow conv: bit-exact PCM against the previous build
# (libq3t_head.so), then per-grid kernel traces with Q3T_CONV_XCD=0 / 1
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
Q3T_DEV_LIB=head timeout -k 10 120 python3 tools/dev/voc_dump.py gpurun_out/voc_head.npz || exit 1
timeout -k 10 120 python3 tools/dev/voc_dump.py gpurun_out/voc_new.npz || exit 1
python3 tools/dev/voc_dump.py --cmp gpurun_out/voc_head.npz gpurun_out/voc_new.npz || exit 1
for V in 0 1; do
  Q3T_CONV_XCD=$V bash tools/dev/gpu.sh trace voc_x$V "python3 $R/tools/dev/voc_only.py 512" --by-grid > /dev/null || exit 1
  grep -E "conv_mt<|conv_pd<|total" gpurun_out/prof_voc_x${V}_summary.txt
done
