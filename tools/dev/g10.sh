# dev (round 6): the 192-channel 7-tap conv on k_conv_pd (Q3T_CONV_PD_MINC=192) or k_conv_mt (384), both in XCD order
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
for V in 192 384; do
  Q3T_CONV_PD_MINC=$V bash tools/dev/gpu.sh trace voc_m$V "python3 $R/tools/dev/voc_only.py 512" --by-grid > /dev/null || exit 1
  grep -E "g163840x2|g327680x2|total" gpurun_out/prof_voc_m${V}_summary.txt
done
