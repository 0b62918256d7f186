#!/bin/bash
# MFMA-utilisation tables (tools/dev/gpu_mfma.sh) for the 512-frame vocoder, the 64-slot talker step and the 64-slot
# code-predictor frame, tagged rNN
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
TAG=${1:-r02d}
bash tools/dev/gpu_mfma.sh ${TAG}_vocoder "python3 $R/tools/dev/voc_only.py 512" > /dev/null || exit 1
bash tools/dev/gpu_mfma.sh ${TAG}_talker_b64 "python3 $R/tools/dev/stage_only.py 0 64 266 5" > /dev/null || exit 1
bash tools/dev/gpu_mfma.sh ${TAG}_cp_b64 "python3 $R/tools/dev/stage_only.py 1 64 266 2" > /dev/null || exit 1
head -6 gpurun_out/mfma_${TAG}_vocoder.txt
