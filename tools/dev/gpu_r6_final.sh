#!/bin/bash
# dev (round 6): end-of-round check of the code that ships: GPU tests + smoke + bench (gpu_final.sh), then the MFMA /
# FETCH / WRITE table of one 512-frame FULL vocoder decode (profiles/rNN_pmc_mfma_vocoder.txt)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
bash tools/dev/gpu_final.sh || exit 1
bash tools/dev/gpu.sh mfma r06y_vocoder "python3 $R/tools/dev/voc_only.py 512" > gpurun_out/r06y_voc_mfma.log 2>&1 || { tail -20 gpurun_out/r06y_voc_mfma.log; exit 1; }
head -30 gpurun_out/mfma_r06y_vocoder.txt
