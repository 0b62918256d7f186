#!/bin/bash
# dev (round 4): the profile set committed under profiles/r04_*: FETCH passes of the talker step (1 and 64 slots), the
# kernel trace of a short B=1 bench split into phases, and MFMA / FETCH / WRITE tables of the vocoder and the 64-slot
# talker step and code-predictor frame.  Stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
bash tools/dev/gpu.sh fetch r04 1 64 || exit 1
bash tools/dev/gpu.sh phases r04 || exit 1
bash tools/dev/gpu.sh mfma r04voc "python3 $R/tools/dev/voc_only.py 512" || exit 1
bash tools/dev/gpu.sh mfma r04tk64 "python3 $R/tools/dev/stage_only.py 0 64 266 5" || exit 1
bash tools/dev/gpu.sh mfma r04cp64 "python3 $R/tools/dev/stage_only.py 1 64 266 5" || exit 1
