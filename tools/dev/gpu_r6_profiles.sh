#!/bin/bash
# dev (round 6): the profiles of the code that ships, one box: kernel traces of the 1-slot talker step and CP frame
# replays at KV position 266 (the bench's launch_ms / cp_frame_ms configuration), the B=1 bench kernel trace split into phases (the bench's talker
# step / CP frame launches), FETCH_SIZE passes over the 1- and 64-slot talker-step replays, kernel traces of the
# 64-slot talker step and CP frame (one persistent launch each), MFMA / FETCH / WRITE tables of those two.  Outputs
# under gpurun_out/ (tools/dev/gpu.sh names); stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
bash tools/dev/gpu.sh trace r06x_stage1_talker "python3 $R/tools/dev/stage_only.py 0 1 266 50" || exit 1
bash tools/dev/gpu.sh trace r06x_stage1_cp "python3 $R/tools/dev/stage_only.py 1 1 266 50" || exit 1
bash tools/dev/gpu.sh phases r06x || exit 1
bash tools/dev/gpu.sh fetch r06x 1 64 || exit 1
bash tools/dev/gpu.sh trace r06x_stage64_talker "python3 $R/tools/dev/stage_only.py 0 64 266 20" || exit 1
bash tools/dev/gpu.sh trace r06x_stage64_cp "python3 $R/tools/dev/stage_only.py 1 64 266 20" || exit 1
bash tools/dev/gpu.sh mfma r06x_talker_b64 "python3 $R/tools/dev/stage_only.py 0 64 266 5" || exit 1
bash tools/dev/gpu.sh mfma r06x_cp_b64 "python3 $R/tools/dev/stage_only.py 1 64 266 5" || exit 1
echo done
