"""dev: dump the raw persistent-kernel timeline (Q3T_PERSIST_PROF=1) of the talker step (stage 0) or the
code-predictor frame (stage 1) to gpurun_out/tl_<tag>.npy ([256 workgroups][PROF_PH phases][4] s_memrealtime
stamps: wait start, input arrived, output published, mid) for offline analysis (tools/dev/persist_tl_report.py).
usage: persist_dump.py STAGE TAG [POS [MAX_CTX]]"""
import os
import sys

import numpy as np

R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(R, "qwen3-tts-jetson_amd"), os.path.join(R, "tests")]
os.environ["Q3T_PERSIST_PROF"] = "1"
os.environ.setdefault("Q3T_DEV_LIB", "1")
import q3t  # noqa: E402
from q3t_testutil import synth_dir  # noqa: E402

stage, tag = int(sys.argv[1]), sys.argv[2]
pos = int(sys.argv[3]) if len(sys.argv) > 3 else 266
ctx = int(sys.argv[4]) if len(sys.argv) > 4 else pos + 64
tts, _ = synth_dir("full")
eng = q3t.Engine(tts, None, device=0, max_slots=1, max_ctx=ctx)
assert eng.persist_status() == 0
ms = eng.time_stage(stage, 1, pos, 20)
PH = 448
T = eng.debug_read(5, 512 * PH * 4 * 8).view(np.uint64).reshape(512, PH, 4)
os.makedirs(os.path.join(R, "gpurun_out"), exist_ok=True)
np.save(os.path.join(R, "gpurun_out", f"tl_{tag}.npy"), T)
print(f"{tag}: stage {stage} pos {pos}: {ms:.4f} ms per replay (timeline build)")
eng.close()
