"""dev: batched code-predictor frame, persistent (persist_cpb.hip) vs the launch-per-op graph, per slot count
(time_stage replays of the frame graph, HIP events)."""
import os
import sys

R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(R, "qwen3-tts-jetson_amd"), os.path.join(R, "tests")]
import q3t  # noqa: E402
from q3t_testutil import synth_dir  # noqa: E402

tts, _ = synth_dir("full")
engs = {}
for cpb in ("1", "0"):
    os.environ["Q3T_PERSIST_CPB"] = cpb
    engs[cpb] = q3t.Engine(tts, None, device=0, max_slots=64, max_ctx=96)
print("slots  persistent_ms  per_op_ms")
for S in [int(a) for a in (sys.argv[1:] or ["4", "8", "16", "24", "32", "33", "48", "64"])]:
    t = {k: min(e.time_stage(1, S, 0, 10) for _ in range(3)) for k, e in engs.items()}
    print(f"{S:5d}  {t['1']:13.3f}  {t['0']:9.3f}", flush=True)
assert engs["1"].persist_status() == 0
