"""dev: mean device time of the captured talker-step (stage 0) and code-predictor frame (stage 1) graphs at a slot
count, for A/B runs of build / env variants (Q3T_DEV_LIB=1 selects the development library and its knobs)."""
import os
import sys

R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(R, "qwen3-tts-jetson_amd"), os.path.join(R, "tests")]
import q3t  # noqa: E402
from q3t_testutil import synth_dir  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
pos = int(sys.argv[2]) if len(sys.argv) > 2 else 266
tag = os.environ.get("TAG", "")
tts, _ = synth_dir("full")
eng = q3t.Engine(tts, None, max_slots=B, max_ctx=pos + 64)
t0 = min(eng.time_stage(0, B, pos, 20) for _ in range(3))
t1 = min(eng.time_stage(1, B, pos, 10) for _ in range(3))
print(f"{tag} B={B} pos={pos}: talker step {t0:.4f} ms, code-predictor frame {t1:.4f} ms", flush=True)
eng.close()
