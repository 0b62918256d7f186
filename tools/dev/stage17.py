"""dev: code-predictor frame replay time of the 1.7B layout (synthetic full17) with the current kernels and with
Q3T_CP_ROLES=0 (the all-role k_persist<2,16>) -- run each in its own process: python3 stage17.py [roles 0|1]"""
import os
import sys

R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(R, "qwen3-tts-jetson_amd"), os.path.join(R, "tests")]
if len(sys.argv) > 1:
    os.environ["Q3T_CP_ROLES"] = sys.argv[1]
import q3t  # noqa: E402
from q3t_testutil import synth_dir  # noqa: E402

tts, _ = synth_dir("full17")
eng = q3t.Engine(tts, None, max_slots=1, max_ctx=330)
print(f"full17 CP frame (kernels {eng.persist_kernels()}): {eng.time_stage(1, 1, 266, 50):.4f} ms; "
      f"talker step: {eng.time_stage(0, 1, 266, 20):.4f} ms")
eng.close()
