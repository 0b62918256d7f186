"""dev: one small generate() on the tiny config (profiler bring-up)."""
import os
import sys

import numpy as np

R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(R, "qwen3-tts-jetson_amd"), os.path.join(R, "tests")]
import q3t  # noqa: E402
from q3t_testutil import prompt, synth_dir  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "tiny"
F = int(sys.argv[2]) if len(sys.argv) > 2 else 8
CTX = int(sys.argv[3]) if len(sys.argv) > 3 else 96
tts, tok = synth_dir(cfg)
eng = q3t.Engine(tts, None, max_slots=1, max_ctx=CTX)
print("created", flush=True)
codes = eng.generate([prompt(cfg)], speakers=[np.zeros(eng.cfg["hidden"], np.float32)], max_len=F, temperature=0.9,
                     force_frames=F)
print("generated", codes[0].shape, flush=True)
eng.close()
