"""dev: repeatability of the GPU speaker mel / embedding against the oracle (fresh engines and repeated calls)"""
import os
import sys
import numpy as np
R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(R, "qwen3-tts-jetson_amd"), os.path.join(R, "tests")]
import q3t  # noqa: E402
from oracle_py import Oracle  # noqa: E402
from q3t_testutil import synth_dir  # noqa: E402
from test_speaker import voice_like  # noqa: E402
tts, tok = synth_dir("full")
o = Oracle(tts, tok)
x = voice_like(0.25)
r = o.mel(x)
for rep in range(4):
    eng = q3t.Engine(tts, None, device=0, max_slots=1, max_ctx=256)
    for it in range(10):
        g = eng.speaker_mel(x)
        r2 = o.mel(x)
        d, d2 = np.abs(g - r).max(), np.abs(r2 - r).max()
        if d > 1e-3 or d2 > 0:
            print(f"engine {rep} call {it}: gpu diff {d:.3g} (g min {g.min():.3f} max {g.max():.3f}); oracle diff {d2:.3g} (min {r2.min():.3f})", flush=True)
    e1 = eng.encode_speaker(voice_like(3.0))
    e2 = eng.encode_speaker(voice_like(3.0))
    print(f"engine {rep}: embed repeat diff {np.abs(e1 - e2).max():.3g}", flush=True)
    eng.close()
print("done")
