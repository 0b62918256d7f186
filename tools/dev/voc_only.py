"""dev: run the FULL vocoder on N random frames (for rocprofv3 kernel traces of the conv stack); with a third
argument U > 0 also U utterances of N frames through q3t_vocoder_decode_batch (per-utterance time)."""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "qwen3-tts-jetson_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import q3t  # noqa: E402
from q3t_testutil import synth_dir  # noqa: E402

F = int(sys.argv[1]) if len(sys.argv) > 1 else 512
mode = int(sys.argv[2]) if len(sys.argv) > 2 else 0
U = int(sys.argv[3]) if len(sys.argv) > 3 else 0
tts, tok = synth_dir("full")
eng = q3t.Engine(tts, tok, device=0, max_slots=1, max_ctx=64)
codes = np.random.default_rng(0).integers(0, 2048, (F, 16)).astype(np.int32)
for i in range(3):
    t = time.perf_counter()
    pcm = eng.vocoder(codes, mode)
    print(f"vocoder {F} frames mode {mode}: {(time.perf_counter() - t) * 1e3:.2f} ms, {len(pcm)} samples", flush=True)
if U > 0:
    cl = [np.random.default_rng(u).integers(0, 2048, (F, 16)).astype(np.int32) for u in range(U)]
    for bf in (4096, 8192):
        eng.vocoder_set_batch_frames(bf)
        for i in range(2):
            t = time.perf_counter()
            outs = eng.vocoder_batch(cl, mode)
            dt = time.perf_counter() - t
            print(f"vocoder batch {U} x {F} frames (batch_frames {bf}): {dt * 1e3:.1f} ms, "
                  f"{dt * 1e3 / U:.2f} ms per utterance", flush=True)
eng.close()
