"""dev: which earlier activity in a process changes a later context's continuous batching?  Recreates
tests/test_gpu_mfma.py's full-model fixture (a 64-slot context under q3t_set_mfma_min_batch(1) with the tokenizer, a
2-slot one under (0)), runs the calls named in argv[1] (comma-separated: tf, cp, pt, g8, g64, none), closes both, then
runs the 24-slot queue with 24 and 3 slots in flight and counts the utterances whose codes differ."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "qwen3-tts-jetson_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import q3t  # noqa: E402
from q3t_testutil import prompt, synth_dir  # noqa: E402

calls = sys.argv[1].split(",")
tts, tok = synth_dir("full")
q3t.set_mfma_min_batch(1)
eng = q3t.Engine(tts, tok, device=0, max_slots=64, max_ctx=96)
q3t.set_mfma_min_batch(0)
vec = q3t.Engine(tts, None, device=0, max_slots=2, max_ctx=96)
q3t.set_mfma_min_batch(4)
H = eng.cfg["hidden"]
rng = np.random.default_rng(3)
base = prompt("full")
if "tf" in calls:
    for pos in range(4):
        e = (rng.standard_normal(H) * 0.5).astype(np.float32)
        eng.talker_forward(e[None], [pos])
        vec.talker_forward(e[None], [pos])
if "cp" in calls:
    hid = rng.standard_normal((5, H)).astype(np.float32)
    eng.codepred_frame(hid, np.array([1, 77, 2047, 300, 5], np.int32), temperature=0.0, want_logits=True)
if "pt" in calls:
    eng.project_text(base)
for n in (8, 64):
    if f"g{n}" in calls:
        ps = [base[:4] + [(t + 13 * i) % 900 + 20 for t in base[4:]] for i in range(n)]
        eng.generate(ps, speakers=[np.zeros(H, np.float32)] * n, max_len=8, temperature=0.0, force_frames=8)
vec.close()
eng.close()
slots, n_utt, nf = 24, 40, 48
q = q3t.Engine(tts, None, device=0, max_slots=slots, max_ctx=nf + 40)
rng = np.random.default_rng(slots)
prompts = []
for i in range(n_utt):
    k = int(rng.integers(5, 13))
    tail = [(t + 13 * i) % 900 + 20 for t in base[4:]]
    prompts.append(base[:4] + tail[:k - 4])
kw = dict(speakers=[np.zeros(H, np.float32)] * n_utt, max_len=nf, temperature=0.9, top_k=50, seed=123)
r24 = q.generate_queue(prompts, max_active=24, **kw)
r3 = q.generate_queue(prompts, max_active=3, **kw)
diff = [u for u in range(n_utt) if not np.array_equal(r24[u], r3[u])]
print(f"calls {sys.argv[1]}: {len(diff)} utterances differ", flush=True)
q.close()
