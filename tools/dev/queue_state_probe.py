"""dev: does an engine created under another q3t_set_mfma_min_batch setting change a later context's continuous
batching?  argv[1]: the min batch during the first engine's life (0 = vector path only, 1 = matrix cores always)."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "qwen3-tts-jetson_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import q3t  # noqa: E402
from q3t_testutil import prompt, synth_dir  # noqa: E402

mb, slots_first, use_first = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
tts, _ = synth_dir("full")
q3t.set_mfma_min_batch(mb)
first = q3t.Engine(tts, None, device=0, max_slots=slots_first, max_ctx=96)
q3t.set_mfma_min_batch(4)
H = first.cfg["hidden"]
if use_first:
    rng = np.random.default_rng(1)
    first.talker_forward((rng.standard_normal((slots_first, H)) * 0.5).astype(np.float32), [0] * slots_first)
first.close()
slots, n_utt, nf = 24, 40, 48
eng = q3t.Engine(tts, None, device=0, max_slots=slots, max_ctx=nf + 40)
base = prompt("full")
rng = np.random.default_rng(slots)
prompts = []
for i in range(n_utt):
    k = int(rng.integers(5, 13))
    tail = [(t + 13 * i) % 900 + 20 for t in base[4:]]
    prompts.append(base[:4] + tail[:k - 4])
kw = dict(speakers=[np.zeros(H, np.float32)] * n_utt, max_len=nf, temperature=0.9, top_k=50, seed=123)
r24 = eng.generate_queue(prompts, max_active=24, **kw)
r3 = eng.generate_queue(prompts, max_active=3, **kw)
diff = [u for u in range(n_utt) if not np.array_equal(r24[u], r3[u])]
print(f"min_batch {mb} first engine {slots_first} slots used {use_first}: {len(diff)} utterances differ", flush=True)
eng.close()
