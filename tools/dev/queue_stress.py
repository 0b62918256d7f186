"""dev: determinism of continuous batching: the same queue (24 slots, 40 utterances) run several times with 24 and 3
slots in flight; every run must give the same codes."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "qwen3-tts-jetson_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import q3t  # noqa: E402
from q3t_testutil import prompt, synth_dir  # noqa: E402

slots, n_utt, nf = 24, 40, 48
tts, _ = synth_dir("full")
eng = q3t.Engine(tts, None, device=0, max_slots=slots, max_ctx=nf + 40)
H = eng.cfg["hidden"]
base = prompt("full")
rng = np.random.default_rng(slots)
prompts = []
for i in range(n_utt):
    k = int(rng.integers(5, 13))
    tail = [(t + 13 * i) % 900 + 20 for t in base[4:]]
    prompts.append(base[:4] + tail[:k - 4])
kw = dict(speakers=[np.zeros(H, np.float32)] * n_utt, max_len=nf, temperature=0.9, top_k=50, seed=123)
ref = None
bad = 0
for it in range(int(sys.argv[1]) if len(sys.argv) > 1 else 4):
    for a in (slots, 3):
        out = eng.generate_queue(prompts, max_active=a, **kw)
        if ref is None:
            ref = out
            continue
        diff = [u for u in range(n_utt) if not np.array_equal(out[u], ref[u])]
        if diff:
            bad += 1
            u = diff[0]
            fr = next((f for f in range(min(len(out[u]), len(ref[u]))) if not np.array_equal(out[u][f], ref[u][f])), -1)
            print(f"iter {it} max_active {a}: {len(diff)} utterances differ, first {u} at frame {fr}", flush=True)
print(f"queue stress: {bad} mismatching runs", flush=True)
eng.close()
