"""dev: dump the per-op batched talker's outputs (k_attn_seq, Q3T_PERSIST_TKB=0) over a run of positions crossing
several chunk boundaries, to compare two library variants bit for bit.  Usage: attn_ab.py OUT.npz"""
import os
import sys

import numpy as np

R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(R, "qwen3-tts-jetson_amd"), os.path.join(R, "tests")]
os.environ["Q3T_PERSIST_TKB"] = "0"
import q3t  # noqa: E402
from q3t_testutil import synth_dir  # noqa: E402

tts, _ = synth_dir("full")
eng = q3t.Engine(tts, None, device=0, max_slots=32, max_ctx=300)
H = eng.cfg["hidden"]
rng = np.random.default_rng(5)
hs, ls = [], []
for step in range(0, 270, 7):
    pos = (step + np.arange(32) % 13).astype(np.int32)
    h, l = eng.talker_forward((rng.standard_normal((32, H)) * 0.5).astype(np.float32), pos)
    hs.append(h)
    ls.append(l)
np.savez(sys.argv[1], h=np.array(hs), l=np.array(ls))
print("saved", len(hs), "steps")
