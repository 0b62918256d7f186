"""dev: FULL-vocoder PCM of fixed random codes (512 frames single, and a 3-utterance batch) into an .npz, for bit-exact
A/B between two builds (Q3T_DEV_LIB=<name> loads libq3t_<name>.so).  Usage: python tools/dev/voc_dump.py OUT.npz
python tools/dev/voc_dump.py --cmp A.npz B.npz"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if sys.argv[1] == "--cmp":
    a, b = np.load(sys.argv[2]), np.load(sys.argv[3])
    bad = [k for k in a.files if not np.array_equal(a[k], b[k])]
    for k in a.files:
        print(k, a[k].shape, "max|d| %.3e" % float(np.abs(a[k] - b[k]).max()))
    sys.exit(1 if bad else 0)
sys.path.insert(0, os.path.join(REPO, "qwen3-tts-jetson_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import q3t  # noqa: E402
from q3t_testutil import synth_dir  # noqa: E402

_, tok = synth_dir("full")
eng = q3t.Engine(None, tok, device=0)
cl = [np.random.default_rng(7 + u).integers(0, 2048, (F, 16)).astype(np.int32) for u, F in enumerate((512, 300, 280, 271))]
out = {"single": eng.vocoder(cl[0], 0)}
for i, x in enumerate(eng.vocoder_batch(cl[1:], 0)):
    out[f"batch{i}"] = x
np.savez(sys.argv[1], **out)
print("saved", sys.argv[1], {k: v.shape for k, v in out.items()})
eng.close()
