"""dev: voice-cloning generate under engine options (tests/test_speaker.py::test_gpu_speaker_embedding_drives_generation
probe): GPU vs oracle speaker embedding, repeated calls, per configuration."""
import os
import sys

import numpy as np

R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(R, "tests"))
sys.path.insert(0, os.path.join(R, "qwen3-tts-jetson_amd"))
from oracle_py import Oracle  # noqa: E402
from q3t_testutil import prompt, synth_dir  # noqa: E402
from test_speaker import voice_like  # noqa: E402

import q3t  # noqa: E402

tts, tok = synth_dir("full")
o = Oracle(tts, tok)
x = voice_like(2.0)
so = o.encode_speaker(x)
res = {}
for cfg in sys.argv[1:] or ["default"]:
    env = dict(kv.split("=") for kv in cfg.split(",") if "=" in kv)
    os.environ.update(env)
    eng = q3t.Engine(tts, None, device=0, max_slots=1, max_ctx=256)
    sg = eng.encode_speaker(x)
    g = lambda s: eng.generate([prompt("full")], speakers=[s] if s is not None else None, max_len=8, temperature=0.0,
                               force_frames=8)[0]
    a, b, c, n, n2 = g(sg), g(so), g(sg), g(None), g(None)
    print(f"{cfg}: spk rel {np.abs(sg - so).max() / np.abs(so).max():.2e}  a==b {(a == b).mean():.3f}  "
          f"a==a' {(a == c).mean():.3f}  none==none' {(n == n2).mean():.3f}  a==none {(a == n).mean():.3f}", flush=True)
    print("   a[0]", a[0, :8], " b[0]", b[0, :8], " n[0]", n[0, :8], flush=True)
    res[cfg] = (a, b, n)
    eng.close()
    for k in env:
        del os.environ[k]
ks = list(res)
for k in ks[1:]:
    print(f"{ks[0]} vs {k}: a {(res[ks[0]][0] == res[k][0]).mean():.3f} b {(res[ks[0]][1] == res[k][1]).mean():.3f} "
          f"none {(res[ks[0]][2] == res[k][2]).mean():.3f}")
