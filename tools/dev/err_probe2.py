import os, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "tests")); sys.path.insert(0, os.path.join(REPO, "qwen3-tts-jetson_amd"))
import q3t
from oracle_py import Oracle
from q3t_testutil import synth_dir, prompt
for cfg in ["tiny1", "tiny"]:
    tts, tok = synth_dir(cfg)
    eng = q3t.Engine(tts, tok, device=0, max_slots=4, max_ctx=128)
    orc = Oracle(tts, tok)
    H = eng.cfg["hidden"]
    toks = prompt("tiny")
    a, b = eng.project_text(toks), orc.project_text(toks)
    print(cfg, "project_text maxabs %.3e max %.3f nexact %d/%d" % (np.abs(a-b).max(), np.abs(b).max(), (a==b).sum(), a.size))
    rng = np.random.default_rng(3)
    kv = orc.kv_new(128, 0)
    for pos in range(4):
        e = (rng.standard_normal(H) * 0.5).astype(np.float32)
        hg, lg = eng.talker_forward(e[None], [pos])
        ho, lo = orc.talker_step(kv, e, pos)
        d = np.abs(hg[0]-ho)
        print(cfg, "talker pos", pos, "hidden maxabs %.3e (max %.2f) n_exact %d/%d" % (d.max(), np.abs(ho).max(), (d==0).sum(), d.size),
              "logits maxabs %.3e" % np.abs(lg[0]-lo).max())
