"""Dev probe: magnitude of GPU-vs-oracle differences per stage (prints numbers, asserts nothing)."""
import os, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "tests")); sys.path.insert(0, os.path.join(REPO, "qwen3-tts-jetson_amd"))
import q3t
from oracle_py import Oracle
from q3t_testutil import synth_dir, prompt
for cfg in sys.argv[1:] or ["tiny", "full"]:
    tts, tok = synth_dir(cfg)
    eng = q3t.Engine(tts, tok, device=0, max_slots=4, max_ctx=128)
    orc = Oracle(tts, tok)
    H = eng.cfg["hidden"]
    rng = np.random.default_rng(3)
    kv = orc.kv_new(128, 0)
    for pos in range(12):
        e = (rng.standard_normal(H) * 0.5).astype(np.float32)
        hg, lg = eng.talker_forward(e[None], [pos])
        ho, lo = orc.talker_step(kv, e, pos)
        print(cfg, "talker pos", pos, "hidden maxabs %.3e (max %.2f)" % (np.abs(hg[0]-ho).max(), np.abs(ho).max()),
              "logits maxabs %.3e (max %.2f) top2gap %.3f" % (np.abs(lg[0]-lo).max(), np.abs(lo).max(), np.diff(np.sort(lo[:2048])[-2:])[0]))
    hid = rng.standard_normal((1, H)).astype(np.float32)
    codes, lg = eng.codepred_frame(hid, [137], temperature=0.0, want_logits=True)
    oc, ol = orc.cp_frame(hid[0], 137, temperature=0.0, want_logits=True)
    for s in range(15):
        print(cfg, "cp step", s, "logit maxabs %.3e max %.2f" % (np.abs(lg[0, s]-ol[s]).max(), np.abs(ol[s]).max()), codes[0, s], oc[s])
