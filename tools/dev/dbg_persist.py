"""dev: compare the persistent single-slot talker step with the launch-per-phase graph (K/V caches, and with
Q3T_TALKER_LAYERS=1 Q3T_PERSIST_DBG=1 the layer-0 QKV rows and attention output)."""
import os, sys
import numpy as np
R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(R, "qwen3-tts-jetson_amd"), os.path.join(R, "tests")]
import q3t
from q3t_testutil import synth_dir
tts, tok = synth_dir("full")
def mk(flag):
    os.environ["Q3T_PERSIST"] = flag
    return q3t.Engine(tts, None, device=0, max_slots=1, max_ctx=320)
ep, eg = mk("1"), mk("0")
print("persist", ep.persist_status(), eg.persist_status())
H = 1024; L = int(os.environ.get("Q3T_TALKER_LAYERS", "28")); CTX = 320
rng = np.random.default_rng(11)
nb = L * 8 * CTX * 128 * 2
for pos in range(4):
    e = (rng.standard_normal(H) * 0.5).astype(np.float32)
    hp, lp = ep.talker_forward(e[None], [pos]); hg, lg = eg.talker_forward(e[None], [pos])
    print("pos", pos, "hidden maxdiff", np.abs(hp - hg).max(), "logits", np.abs(lp - lg).max())
    for which in (0, 1):
        a = ep.debug_read(which, nb).view(np.float16).reshape(L, 8, CTX, 128).astype(np.float32)
        b = eg.debug_read(which, nb).view(np.float16).reshape(L, 8, CTX, 128).astype(np.float32)
        for p2 in range(pos + 1):
            d = np.abs(a[:, :, p2] - b[:, :, p2]).max(axis=(1, 2))
            first = int(np.argmax(d > 0)) if (d > 0).any() else -1
            print(f"  {'KV'[which]}[{p2}] first differing layer {first}, max {d.max():.3g}")
    if os.environ.get("Q3T_PERSIST_DBG") and L == 1:
        qa = ep.debug_read(2, 4096 * 4).view(np.float32); qb = eg.debug_read(2, 4096 * 4).view(np.float32)
        print("  layer-0 qkv maxdiff", np.abs(qa - qb).max())
        aa = ep.debug_read(3, 2048 * 2).view(np.float16).astype(np.float32)
        ab = eg.debug_read(3, 2048 * 2).view(np.float16).astype(np.float32)
        dd = np.abs(aa - ab).reshape(16, 128).max(axis=1)
        print("  layer-0 attention maxdiff per head", np.round(dd, 5))
