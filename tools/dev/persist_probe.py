"""dev: where does the persistent talker step (k_persist<0>) first differ from the launch-per-op graph?  Truncated
talker stacks (Q3T_TALKER_LAYERS, development library): the first differing position and the K/V cache rows."""
import os
import sys

import numpy as np

R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(R, "qwen3-tts-jetson_amd"), os.path.join(R, "tests")]
os.environ["Q3T_DEV_LIB"] = "1"
import q3t  # noqa: E402
from q3t_testutil import synth_dir  # noqa: E402

tts, _ = synth_dir("full")
CTX = 160


def eng(persist, n):
    os.environ["Q3T_PERSIST"] = "1" if persist else "0"
    os.environ["Q3T_CP_FUSED_ATTN"] = "1" if persist else "0"
    os.environ["Q3T_TALKER_LAYERS"] = str(n)
    return q3t.Engine(tts, None, device=0, max_slots=1, max_ctx=CTX)


for n in [int(a) for a in sys.argv[1:]] or [1]:
    ep, eg = eng(True, n), eng(False, n)
    rng = np.random.default_rng(5)
    H = ep.cfg["hidden"]
    first = None
    diffs = []
    for pos in range(0, 72):
        e = (rng.standard_normal(H) * 0.5).astype(np.float32)
        hp, lp = ep.talker_forward(e[None], [pos])
        hg, lg = eg.talker_forward(e[None], [pos])
        d = np.abs(hp - hg).max()
        if d > 0:
            diffs.append(pos)
        if d > 0 and first is None:
            first = pos
            kb = n * 8 * CTX * 128 * 2
            kp = ep.debug_read(0, kb).view(np.uint16).reshape(n, 8, CTX, 128)
            kg = eg.debug_read(0, kb).view(np.uint16).reshape(n, 8, CTX, 128)
            vp = ep.debug_read(1, kb).view(np.uint16).reshape(n, 8, CTX, 128)
            vg = eg.debug_read(1, kb).view(np.uint16).reshape(n, 8, CTX, 128)
            bad_k = np.argwhere((kp[:, :, :pos + 1] != kg[:, :, :pos + 1]).any(-1))
            bad_v = np.argwhere((vp[:, :, :pos + 1] != vg[:, :, :pos + 1]).any(-1))
            print(f"layers {n}: first hidden difference at pos {pos} (max {d:.2e}); K rows differing (layer, kv, pos): "
                  f"{bad_k[:12].tolist()} ({len(bad_k)}); V rows: {bad_v[:12].tolist()} ({len(bad_v)})", flush=True)
    print(f"layers {n}: positions with a hidden difference: {diffs}", flush=True)
    ep.close()
    eg.close()
