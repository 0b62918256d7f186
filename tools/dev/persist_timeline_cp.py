"""dev: timeline of the persistent code-predictor frame (Q3T_PERSIST_PROF=1): per phase type, the median wait, the
edge (input arrival after the last producer published) and the body, over the 16 passes; plus the head + selection
phases.  Clock: s_memrealtime (100 MHz)."""
import os
import sys

import numpy as np

R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(R, "qwen3-tts-jetson_amd"), os.path.join(R, "tests")]
os.environ["Q3T_PERSIST_PROF"] = "1"
os.environ.setdefault("Q3T_DEV_LIB", "1")   # needs the development build: make -C qwen3-tts-jetson_amd/csrc DEV=1
import q3t  # noqa: E402
from q3t_testutil import synth_dir  # noqa: E402

tts, _ = synth_dir("full")
eng = q3t.Engine(tts, None, device=0, max_slots=1, max_ctx=320)
assert eng.persist_status() == 0
ms = eng.time_stage(1, 1, 100, 20)
PH = 448
T = eng.debug_read(5, 256 * PH * 4 * 8).view(np.uint64).reshape(256, PH, 4).astype(np.int64)
t0 = T[:, 0, 3].min()
T = np.where(T > 0, T - t0, -1) * 10e-3   # -> microseconds
NL, PPH = 5, 26
last = T[:, 15 * PPH + 25, 2].max()
print(f"code-predictor frame: {ms * 1e3:.1f} us per replay (HIP events); launch span {last:.1f} us")
names = ["A qkv", "B attn", "C oproj", "D gateup", "E down"]
print(f"{'phase':10s} {'wait (med)':>11s} {'arrive-lastpub':>15s} {'body (med)':>11s}   [us, mean over passes x layers]")
for k in range(5):
    waits, edges, bodies = [], [], []
    for ps in range(16):
        for l in range(NL):
            if l == 0 and k == 0:
                continue
            ph = ps * PPH + 5 * l + k
            prod = ph - 1
            if k == 2 and not (T[:, prod, 2] >= 0).any():
                prod = ph - 2   # fused code-predictor attention: C waits on A's QKV rows (no phase B)
            st, arr, pub = T[:, ph, 0], T[:, ph, 1], T[:, ph, 2]
            ok = (arr >= 0) & (pub >= 0)
            if not ok.any() or not (T[:, prod, 2] >= 0).any():
                continue
            waits.append(np.median(arr[ok] - st[ok]))
            edges.append(np.median(arr[ok]) - T[:, prod, 2][T[:, prod, 2] >= 0].max())
            bodies.append(np.median(pub[ok] - arr[ok]))
    print(f"{names[k]:10s} {np.mean(waits):11.2f} {np.mean(edges):15.2f} {np.mean(bodies):11.2f}")
pre, post = [], []
for ps in range(16):
    for l in range(NL):
        ph = ps * PPH + 5 * l + 1
        ok = (T[:, ph, 3] >= 0) & (T[:, ph, 1] >= 0) & (T[:, ph, 2] >= 0)
        if ok.any():
            pre.append(np.median(T[ok, ph, 3] - T[ok, ph, 1]))
            post.append(np.median(T[ok, ph, 2] - T[ok, ph, 3]))
print(f"B body split: arrive -> q/k normed + RoPE {np.mean(pre):.2f} us, -> published {np.mean(post):.2f} us")
hd = []
for ps in range(1, 16):
    h = ps * PPH + 25
    e_last = T[:, ps * PPH + 24, 2].max()
    nxt = (ps + 1) * PPH + 0 if ps < 15 else None
    arr = np.median(T[:, h, 1][T[:, h, 1] >= 0])
    pub = T[:, h, 2][T[:, h, 2] >= 0].max()
    a_next = np.median(T[:, nxt, 2][T[:, nxt, 2] >= 0]) if nxt is not None else np.nan
    hd.append((arr - e_last, pub - arr, a_next - pub))
hd = np.array(hd)
print(f"head: edge {np.nanmean(hd[:, 0]):.2f}, body to last logits {np.nanmean(hd[:, 1]):.2f}, "
      f"last logits -> next pass A published (median) {np.nanmean(hd[:, 2]):.2f} us")
sel = []
for ps in range(1, 16):
    h = ps * PPH + 25
    st = T[:, h, 3][(T[:, h, 3] >= 0) & (np.arange(256) != 0)]
    if len(st) and T[0, h, 3] >= 0:
        sel.append(T[0, h, 3] - st.max())
if sel:
    print(f"selection (last workgroup, select_token): {np.mean(sel):.2f} us per pass")
per_pass = np.diff([T[:, ps * PPH + 24, 2].max() for ps in range(16)])
print(f"per-pass span: mean {per_pass.mean():.2f} us (min {per_pass.min():.2f}, max {per_pass.max():.2f})")
eng.close()
