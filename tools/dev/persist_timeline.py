"""dev: timeline of the persistent talker step (Q3T_PERSIST_PROF=1): per phase type, how long a workgroup waits for
its input, how late the input arrives after the last producer published it (edge latency), and how long the phase
body takes from input arrival to its own publish.  Clock: s_memrealtime (100 MHz)."""
import os
import sys

import numpy as np

R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(R, "qwen3-tts-jetson_amd"), os.path.join(R, "tests")]
os.environ["Q3T_PERSIST_PROF"] = "1"
os.environ["Q3T_DEV_LIB"] = "1"   # needs the development build: make -C qwen3-tts-jetson_amd/csrc DEV=1
import q3t  # noqa: E402
from q3t_testutil import synth_dir  # noqa: E402

pos = int(sys.argv[1]) if len(sys.argv) > 1 else 266
tts, _ = synth_dir("full")
eng = q3t.Engine(tts, None, device=0, max_slots=1, max_ctx=pos + 64)
assert eng.persist_status() == 0
ms = eng.time_stage(0, 1, pos, 20)
PH = 448   # persist.h PROF_PH
T = eng.debug_read(5, 256 * PH * 4 * 8).view(np.uint64).reshape(256, PH, 4).astype(np.int64)
t0 = T[:, 0, 3].min()
T = np.where(T > 0, T - t0, -1) * 10e-3   # -> microseconds
L = 28
print(f"talker step at pos {pos}: {ms * 1e3:.1f} us per replay (HIP events); launch span {T[:, 140, 2].max():.1f} us "
      f"(first wg start -> last head publish); wg start skew {T[:, 0, 3].max():.2f} us")
names = ["A qkv", "B attn", "C oproj", "D gateup", "E down"]
prev_pub = None
rows = []
for k in range(5):
    waits, edges, bodies = [], [], []
    for l in range(L):
        ph = 5 * l + k
        st, arr, pub = T[:, ph, 0], T[:, ph, 1], T[:, ph, 2]
        ok = (arr >= 0) & (pub >= 0)
        if l == 0 and k == 0:
            continue
        prod = 5 * l + k - 1
        last_pub = T[:, prod, 2][T[:, prod, 2] >= 0].max() if (T[:, prod, 2] >= 0).any() else np.nan
        waits.append(np.median(arr[ok] - st[ok]))
        edges.append(np.median(arr[ok]) - last_pub)
        bodies.append(np.median(pub[ok] - arr[ok]))
    rows.append((names[k], np.mean(waits), np.mean(edges), np.mean(bodies)))
print(f"{'phase':10s} {'wait (med)':>11s} {'arrive-lastpub':>15s} {'body (med)':>11s}   [us, mean over layers]")
for n, a, b, c in rows:
    print(f"{n:10s} {a:11.2f} {b:15.2f} {c:11.2f}")
per_layer = np.diff([T[:, 5 * l + 4, 2].max() for l in range(L)])
print(f"per-layer span (last E publish to last E publish): mean {per_layer.mean():.2f} us, min {per_layer.min():.2f}, max {per_layer.max():.2f}")
# publish skew within a phase: last - median publish
skew = [np.max(T[:, 5 * l + k, 2]) - np.median(T[:, 5 * l + k, 2][T[:, 5 * l + k, 2] >= 0]) for l in range(L) for k in (0, 2, 3, 4)]
print(f"producer publish skew (last - median) over A/C/D/E: mean {np.mean(skew):.2f} us, max {np.max(skew):.2f}")
for k, n in ((0, "A"), (3, "D")):
    pre = [np.median(T[:, 5 * l + k, 3] - T[:, 5 * l + k, 1]) for l in range(1, L)]
    post = [np.median(T[:, 5 * l + k, 2] - T[:, 5 * l + k, 3]) for l in range(1, L)]
    print(f"{n} body split: arrive -> after RMS {np.mean(pre):.2f} us, -> published {np.mean(post):.2f} us")
pre, post = [], []
for l in range(L):
    ph = 5 * l + 1
    ok = (T[:, ph, 3] >= 0) & (T[:, ph, 1] >= 0) & (T[:, ph, 2] >= 0)
    if ok.any():
        pre.append(np.median(T[ok, ph, 3] - T[ok, ph, 1]))
        post.append(np.median(T[ok, ph, 2] - T[ok, ph, 3]))
print(f"B body split: arrive -> q/k normed + RoPE {np.mean(pre):.2f} us, -> published {np.mean(post):.2f} us")
eng.close()
