"""dev: timeline of the batched persistent talker step (persist_tkb.hip, Q3T_PERSIST_PROF=1, development library).
Per hand-off kind, averaged over layers 1..26: the producers' publish skew, the edge (median consumer data-ready minus
the LAST producer's publish) and the consumers' span from data-ready to their own publish.  Clock: s_memrealtime
(100 MHz).  Usage: python tools/dev/tkb_timeline.py [slots] [pos]"""
import os
import sys

import numpy as np

R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(R, "qwen3-tts-jetson_amd"), os.path.join(R, "tests")]
os.environ["Q3T_PERSIST_PROF"] = "1"
os.environ.setdefault("Q3T_DEV_LIB", "1")
import q3t  # noqa: E402
from q3t_testutil import synth_dir  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 64
POS = int(sys.argv[2]) if len(sys.argv) > 2 else 266
tts, _ = synth_dir("full")
eng = q3t.Engine(tts, None, device=0, max_slots=S, max_ctx=POS + 8)
assert eng.persist_kernels() & 32
ms = eng.time_stage(0, S, POS, 10)
T = eng.debug_read(5, 256 * 768 * 4 * 8).view(np.uint64)[: 256 * 768 * 4].reshape(256, 768, 4).astype(np.int64)
valid = T > 0
t0 = T[valid].min()
T = np.where(valid, (T - t0) * 1e-2, np.nan)   # microseconds
print(f"{S}-slot talker step at position {POS}: {ms * 1e3:.1f} us per replay; stamped span {np.nanmax(T) - np.nanmin(T):.1f} us")
NAMES = ["RN_A", "QKV", "ATT", "O", "RN_F", "GU", "DN", "HEAD"]
NEXT = {0: 1, 1: 2, 2: 3, 3: 4, 4: 5, 5: 6, 6: 0, 7: None}


def ph(l, k):
    return l * 8 + k


rows = {k: ([], [], [], []) for k in range(8)}
for l in range(1, 27):
    for k in range(7):
        x = ph(l, k)
        pub = T[:, x, 2]
        rdy = T[:, x, 1]
        if np.isnan(pub).all() or np.isnan(rdy).all():
            continue
        last = np.nanmax(pub)
        nk = NEXT[k]
        nl = l + 1 if nk == 0 else l
        y = ph(nl, nk)
        c = ~np.isnan(rdy) & ~np.isnan(T[:, y, 2])
        span = np.nanmedian(T[c, y, 2] - rdy[c]) if c.any() else np.nan
        c3 = c & ~np.isnan(T[:, y, 3])
        comp = np.nanmedian(T[c3, y, 3] - rdy[c3]) if c3.any() else np.nan
        rows[k][0].append(last - np.nanmin(pub))
        rows[k][1].append(np.nanmedian(rdy) - last)
        rows[k][2].append(span)
        rows[k][3].append(comp)
print(f"{'hand-off':8s} {'pub skew':>9s} {'edge':>7s} {'consumer body':>14s} {'(ready->computed)':>18s}   [us, mean over layers 1..26]")
for k in range(7):
    s, e, b, c = (np.nanmean(v) if len(v) and not np.isnan(v).all() else np.nan for v in rows[k])
    print(f"{NAMES[k]:8s} {s:9.2f} {e:7.2f} {b:14.2f} {c:18.2f}")
lay = [np.nanmax(T[:, ph(l + 1, 6), 2]) - np.nanmax(T[:, ph(l, 6), 2]) for l in range(1, 26)]
print(f"layer (DN publish to DN publish): {np.nanmean(lay):.2f} us")
att = [np.nanmedian(T[:, ph(l, 2), 3] - T[:, ph(l, 1), 0]) for l in range(1, 27)]
print(f"attention unit (first unit: start -> computed, median): {np.nanmean(att):.2f} us")
head = np.nanmax(T[:, ph(28, 7), 2]) - np.nanmax(T[:, ph(28, 0), 2])
sel = np.nanmax(T[:, ph(28, 7), 3]) - np.nanmax(T[:, ph(28, 7), 2])
print(f"final norm -> head published {head:.2f} us; head published -> selected {sel:.2f} us")
