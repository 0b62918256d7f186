"""dev: timeline of the batched persistent code-predictor frame (persist_cpb.hip, Q3T_PERSIST_PROF=1, development
library).  Per hand-off kind, averaged over passes 1..15 and layers: the producers' publish skew, the edge (median
consumer data-ready minus the LAST producer's publish) and the consumers' span from data-ready to their own publish.
Clock: s_memrealtime (100 MHz).  Usage: python tools/dev/cpb_timeline.py [slots]"""
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
tts, _ = synth_dir("full")
eng = q3t.Engine(tts, None, device=0, max_slots=S, max_ctx=96)
assert eng.persist_kernels() & 16
ms = eng.time_stage(1, S, 0, 10)
T = eng.debug_read(5, 256 * 768 * 4 * 8).view(np.uint64)[: 256 * 768 * 4].reshape(256, 768, 4).astype(np.int64)
valid = T > 0
t0 = T[valid].min()
T = np.where(valid, (T - t0) * 1e-2, np.nan)   # microseconds
print(f"{S}-slot code-predictor frame: {ms * 1e3:.1f} us per replay; stamped span {np.nanmax(T) - np.nanmin(T):.1f} us")
NAMES = ["RN_A", "QKV", "ATT", "O", "RN_F", "GU", "DN", "HEAD"]
# producer kind -> the kind its consumers publish
NEXT = {0: 1, 1: 2, 2: 3, 3: 4, 4: 5, 5: 6, 6: 0, 7: None}


def ph(p, l, k):
    return p * 48 + l * 8 + k


rows = {k: ([], [], [], []) for k in range(8)}
for p in range(1, 16):
    for l in range(6):
        for k in range(8):
            x = ph(p, l, k)
            pub = T[:, x, 2]
            rdy = T[:, x, 1]
            if np.isnan(pub).all() or np.isnan(rdy).all():
                continue
            last = np.nanmax(pub)
            skew = last - np.nanmin(pub)
            edge = np.nanmedian(rdy) - last
            nk = NEXT[k]
            span = np.nan
            comp = np.nan
            if nk is not None:
                nl = l + 1 if nk == 0 else l
                if nk == 0 and l == 4:
                    nl = 5
                y = ph(p, nl, nk)
                c = ~np.isnan(rdy) & ~np.isnan(T[:, y, 2])
                if c.any():
                    span = np.nanmedian(T[c, y, 2] - rdy[c])
                    c3 = c & ~np.isnan(T[:, y, 3])
                    if c3.any():
                        comp = np.nanmedian(T[c3, y, 3] - rdy[c3])
            rows[k][0].append(skew)
            rows[k][1].append(edge)
            rows[k][2].append(span)
            rows[k][3].append(comp)
print(f"{'hand-off':8s} {'pub skew':>9s} {'edge':>7s} {'consumer body':>14s} {'(ready->computed)':>18s}   [us, mean over passes 1..15]")
for k in range(8):
    s, e, b, c = (np.nanmean(v) if len(v) and not np.isnan(v).all() else np.nan for v in rows[k])
    print(f"{NAMES[k]:8s} {s:9.2f} {e:7.2f} {b:14.2f} {c:18.2f}")
# one pass end to end
for p in (1, 8):
    a = np.nanmin(T[:, ph(p, 0, 0):ph(p + 1, 0, 0), :]) if p < 15 else np.nan
    b = np.nanmin(T[:, ph(p + 1, 0, 0):ph(p + 2, 0, 0), :]) if p < 14 else np.nan
    print(f"pass {p}: {b - a:.1f} us")
head = [np.nanmax(T[:, ph(p, 5, 7), 2]) - np.nanmax(T[:, ph(p, 5, 0), 2]) for p in range(1, 16)]
sel = [np.nanmax(T[:, ph(p, 5, 7), 3]) - np.nanmax(T[:, ph(p, 5, 7), 2]) for p in range(1, 16)]
print(f"final norm -> head published {np.nanmean(head):.2f} us; head published -> selected {np.nanmean(sel):.2f} us")
# one layer in detail: per kind, percentiles of data-ready and publish over the workgroups that stamped them, relative
# to the previous layer's last DN publish, with the workgroup ranges of the slowest publishers
if len(sys.argv) > 2:
    p, l = 8, 2
    base = np.nanmax(T[:, ph(p, l - 1, 6), 2])
    for k in range(8):
        x = ph(p, l if k else l, k)
        for lab, col in (("ready", 1), ("computed", 3), ("publish", 2)):
            v = T[:, x, col] - base
            ok = ~np.isnan(v)
            if not ok.any():
                continue
            q = np.percentile(v[ok], [0, 10, 50, 90, 100])
            slow = np.argsort(np.where(ok, v, -1e9))[-6:][::-1]
            print(f"{NAMES[k]:5s} {lab:8s} n={ok.sum():3d}  min {q[0]:6.2f} p10 {q[1]:6.2f} p50 {q[2]:6.2f} p90 {q[3]:6.2f} max {q[4]:6.2f}  slowest wg {list(slow)}")
# attention detail (variant build with -DCPB_ATT_STAMPS): wave 0 of every slot workgroup, per layer l >= 1, deltas between
# the QKV data ready, the stamps inside attn_small_compute (0: before the 1st LDS fence, 1: after it, 2: before the 2nd,
# 3: after it) and computed
if os.environ.get("Q3T_DEV_LIB", "1") != "1":
    d = {k: [] for k in ("ready->s0", "s0->s1", "s1->s2", "s2->s3", "s3->computed")}
    for p in range(1, 16):
        for l in range(1, 5):
            rdy = T[128:, ph(p, l, 1), 1]
            st = [T[128:, p * 48 + 41 + l, k] for k in range(4)]
            cmp_ = T[128:, ph(p, l, 2), 3]
            seq = [rdy] + st + [cmp_]
            for (k, a, b_) in zip(d.keys(), seq[:-1], seq[1:]):
                d[k].append(np.nanmedian(b_ - a))
    print("attention (slot workgroups, median):", "  ".join(f"{k} {np.nanmean(v):.2f}" for k, v in d.items()), "us")
