"""dev: offline report of the role-specialised code-predictor frame's timeline (persist_cp.hip; raw dump of
tools/dev/persist_dump.py 1 TAG).  Per phase: edge = consumer arrival (median / max) after the last producer published,
body = publish - arrival (median / max), step = last publish of the phase - last publish of its input phase."""
import sys

import numpy as np

T = np.load(sys.argv[1]).astype(np.int64)
t0 = T[T > 0].min()
T = np.where(T > 0, T - t0, -1) * 10e-3   # us
ROLES = {"QKV": range(0, 64), "ATT": range(64, 72), "O": range(72, 104), "GU": range(104, 200), "DN": range(200, 256)}
PPH, NL = 26, 5
role_of_k = {0: "QKV", 1: "ATT", 2: "O", 3: "GU", 4: "DN"}


def stamps(ph, role, k):
    w = np.array(list(ROLES[role]))
    v = T[w, ph, k]
    return v[v >= 0]


rows = {}
seq = []   # (label, ph, role) in chain order
for ps in range(16):
    for l in range(NL):
        for k in range(5):
            if ps >= 1 and l == 0 and k == 0:
                continue   # table
            if ps == 0 and l == NL - 1 and k >= 2:
                continue   # skipped
            seq.append((f"{'ABCDE'[k]}", ps * PPH + 5 * l + k, role_of_k[k]))
    if ps >= 1:
        seq.append(("head", ps * PPH + 25, "QKV"))
        seq.append(("sel", ps * PPH + 25, "ATT"))
prev_last = None
for lab, ph, role in seq:
    arr, pub = stamps(ph, role, 1), stamps(ph, role, 2)
    if len(pub) == 0:
        continue
    last = pub.max()
    if prev_last is not None and len(arr):
        r = rows.setdefault(lab, [])
        r.append((np.median(arr) - prev_last, arr.max() - prev_last, np.median(pub) - np.median(arr), pub.max() - prev_last - (arr.max() - prev_last), last - prev_last))
    elif prev_last is not None:   # table-fed attention: no arrival stamp
        rows.setdefault(lab + "(tab)", []).append((np.nan, np.nan, np.nan, np.nan, last - prev_last))
    prev_last = last
print(f"{'phase':8s} {'edge_med':>8s} {'edge_max':>8s} {'body_med':>8s} {'tail':>8s} {'step':>8s}  n   (us)")
tot = 0
for lab, r in rows.items():
    a = np.array(r)
    m = np.nanmean(a, axis=0)
    tot += np.nansum(a[:, 4])
    print(f"{lab:8s} " + " ".join(f"{v:8.2f}" for v in m) + f"  {len(a)}")
ends = [stamps(ps * PPH + 25, "ATT", 2).max() for ps in range(1, 16)]
print(f"per-pass span (selection to selection) {np.mean(np.diff(ends)):.2f} us; total steps {tot:.1f} us; last selection {ends[-1]:.1f} us")
# selection split (ATT workgroups: [1] logits arrived, [3] token selected, [2] committed / published)
a, b, c = [], [], []
for ps in range(1, 16):
    h = ps * PPH + 25
    for w in ROLES["ATT"]:
        if T[w, h, 1] >= 0 and T[w, h, 3] >= 0 and T[w, h, 2] >= 0:
            a.append(T[w, h, 3] - T[w, h, 1]); b.append(T[w, h, 2] - T[w, h, 3])
if a:
    print(f"selection: select_token_pre {np.median(a):.2f} us, commit + publish {np.median(b):.2f} us (median over passes x 8)")
# selection stage stamps of the last pass (development builds: select.h SEL_STAMP -> phase slots 440..442)
st = T[64:72, 440:443].reshape(8, -1)
if (st[:, 1:9] >= 0).all():
    names = ["minmax", "hist", "bin", "cand", "rank", "exp", "scan", "pick"]
    rel = np.median(st[:, 1:9] - st[:, 1:2], axis=0)
    print("selection stages (us after minmax): " + ", ".join(f"{n} {v:.2f}" for n, v in zip(names[1:], rel[1:])))
