"""dev: offline report of the role-specialised talker step's timeline (persist_tk.hip; raw dump of
tools/dev/persist_dump.py 0 TAG POS CTX).  usage: persist_tl_tk.py FILE.npy NSPLIT [PAIR]"""
import sys

import numpy as np

T = np.load(sys.argv[1]).astype(np.int64)
S = int(sys.argv[2])
t0 = T[T > 0].min()
T = np.where(T > 0, T - t0, -1) * 10e-3
AW = 248
# role layout of persist_tk.hip (Q3T_TK_PAIR = 1: down, O, gate/up, QKV; a third argument 0 = the other layout)
PAIR = int(sys.argv[3]) if len(sys.argv) > 3 else 1
OR, GR, DR = (range(56, 88), range(88, 184), range(0, 56)) if PAIR else (range(0, 32), range(32, 128), range(128, 184))
ROLES = {"O": OR, "GU": GR, "DN": DR, "QKV": range(184, 248),
         "ATT": range(AW, AW + 8 * S), "SEL": range(AW + 8 * S, AW + 8 * S + 1)}
NL = 28
role_of_k = {0: "QKV", 1: "ATT", 2: "O", 3: "GU", 4: "DN"}


def st(ph, role, k):
    w = np.array(list(ROLES[role]))
    v = T[w, ph, k]
    return v[v >= 0]


seq = []
for l in range(NL):
    for k in range(5):
        seq.append(("ABCDE"[k], 5 * l + k, role_of_k[k]))
seq.append(("head", 140, "QKV"))
seq.append(("sel", 140, "SEL"))
rows = {}
prev = None
for lab, ph, role in seq:
    arr, pub = st(ph, role, 1), st(ph, role, 2)
    if len(pub) == 0:
        continue
    last = pub.max()
    if prev is not None and len(arr):
        rows.setdefault(lab, []).append((np.median(arr) - prev, arr.max() - prev, np.median(pub - arr) if len(pub) == len(arr) else np.nan,
                                         last - prev))
    elif prev is not None:
        rows.setdefault(lab, []).append((np.nan, np.nan, np.nan, last - prev))
    prev = last
print(f"{'phase':6s} {'edge_med':>8s} {'edge_max':>8s} {'body_med':>8s} {'step':>8s}  (us)")
for lab, r in rows.items():
    m = np.nanmean(np.array(r), axis=0)
    print(f"{lab:6s} " + " ".join(f"{v:8.2f}" for v in m) + f"  n={len(r)}")
# attention split spread and the O workgroups' combine
for l in [5, 15]:
    ph = 5 * l + 1
    a = T[AW:AW + 8 * S, ph]
    o = T[list(OR), ph + 1]
    print(f"layer {l} B: splits arrive {np.median(a[:,1]):.2f} pub med {np.median(a[:,2]):.2f} max {a[:,2].max():.2f}; "
          f"QKV last pub {T[184:248, 5*l, 2].max():.2f}; O arrive med {np.median(o[:,1]):.2f} combined {np.median(o[:,3]):.2f} pub {np.median(o[:,2]):.2f}")
print(f"span {T[:, 140, 2].max():.1f} us")
# attention body split (stamps 200 + l: 0 normed, 1 scores + max, 2 P.V reduced)
segs = {"arrive->norm": [], "norm->scores": [], "scores->pv": [], "pv->pub": [], "O arrive->combined": [], "O combined->pub": [],
        "O arrive->weights": [], "O weights->w0 combine": [], "O w0 combine->barrier": []}
for l in range(1, NL):
    ph = 5 * l + 1
    for w in ROLES["ATT"]:
        a, n0, n1, n2, pb = T[w, ph, 1], T[w, 200 + l, 0], T[w, 200 + l, 1], T[w, 200 + l, 2], T[w, ph, 2]
        if min(a, n0, n1, n2, pb) < 0:
            continue
        segs["arrive->norm"].append(n0 - a)
        segs["norm->scores"].append(n1 - n0)
        segs["scores->pv"].append(n2 - n1)
        segs["pv->pub"].append(pb - n2)
    for w in ROLES["O"]:
        a, c, pb = T[w, ph + 1, 1], T[w, ph + 1, 3], T[w, ph + 1, 2]
        if min(a, c, pb) >= 0:
            segs["O arrive->combined"].append(c - a)
            segs["O combined->pub"].append(pb - c)
            b0, b1 = T[w, 200 + l, 0], T[w, 200 + l, 1]
            if min(b0, b1) >= 0:
                segs["O arrive->weights"].append(b0 - a)
                segs["O weights->w0 combine"].append(b1 - b0)
                segs["O w0 combine->barrier"].append(c - b1)
print("attention body: " + ", ".join(f"{k} {np.median(v):.2f}" for k, v in segs.items() if v))
