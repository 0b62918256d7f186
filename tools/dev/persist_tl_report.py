"""dev: offline report of a raw persistent-kernel timeline (tools/dev/persist_dump.py output).
Per phase type: producer skew (last - median publish of the phase's input), edge (consumer arrival median / max after
the last producer published), body (publish - arrival, median over the phase's workgroups) and the critical-path
step (last publish of this phase - last publish of the previous one).  usage: persist_tl_report.py FILE.npy STAGE"""
import sys

import numpy as np

T = np.load(sys.argv[1]).astype(np.int64)
stage = int(sys.argv[2])
nsplit = int(sys.argv[3]) if len(sys.argv) > 3 else (5 if stage == 0 else 1)
t0 = T[:, 0, 3][T[:, 0, 3] > 0].min()
T = np.where(T > 0, T - t0, -1) * 10e-3   # microseconds (100 MHz clock)
W = np.arange(256)
att = W < 8 * nsplit
if stage == 0:
    NL, npass, PPH = 28, 1, 141
else:
    NL, npass, PPH = 5, 16, 26
names = ["A qkv", "B attn", "C oproj", "D gateup", "E down"]
rows = {k: [] for k in range(6)}
steps = []
prev_last = None
for ps in range(npass):
    for l in range(NL):
        for k in range(5):
            ph = ps * PPH + 5 * l + k
            cons = att if k == 1 else np.ones(256, bool)
            if k == 0:
                prod_ph = ph - 1 if l > 0 else None
                if l == 0 and ps > 0:
                    prod_ph = ps * PPH - 1   # previous pass head
            else:
                prod_ph = ph - 1
            pub = T[:, ph, 2]
            arr = T[:, ph, 1]
            okc = cons & (arr >= 0) & (pub >= 0)
            last_pub = pub[cons & (pub >= 0)].max() if (cons & (pub >= 0)).any() else np.nan
            if prod_ph is not None and okc.any():
                pm = att if (prod_ph % PPH) % 5 == 1 and (prod_ph % PPH) < 5 * NL else np.ones(256, bool)
                pp = T[:, prod_ph, 2][pm & (T[:, prod_ph, 2] >= 0)]
                if len(pp):
                    rows[k].append((pp.max() - np.median(pp), np.median(arr[okc]) - pp.max(), arr[okc].max() - pp.max(),
                                    np.median(pub[okc] - arr[okc]), np.max(pub[okc] - arr[okc]), last_pub - pp.max()))
    h = ps * PPH + 5 * NL
    if stage == 0 or ps > 0:
        pub, arr = T[:, h, 2], T[:, h, 1]
        ok = (arr >= 0) & (pub >= 0)
        pp = T[:, h - 1, 2][T[:, h - 1, 2] >= 0]
        if ok.any():
            rows[5].append((pp.max() - np.median(pp), np.median(arr[ok]) - pp.max(), arr[ok].max() - pp.max(),
                            np.median(pub[ok] - arr[ok]), np.max(pub[ok] - arr[ok]), pub[ok].max() - pp.max()))
print(f"{'phase':9s} {'prodskew':>8s} {'edge_med':>8s} {'edge_max':>8s} {'body_med':>8s} {'body_max':>8s} {'step':>7s}  (us, mean over layers/passes; n)")
tot = 0.0
for k in range(6):
    if not rows[k]:
        continue
    a = np.array(rows[k])
    nm = names[k] if k < 5 else "head"
    m = np.nanmean(a, axis=0)
    print(f"{nm:9s} " + " ".join(f"{v:8.2f}" for v in m[:5]) + f" {m[5]:7.2f}  n={len(a)}")
    tot += m[5] * (NL if k < 5 else 1)
if stage == 0:
    end = T[:, 140, 2].max()
    print(f"launch span to last head publish {end:.1f} us; layer step sum {tot:.1f}")
else:
    ends = [T[:, ps * PPH + 24, 2].max() for ps in range(16)]
    print(f"per-pass span mean {np.mean(np.diff(ends)):.2f} us; last layer-E publish {ends[-1]:.1f} us")
    # head -> next pass: selection + token hand-off + first phase of next pass
    d = []
    for ps in range(1, 15):
        h = ps * PPH + 25
        hl = T[:, h, 2].max()
        nb = (ps + 1) * PPH + 1   # next pass B (layer 0 from table)
        barr = T[att, nb, 1]
        bpub = T[att, nb, 2]
        d.append((hl - T[:, h - 1, 2].max(), np.median(barr[barr >= 0]) - hl, bpub[bpub >= 0].max() - hl))
    d = np.array(d)
    print(f"head body(last logits - last E) {d[:,0].mean():.2f}; last logits -> next-pass B arrival (selection) {d[:,1].mean():.2f}; -> next B published {d[:,2].mean():.2f}")
