"""dev: split of the code-predictor lm_head phase (QKV workgroups, persist_cp.hip PROF slots 1 / 3 / 2: rows arrived,
rows reduced, published) from a raw timeline (tools/dev/persist_dump.py 1 TAG)."""
import sys

import numpy as np

T = np.load(sys.argv[1]).astype(np.int64)
a, b = [], []
for ps in range(1, 16):
    h = ps * 26 + 25
    for w in range(64):
        t1, t3, t2 = T[w, h, 1], T[w, h, 3], T[w, h, 2]
        if t1 > 0 and t3 > 0 and t2 > 0:
            a.append((t3 - t1) / 100)
            b.append((t2 - t3) / 100)
print(f"head: arrive -> rows reduced {np.median(a):.2f} us, reduced -> published {np.median(b):.2f} us (median, n={len(a)})")
