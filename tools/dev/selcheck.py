"""dev: compare the token files of two selbench builds (tools/dev/selbench.hip) and check every token against a float64
restatement of top-k sampling (the rows and u regenerated as selbench makes them).  usage: selcheck.py V A.bin B.bin"""
import sys

import numpy as np

V = int(sys.argv[1])
A = np.fromfile(sys.argv[2], dtype=np.int32)
B = np.fromfile(sys.argv[3], dtype=np.int32)
R, NROW, K = len(A), 64, 50
M64 = (1 << 64) - 1


def mix64(z):
    z = (z + 0x9E3779B97F4A7C15) & M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def uniform24(seed, utt, frame, cb):
    h = mix64((mix64(seed ^ ((utt * 0xD1B54A32D192ED03) & M64)) + frame * 16 + cb) & M64)
    return np.float32((h >> 40) * (1.0 / 16777216.0))


z = 7


def rnd():
    global z
    z = (z * 1664525 + 1013904223) & 0xFFFFFFFF
    return np.float32((z >> 8) * (1.0 / 16777216.0))


rows = np.zeros((NROW, V), np.float32)
for r in range(NROW):
    x = rows[r]
    for i in range(V):
        s = np.float32(0)
        for k in range(4):
            s = np.float32(s + np.float32(rnd() - np.float32(0.5)))
        x[i] = np.float32(np.float32(s * np.float32(4.0)) * np.float32(1.7))
    kind = r % 8
    if kind == 1:
        for k in range(3):
            j = int(rnd() * V)
            x[j] = np.float32(x[j] + np.float32(80.0))
    if kind == 2:
        x[:] = np.floor(x * np.float32(2.0)) * np.float32(0.5)
    if kind == 3:
        for i in range(V - 1024, V):
            if i != V - 3:
                x[i] = -np.inf
    if kind == 4:
        x[:] = np.floor(x * np.float32(0.25))
    if kind == 5:
        x[:] = x * np.float32(0.05)
    if kind == 6:
        x[:] = -np.inf
        for k in range(30):
            val = rnd()   # C++17: the right operand of = is sequenced first
            x[int(rnd() * V)] = val
    if kind == 7:
        x[5] = np.float32(1e30)
bad = 0
for r in range(R):
    T = np.float32(0.9) if (r & 4) else np.float32(0.7)
    keep = V - 1 - (r % 7) * 131 if r % 3 == 0 else -1
    v = (rows[r % NROW] / T).astype(np.float32)
    kv = v[keep] if keep >= 0 else None
    thr = np.sort(v)[::-1][K - 1]
    w = np.where(v < thr, -np.inf, v)
    if keep >= 0:
        w[keep] = kv
    p = np.exp((w - w.max()).astype(np.float64))
    c = np.cumsum(p)
    u = float(uniform24(1, 0, r, 3)) * c[-1]
    for name, tok in (("A", A[r]), ("B", B[r])):
        lo = c[tok - 1] if tok > 0 else 0.0
        ok = p[tok] > 0 and lo - 1e-5 * c[-1] <= u <= c[tok] + 1e-5 * c[-1]
        if not ok:
            bad += 1
            print(f"r {r} kind {r % 64 % 8} {name} tok {tok} p {p[tok]:.3g} interval [{lo:.6g}, {c[tok]:.6g}] u {u:.6g}")
diff = np.nonzero(A != B)[0]
print(f"{R} selections: {len(diff)} differ between the builds, {bad} tokens outside their float64 CDF interval (1e-5)")
for r in diff[:10]:
    print(f"  r {r} kind {r % 64 % 8}: {A[r]} vs {B[r]}")
