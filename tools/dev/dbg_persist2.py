"""dev: head 10/11 (kv group 5) attention at pos 1, layer 0: persistent dump vs graph output vs float64."""
import os, sys
import numpy as np
R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(R, "qwen3-tts-jetson_amd"), os.path.join(R, "tests")]
os.environ["Q3T_TALKER_LAYERS"] = "1"; os.environ["Q3T_PERSIST_DBG"] = "1"
import q3t
from q3t_testutil import synth_dir
tts, tok = synth_dir("full")
def mk(flag):
    os.environ["Q3T_PERSIST"] = flag
    return q3t.Engine(tts, None, device=0, max_slots=1, max_ctx=320)
ep, eg = mk("1"), mk("0")
H = 1024; CTX = 320
rng = np.random.default_rng(11)
nb = 1 * 8 * CTX * 128 * 2
for pos in range(2):
    e = (rng.standard_normal(H) * 0.5).astype(np.float32)
    ep.talker_forward(e[None], [pos]); eg.talker_forward(e[None], [pos])
K = ep.debug_read(0, nb).view(np.float16).reshape(8, CTX, 128).astype(np.float64)[5]
V = ep.debug_read(1, nb).view(np.float16).reshape(8, CTX, 128).astype(np.float64)[5]
dd = ep.debug_read(4, 8 * 32 * 2 * 130 * 4).view(np.float32)[16384:16384 + 1024]
q = dd[:256].reshape(2, 128).astype(np.float64); kn = dd[256:384]; vn = dd[384:512]
print("kn == K[1]:", np.array_equal(np.float16(kn).astype(np.float64), K[1]), " vn == V[1]:", np.array_equal(np.float16(vn).astype(np.float64), V[1]))
print("M, L dumped:", dd[512:516])
dg = eg.debug_read(4, 16 * 5 * 130 * 4).view(np.float32)[16384 - 16384:][:0]
try:
    dg = eg.debug_read(4, 1024 * 4).view(np.float32)[:1024]
    print("graph q vs persist q: maxdiff", np.abs(dg[:256] - dd[:256]).max(), "kn", np.abs(dg[256:384] - kn).max(), "vn", np.abs(dg[384:512] - vn).max())
    print("graph M,L:", dg[512:516])
    i = np.argmax(np.abs(dg[:256] - dd[:256])); print("  q idx", i, dg[i], dd[i])
except Exception as ex:
    print("graph dump failed", ex)
ap = ep.debug_read(3, 4096).view(np.float16).astype(np.float64).reshape(16, 128)
ag = eg.debug_read(3, 4096).view(np.float16).astype(np.float64).reshape(16, 128)
for h in range(2):
    s = (K[:2] @ q[h]) / np.sqrt(128.0)
    p = np.exp(s - s.max()); o = (p @ V[:2]) / p.sum()
    f32 = dd[516 + h * 128: 516 + (h + 1) * 128]
    dp = np.abs(ap[10 + h] - ag[10 + h])
    i = int(np.argmax(dp))
    print(f"head {10+h}: scores {s}, M {s.max():.7f}; max|persist-graph| {dp.max():.3g} at d={i}: persist {ap[10+h][i]!r} graph {ag[10+h][i]!r} f32 {f32[i]!r} f64 {o[i]!r}")
