"""dev: do several contexts on one GPU (each its own stream and graphs, weights copied device to device) overlap their
latency-bound batched frame loops?  Times N utterances x F frames through one context of N slots, then through R
replicas of N/R slots driven from R host threads concurrently."""
import os
import sys
import threading
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "qwen3-tts-jetson_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import q3t  # noqa: E402
from q3t_testutil import prompt as make_prompt, synth_dir  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 64
F = int(sys.argv[2]) if len(sys.argv) > 2 else 128
tts, tok = synth_dir("full")
pr = make_prompt("full")
kw = dict(max_len=F, temperature=0.9, top_k=50, repetition_penalty=1.05, force_frames=F)
base = q3t.Engine(tts, None, device=0, max_slots=N, max_ctx=F + 32)
H = base.cfg["hidden"]


def run(eng, n, seed):
    return eng.generate([pr] * n, speakers=[np.zeros(H, np.float32)] * n, seed=seed, **kw)


run(base, N, 1)
base.synchronize()
t = time.perf_counter()
ref = run(base, N, 1)
base.synchronize()
t1 = time.perf_counter() - t
print(f"1 context x {N} slots: {t1 * 1e3:.1f} ms, {N * F / t1:.0f} frames/s", flush=True)
RS = [int(x) for x in sys.argv[3].split(",")] if len(sys.argv) > 3 else [2, 4]
PER = int(sys.argv[4]) if len(sys.argv) > 4 else 0   # slots per replica (0: N / R)
for R in RS:
    n = PER or N // R
    engs = [base.replica(0, n, F + 32) for _ in range(R)]
    for e in engs:
        run(e, n, 1)
        e.synchronize()
    outs = [None] * R

    def work(i):
        outs[i] = run(engs[i], n, 1)
        engs[i].synchronize()
    th = [threading.Thread(target=work, args=(i,)) for i in range(R)]
    t = time.perf_counter()
    for x in th:
        x.start()
    for x in th:
        x.join()
    tr = time.perf_counter() - t
    print(f"{R} contexts x {n} slots concurrently: {tr * 1e3:.1f} ms, {R * n * F / tr:.0f} frames/s", flush=True)
    # serial for comparison
    t = time.perf_counter()
    for i in range(R):
        work(i)
    ts = time.perf_counter() - t
    print(f"{R} contexts x {n} slots one after another: {ts * 1e3:.1f} ms", flush=True)
    for e in engs:
        e.close()
base.close()
