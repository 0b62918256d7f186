"""dev: split a frame-loop kernel trace into code-predictor and talker phases.  Frames are delimited by k_advance (or,
when the persistent talker step folds the advance in, by that step);
the talker phase is the last TALKER_KERNELS (5 per layer x 28 + codec head = 141) kernels before it, everything
earlier in the frame is the code-predictor phase.  Prints per-kernel avg durations and per-phase spans."""
import collections
import csv
import re
import sys

rows = []
with open(sys.argv[1]) as f:
    for r in csv.DictReader(f):
        n = r["Kernel_Name"].replace("(anonymous namespace)::", "")   # the role kernels sit in an anonymous namespace
        n = re.sub(r"\(.*", "", n).replace("void q3t::", "").replace("q3t::", "")
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), n, r["Grid_Size_X"], r["Grid_Size_Y"]))
rows.sort()
# the 1-slot talker step is ONE persistent launch when the persistent kernels run (k_tk_roles / k_persist<0, *>)
persistent = any(n.startswith(("k_tk_roles", "k_persist<0")) for _, _, n, _, _ in rows)
TALKER_KERNELS = int(sys.argv[2]) if len(sys.argv) > 2 else (1 if persistent else 141)
frames, cur = [], []
for row in rows:
    if row[2] == "k_advance":
        frames.append(cur)
        cur = []
    else:
        cur.append(row)
        # the persistent talker step folds the advance in (no k_advance launch): it closes the frame itself
        if persistent and row[2].startswith(("k_tk_roles", "k_persist<0")) and not any(r[2] == "k_advance" for r in rows):
            frames.append(cur)
            cur = []
print(f"({len(rows)} kernels, {sum(1 for r in rows if r[2] == 'k_advance')} k_advance, {len(frames)} chunks, "
      f"persistent={persistent}, chunk sizes {[len(f) for f in frames[:6]]})")
frames = [f for f in frames[1:] if len(f) > TALKER_KERNELS]
if persistent:   # the frame loop's first chunk ends in the prefill; every later chunk is [cp frame, talker step]
    frames = [f for f in frames if len(f) >= 2]   # first chunk holds prefill/setup kernels
    # folded advance: keep the frame-loop chunks [code-predictor frame, talker step] (the later chunks hold the vocoder
    # and the time_stage replays)
    frames = [f for f in frames if len(f) <= 4 and f[-2][2].startswith(("k_cp_roles", "k_persist<1"))]
agg = {"cp": collections.defaultdict(list), "talker": collections.defaultdict(list)}
spans = {"cp": [], "talker": [], "frame": []}
for f in frames:
    cp, tk = f[:-TALKER_KERNELS], f[-TALKER_KERNELS:]
    for ph, ks in (("cp", cp), ("talker", tk)):
        spans[ph].append(ks[-1][1] - ks[0][0])
        for s, e, n, gx, gy in ks:
            agg[ph][f"{n} g{gx}x{gy}"].append(e - s)
    spans["frame"].append(f[-1][1] - f[0][0])
for ph in ("cp", "talker"):
    sp = spans[ph]
    nph = max(1, len(sp))
    print(f"== {ph}: {len(sp)} frames, mean span {sum(sp) / nph / 1e3:.1f} us")
    tot = 0
    for k, v in sorted(agg[ph].items(), key=lambda kv: -sum(kv[1])):
        tot += sum(v) / nph
        print(f"  {len(v) / nph:6.1f}/frame x {sum(v) / len(v) / 1e3:7.2f} us = {sum(v) / nph / 1e3:8.1f} us  {k}")
    print(f"  sum of kernel time per frame {tot / 1e3:.1f} us")
sp = spans["frame"]
print(f"== frame: {len(sp)} frames, mean span {sum(sp) / max(1, len(sp)) / 1e3:.1f} us (k_advance excluded)")

# ---- time_stage replays at the end of a bench trace: 21 talker-step replays (1 warm + 20 timed, 141 kernels each)
# then 11 code-predictor-frame replays (1 warm + 10 timed).  Mean replay span = first kernel start -> last kernel end.
TR, CR = 21, 11
CPK = max(1, round(sum(len(f) - TALKER_KERNELS for f in frames) / max(1, len(frames)))) if frames else 335
qrows = [r for r in rows if not r[2].startswith("__amd")]   # runtime copy/fill kernels of time_stage's setup
tail = qrows[-(TR * TALKER_KERNELS + CR * CPK):] if len(qrows) >= TR * TALKER_KERNELS + CR * CPK else []
if tail:
    talk = tail[:TR * TALKER_KERNELS]
    reps = [talk[i * TALKER_KERNELS:(i + 1) * TALKER_KERNELS] for i in range(TR)][1:]
    spans_r = [r[-1][1] - r[0][0] for r in reps]
    busy_r = [sum(e - s for s, e, *_ in r) for r in reps]
    print(f"== time_stage talker replays: {len(reps)} timed, mean span {sum(spans_r) / len(reps) / 1e3:.1f} us, "
          f"mean kernel-busy {sum(busy_r) / len(reps) / 1e3:.1f} us; first kernel {reps[0][0][2]}, last {reps[0][-1][2]}")
    agg_r = collections.defaultdict(list)
    for r in reps:
        for s, e, n, gx, gy in r:
            agg_r[f"{n} g{gx}x{gy}"].append(e - s)
    for k, v in sorted(agg_r.items(), key=lambda kv: -sum(kv[1])):
        print(f"  {len(v) / len(reps):6.1f}/replay x {sum(v) / len(v) / 1e3:7.2f} us = {sum(v) / len(reps) / 1e3:8.1f} us  {k}")
