"""dev: split a frame-loop kernel trace into the code-predictor phase (after k_cb0 up to the 15th k_cpsel) and the
talker phase (from there to k_advance); per-kernel avg durations inside each phase and per-phase span."""
import collections
import csv
import re
import sys

rows = []
with open(sys.argv[1]) as f:
    for r in csv.DictReader(f):
        n = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void q3t::", "").replace("q3t::", "")
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), n, r["Grid_Size_X"], r["Grid_Size_Y"]))
rows.sort()
agg = {"talker": collections.defaultdict(list), "cp": collections.defaultdict(list), "frame": collections.defaultdict(list)}
spans = {"talker": [], "cp": [], "frame": []}
phase, start, nsel, fstart, last_e = None, None, 0, None, 0


def close(ph):
    if start is not None:
        spans[ph].append(last_e - start)


for s, e, n, gx, gy in rows:
    key = f"{n} g{gx}x{gy}"
    if n == "k_cb0":
        phase, start, nsel, fstart = "cp", None, 0, s
        agg["frame"][key].append(e - s)
        continue
    if phase is None:
        continue
    if n == "k_advance":
        close(phase)
        spans["frame"].append(e - fstart)
        agg["frame"][key].append(e - s)
        phase = None
        continue
    if start is None:
        start = s
    last_e = e
    agg[phase][key].append(e - s)
    if n == "k_cpsel" and phase == "cp":
        nsel += 1
        if nsel == 15:
            close("cp")
            phase, start = "talker", None
for ph in ("cp", "talker", "frame"):
    sp = spans[ph]
    nph = max(1, len(sp))
    print(f"== {ph}: {len(sp)} phases, mean span {sum(sp) / nph / 1e3:.1f} us")
    tot = 0
    for k, v in sorted(agg[ph].items(), key=lambda kv: -sum(kv[1])):
        tot += sum(v) / nph
        print(f"  {len(v) / nph:6.1f}/phase x {sum(v) / len(v) / 1e3:7.2f} us = {sum(v) / nph / 1e3:8.1f} us  {k}")
    print(f"  sum of kernel time per phase {tot / 1e3:.1f} us")
