"""dev: split a frame-loop kernel trace into talker (after k_step_embd .. k_advance) and CP (after k_cb0 ..
k_step_embd) phases; per-kernel avg durations inside each phase and per-phase span."""
import collections, csv, re, sys
rows = []
with open(sys.argv[1]) as f:
    for r in csv.DictReader(f):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void q3t::", "").replace("q3t::", ""), r["Grid_Size_X"], r["Grid_Size_Y"]))
rows.sort()
phase = None
agg = {"talker": collections.defaultdict(list), "cp": collections.defaultdict(list)}
spans = {"talker": [], "cp": []}
start = None
for s, e, n, gx, gy in rows:
    if n == "k_cb0":
        phase, start = "cp", None
        continue
    if n == "k_step_embd":
        if phase == "cp" and start is not None: spans["cp"].append(last_e - start)
        phase, start = "talker", None
        continue
    if n == "k_advance":
        if phase == "talker" and start is not None: spans["talker"].append(last_e - start)
        phase = None
        continue
    if phase:
        if start is None: start = s
        last_e = e
        agg[phase][f"{n} g{gx}x{gy}"].append(e - s)
for ph in ("talker", "cp"):
    sp = spans[ph]
    print(f"== {ph}: {len(sp)} phases, mean span {sum(sp)/max(1,len(sp))/1e3:.1f} us")
    tot = 0
    for k, v in sorted(agg[ph].items(), key=lambda kv: -sum(kv[1])):
        per = len(v) / max(1, len(sp))
        tot += sum(v) / max(1, len(sp))
        print(f"  {per:6.1f}/phase x {sum(v)/len(v)/1e3:7.2f} us = {sum(v)/max(1,len(sp))/1e3:8.1f} us  {k}")
    print(f"  sum of kernel time per phase {tot/1e3:.1f} us")
