"""Join a rocprofv3 kernel trace with PMC passes per kernel (name + grid): mean duration, MFMA instructions and the
TFLOP/s they imply (v_mfma_f32_32x32x16_f16 = 32768 FLOP per wave instruction; 16x16x32 likewise 16384), MFMA busy
cycles, HBM bytes (FETCH_SIZE x2: the gfx950 correction of MI355X_MICROARCH.md, WRITE_SIZE as reported).
usage: mfma_table.py DIR [top]"""
import collections
import csv
import glob
import re
import sys

root = sys.argv[1]
top = int(sys.argv[2]) if len(sys.argv) > 2 else 25
PEAK_TF, HBM = 2500.0, 8000.0


def key(name, grid):
    s = re.sub(r"\(.*", "", name.replace("void ", "").replace("q3t::", "").replace("(anonymous namespace)::", ""))
    return f"{s[:44]} g{grid}"


dur = collections.defaultdict(list)
for f in glob.glob(f"{root}/trace/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        g = (int(r.get("Grid_Size_X", 1)) * int(r.get("Grid_Size_Y", 1)) * int(r.get("Grid_Size_Z", 1))
             if "Grid_Size_X" in r else r.get("Grid_Size", "?"))   # the counter CSVs report the total
        dur[key(r["Kernel_Name"], g)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
cnt = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{root}/p*/**/*counter_collection.csv", recursive=True):
    per = collections.defaultdict(float)
    for r in csv.DictReader(open(f)):
        d = (r.get("Dispatch_Id") or r.get("Correlation_Id"), key(r["Kernel_Name"], r.get("Grid_Size", "?")), r["Counter_Name"])
        per[d] += float(r["Counter_Value"])
    for (_, k, c), v in per.items():
        cnt[k][c].append(v)
mean = lambda v: sum(v) / len(v) if v else 0.0
rows = []
for k, ds in dur.items():
    c = cnt.get(k, {})
    us = mean(ds)
    mf = mean(c.get("SQ_INSTS_MFMA", []))
    tf = mf * 32768 / (us * 1e-6) / 1e12 if us else 0.0
    fb = 2 * mean(c.get("FETCH_SIZE", [])) * 1024   # FETCH_SIZE is in KB
    wb = mean(c.get("WRITE_SIZE", [])) * 1024
    rows.append((sum(ds), k, len(ds), us, mf, tf, mean(c.get("SQ_VALU_MFMA_BUSY_CYCLES", [])), fb, wb))
rows.sort(reverse=True)
tot = sum(r[0] for r in rows)
print(f"total kernel time {tot / 1e3:.2f} ms; TFLOP/s from SQ_INSTS_MFMA x 32768 (32x32x16 f16) / mean duration; "
      f"peak {PEAK_TF:.0f} TF dense f16, HBM {HBM:.0f} GB/s")
print(f"{'kernel':52s} {'n':>4s} {'avg us':>9s} {'MFMA inst':>11s} {'TFLOP/s':>8s} {'%pk':>5s} {'busy cyc':>11s} "
      f"{'read MB':>8s} {'write MB':>8s} {'GB/s':>7s}")
for t, k, n, us, mf, tf, busy, fb, wb in rows[:top]:
    gbs = (fb + wb) / (us * 1e-6) / 1e9 if us else 0.0
    print(f"{k[:52]:52s} {n:4d} {us:9.2f} {mf:11.4g} {tf:8.1f} {100 * tf / PEAK_TF:5.1f} {busy:11.4g} "
          f"{fb / 1e6:8.1f} {wb / 1e6:8.1f} {gbs:7.0f}")
