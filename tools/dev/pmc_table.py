"""dev: per-kernel (name + grid) mean of every counter over all rocprofv3 --pmc passes under a directory."""
import collections
import csv
import glob
import sys

root = sys.argv[1]
top = int(sys.argv[2]) if len(sys.argv) > 2 else 14
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
    per_disp = collections.defaultdict(float)
    meta = {}
    for row in csv.DictReader(open(f)):
        name = row["Kernel_Name"]
        short = name.split("(")[0].replace("void ", "").replace("q3t::", "").replace("(anonymous namespace)::", "")
        key = f"{short[:46]} g{row.get('Grid_Size', '')}"
        d = (row.get("Dispatch_Id") or row.get("Correlation_Id"), key, row["Counter_Name"])
        per_disp[d] += float(row["Counter_Value"])   # sum over dimensions / XCDs of one dispatch
    for (disp, key, cn), v in per_disp.items():
        agg[key][cn].append(v)
rows = sorted(agg.items(), key=lambda kv: -max((sum(v) for v in kv[1].values()), default=0))
counters = sorted({c for _, d in rows for c in d})
print("kernel".ljust(58) + " n  " + "  ".join(c[-22:].rjust(14) for c in counters))
for key, d in rows[:top]:
    n = max(len(v) for v in d.values())
    print(key[:58].ljust(58) + f"{n:3d} " + "  ".join((f"{sum(d[c]) / len(d[c]):14.4g}" if c in d else " " * 14) for c in counters))
