"""Summarise a rocprofv3 kernel trace (rocpd .db or kernel_trace.csv): per-kernel count / total / avg us."""
import csv, glob, sqlite3, sys, collections, re
def short(n):
    n = re.sub(r"\(.*", "", n)
    return n[:110]
def from_db(path):
    con = sqlite3.connect(path); cur = con.cursor()
    t = {r[0].split("_0")[0] if False else r[0]: r[0] for r in cur.execute("select name from sqlite_master where type='table'")}
    kd = [v for v in t if v.startswith("rocpd_kernel_dispatch")][0]
    ks = [v for v in t if v.startswith("rocpd_info_kernel_symbol")][0]
    cols = [r[1] for r in cur.execute(f"pragma table_info({ks})")]
    namecol = "kernel_name" if "kernel_name" in cols else ("display_name" if "display_name" in cols else cols[2])
    names = {r[0]: r[1] for r in cur.execute(f"select id, {namecol} from {ks}")}
    rows = cur.execute(f"select kernel_id, start, end from {kd}").fetchall()
    return [(names.get(k, str(k)), (e - s) / 1e3) for k, s, e in rows]
def from_csv(path):
    out = []
    with open(path) as f:
        for r in csv.DictReader(f):
            out.append((r["Kernel_Name"], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
    return out
p = sys.argv[1]
ev = from_db(p) if p.endswith(".db") else from_csv(p)
agg = collections.defaultdict(lambda: [0, 0.0])
for n, us in ev:
    a = agg[short(n)]; a[0] += 1; a[1] += us
tot = sum(v[1] for v in agg.values())
print(f"total kernel time {tot/1e3:.1f} ms over {sum(v[0] for v in agg.values())} dispatches")
for n, (c, s) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:40]:
    print(f"{s/1e3:9.2f} ms {100*s/tot:5.1f}% {c:8d} x {s/c:8.2f} us  {n}")
