"""Summarise a rocprofv3 kernel trace (rocpd .db or kernel_trace.csv): per-kernel count / total / avg us, plus
busy-vs-span (launch gaps) over the densest window.  Usage: prof_stats.py TRACE [--by-grid]"""
import collections
import csv
import re
import sqlite3
import sys


def short(n):
    n = n.replace("(anonymous namespace)::", "")
    n = re.sub(r"\(.*", "", n)
    return n[:110]


def from_db(path):
    con = sqlite3.connect(path)
    cur = con.cursor()
    t = [r[0] for r in cur.execute("select name from sqlite_master where type='table'")]
    kd = [v for v in t if v.startswith("rocpd_kernel_dispatch")][0]
    ks = [v for v in t if v.startswith("rocpd_info_kernel_symbol")][0]
    cols = [r[1] for r in cur.execute(f"pragma table_info({ks})")]
    namecol = "kernel_name" if "kernel_name" in cols else ("display_name" if "display_name" in cols else cols[2])
    names = {r[0]: r[1] for r in cur.execute(f"select id, {namecol} from {ks}")}
    rows = cur.execute(f"select kernel_id, start, end from {kd}").fetchall()
    return [(names.get(k, str(k)), s, e, "") for k, s, e in rows]


def from_csv(path):
    out = []
    with open(path) as f:
        for r in csv.DictReader(f):
            g = f"g{r.get('Grid_Size_X', r.get('Grid_Size', '?'))}x{r.get('Grid_Size_Y', '')}"
            out.append((r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"]), g))
    return out


def main():
    p = sys.argv[1]
    by_grid = "--by-grid" in sys.argv
    ev = from_db(p) if p.endswith(".db") else from_csv(p)
    if "--seq" in sys.argv:   # the last N dispatches in time order
        n = int(sys.argv[sys.argv.index("--seq") + 1])
        ev.sort(key=lambda x: x[1])
        for name, s, e, g in ev[-n:]:
            print(f"{(e - s) / 1e3:9.2f} us  {short(name)} {g}")
        return
    agg = collections.defaultdict(lambda: [0, 0.0])
    for n, s, e, g in ev:
        a = agg[short(n) + (" " + g if by_grid else "")]
        a[0] += 1
        a[1] += (e - s) / 1e3
    tot = sum(v[1] for v in agg.values())
    print(f"total kernel time {tot / 1e3:.1f} ms over {sum(v[0] for v in agg.values())} dispatches")
    for n, (c, s) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:45]:
        print(f"{s / 1e3:9.2f} ms {100 * s / tot:5.1f}% {c:8d} x {s / c:8.2f} us  {n}")
    # busy vs span: merge intervals, report idle gaps between consecutive kernels
    ev.sort(key=lambda x: x[1])
    if ev:
        span = (ev[-1][2] - ev[0][1]) / 1e3
        busy = 0.0
        cur_s, cur_e = ev[0][1], ev[0][2]
        gaps = []
        for _, s, e, _ in ev[1:]:
            if s > cur_e:
                busy += cur_e - cur_s
                gaps.append(s - cur_e)
                cur_s, cur_e = s, e
            else:
                cur_e = max(cur_e, e)
        busy += cur_e - cur_s
        small = [g for g in gaps if g < 50_000]  # ignore host-side pauses > 50 us
        print(f"span {span / 1e3:.1f} ms, busy {busy / 1e6:.1f} ms; {len(small)} inter-kernel gaps < 50us avg "
              f"{(sum(small) / max(1, len(small))) / 1e3:.2f} us (total {sum(small) / 1e6:.1f} ms)")


if __name__ == "__main__":
    main()
