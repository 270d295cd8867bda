"""Summarise a rocprofv3 kernel trace (.db from --kernel-trace, or the CSV from
--output-format csv) into per-kernel count / total / average duration."""
import csv
import glob
import os
import sqlite3
import sys
from collections import defaultdict

BY_GRID = "--by-grid" in sys.argv


def from_db(path):
    con = sqlite3.connect(path)
    cur = con.cursor()
    tabs = [r[0] for r in cur.execute("select name from sqlite_master where type='table'")]
    kd = [t for t in tabs if t.startswith("rocpd_kernel_dispatch")][0]
    ks = [t for t in tabs if t.startswith("rocpd_info_kernel_symbol")][0]
    rows = cur.execute(
        f"select s.kernel_name, d.end - d.start, d.grid_size_x from {kd} d "
        f"join {ks} s on d.kernel_id = s.id")
    return [(f"{n} [grid={g}]" if BY_GRID else n, dur) for n, dur, g in rows]


def from_csv(path):
    out = []
    with open(path) as f:
        for r in csv.DictReader(f):
            out.append((r["Kernel_Name"], int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    return out


def summarise(rows, top=25):
    agg = defaultdict(lambda: [0, 0])
    for n, d in rows:
        agg[n][0] += 1
        agg[n][1] += d
    tot = sum(v[1] for v in agg.values())
    lines = [f"{'calls':>7} {'total_us':>11} {'avg_us':>9} {'pct':>6}  kernel"]
    for n, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
        short = n if len(n) < 110 else n[:60] + "..." + n[-45:]
        lines.append(f"{c:7d} {t/1e3:11.1f} {t/c/1e3:9.2f} {100*t/tot:6.2f}  {short}")
    return "\n".join(lines)


if __name__ == "__main__":
    p = [a for a in sys.argv[1:] if not a.startswith("--")][0]
    if os.path.isdir(p):
        cands = glob.glob(os.path.join(p, "**", "*.db"), recursive=True) + \
            glob.glob(os.path.join(p, "**", "*kernel_trace.csv"), recursive=True)
        p = cands[0]
    rows = from_db(p) if p.endswith(".db") else from_csv(p)
    top = [int(a.split("=", 1)[1]) for a in sys.argv[1:] if a.startswith("--top=")]
    print(summarise(rows, top[0] if top else 25))
