"""Per-kernel durations of the scan calls in a rocprofv3 kernel trace (.db):
median duration of each kernel (by name and grid) and of the gap before it.

    python tools/call_timeline.py <rocprofv3 output dir>"""
import glob
import sqlite3
import statistics
import sys
from collections import defaultdict


def main():
    db = glob.glob(f"{sys.argv[1]}/**/*.db", recursive=True)[0]
    cur = sqlite3.connect(db).cursor()
    tabs = [r[0] for r in cur.execute("select name from sqlite_master where type='table'")]
    kd = [t for t in tabs if t.startswith("rocpd_kernel_dispatch")][0]
    ks = [t for t in tabs if t.startswith("rocpd_info_kernel_symbol")][0]
    rows = cur.execute(f"select s.kernel_name, d.start, d.end, d.grid_size_x, d.workgroup_size_x "
                       f"from {kd} d join {ks} s on d.kernel_id = s.id order by d.start").fetchall()
    dur, gap, order = defaultdict(list), defaultdict(list), []
    for i, (n, s, e, g, w) in enumerate(rows):
        name = n.split("(")[0].replace("_ZN3irc4scan", "scan::").replace("_ZN3irc3gpp", "gpp::")[:58]
        prev = rows[i - 1][0].split("(")[0][-40:-20] if i else ""
        key = f"{name} wgs={g // max(w, 1)}" + (f" after ..{prev}" if "select" in name else "")
        if key not in dur:
            order.append(key)
        dur[key].append((e - s) / 1e3)
        if i:
            gap[key].append((s - rows[i - 1][2]) / 1e3)
    for key in order:
        if len(dur[key]) < 5:
            continue
        print(f"{key:100s} n={len(dur[key]):4d} med {statistics.median(dur[key]):8.2f} us  "
              f"gap before {statistics.median(gap[key]) if gap[key] else 0:6.2f} us")


if __name__ == "__main__":
    main()
