"""Per-kernel totals of a rocprofv3 --kernel-trace run (the rocpd .db it writes):
calls, total and average us, sorted by total.

    python tools/trace_top.py <rocprofv3 output dir> [--top 30]"""
import argparse
import glob
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--top", type=int, default=30)
    a = ap.parse_args()
    db = glob.glob(f"{a.dir}/**/*.db", recursive=True)[0]
    c = sqlite3.connect(db)
    rows = list(c.execute("select name, total_calls, total_duration, average from top_kernels"))
    tot = sum(r[2] for r in rows)
    print(f"{'calls':>7} {'total_us':>11} {'avg_us':>9} {'pct':>6}  kernel")
    for name, n, t, avg in rows[:a.top]:
        print(f"{n:7d} {t:11.1f} {avg:9.2f} {100 * t / tot:6.2f}  {name[:110]}")


if __name__ == "__main__":
    main()
