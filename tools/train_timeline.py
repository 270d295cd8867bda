"""Occupancy of the GPU over the last N kernels' span in a rocprofv3 kernel trace
(.db): union of busy intervals overall and per queue, idle gaps, and the kernel
families that run while only one queue is busy.

    python tools/train_timeline.py <rocprofv3 output dir> [--last 3000]"""
import argparse
import glob
import sqlite3
from collections import defaultdict


def union(iv):
    iv = sorted(iv)
    out, tot = [], 0
    for s, e in iv:
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    for s, e in out:
        tot += e - s
    return out, tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--last", type=int, default=3000)
    a = ap.parse_args()
    db = glob.glob(f"{a.dir}/**/*.db", recursive=True)[0]
    cur = sqlite3.connect(db).cursor()
    tabs = [r[0] for r in cur.execute("select name from sqlite_master where type='table'")]
    kd = [t for t in tabs if t.startswith("rocpd_kernel_dispatch")][0]
    ks = [t for t in tabs if t.startswith("rocpd_info_kernel_symbol")][0]
    rows = cur.execute(f"select s.kernel_name, d.start, d.end, d.queue_id from {kd} d join {ks} s "
                       f"on d.kernel_id = s.id order by d.start").fetchall()
    rows = rows[-a.last:]
    t0, t1 = rows[0][1], max(r[2] for r in rows)
    span = (t1 - t0) / 1e3
    _, busy = union([(r[1], r[2]) for r in rows])
    print(f"span {span:.0f} us over {len(rows)} kernels; GPU busy (any queue) {busy / 1e3:.0f} us "
          f"({busy / 1e3 / span:.1%})")
    byq = defaultdict(list)
    for r in rows:
        byq[r[3]].append((r[1], r[2]))
    for q, iv in sorted(byq.items()):
        _, b = union(iv)
        print(f"  queue {q}: {len(iv)} kernels, busy {b / 1e3:.0f} us ({b / 1e3 / span:.1%})")
    fam = defaultdict(float)
    for n, s, e, q in rows:
        name = n.split("(")[0]
        for key in ("gemm_big", "gemm_pp", "gemm_kernel", "attention", "layernorm", "embed_ln",
                    "lstm_fwd_coop", "lstm_bwd_coop", "nce", "adam", "momentum", "enqueue"):
            if key in name:
                name = key
                break
        else:
            name = name[-40:]
        fam[name] += (e - s) / 1e3
    print("kernel time by family (us, summed, overlaps counted twice):")
    for k, v in sorted(fam.items(), key=lambda x: -x[1])[:18]:
        print(f"  {v:9.0f}  {k}")


if __name__ == "__main__":
    main()
