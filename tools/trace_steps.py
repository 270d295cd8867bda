"""Per-step timeline of a rocprofv3 --kernel-trace run of the training step: between
consecutive optimizer launches (adam_kernel / sgd_kernel), the wall time, the time
some kernel was running (union), the time kernels of two streams overlapped, and
per-stream busy time with its top kernels -- where a step's wall clock goes when
the BERT prefetch stream and the heads stream share the chip.

    python tools/trace_steps.py <rocprofv3 output dir> [--skip 5] [--steps 20]"""
import argparse
import collections
import glob
import sqlite3


def union(iv):
    tot, cur_s, cur_e = 0, None, None
    for s, e in sorted(iv):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--skip", type=int, default=5)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--top", type=int, default=8)
    a = ap.parse_args()
    db = glob.glob(f"{a.dir}/**/*.db", recursive=True)[0]
    c = sqlite3.connect(db)
    ks = list(c.execute("select name, stream_id, queue_id, start, end from kernels order by start"))
    marks = [k[4] for k in ks if "adam_kernel" in k[0] or "sgd_kernel" in k[0]]
    marks = marks[a.skip:a.skip + a.steps + 1]
    walls, unions, per_stream, per_kernel = [], [], collections.Counter(), collections.Counter()
    for t0, t1 in zip(marks, marks[1:]):
        iv = [(max(s, t0), min(e, t1)) for n, sid, q, s, e in ks if e > t0 and s < t1]
        walls.append(t1 - t0)
        unions.append(union(iv))
        for n, sid, q, s, e in ks:
            if e > t0 and s < t1:
                d = min(e, t1) - max(s, t0)
                per_stream[(sid, q)] += d
                per_kernel[((sid, q), n.split("(")[0][:70])] += d
    n = len(walls)
    ms = lambda v: v / n / 1e6
    print(f"steps {n}: wall {ms(sum(walls)):.3f} ms  busy(union) {ms(sum(unions)):.3f} ms  "
          f"idle {ms(sum(walls) - sum(unions)):.3f} ms")
    for key, t in per_stream.most_common():
        print(f"  stream {key}: {ms(t):.3f} ms of kernel time")
        for (k2, name), t2 in per_kernel.most_common():
            if k2 == key and t2 / n / 1e6 > 0.02:
                print(f"      {ms(t2):7.3f}  {name}")


if __name__ == "__main__":
    main()
