"""C2 retrieval (100k x 768 bf16 shard, Q = 256, k = 100): per-batch time of serial
search() calls and of search_many() at 1..4 batches in flight -- the one-call native loop
(irc_scan_topk_many), the per-stream HIP graphs, and the per-batch Python loop search_many
ran before (search() per batch on the depth streams) -- with the host's issue time of each
(the call alone, before the synchronize).  Diagnostic for the serving leg's depth choice.

    python tools/scan_depth.py [--reps 200]
"""
import argparse
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "information-retrieval-with-contrastive-learning_amd"))

from irc_amd import retrieval  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--n", type=int, default=100_000)
    ap.add_argument("--q", type=int, default=256)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(2024)
    shard = torch.nn.functional.normalize(torch.randn(a.n, 768, generator=g, device=dev)).bfloat16()
    q = torch.nn.functional.normalize(torch.randn(a.q, 768, device=dev)).bfloat16()
    index = retrieval.ShardedDenseIndex(shard, doc_offset=0)
    ref = index.search(q, 100, equal_counts=True)
    batches = [q] * a.reps

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        return (t2 - t0) * 1e6 / a.reps, (t1 - t0) * 1e6 / a.reps

    def pyloop(bs, depth):
        cur = torch.cuda.current_stream(dev)
        streams = retrieval._search_streams(dev, depth)
        out = []
        for n, qb in enumerate(bs):
            st = streams[n % depth]
            st.wait_stream(cur)
            with torch.cuda.stream(st):
                out.append(index.search(qb, 100, equal_counts=True, ws_tag=f"scan{n % depth}"))
        for st in streams:
            cur.wait_stream(st)
        return out

    def serial():
        for _ in range(a.reps):
            index.search(q, 100, equal_counts=True)

    us, host = timed(serial)
    print(f"serial search(): {us:.1f} us/batch (host {host:.1f})", flush=True)
    for rep in range(2):
        for mode in ("native", "python", "graphs"):
            for depth in (1, 2, 3, 4):
                if mode == "python":
                    fn = lambda bs: pyloop(bs, depth)  # noqa: E731
                else:
                    fn = lambda bs: index.search_many(  # noqa: E731
                        bs, 100, depth=depth, equal_counts=True, graphs=mode == "graphs")
                us, host = timed(lambda: fn(batches))
                out = fn(batches[:depth + 1])
                same = all(torch.equal(s, ref[0]) and torch.equal(i, ref[1]) for s, i in out)
                print(f"rep {rep} {mode:6s} depth {depth}: {us:6.1f} us/batch (host {host:5.1f})"
                      f"{'' if same else '  RESULTS DIFFER'}", flush=True)


if __name__ == "__main__":
    main()
