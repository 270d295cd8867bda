"""A/B of the single-pass GEMM filter (irc_scan_set_ppl_min_q) against the sampled-
threshold pipeline: whole irc_scan_topk call time per Q on a shard (default: the C2
100k x 768 shard and the C3 250k x 768 shard), both modes interleaved in one process,
plus the rescan counters of the single-pass runs.

    python tools/scan_ppl_ab.py [--reps 50]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "information-retrieval-with-contrastive-learning_amd"))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--qs", default="64,96,128,192,256")
    args = ap.parse_args()
    from irc_amd import retrieval

    dev = torch.device("cuda:0")
    for n in (100_000, 250_000):
        g = torch.Generator(device=dev).manual_seed(2024)
        d = torch.nn.functional.normalize(torch.randn(n, 768, generator=g, device=dev)).bfloat16()
        for q in [int(x) for x in args.qs.split(",")]:
            gq = torch.Generator().manual_seed(11 + q)
            qq = torch.nn.functional.normalize(torch.randn(q, 768, generator=gq)).bfloat16().to(dev)
            res = {}
            for rnd in range(2):
                for mode, mq in (("single", 1), ("sampled", 1 << 20)):
                    prev = retrieval.set_single_pass_min_q(mq)
                    for _ in range(3):
                        retrieval.scan_topk(qq, d, 100)
                    torch.cuda.synchronize()
                    if mode == "single":
                        retrieval.rescan_stats(reset=True)
                    t0 = time.perf_counter()
                    for _ in range(args.reps):
                        retrieval.scan_topk(qq, d, 100)
                    torch.cuda.synchronize()
                    dt = (time.perf_counter() - t0) / args.reps * 1e6
                    res.setdefault(mode, []).append(dt)
                    if mode == "single":
                        res["rescans"] = retrieval.rescan_stats(reset=True)
                    retrieval.set_single_pass_min_q(prev)
            alg = n * 768 * 2 + q * 768 * 2 + q * 100 * 8
            s, p = min(res["single"]), min(res["sampled"])
            print(f"N={n} Q={q:4d}  single {s:7.1f} us ({alg / s / 8e6:.3f} of HBM)  sampled "
                  f"{p:7.1f} us ({alg / p / 8e6:.3f})  rescans (queries, tiles) over "
                  f"{args.reps + 3} calls: {res['rescans']}", flush=True)
        del d
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
