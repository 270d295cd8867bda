"""One retrieval configuration's whole irc_scan_topk call, repeated, for a kernel
trace (rocprofv3 --kernel-trace --stats) of where the call's time goes.

    python tools/scan_call_prof.py --n 625000 --d 1024 --q 2048 [--fp8] [--reps 10]
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
    ap.add_argument("--n", type=int, default=625_000)
    ap.add_argument("--d", type=int, default=1024)
    ap.add_argument("--q", type=int, default=2048)
    ap.add_argument("--k", type=int, default=100)
    ap.add_argument("--fp8", action="store_true")
    ap.add_argument("--reps", type=int, default=10)
    args = ap.parse_args()
    from irc_amd import retrieval

    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(2024)
    d = torch.nn.functional.normalize(torch.randn(args.n, args.d, generator=g, device=dev))
    gq = torch.Generator().manual_seed(7)
    q = torch.nn.functional.normalize(torch.randn(args.q, args.d, generator=gq)).to(dev)
    if args.fp8:
        d8, q8 = retrieval.quantize_fp8(d), retrieval.quantize_fp8(q)
        del d
        fn = lambda: retrieval.scan_topk_fp8(q8, d8, args.k, 0, 1.0 / 256)  # noqa: E731
    else:
        db, qb = d.bfloat16(), q.bfloat16()
        del d
        fn = lambda: retrieval.scan_topk(qb, db, args.k)  # noqa: E731
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.reps):
        fn()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / args.reps
    print(f"N={args.n} D={args.d} Q={args.q} fp8={args.fp8}: {dt * 1e6:.1f} us per call, "
          f"{args.q / dt:.0f} queries/s", flush=True)


if __name__ == "__main__":
    main()
