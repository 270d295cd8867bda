"""Scan filter microbenchmark: C2 corpus (100k x 768 bf16), Q in {1,16,64,256}.

    python tools/scan_bench.py [--n 100000] [--reps 30]

Prints per Q: filter kernel us (HIP events via the library's profiler), its
algorithmic GB/s (N*D*2 + Q*D*2) and HBM fraction, and the whole call's us."""
import argparse
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "information-retrieval-with-contrastive-learning_amd"))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=100_000)
    ap.add_argument("--d", type=int, default=768)
    ap.add_argument("--k", type=int, default=100)
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--q", type=int, nargs="*", default=[1, 16, 64, 256])
    ap.add_argument("--fp8", action="store_true", help="e4m3 corpus and queries")
    args = ap.parse_args()
    from irc_amd import _lib, retrieval

    lib = _lib.load()
    dev = torch.device("cuda:0")
    g = torch.Generator().manual_seed(2024)
    docs = torch.nn.functional.normalize(torch.randn(args.n, args.d, generator=g)).bfloat16().to(dev)
    search = retrieval.scan_topk
    if args.fp8:
        docs = retrieval.quantize_fp8(docs)
        search = lambda qq, dd, k: retrieval.scan_topk_fp8(qq, dd, k, 0, 1 / 256)  # noqa: E731
    eb = 1 if args.fp8 else 2
    for q in args.q:
        qq = torch.nn.functional.normalize(torch.randn(q, args.d, generator=g)).bfloat16().to(dev)
        if args.fp8:
            qq = retrieval.quantize_fp8(qq)
        for _ in range(3):
            search(qq, docs, args.k)
        torch.cuda.synchronize()
        lib.irc_prof_reset()
        lib.irc_prof_enable(1)
        t0 = time.perf_counter()
        for _ in range(args.reps):
            search(qq, docs, args.k)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / args.reps
        lib.irc_prof_enable(0)
        tot, cnt, work = ctypes.c_double(0), ctypes.c_int64(0), ctypes.c_double(0)
        lib.irc_prof_query(b"scan_filter", ctypes.byref(tot), ctypes.byref(cnt), ctypes.byref(work))
        us = tot.value * 1e3 / max(cnt.value, 1)
        gbs = work.value / max(cnt.value, 1) / (us * 1e-6) / 1e9
        print(f"{'fp8 ' if args.fp8 else ''}Q={q:4d} filter {us:7.1f} us  {gbs:7.0f} GB/s  {gbs / 8000:.1%} of HBM   call "
              f"{dt * 1e6:7.1f} us", flush=True)


if __name__ == "__main__":
    main()
