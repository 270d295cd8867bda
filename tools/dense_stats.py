"""Diagnostic (library built with -DIRC_SCAN_STAMPS, loaded via IRC_LIB_PATH):
how many select_dense blocks rescanned workers, per scan_topk call."""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "information-retrieval-with-contrastive-learning_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=100_000)
    ap.add_argument("--d", type=int, default=768)
    ap.add_argument("--k", type=int, default=100)
    ap.add_argument("--q", type=int, nargs="*", default=[1, 64, 128])
    ap.add_argument("--fp8", action="store_true")
    args = ap.parse_args()
    from irc_amd import _lib, retrieval

    lib = _lib.load()
    dev = torch.device("cuda:0")
    g = torch.Generator().manual_seed(2024)
    docs = torch.nn.functional.normalize(torch.randn(args.n, args.d, generator=g)).bfloat16().to(dev)
    if args.fp8:
        docs = retrieval.quantize_fp8(docs)
    buf = np.zeros((4, 32), dtype=np.uint64)
    for q in args.q:
        qq = torch.nn.functional.normalize(torch.randn(q, args.d, generator=g)).bfloat16().to(dev)
        if args.fp8:
            qq = retrieval.quantize_fp8(qq)
        lib.irc_scan_dbg_stamps(buf.ctypes.data_as(ctypes.c_void_p))
        before = buf[3, 28:32].copy()
        reps = 10
        for _ in range(reps):
            if args.fp8:
                retrieval.scan_topk_fp8(qq, docs, args.k, 0, 1 / 256)
            else:
                retrieval.scan_topk(qq, docs, args.k)
        torch.cuda.synchronize()
        lib.irc_scan_dbg_stamps(buf.ctypes.data_as(ctypes.c_void_p))
        d = (buf[3, 28:32] - before) / reps
        print(f"{'fp8 ' if args.fp8 else ''}Q={q}: LTOP insertion steps (wave 0, blocks < 256) "
              f"per call {d[0]:.0f}; rescanned workers per call "
              f"{d[2]:.2f}, queries with a rescan per call {d[3]:.2f}", flush=True)


if __name__ == "__main__":
    main()
