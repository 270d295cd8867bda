"""Diagnostic (library built with -DIRC_SCAN_STAMPS, loaded via IRC_LIB_PATH): phase
times of select_dense_kernel's block 0 (query 0) on a C3-sized shard, per Q.
Stamps are s_memrealtime (100 MHz): 16 start, 25 keys loaded + min/max/count, 26/27
radix passes 0/1 done, 17 first dense_kth done, 18 truncated lists flagged, 19 rescan
done, 20 results written; [24] radix passes."""
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
    ap.add_argument("--n", type=int, default=250_000)
    ap.add_argument("--d", type=int, default=768)
    ap.add_argument("--k", type=int, default=100)
    ap.add_argument("--q", type=int, nargs="*", default=[1, 16, 64])
    args = ap.parse_args()
    from irc_amd import _lib, retrieval

    lib = _lib.load()
    dev = torch.device("cuda:0")
    g = torch.Generator().manual_seed(2024)
    docs = torch.nn.functional.normalize(torch.randn(args.n, args.d, generator=g)).bfloat16().to(dev)
    buf = np.zeros((4, 32), dtype=np.uint64)
    for q in args.q:
        qq = torch.nn.functional.normalize(torch.randn(q, args.d, generator=g)).bfloat16().to(dev)
        rows = []
        for _ in range(12):
            retrieval.scan_topk(qq, docs, args.k)
            torch.cuda.synchronize()
            lib.irc_scan_dbg_stamps(buf.ctypes.data_as(ctypes.c_void_p))
            st = buf[2].astype(np.int64)
            rows.append([(st[i] - st[16]) * 10 / 1000 for i in (25, 26, 27, 17, 18, 19, 20)] + [st[24]])
        r = np.array(rows[2:])
        med = np.median(r, axis=0)
        print(f"Q={q}: select_dense block 0 (us from start): loads+minmax {med[0]:.2f}  pass0 {med[1]:.2f}  "
              f"pass1 {med[2]:.2f}  kth {med[3]:.2f}  flags {med[4]:.2f}  "
              f"rescan {med[5]:.2f}  end {med[6]:.2f}  radix passes {med[7]:.0f}", flush=True)


if __name__ == "__main__":
    main()
