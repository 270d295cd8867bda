"""Fused InfoNCE kernels alone (csrc/nce_fused.hip): forward (partials + combine)
and backward (partials + reduce) timed with HIP events on the launch stream, at
the C2 / C3 / C4 global batches (N = 256 / 1024 / 2048, D = 128, 12544-key
queue), against the exact-fp32 MFMA peak on the algorithmic flops.

    python tools/nce_bench.py [--iters 20]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "information-retrieval-with-contrastive-learning_amd"))

import torch  # noqa: E402

FP32_MFMA_PEAK = 157.3e12  # MI355X dense fp32 matrix


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--n", type=int, nargs="*", default=[256, 1024, 2048])
    ap.add_argument("--d", type=int, default=128)
    ap.add_argument("--k", type=int, default=12544)
    args = ap.parse_args()
    from irc_amd import nce

    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    for n in args.n:
        D, K = args.d, args.k
        F = torch.nn.functional.normalize(torch.randn(2 * n, D, generator=g, device=dev), dim=1)
        qu = torch.nn.functional.normalize(torch.randn(D, K, generator=g, device=dev), dim=0)
        lse = torch.empty(2 * n, device=dev)
        loss_row = torch.empty(2 * n, device=dev)
        gs = torch.ones(1, device=dev)
        # algorithmic flops: S (2N x 2N) and LQ (N x K) once in the forward, recomputed
        # and multiplied back in the backward (2x)
        fl = 2.0 * D * (2 * n * 2 * n + n * K)
        res = {}
        for name, fn in (("fwd", lambda: nce._fused_fwd(F, qu, n, 0.05, 0, n, lse, loss_row)),
                         ("bwd", lambda: nce._fused_bwd(F, qu, lse, n, 0.05, gs, 0, n))):
            for _ in range(3):
                fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.iters):
                fn()
            e1.record()
            torch.cuda.synchronize()
            res[name] = e0.elapsed_time(e1) / args.iters * 1e3
        tf = fl / (res["fwd"] * 1e-6) / 1e12
        tb = 2 * fl / (res["bwd"] * 1e-6) / 1e12
        print(f"N={n:5d} D={D} K={K}: fwd {res['fwd']:7.1f} us ({tf:6.1f} TF/s, "
              f"{tf * 1e12 / FP32_MFMA_PEAK:.0%} of fp32 MFMA)  bwd {res['bwd']:7.1f} us "
              f"({tb:6.1f} TF/s, {tb * 1e12 / FP32_MFMA_PEAK:.0%})", flush=True)


if __name__ == "__main__":
    main()
