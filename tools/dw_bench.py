"""The LSTM heads' weight-gradient GEMMs at C2 (B L = 16384 tokens, both directions as
one batched call, K-outer x K-outer, fp32 accumulate into the flat gradient), exactly as
lstm_head._layer_bwd_mfma issues them: us per launch (HIP events).

    python tools/dw_bench.py [--iters 20]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "information-retrieval-with-contrastive-learning_amd"))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    from irc_amd import ops

    dev = torch.device("cuda:0")
    BL, H, nd = 16384, 256, 2
    dg = torch.randn(BL, nd * 4 * H, device=dev).bfloat16()
    st = torch.cuda.current_stream()
    for name, In in (("dW_ih l0", 768), ("dW_ih l1", 512), ("dW_hh", None)):
        if In is None:
            x = torch.randn(nd, BL, H, device=dev).bfloat16()
            g = torch.zeros(nd * 4 * H * H, device=dev)
            run = lambda: ops.gemm_strided(dg, x, g, M=4 * H, N=H, K=BL, batch=nd, lda=nd * 4 * H,
                                           sA=4 * H, ldb=H, sB=BL * H, ldc=H, sC=4 * H * H,
                                           trans_a=True, b_is_nk=False, accumulate=True)
            n = H
        else:
            x = torch.randn(BL, In, device=dev).bfloat16()
            g = torch.zeros(nd * 4 * H * In, device=dev)
            run = lambda: ops.gemm_strided(dg, x, g, M=4 * H, N=In, K=BL, batch=nd, lda=nd * 4 * H,
                                           sA=4 * H, ldb=x.stride(0), sB=0, ldc=In, sC=4 * H * In,
                                           trans_a=True, b_is_nk=False, accumulate=True)
            n = In
        for _ in range(3):
            run()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(a.iters):
            run()
        e1.record(st)
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / a.iters
        tf = 2.0 * nd * 4 * H * n * BL / us / 1e6
        print(f"{name:9s} M={4 * H} N={n} K={BL} batch={nd}  {us:8.1f} us  {tf:6.1f} TF/s  "
              f"{tf / 2500:.1%}", flush=True)


if __name__ == "__main__":
    main()
