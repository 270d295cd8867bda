"""Wave-tail form of the big-tile GEMM against the plain form on the BERT shapes at
M = 512 L (a C2 micro-batch of 256 pairs jointly padded to L).

    python tools/tail_bench.py [--lens 64,65,66,68,72] [--iters 30]

One line per (L, shape): the tail plan (whole-tile rows, tail tiles x K pieces) and
us per launch with the tail form on and off (HIP events on the launch stream,
interleaved)."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "information-retrieval-with-contrastive-learning_amd"))

import torch  # noqa: E402

SHAPES = [("qkv", 2304, 768, 1), ("out+res", 768, 768, 3), ("ffn1+gelu", 3072, 768, 2),
          ("ffn2+res", 768, 3072, 3)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lens", default="64,65,66,68,72")
    ap.add_argument("--iters", type=int, default=30)
    a = ap.parse_args()
    from irc_amd import ops

    dev = torch.device("cuda:0")
    for L in (int(v) for v in a.lens.split(",")):
        M = 512 * L
        for name, N, K, epi in SHAPES:
            x = (torch.randn(M, K, device=dev) * 0.5).bfloat16()
            w = (torch.randn(N, K, device=dev) / K ** 0.5).bfloat16()
            bias = torch.randn(N, device=dev)
            res = torch.randn(M, N, device=dev).bfloat16() if epi == 3 else None
            plan = ops.gemm_tail_plan(M, N, K)
            t = {True: [], False: []}
            for it in range(a.iters + 3):
                for on in (True, False):
                    ops.gemm_set_tail(on)
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    ops.gemm(x, w, bias=bias, epilogue=epi, residual=res)
                    e1.record()
                    e1.synchronize()
                    if it >= 3:
                        t[on].append(e0.elapsed_time(e1) * 1e3)
            ops.gemm_set_tail(True)
            med = {k: sorted(v)[len(v) // 2] for k, v in t.items()}
            print(f"L={L:3d} {name:10s} M={M:6d} plan={plan}  tail {med[True]:7.1f} us  "
                  f"plain {med[False]:7.1f} us", flush=True)


if __name__ == "__main__":
    main()
