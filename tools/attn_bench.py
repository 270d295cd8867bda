"""Attention kernels alone at a fixed token count and growing L (the joint padding of a
batch, contrastive_module.py:38): forward (irc_attention: whole-row MFMA kernel at
L <= 128, streamed keys above), MX-output forward (irc_attention_mx) and backward
(irc_attention_bwd).

    python tools/attn_bench.py [--tokens 32768] [--h 768] [--iters 20]

Prints us per call (HIP events on the launch stream) and the algorithmic rate:
flops 4 B L^2 H forward (S = Q K^T and P V), 8 B L^2 H backward (dP, dV, dK, dQ;
the recomputed S's not counted), against the 2.5 PF bf16 dense peak.
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "information-retrieval-with-contrastive-learning_amd"))

import torch  # noqa: E402


def timed(fn, iters):
    for _ in range(3):
        fn()
    st = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(iters):
        fn()
    e1.record(st)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=32768)
    ap.add_argument("--h", type=int, default=768)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--lens", default="64,96,100,128,129,192,256,384,512")
    a = ap.parse_args()
    from irc_amd import ops

    dev = torch.device("cuda:0")
    H = a.h
    heads = H // 64
    for L in (int(x) for x in a.lens.split(",")):
        B = max(1, a.tokens // L)
        qkv = torch.randn(B * L, 3 * H, device=dev).bfloat16()
        mask = torch.ones(B, L, dtype=torch.int64, device=dev)
        mask[1::2, L * 3 // 4:] = 0
        ctx = torch.empty(B * L, H, dtype=torch.bfloat16, device=dev)
        dctx = torch.randn(B * L, H, device=dev).bfloat16()
        fl = 4.0 * B * L * L * H
        fwd = timed(lambda: ops.attention(qkv, mask, B, L, H, heads, out=ctx), a.iters)
        mx = timed(lambda: ops.attention_mx(qkv, mask, B, L, H, heads), a.iters)
        bwd = timed(lambda: ops.attention_bwd(qkv, mask, ctx, dctx, B, L, H, heads), a.iters)
        print(f"L={L:4d} B={B:4d}  fwd {fwd:8.1f} us {fl / fwd / 1e6:6.1f} TF/s ({fl / fwd / 2.5e9:.3f})"
              f"  mx {mx:8.1f} us  bwd {bwd:8.1f} us {2 * fl / bwd / 1e6:6.1f} TF/s"
              f" ({2 * fl / bwd / 2.5e9:.3f})", flush=True)


if __name__ == "__main__":
    main()
