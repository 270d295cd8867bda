"""GEMM microbenchmark on the training-step shapes (C2: 2x256 sequences x L=64).

    python tools/gemm_bench.py [--iters 20]

Prints one line per shape: M N K epilogue, us per launch (HIP events on the
launch stream), TFLOP/s and the fraction of the 2.5 PF dense bf16 peak.
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "information-retrieval-with-contrastive-learning_amd"))

import torch  # noqa: E402

SHAPES = [  # (name, M, N, K, epilogue)
    ("qkv", 32768, 2304, 768, 1),
    ("attn_out+res", 32768, 768, 768, 3),
    ("ffn1+gelu", 32768, 3072, 768, 2),
    ("ffn1+bias", 32768, 3072, 768, 1),   # the GELU epilogue's cost = the difference
    ("ffn2+res", 32768, 768, 3072, 3),
    ("lstm_xp_l0", 16384, 2048, 768, 1),
    ("lstm_xp_l12", 16384, 2048, 512, 1),
    ("lstm_dx", 16384, 512, 2048, 0),
    ("square4k", 4096, 4096, 4096, 0),
    ("dW_ih^T", 1024, 768, 16384, -1),   # dg^T x: both operands K-outer, split-K
    ("dW_hh^T", 1024, 256, 16384, -1),
    # trainable BERT-base forward at 256 anchors x L=64 = 16384 rows (epi 6: bias + GELU,
    # pre-activation saved for the backward)
    ("bert_fwd_qkv", 16384, 2304, 768, 1),
    ("bert_fwd_o", 16384, 768, 768, 3),
    ("bert_fwd_ffn1", 16384, 3072, 768, 6),
    ("bert_fwd_ffn2", 16384, 768, 3072, 3),
    # trainable BERT-base backward (256 anchors x L=64 -> 16384 rows)
    ("bert_dx_ffn2", 16384, 3072, 768, 5),   # dU = (dS2 W2) * gelu'(u)
    ("bert_dx_ffn1", 16384, 768, 3072, 4),   # dA = dU W1 + dS2
    ("bert_dx_qkv", 16384, 768, 2304, 4),
    ("bert_dW_ffn1", 3072, 768, 16384, -1),
    ("bert_dW_qkv", 2304, 768, 16384, -1),
    ("bert_dW_o", 768, 768, 16384, -1),
    # scan-shaped (C = Q . Docs^T): one shared 256-row operand vs the roles swapped
    ("scan_q256", 256, 100352, 768, 0),
    ("scan_swap", 100352, 256, 768, 0),
    ("scan_q1024", 1024, 100352, 768, 0),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--layouts", action="store_true")
    ap.add_argument("--only", default="", help="comma-separated shape names")
    ap.add_argument("--mx", action="store_true", help="MX-fp8 GEMMs (irc_gemm_mx) of the BERT shapes")
    ap.add_argument("--mf16", default="", help="big-tile MFMA shape: 0, 1 or 'ab' (interleaved); "
                    "default: the library's setting")
    args = ap.parse_args()
    only = set(filter(None, args.only.split(",")))
    if args.mx:
        return mx_shapes(args)
    from irc_amd import ops

    dev = torch.device("cuda:0")
    if args.layouts:  # 4096^3 mainloop efficiency of every operand layout (bf16 out)
        for ta, nk in ((False, True), (False, False), (True, True), (True, False)):
            M = N = K = 4096
            a = torch.randn((K, M) if ta else (M, K), device=dev).to(torch.bfloat16)
            b = torch.randn((N, K) if nk else (K, N), device=dev).to(torch.bfloat16)
            out = torch.empty((M, N), device=dev, dtype=torch.bfloat16)
            run = lambda: ops.gemm(a, b, trans_a=ta, b_is_nk=nk, out=out)
            for _ in range(3):
                run()
            st = torch.cuda.current_stream()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(args.iters):
                run()
            e1.record(st)
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / args.iters
            tf = 2.0 * M * N * K / us / 1e6
            lay = ("COL" if ta else "ROW") + ("NK" if nk else "KN")
            print(f"square4k {lay:6s} {us:9.1f} us  {tf:7.1f} TF/s  {tf / 2500:.1%}", flush=True)
        return
    for name, M, N, K, epi in SHAPES:
        if only and name not in only:
            continue
        if epi < 0:  # K-outer operands: C[M,N] = A[K,M]^T B[K,N], fp32 accumulate
            a = torch.randn((K, M), device=dev).to(torch.bfloat16)
            b = torch.randn((K, N), device=dev).to(torch.bfloat16)
            out = torch.zeros((M, N), device=dev)
            run = lambda: ops.gemm(a, b, trans_a=True, b_is_nk=False, out=out, accumulate=True)
            for _ in range(3):
                run()
            st = torch.cuda.current_stream()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(args.iters):
                run()
            e1.record(st)
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / args.iters
            tf = 2.0 * M * N * K / us / 1e6
            print(f"{name:14s} M={M:6d} N={N:5d} K={K:5d} COLCOL  {us:9.1f} us  {tf:7.1f} TF/s  "
                  f"{tf / 2500:.1%}", flush=True)
            continue
        a = torch.randn((M, K), device=dev).to(torch.bfloat16)
        b = torch.randn((N, K), device=dev).to(torch.bfloat16)
        bias = torch.randn((N,), device=dev) if epi in (1, 2, 3, 6) else None
        res = torch.randn((M, N), device=dev).to(torch.bfloat16) if epi in (3, 4, 5, 6) else None
        od = torch.float32 if name in ("lstm_dx",) or name.startswith("lstm_xp") else torch.bfloat16
        if name.startswith("scan"):
            od = torch.bfloat16
        if res is not None:
            res = res.to(od)
        out = torch.empty((M, N), device=dev, dtype=od)
        modes = (0, 1, 0, 1) if args.mf16 == "ab" else ((int(args.mf16),) if args.mf16 else (None,))
        prev = None
        for mode in modes:
            if mode is not None:
                p0 = ops.gemm_set_big_mf16(mode)
                prev = p0 if prev is None else prev
            for _ in range(3):
                ops.gemm(a, b, bias=bias, epilogue=epi, residual=res, out=out)
            st = torch.cuda.current_stream()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(args.iters):
                ops.gemm(a, b, bias=bias, epilogue=epi, residual=res, out=out)
            e1.record(st)
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / args.iters
            tf = 2.0 * M * N * K / us / 1e6
            tag = f" mf16={mode}" if mode is not None else ""
            print(f"{name:14s} M={M:6d} N={N:5d} K={K:5d} epi={epi}{tag}  {us:9.1f} us  "
                  f"{tf:7.1f} TF/s  {tf / 2500:.1%}", flush=True)
        if prev is not None:
            ops.gemm_set_big_mf16(prev)


def mx_shapes(args):
    """The frozen encoder's four linear layers on MX-fp8 at M = 32768 (C5): HIP-event
    time per launch and the fraction of the 5 PF dense fp8 peak."""
    from irc_amd import ops

    dev = torch.device("cuda:0")
    for name, M, N, K, epi, omx in (("qkv", 32768, 2304, 768, 1, False),
                                    ("attn_out+res", 32768, 768, 768, 3, False),
                                    ("ffn1+gelu>mx", 32768, 3072, 768, 2, True),
                                    ("ffn1+gelu", 32768, 3072, 768, 2, False),
                                    ("ffn2+res", 32768, 768, 3072, 3, False)):
        a = ops.quantize_mx(torch.randn((M, K), device=dev).to(torch.bfloat16))
        w = ops.quantize_mx(torch.randn((N, K), device=dev) * 0.03)
        bias = torch.randn((N,), device=dev)
        res = torch.randn((M, N), device=dev).to(torch.bfloat16) if epi == 3 else None
        run = lambda: ops.gemm_mx(a, w, bias=bias, epilogue=epi, residual=res, out_mx=omx)  # noqa: E731
        for _ in range(3):
            run()
        st = torch.cuda.current_stream()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(args.iters):
            run()
        e1.record(st)
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / args.iters
        tf = 2.0 * M * N * K / us / 1e6
        print(f"mx {name:14s} M={M:6d} N={N:5d} K={K:5d} epi={epi}  {us:9.1f} us  {tf:7.1f} TF/s  "
              f"{tf / 5000:.1%}", flush=True)


if __name__ == "__main__":
    main()
