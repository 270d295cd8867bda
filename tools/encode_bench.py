"""Frozen-encoder forward alone (BERT-base, C2 micro-batch: 2 x 256 sequences x
L = 64), bf16 against MX-fp8 weights, with the per-kernel split from the
library's profiler (HIP events per launch; the profiled pass is separate from the
clean timing).

    python tools/encode_bench.py [--iters 20] [--batch 512] [--large]
"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "information-retrieval-with-contrastive-learning_amd"))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--seq", type=int, default=64)
    ap.add_argument("--large", action="store_true")
    args = ap.parse_args()
    from irc_amd import _lib
    from irc_amd.bert import BertConfig, BertModel

    lib = _lib.load()
    dev = torch.device("cuda:0")
    cfg = BertConfig(hidden_size=1024, num_hidden_layers=24, num_attention_heads=16,
                     intermediate_size=4096) if args.large else BertConfig()
    torch.manual_seed(0)
    m = BertModel(cfg).to(dev).eval()
    g = torch.Generator().manual_seed(1)
    ids = torch.randint(1000, 30000, (args.batch, args.seq), generator=g).to(dev)
    mask = torch.ones_like(ids)
    for fmt in ("bf16", "fp8"):
        m.set_weight_format(fmt)
        with torch.no_grad():
            for _ in range(3):
                m.encode(ids, mask)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.iters):
                m.encode(ids, mask)
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / args.iters
            lib.irc_prof_reset()
            lib.irc_prof_enable(1)
            for _ in range(args.iters):
                m.encode(ids, mask)
            torch.cuda.synchronize()
            lib.irc_prof_enable(0)
        print(f"{fmt}: encode {ms:.3f} ms per micro-batch ({args.batch} x {args.seq})", flush=True)
        for k in ("gemm_bf16", "gemm_fp8", "attention", "layernorm"):  # the profiler's tags
            tot, cnt, work = ctypes.c_double(0), ctypes.c_int64(0), ctypes.c_double(0)
            lib.irc_prof_query(k.encode(), ctypes.byref(tot), ctypes.byref(cnt), ctypes.byref(work))
            if cnt.value:
                print(f"   {k:16s} {tot.value / args.iters:8.3f} ms/encode  {cnt.value // args.iters:4d} "
                      f"launches", flush=True)


if __name__ == "__main__":
    main()
