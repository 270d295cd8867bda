"""Bit-for-bit comparison of two builds of the library on the BERT GEMM shapes: run once
per build (IRC_LIB_PATH selects the variant) with --save / --check.

    python tools/variant_bitcheck.py --save gpurun_out/base.pt
    IRC_LIB_PATH=.../variants/x.so python tools/variant_bitcheck.py --check gpurun_out/base.pt
    (or an A/B environment switch such as IRC_LN_ROWS=4 instead of IRC_LIB_PATH)
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "information-retrieval-with-contrastive-learning_amd"))

import torch  # noqa: E402

CASES = [("qkv", 32768, 2304, 768, 1), ("out", 32768, 768, 768, 3), ("ffn2", 32768, 768, 3072, 3),
         ("ragged", 32700, 768, 768, 3), ("k64", 4096, 768, 64, 1), ("c4_out", 32768, 1024, 1024, 3),
         ("ffn1", 32768, 3072, 768, 2), ("ffn1_bias", 32768, 3072, 768, 1),
         ("pp_ragged", 4000, 3072, 768, 2)]


def run():
    from irc_amd import ops

    dev = torch.device("cuda:0")
    out = {}
    for name, M, N, K, epi in CASES:
        g = torch.Generator(device=dev).manual_seed(M + N + K)
        a = torch.randn(M, K, device=dev, generator=g).bfloat16()
        b = (torch.randn(N, K, device=dev, generator=g) * 0.05).bfloat16()
        bias = torch.randn(N, device=dev, generator=g)
        r = torch.randn(M, N, device=dev, generator=g).bfloat16() if epi == 3 else None
        if name.startswith("ffn1") or name == "pp_ragged":  # typical pre-activation scale
            b = b * 0.3
        out[name] = ops.gemm(a, b, bias=bias, epilogue=epi, residual=r).cpu()
    for name, rows in (("ln", 32768), ("ln_ragged", 1003)):
        g = torch.Generator(device=dev).manual_seed(rows)
        x = (torch.randn(rows, 768, device=dev, generator=g) * 3 + 1).bfloat16()
        gm = torch.rand(768, device=dev, generator=g) + 0.5
        bt = torch.randn(768, device=dev, generator=g)
        out[name] = ops.layernorm(x, gm, bt, 1e-12).cpu()
    B, L, H = 512, 64, 768
    g = torch.Generator(device=dev).manual_seed(9)
    x = torch.randn(B * L, H, device=dev, generator=g).bfloat16()
    w = (torch.randn(3 * H, H, device=dev, generator=g) * 0.05).bfloat16()
    bq = torch.randn(3 * H, device=dev, generator=g)
    mask = torch.ones(B, L, dtype=torch.int64, device=dev)
    perm = ops.qkv_perm_index(H, dev)
    out["qkv_attn"] = ops.qkv_attention(x, w.index_select(0, perm).contiguous(),
                                        bq.index_select(0, perm).contiguous(), mask, B, L, H,
                                        12).cpu()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--save")
    ap.add_argument("--check")
    a = ap.parse_args()
    out = run()
    if a.save:
        torch.save(out, a.save)
        print("saved", len(out), "outputs")
        return
    ref = torch.load(a.check, weights_only=True)
    bad = [k for k in ref if not torch.equal(ref[k], out[k])]
    for k in ref:
        print(f"{k:10s} {'IDENTICAL' if k not in bad else 'DIFFERENT'}")
    if bad:
        raise SystemExit(f"{len(bad)} outputs differ")


if __name__ == "__main__":
    main()
