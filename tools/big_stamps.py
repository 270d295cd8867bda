"""Per-K-tile phase stamps of the big-tile GEMM's 16x16x32 main loop (block 0, wave 0),
from the diagnostic build `tools/build_variant.sh bigstamps gemm.hip -DIRC_BIG_STAMPS`:

    IRC_LIB_PATH=.../variants/bigstamps.so python tools/big_stamps.py [--shape ffn2]

Phases of one K-tile: DMA issue (next K-tile), fragment reads + MFMA issue, the vmcnt(0)
wait, the barrier.  Prints the mean shader cycles and ns of each phase over the middle
K-tiles, the clock (shader cycles / realtime), and the K-tile total.
"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "information-retrieval-with-contrastive-learning_amd"))

import torch  # noqa: E402

SHAPES = {"qkv": (32768, 2304, 768, 1), "out": (32768, 768, 768, 3), "ffn2": (32768, 768, 3072, 3),
          "ffn1": (32768, 3072, 768, 2)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="ffn2")
    ap.add_argument("--iters", type=int, default=200)
    a = ap.parse_args()
    from irc_amd import _lib, ops

    M, N, K, epi = SHAPES[a.shape]
    dev = torch.device("cuda:0")
    x = torch.randn(M, K, device=dev).bfloat16()
    w = torch.randn(N, K, device=dev).bfloat16()
    b = torch.randn(N, device=dev)
    r = torch.randn(M, N, device=dev).bfloat16() if epi == 3 else None
    out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    os.environ.setdefault("IRC_GEMM_PP", "0")
    for _ in range(a.iters):  # >= a second of back-to-back launches: the loaded clock
        ops.gemm(x, w, bias=b, epilogue=epi, residual=r, out=out)
    torch.cuda.synchronize()
    lib = _lib.load()
    buf = (ctypes.c_uint64 * (64 * 5 * 2))()
    if lib.irc_big_dbg_stamps(buf) != 0:
        raise SystemExit("irc_big_dbg_stamps failed (not the stamps build?)")
    nk = K // 64
    st = [[(buf[(kt * 5 + p) * 2], buf[(kt * 5 + p) * 2 + 1]) for p in range(5)] for kt in range(min(nk, 64))]
    names = ["dma issue", "frags + mfma issue", "vmcnt(0)", "barrier"]
    mid = range(1, min(nk, 64) - 1)
    cyc = [0.0] * 4
    ns = [0.0] * 4
    tot_c = tot_n = 0.0
    for kt in mid:
        for p in range(4):
            cyc[p] += st[kt][p + 1][0] - st[kt][p][0]
            ns[p] += (st[kt][p + 1][1] - st[kt][p][1]) * 10.0
        nxt = st[kt + 1][0] if kt + 1 < len(st) else st[kt][4]
        tot_c += nxt[0] - st[kt][0][0]
        tot_n += (nxt[1] - st[kt][0][1]) * 10.0
    n = len(mid)
    print(f"{a.shape}: M={M} N={N} K={K}, {nk} K-tiles, block 0 wave 0, mean over {n} middle K-tiles")
    for p in range(4):
        print(f"  {names[p]:20s} {cyc[p] / n:8.0f} cycles {ns[p] / n:8.0f} ns")
    print(f"  K-tile total        {tot_c / n:8.0f} cycles {tot_n / n:8.0f} ns  "
          f"clock {tot_c / tot_n:.2f} GHz; MFMA floor 3072 cycles (192 x 16 per SIMD)")


if __name__ == "__main__":
    main()
