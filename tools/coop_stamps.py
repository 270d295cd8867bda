"""Per-step phase stamps of the cluster LSTM forward (block 0 = member 0 of cluster 0,
direction 0, wave 0), from the diagnostic build
`tools/build_variant.sh coopstamps lstm_coop.hip -DIRC_COOP_STAMPS`:

    IRC_LIB_PATH=.../variants/coopstamps.so python tools/coop_stamps.py

Phases of one step: MFMA issue, the first barrier (every wave's MFMAs and h reads),
cell update + publish, the gather sweep (waiting for the other three members), the
gathered h into LDS + saves, the last barrier.  Mean shader cycles and ns over the
middle steps, and the clock."""
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
    a = ap.parse_args()
    from irc_amd import _lib, ops

    B, L, H, nd = 256, 64, 256, 2
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    whh = torch.randn(nd * 4 * H, H, device=dev) * 0.06
    xp = torch.randn(B * L, nd * 4 * H, device=dev) * 0.5
    wf, wb = ops.lstm_coop_pack(whh, H, nd)
    for _ in range(a.iters):
        h, g, c, hp, sync = ops.lstm_fwd_coop(xp, wf, B, L, H, nd, save=True)
    torch.cuda.synchronize()
    lib = _lib.load()
    buf = (ctypes.c_uint64 * (64 * 7 * 2))()
    if lib.irc_coop_dbg_stamps(buf) != 0:
        raise SystemExit("irc_coop_dbg_stamps failed (not the stamps build?)")
    st = [[(buf[(s * 7 + p) * 2], buf[(s * 7 + p) * 2 + 1]) for p in range(7)] for s in range(L)]
    names = ["MFMA issue", "barrier 1", "cell update + publish", "gather sweep",
             "h to LDS + saves", "barrier 2"]
    mid = range(2, L - 2)
    cyc = [0.0] * 6
    ns = [0.0] * 6
    for s in mid:
        for p in range(6):
            cyc[p] += st[s][p + 1][0] - st[s][p][0]
            ns[p] += (st[s][p + 1][1] - st[s][p][1]) * 10.0
    n = len(mid)
    tot_c = sum(st[s + 1][0][0] - st[s][0][0] for s in mid) / n
    tot_ns = sum(st[s + 1][0][1] - st[s][0][1] for s in mid) * 10.0 / n
    print(f"cluster forward, B = {B}, block 0 wave 0, mean over {n} steps")
    for p in range(6):
        print(f"  {names[p]:24s} {cyc[p] / n:8.0f} cycles {ns[p] / n:8.0f} ns")
    print(f"  step {tot_c:8.0f} cycles {tot_ns:8.0f} ns  clock {tot_c / tot_ns:.2f} GHz")


if __name__ == "__main__":
    main()
