"""Run-to-run reproducibility of the cluster LSTM recurrences at the C2 head shapes: the same
inputs through lstm_fwd_coop / lstm_bwd_coop N times per hand-off form; prints how many
outputs differ bitwise from the first call and the largest difference, per form, and the
distance of each form from the single-CU MFMA recurrence.

    python tools/lstm_coop_repro.py [--n 8]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "information-retrieval-with-contrastive-learning_amd"))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=8)
    ap.add_argument("--b", type=int, default=256)
    ap.add_argument("--l", type=int, default=64)
    a = ap.parse_args()
    from irc_amd import ops

    dev = torch.device("cuda:0")
    B, L, H, nd = a.b, a.l, 256, 2
    torch.manual_seed(0)
    whh = torch.randn(nd * 4 * H, H, device=dev) * 0.06
    xp = torch.randn(B * L, nd * 4 * H, device=dev) * 0.5
    dy = torch.randn(B * L, nd * H, device=dev) * 0.1
    wf, wb = ops.lstm_coop_pack(whh, H, nd)
    h0, g, c, hp, sync = ops.lstm_fwd_coop(xp, wf, B, L, H, nd, save=True)
    nh = 0
    for _ in range(a.n):
        h, *_ = ops.lstm_fwd_coop(xp, wf, B, L, H, nd, save=True)
        nh += int(not torch.equal(h, h0))
    print(f"fwd: {nh} of {a.n} calls differ from the first", flush=True)
    firsts = {}
    for form in ("0", "1", "2"):
        os.environ["IRC_LSTM_COOP_BWD_TAGGED"] = form
        d0, s0 = ops.lstm_bwd_coop(dy, wb, g, c, B, L, H, nd)
        assert not ops.lstm_coop_timed_out(s0, B, nd)
        firsts[form] = d0
        bad, worst = 0, 0.0
        for _ in range(a.n):
            d, s = ops.lstm_bwd_coop(dy, wb, g, c, B, L, H, nd)
            assert not ops.lstm_coop_timed_out(s, B, nd)
            if not torch.equal(d, d0):
                bad += 1
                worst = max(worst, (d.float() - d0.float()).abs().max().item())
        print(f"bwd tagged={form}: {bad} of {a.n} calls differ from the first (max |diff| {worst:.3e})",
              flush=True)
    os.environ.pop("IRC_LSTM_COOP_BWD_TAGGED")
    for other in ("1", "2"):
        d01 = (firsts["0"].float() - firsts[other].float()).abs()
        print(f"bwd form 0 vs {other}: {int((d01 > 0).sum())} elements differ, max "
              f"{d01.max().item():.3e}", flush=True)
    # the single-CU recurrence on the same W_hh (its own packing) as the outside reference
    wih = torch.zeros(nd * 4 * H, 64, device=dev)
    bz = torch.zeros(nd * 4 * H, device=dev)
    _, _, w, wT = ops.lstm_pack(wih, bz, bz, whh, H, nd)
    hm, gm, cm, _ = ops.lstm_fwd_mfma(xp, w, B, L, H, nd, save=True)
    dm = ops.lstm_bwd_mfma(dy, wT, gm, cm, B, L, H, nd)
    for form, d in firsts.items():
        err = ((d.float() - dm.float()).norm() / dm.float().norm()).item()
        print(f"bwd tagged={form} vs single-CU: rel Frobenius {err:.3e}", flush=True)


if __name__ == "__main__":
    main()
