"""Cluster LSTM recurrences alone at the C2 head shapes (B = 256, L = 64, H = 256, BiLSTM):
forward (with saves, as the query encoder) and backward, us per launch (HIP events on the
launch stream), with the library knobs given as A/B pairs of environment settings.

    python tools/lstm_coop_bench.py [--iters 20] [--ab IRC_LSTM_COOP_SENTINELS=1,IRC_LSTM_COOP_SENTINELS=0]

The knobs are read by the library per call, so the variants interleave in one process.
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "information-retrieval-with-contrastive-learning_amd"))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--b", type=int, default=256)
    ap.add_argument("--l", type=int, default=64)
    ap.add_argument("--ab", default="IRC_LSTM_COOP_SENTINELS=1,IRC_LSTM_COOP_SENTINELS=0")
    a = ap.parse_args()
    from irc_amd import ops

    dev = torch.device("cuda:0")
    B, L, H, nd = a.b, a.l, 256, 2
    torch.manual_seed(0)
    whh = torch.randn(nd * 4 * H, H, device=dev) * 0.06
    xp = torch.randn(B * L, nd * 4 * H, device=dev) * 0.5
    dy = torch.randn(B * L, nd * H, device=dev) * 0.1
    wf, wb = ops.lstm_coop_pack(whh, H, nd)
    variants = [v.split("=", 1) for v in a.ab.split(",") if v]
    ref = None
    for rnd in range(2):
        for k, v in variants:
            os.environ[k] = v
            h, g, c, hp, sync = ops.lstm_fwd_coop(xp, wf, B, L, H, nd, save=True)
            dg, sync_b = ops.lstm_bwd_coop(dy, wb, g, c, B, L, H, nd)
            assert not ops.lstm_coop_timed_out(sync, B, nd)
            assert not ops.lstm_coop_timed_out(sync_b, B, nd)
            if ref is None:
                ref = (h.clone(), dg.clone())
            same = torch.equal(ref[0], h) and torch.equal(ref[1], dg)
            st = torch.cuda.current_stream()
            out = []
            for name, fn in (("fwd", lambda: ops.lstm_fwd_coop(xp, wf, B, L, H, nd, save=True)),
                             ("bwd", lambda: ops.lstm_bwd_coop(dy, wb, g, c, B, L, H, nd))):
                for _ in range(3):
                    fn()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                for _ in range(a.iters):
                    fn()
                e1.record(st)
                torch.cuda.synchronize()
                us = e0.elapsed_time(e1) * 1e3 / a.iters
                out.append(f"{name} {us:7.1f} us ({us / L:5.2f} us/step)")
            print(f"round {rnd} {k}={v:4s} " + "  ".join(out) + f"  bit-identical to first: {same}",
                  flush=True)
        for k, _ in variants:
            os.environ.pop(k, None)


if __name__ == "__main__":
    main()
