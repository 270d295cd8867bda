"""LayerNorm [32768, 768] bf16 (the encoder's shape): HIP-event time per launch.

    IRC_LN_ROWS=4 python tools/ln_bench.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "information-retrieval-with-contrastive-learning_amd"))

import torch  # noqa: E402


def main():
    from irc_amd import ops

    dev = torch.device("cuda:0")
    x = torch.randn(32768, 768, device=dev).bfloat16()
    g = torch.rand(768, device=dev) + 0.5
    b = torch.randn(768, device=dev)
    y = torch.empty_like(x)
    for _ in range(5):
        ops.layernorm(x, g, b, 1e-12, out=y)
    st = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(100):
        ops.layernorm(x, g, b, 1e-12, out=y)
    e1.record(st)
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / 100
    print(f"layernorm rows={os.environ.get('IRC_LN_ROWS', '1')}: {us:.2f} us, "
          f"{2 * x.numel() * 2 / us / 1e6:.2f} TB/s", flush=True)


if __name__ == "__main__":
    main()
