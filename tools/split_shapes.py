"""Every split-K-capable GEMM of the C2 training step (bench.py --part train): shape,
caller and the split workspace under the default cap and under a cap of 128 blocks.
Diagnostic for the split-K block budget.

    python tools/split_shapes.py
"""
import argparse
import collections
import os
import sys
import traceback

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "information-retrieval-with-contrastive-learning_amd"))

import bench  # noqa: E402
from irc_amd import _lib, ops  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    lib = _lib.load()
    seen = collections.OrderedDict()
    orig = ops._splitk_ws

    def spy(a, out, epilogue, M, N, K, batch, max_blocks=0):
        fr = [f for f in traceback.extract_stack()[:-1] if "irc_amd/ops.py" not in f.filename][-1]
        key = (ops._code(a), ops._code(out), int(epilogue), M, N, K, batch, int(max_blocks),
               f"{os.path.basename(fr.filename)}:{fr.lineno}")
        seen[key] = seen.get(key, 0) + 1
        return orig(a, out, epilogue, M, N, K, batch, max_blocks)

    ops._splitk_ws = spy
    args = argparse.Namespace(steps=2, warmup=1, gpus=1)
    bench.run_train(args, 0, 1, dev)
    torch.cuda.synchronize()
    print("in out epi M N K batch cap caller calls  ws(cap) ws(cap or 128)")
    for (ci, co, e, M, N, K, b, mb, where), n in seen.items():
        w0 = lib.irc_gemm_workspace_ex(ci, co, e, M, N, K, b, mb)
        w1 = lib.irc_gemm_workspace_ex(ci, co, e, M, N, K, b, mb or 128)
        flag = "  <- differs" if w0 != w1 else ""
        print(f"{ci} {co} {e} {M} {N} {K} {b} {mb} {where} {n}  {w0} {w1}{flag}")


if __name__ == "__main__":
    main()
