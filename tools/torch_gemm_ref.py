"""Calibration only: torch.matmul (hipBLASLt) on the BERT-base GEMM shapes of the
training step, next to irc_gemm, so the headroom of the hand-written kernels is
known.  Nothing in the package calls torch.matmul.

    python tools/torch_gemm_ref.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "information-retrieval-with-contrastive-learning_amd"))

import torch  # noqa: E402

SHAPES = [  # name, M, N, K (C = A[M,K] . B[N,K]^T)
    ("qkv", 32768, 2304, 768),
    ("attn_out", 32768, 768, 768),
    ("ffn1", 32768, 3072, 768),
    ("ffn2", 32768, 768, 3072),
    ("dx_ffn2", 16384, 3072, 768),
    ("square4k", 4096, 4096, 4096),
]


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


TN_SHAPES = [  # dW = A^T B, A [K, M], B [K, N] (both K-outer), batched over layers
    ("dW_ffn1 x12", 12, 3072, 768, 16384),
    ("dW_qkv x12", 12, 2304, 768, 16384),
    ("dW_o x12", 12, 768, 768, 16384),
    ("tn4k", 1, 4096, 4096, 4096),
]


def main():
    from irc_amd import ops

    dev = torch.device("cuda:0")
    for name, L, M, N, K in TN_SHAPES:
        a = torch.randn(L, K, M, device=dev).bfloat16()
        b = torch.randn(L, K, N, device=dev).bfloat16()
        fl = 2.0 * L * M * N * K
        t_ref = timeit(lambda: torch.bmm(a.transpose(1, 2), b), reps=5)
        out = torch.zeros(M, N, device=dev)
        t_irc = timeit(lambda: [ops.gemm(a[i], b[i], trans_a=True, b_is_nk=False, out=out,
                                         accumulate=True) for i in range(L)], reps=5)
        print(f"{name:12s} M={M:5d} N={N:5d} K={K:5d}  torch {t_ref:8.1f} us "
              f"{fl / t_ref / 1e6:6.0f} TF   irc(per-layer calls) {t_irc:8.1f} us "
              f"{fl / t_irc / 1e6:6.0f} TF", flush=True)
    for name, M, N, K in SHAPES:
        a = torch.randn(M, K, device=dev).bfloat16()
        b = torch.randn(N, K, device=dev).bfloat16()
        fl = 2.0 * M * N * K
        t_ref = timeit(lambda: torch.matmul(a, b.t()))
        t_irc = timeit(lambda: ops.gemm(a, b))
        print(f"{name:10s} M={M:6d} N={N:5d} K={K:5d}  torch {t_ref:7.1f} us {fl / t_ref / 1e6:6.0f} TF"
              f"   irc {t_irc:7.1f} us {fl / t_irc / 1e6:6.0f} TF", flush=True)


if __name__ == "__main__":
    main()
