"""Compute-precision switch for the MFMA paths.

"bf16" (default, the production mode): bf16 operands, fp32 accumulation and
fp32 state/statistics.  "fp32": exact-fp32 MFMA operands everywhere -- the
parity mode used to pin the kernels against the fp32 reference oracle tightly.
The InfoNCE loss and the optimizer always run in fp32.
"""
from __future__ import annotations

import os

import torch

_MODE = os.environ.get("IRC_PRECISION", "bf16")


def set_precision(mode: str) -> None:
    global _MODE
    if mode not in ("bf16", "fp32"):
        raise ValueError(f"precision must be 'bf16' or 'fp32', got {mode!r}")
    _MODE = mode


def get_precision() -> str:
    return _MODE


def compute_dtype() -> torch.dtype:
    return torch.bfloat16 if _MODE == "bf16" else torch.float32
