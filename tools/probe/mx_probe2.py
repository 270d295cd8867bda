"""tools/probe/mx_probe2.so: per data lane, the scale lanes that govern its bytes
(and how many of its 32 bytes each governs)."""
import ctypes
import os

import numpy as np
import torch

lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "mx_probe2.so"))
torch.zeros(1, device="cuda")
for mode in (0, 1):
    out = torch.zeros(64 * 64, device="cuda")
    assert lib.mx_probe2(ctypes.c_void_p(out.data_ptr()), mode) == 0
    c = out.cpu().numpy().reshape(64, 64)
    cnt = np.round((c - 32.0) / 1023.0).astype(int)
    print(f"mode {'A' if mode == 0 else 'B'}:")
    for l in range(64):
        gov = {int(T): int(cnt[l, T]) for T in np.nonzero(cnt[l])[0]}
        print(f"  data lane {l:2d}: {gov}")
