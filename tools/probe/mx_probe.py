"""Run tools/probe/mx_probe.so and print, per data lane, which C rows/cols got the
data and log2 of the applied scale (= the lane whose scale byte was used - 32)."""
import ctypes
import os

import numpy as np
import torch

lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "mx_probe.so"))
torch.zeros(1, device="cuda")
for mode in (0, 1):
    for opsel in (0, 1, 3):
        out = torch.zeros(64 * 256, device="cuda")
        assert lib.mx_probe(ctypes.c_void_p(out.data_ptr()), mode, opsel) == 0
        c = out.cpu().numpy().reshape(64, 16, 16)
        rows = []
        for w in range(64):
            nz = np.argwhere(c[w] != 0)
            if mode == 0:
                r = sorted(set(nz[:, 0].tolist()))
            else:
                r = sorted(set(nz[:, 1].tolist()))
            vals = sorted(set(np.round(np.log2(np.abs(c[w][c[w] != 0]) / 32.0), 3).tolist()))
            rows.append((w, r, [v + 32 for v in vals]))
        print(f"mode {'A' if mode == 0 else 'B'} opsel {opsel}:")
        for w, r, v in rows:
            print(f"  lane {w:2d}: {'rows' if mode == 0 else 'cols'} {r} scale-lane {v}")
