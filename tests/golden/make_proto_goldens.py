"""Golden fixtures for the ProtoNCE prototype loss, made by RUNNING the
reference's NCELoss._compute_proto_loss (src/contrastor/contrastive_loss.py:95-135)
and its autograd on seeded inputs.

  python tests/golden/make_proto_goldens.py

Runs only in the build container (imports /root/reference read-only, with the
stand-ins of make_goldens.py).  The negative prototypes come from Python's
`random.sample` over a set, as in the reference; the fixture records the seed
it was called with (random.seed(SEED) right before the call) so the product
replays the same draw.  Saved: q, per-set centroids / density / emb2cluster,
index, the loss and dL/dq (proto.npz).
"""
from __future__ import annotations

import os
import random
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_goldens import _import_ref  # noqa: E402

SEED = 4242


def main():
    _import_ref()
    from src.contrastor.contrastive_loss import NCELoss

    g = torch.Generator().manual_seed(7)
    B, D, n_emb = 8, 16, 60
    ks, r = [24, 30, 20], 4
    cfg = {"temperature": 0.05, "cluster": {"num_cluster": ks, "num_neg_proto": r}}
    crit = NCELoss(cfg)
    q = torch.nn.functional.normalize(torch.randn(B, D, generator=g), dim=1).requires_grad_(True)
    index = torch.randint(0, n_emb, (B,), generator=g)
    res = {"centroids": [], "density": [], "emb2cluster": []}
    out = {"q": q.detach().numpy(), "index": index.numpy(), "ks": np.array(ks),
           "num_neg_proto": np.array(r), "seed": np.array(SEED)}
    for n, k in enumerate(ks):
        c = torch.nn.functional.normalize(torch.randn(k, D, generator=g), dim=1)
        dens = 0.05 * (0.5 + torch.rand(k, generator=g))
        e2c = torch.randint(0, k, (n_emb,), generator=g)
        res["centroids"].append(c)
        res["density"].append(dens)
        res["emb2cluster"].append(e2c)
        out[f"centroids_{n}"] = c.numpy()
        out[f"density_{n}"] = dens.numpy()
        out[f"emb2cluster_{n}"] = e2c.numpy()
    random.seed(SEED)
    loss = crit._compute_proto_loss(q, res, index)
    loss.backward()
    out["loss"] = np.array(loss.item(), np.float64)
    out["dq"] = q.grad.numpy()
    np.savez_compressed(os.path.join(HERE, "proto.npz"), **out)
    print("wrote proto.npz, loss", loss.item())


if __name__ == "__main__":
    main()
