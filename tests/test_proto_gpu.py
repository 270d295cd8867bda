"""ProtoNCE on the GPU (irc_amd.cluster): the prototype loss against the
reference's own _compute_proto_loss run on the same inputs and the same
negative-prototype draw (tests/golden/proto.npz, make_proto_goldens.py), and the
k-means invariants (faiss, the reference's clustering library, is absent: the
clustering itself is parity-unpinned)."""
import random

import numpy as np
import pytest
import torch

from conftest import load_golden

pytestmark = pytest.mark.gpu


def test_proto_loss_matches_reference(gpu):
    from src.contrastor.contrastive_loss import NCELoss

    g = load_golden("proto.npz")
    ks = [int(x) for x in g["ks"]]
    crit = NCELoss({"temperature": 0.05,
                    "cluster": {"num_cluster": ks, "num_neg_proto": int(g["num_neg_proto"])}})
    res = {"centroids": [], "density": [], "emb2cluster": []}
    for n in range(len(ks)):
        res["centroids"].append(torch.from_numpy(g[f"centroids_{n}"]).to(gpu))
        res["density"].append(torch.from_numpy(g[f"density_{n}"]).to(gpu))
        res["emb2cluster"].append(torch.from_numpy(g[f"emb2cluster_{n}"]).to(gpu))
    q = torch.from_numpy(g["q"]).to(gpu).requires_grad_(True)
    random.seed(int(g["seed"]))  # the reference's draw was made right after this seed
    loss = crit._compute_proto_loss(q, res, torch.from_numpy(g["index"]).to(gpu))
    loss.backward()
    np.testing.assert_allclose(loss.item(), float(g["loss"]), rtol=1e-5)
    np.testing.assert_allclose(q.grad.cpu().numpy(), g["dq"], rtol=1e-4, atol=1e-5)


def test_kmeans_lloyd_invariants(gpu):
    from irc_amd import cluster

    rng = np.random.default_rng(0)
    k, D, per = 16, 32, 200
    centers = rng.standard_normal((k, D)) * 4
    x = (centers[:, None, :] + rng.standard_normal((k, per, D))).reshape(-1, D).astype(np.float32)
    c, idx, dist = cluster.kmeans(torch.from_numpy(x).to(gpu), k, niter=15, nredo=3, seed=1)
    c, idx, dist = c.cpu().numpy(), idx.cpu().numpy(), dist.cpu().numpy()
    d2 = ((x[:, None, :] - c[None, :, :]) ** 2).sum(-1)
    # assignment = nearest centroid (up to fp32 ties), distances = squared L2
    np.testing.assert_allclose(d2[np.arange(len(x)), idx], d2.min(1), rtol=1e-4, atol=1e-3)
    np.testing.assert_allclose(dist, d2[np.arange(len(x)), idx], rtol=1e-4, atol=1e-2)
    # Lloyd never increases the objective: more iterations from the same start
    xt = torch.from_numpy(x).to(gpu)
    objs = [float(cluster.kmeans(xt, k, niter=it, nredo=1, seed=5)[2].sum().item())
            for it in (1, 3, 10)]
    assert objs[0] >= objs[1] * (1 - 1e-5) and objs[1] >= objs[2] * (1 - 1e-5), objs
    # well-separated blobs: most of each blob in one cluster (random init may merge two)
    labels = np.repeat(np.arange(k), per)
    purity = sum(np.bincount(idx[labels == b]).max() for b in range(k)) / len(x)
    assert purity > 0.85


def test_run_kmeans_results_shape(gpu):
    from src.contrastor.utils import kmeans_results

    rng = np.random.default_rng(1)
    x = rng.standard_normal((600, 16)).astype(np.float32)
    x /= np.linalg.norm(x, axis=1, keepdims=True)
    cfg = {"temperature": 0.05, "cluster": {"num_cluster": [8, 12], "niter": 5, "nredo": 2,
                                            "max_points_per_centroid": 1000}}
    res = kmeans_results(cfg, x, gpu)
    for n, k in enumerate([8, 12]):
        assert res["centroids"][n].shape == (k, 16)
        assert torch.allclose(res["centroids"][n].norm(dim=1),
                              torch.ones(k, device=gpu), atol=1e-5)
        assert res["emb2cluster"][n].shape == (600,)
        d = res["density"][n].cpu().numpy()
        assert abs(d.mean() - 0.05) < 1e-6 and np.all(d > 0)
