"""ProtoNCE / HProtoNCE on the irc HIP kernels.

* ``proto_loss`` -- NCELoss._compute_proto_loss (src/contrastor/
  contrastive_loss.py:95-135): per cluster set the positive prototype of each
  sample (emb2cluster[index]), ``num_neg_proto`` negatives drawn with Python's
  ``random.sample`` over the set {0 .. max(emb2cluster)-1} minus the positives
  exactly as the reference draws them (its off-by-one included: the last
  cluster id is never a negative), logits q . protos^T / density on the exact
  fp32 MFMA GEMM, CrossEntropy(sum) on ``irc_proto_ce``, averaged over the sets.
* ``kmeans`` -- the clustering run_kmeans does with faiss (src/contrastor/
  utils.py:50-110): Lloyd iterations, nredo restarts keeping the lowest
  objective, then nearest-centroid assignment with squared L2 distances.  faiss
  (unpinned in the reference's requirements, absent here) is replaced by the
  same algorithm on irc_gemm + irc_argmax_bias + irc_centroid_*: parity
  unpinned for the clustering itself (its initialisation RNG is faiss's own);
  tests check the Lloyd invariants.
"""
from __future__ import annotations

import random

import numpy as np
import torch

from . import _lib, ops
from ._torch import ptr, require_hip, stream_ptr


class _ProtoCE(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, protos, temp):
        q = q.float().contiguous()
        logits = ops.gemm(q, protos)  # [B, C] = q . protos^T, exact fp32 MFMA
        B, C = logits.shape
        row = torch.empty((B,), dtype=torch.float32, device=q.device)
        _lib.call("irc_proto_ce", ptr(logits), ptr(temp), B, C, ptr(row), None, None,
                  stream_ptr(q.device))
        ctx.save_for_backward(logits, protos, temp)
        return ops.dsum(row)

    @staticmethod
    def backward(ctx, gloss):
        logits, protos, temp = ctx.saved_tensors
        B, C = logits.shape
        g = gloss.reshape(1).float().contiguous()
        dlog = torch.empty_like(logits)
        _lib.call("irc_proto_ce", ptr(logits), ptr(temp), B, C, None, ptr(dlog), ptr(g),
                  stream_ptr(logits.device))
        dq = ops.gemm(dlog, protos, b_is_nk=False)  # [B, C] @ [C, D]
        return dq, None, None


def proto_loss(q, cluster_result, index, num_cluster, num_neg_proto):
    """contrastive_loss.py:95-135 -> 0-d loss with autograd into q."""
    require_hip(q)
    total = None
    for emb2cluster, prototypes, density in zip(cluster_result["emb2cluster"],
                                                cluster_result["centroids"],
                                                cluster_result["density"]):
        pos_proto_id = emb2cluster[index.tolist()]
        all_proto_id = [i for i in range(int(emb2cluster.max()))]
        neg_proto_id = set(all_proto_id) - set(pos_proto_id.tolist())
        neg_proto_id = random.sample(tuple(neg_proto_id), num_neg_proto)
        ids = torch.cat([pos_proto_id.to(q.device),
                         torch.as_tensor(neg_proto_id, dtype=torch.long, device=q.device)])
        protos = prototypes.to(q.device).float()[ids].contiguous()
        temp = density.to(q.device).float()[ids].contiguous()
        part = _ProtoCE.apply(q, protos, temp)
        total = part if total is None else total + part
    return total / len(num_cluster)


def _assign(x, c, bias, chunk=8192):
    """Nearest centroid per row: (idx int64 [n], val fp32 [n] = max x.c - |c|^2/2)."""
    n, k = x.shape[0], c.shape[0]
    idx = torch.empty((n,), dtype=torch.int64, device=x.device)
    val = torch.empty((n,), dtype=torch.float32, device=x.device)
    for r0 in range(0, n, chunk):
        xs = x[r0:r0 + chunk]
        S = ops.gemm(xs, c)  # [rows, k] fp32
        _lib.call("irc_argmax_bias", ptr(S), ptr(bias), xs.shape[0], k, ptr(idx[r0:]),
                  ptr(val[r0:]), stream_ptr(x.device))
    return idx, val


def kmeans(x, k: int, niter: int = 20, nredo: int = 1, seed: int = 0,
           max_points_per_centroid: int = 256):
    """Lloyd k-means of x [n, D] (device fp32): (centroids [k, D], assignment
    [n] int64, squared L2 distance to the assigned centroid [n])."""
    require_hip(x)
    x = x.float().contiguous()
    n, D = x.shape
    if n < k:
        raise ValueError(f"kmeans: {n} points < {k} clusters")
    dev, st = x.device, stream_ptr(x.device)
    rng = np.random.default_rng(seed)
    # faiss trains on at most k * max_points_per_centroid sampled points
    train = x
    if n > k * max_points_per_centroid:
        train = x[torch.as_tensor(rng.choice(n, k * max_points_per_centroid, replace=False),
                                  device=dev)].contiguous()
    nt = train.shape[0]
    best_obj, best_c = None, None
    sums = torch.empty((k, D), dtype=torch.float32, device=dev)
    counts = torch.empty((k,), dtype=torch.float32, device=dev)
    bias = torch.empty((k,), dtype=torch.float32, device=dev)
    for _ in range(max(nredo, 1)):
        c = train[torch.as_tensor(rng.choice(nt, k, replace=False), device=dev)].contiguous()
        sums.zero_()
        counts.fill_(1.0)  # finalize with counts = 1: bias from the initial centroids
        _lib.call("irc_centroid_finalize", ptr(c), ptr(counts), k, D, ptr(c), ptr(bias), st)
        for _ in range(niter):
            a, _ = _assign(train, c, bias)
            sums.zero_()
            counts.zero_()
            _lib.call("irc_centroid_accumulate", ptr(train), ptr(a), nt, D, ptr(sums),
                      ptr(counts), st)
            _lib.call("irc_centroid_finalize", ptr(sums), ptr(counts), k, D, ptr(c), ptr(bias),
                      st)
        _, val = _assign(train, c, bias)
        obj = float(ops.dsum(val, -2.0).item())  # sum |x|^2 is constant across restarts
        if best_obj is None or obj < best_obj:
            best_obj, best_c = obj, c.clone()
    _lib.call("irc_centroid_finalize", ptr(best_c), ptr(counts.fill_(1.0)), k, D, ptr(best_c),
              ptr(bias), st)
    idx, val = _assign(x, best_c, bias)
    _, nrm = ops.l2norm_fwd(x)
    # squared L2 = |x|^2 - 2 (x.c - |c|^2 / 2): n-element bookkeeping, as faiss' D
    dist = nrm * nrm - 2.0 * val
    return best_c, idx, dist.clamp_min(0.0)


def concentration(assign: np.ndarray, dist: np.ndarray, k: int, temperature: float):
    """utils.py:74-98: per-cluster concentration phi (mean distance / log(n+10),
    singletons -> the max, clipped to the 10-90th percentiles, scaled to mean
    `temperature`).  Host arithmetic on k values, as in the reference."""
    density = np.zeros(k)
    dcl = [[] for _ in range(k)]
    for i, c in enumerate(assign):
        dcl[c].append(dist[i])
    for i, d in enumerate(dcl):
        if len(d) > 1:
            density[i] = (np.asarray(d) ** 0.5).mean() / np.log(len(d) + 10)
    dmax = density.max()
    for i, d in enumerate(dcl):
        if len(d) <= 1:
            density[i] = dmax
    density = density.clip(np.percentile(density, 10), np.percentile(density, 90))
    return temperature * density / density.mean()
