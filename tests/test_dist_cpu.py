"""Multi-process host logic on CPU (gloo, world size 2): the collective plumbing
of the two sharded paths, with the device kernels replaced by test doubles.

* ShardedDenseIndex.search: ragged query all-gather, per-shard
  exact top-k with global doc ids, all-gather + merge.  The local scan / merge
  are the numpy oracle here (test doubles for irc_scan_topk / irc_topk_merge,
  which the GPU tests cover); the result must equal the oracle over the whole
  corpus, bit for bit, on every rank.
* Data-parallel training: irc_amd.dist.gather_rows (global
  in-batch negatives) + the flat-gradient all-reduce must give exactly the
  single-process gradient of the global-batch InfoNCE.  The loss here is a torch
  restatement of contrastive_loss.py:56-93 (the test double for irc_amd.nce).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import irc_oracle as O

WORLD = 2


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _init(rank, port):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)


def _run(fn, *args):
    port = _free_port()
    mp.start_processes(fn, args=(port,) + args, nprocs=WORLD, join=True, start_method="spawn")


# ---------------------------------------------------------------- retrieval
def _corpus():
    rng = np.random.default_rng(3)
    # integer grid values: exact scores, many ties (the tie rule is exercised)
    docs = (rng.integers(-4, 5, size=(301, 16)) / 8.0).astype(np.float32)
    qs = (rng.integers(-4, 5, size=(7, 16)) / 8.0).astype(np.float32)
    return docs, qs


def _index_worker(rank, port, out_dir):
    _init(rank, port)
    import irc_amd.retrieval as R

    docs, qs = _corpus()
    k = 10
    lo, hi = R.shard_bounds(docs.shape[0], WORLD, rank)
    myq = qs[:5] if rank == 0 else qs[5:]  # ragged query split (5 / 2)

    class CpuIndex(R.ShardedDenseIndex):
        def __init__(self, docs, doc_offset, group):
            self.docs, self.doc_offset, self.group = docs, doc_offset, group

        def _local_topk(self, queries, k, ws_tag=None):
            i, s = O.scan_topk(queries.numpy(), self.docs.numpy(), k, self.doc_offset)
            return torch.from_numpy(s), torch.from_numpy(i)

        def _merge(self, scores, idx, k):
            i, s = O.merge_topk(list(idx.numpy()), list(scores.numpy()), k)
            return torch.from_numpy(s), torch.from_numpy(i)

    index = CpuIndex(torch.from_numpy(docs[lo:hi]), lo, dist.group.WORLD)
    s, i = index.search(torch.from_numpy(myq), k)
    np.save(os.path.join(out_dir, f"idx{rank}.npy"), i.numpy())
    np.save(os.path.join(out_dir, f"sc{rank}.npy"), s.numpy())
    dist.destroy_process_group()


def test_sharded_index_search_gloo(tmp_path):
    _run(_index_worker, str(tmp_path))
    docs, qs = _corpus()
    ref_i, ref_s = O.scan_topk(qs, docs, 10)
    for r in range(WORLD):
        np.testing.assert_array_equal(np.load(tmp_path / f"idx{r}.npy"), ref_i)
        np.testing.assert_array_equal(np.load(tmp_path / f"sc{r}.npy"), ref_s)


# ---------------------------------------------------------------- training
def _nce_torch(q, k, queue, T):
    """torch restatement of NCELoss._compute_info_loss (contrastive_loss.py:56-93)."""
    N = q.shape[0]
    F = torch.cat([q, k], 0)
    S = F @ F.t()
    eye = torch.eye(2 * N, dtype=torch.bool)
    S = S[~eye].view(2 * N, 2 * N - 1)
    pos_col = torch.cat([torch.arange(N - 1, 2 * N - 1), torch.arange(0, N)])
    pos = S[torch.arange(2 * N), pos_col].unsqueeze(1)
    keep = torch.ones_like(S, dtype=torch.bool)
    keep[torch.arange(2 * N), pos_col] = False
    neg = S[keep].view(2 * N, 2 * N - 2)
    logits = [pos, neg]
    if queue is not None:
        logits.append((q @ queue).repeat(2, 1))
    logits = torch.cat(logits, 1) / T
    return torch.nn.functional.cross_entropy(logits, torch.zeros(2 * N, dtype=torch.long),
                                             reduction="sum") / 2


def _train_data():
    g = torch.Generator().manual_seed(5)
    W = torch.randn(12, 8, generator=g, dtype=torch.float64)
    xa = torch.randn(6, 12, generator=g, dtype=torch.float64)  # 6 pairs = 2 ranks x 3
    xp = torch.randn(6, 12, generator=g, dtype=torch.float64)
    queue = torch.nn.functional.normalize(torch.randn(8, 10, generator=g, dtype=torch.float64),
                                          dim=0)
    return W, xa, xp, queue


def _dp_worker(rank, port, out_dir):
    _init(rank, port)
    from irc_amd.dist import all_reduce_sum_, gather_rows

    W, xa, xp, queue = _train_data()
    W = W.clone().requires_grad_(True)
    sl = slice(3 * rank, 3 * rank + 3)
    q = torch.nn.functional.normalize(xa[sl] @ W, dim=1)
    with torch.no_grad():
        k = torch.nn.functional.normalize(xp[sl] @ W, dim=1)
    qg = gather_rows(q, dist.group.WORLD)
    kg = gather_rows(k, dist.group.WORLD)
    assert qg.requires_grad and not kg.requires_grad and qg.shape == (6, 8)
    loss = _nce_torch(qg, kg, queue, 0.05)
    loss.backward()
    g = W.grad.clone()
    all_reduce_sum_(g, dist.group.WORLD)
    np.save(os.path.join(out_dir, f"g{rank}.npy"), g.numpy())
    np.save(os.path.join(out_dir, f"l{rank}.npy"), np.array(loss.item()))
    dist.destroy_process_group()


def test_dp_global_negatives_gradient_gloo(tmp_path):
    _run(_dp_worker, str(tmp_path))
    W, xa, xp, queue = _train_data()
    W = W.clone().requires_grad_(True)
    q = torch.nn.functional.normalize(xa @ W, dim=1)
    with torch.no_grad():
        k = torch.nn.functional.normalize(xp @ W, dim=1)
    loss = _nce_torch(q, k, queue, 0.05)
    loss.backward()
    # the torch restatement agrees with the numpy oracle (pinned by the goldens)
    lo, _ = O.nce_info_loss(q.detach().numpy(), k.numpy(), queue.numpy(), 0.05)
    assert abs(float(lo) - loss.item()) <= 1e-9 * abs(float(lo))
    for r in range(WORLD):
        assert abs(float(np.load(tmp_path / f"l{r}.npy")) - loss.item()) <= 1e-12 * loss.item()
        np.testing.assert_allclose(np.load(tmp_path / f"g{r}.npy"), W.grad.numpy(), rtol=1e-10,
                                   atol=1e-12)
