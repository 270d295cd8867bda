"""bench.py's strong-scaling retrieval leg (run_scan_strong) on CPU: a fixed
corpus split n_total / world over two gloo ranks, the same global query batch, the three
steps of a search timed apart.  The device scan and merge are host-side doubles (the numpy
oracle); the GPU tests cover irc_scan_topk / irc_topk_merge themselves.  Checked: every rank
holds its n_total / world slice of the SAME corpus the one-rank run draws, the merged top-k
equals the oracle over the whole corpus, and the JSON fields the driver's scaling run reads
are present.  The ws-2 line is written to the test's tmp dir (profiles/r06_strong_cpu_ws2.json
is one such line)."""
import json
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import irc_oracle as O

N_TOTAL, DIM, NQ, K = 3000, 64, 16, 10


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _double_index(n_total, dim, rank, world, dev, group):
    import bench
    import irc_amd.retrieval as R

    class CpuIndex(R.ShardedDenseIndex):
        def __init__(self, docs, doc_offset, group):
            self.docs, self.doc_offset, self.group, self.dtype = docs, doc_offset, group, "bf16"

        def _local_topk(self, queries, k, ws_tag=None):
            i, s = O.scan_topk(queries.float().numpy(), self.docs.float().numpy(), k,
                               self.doc_offset)
            return torch.from_numpy(s), torch.from_numpy(i)

        def _merge(self, scores, idx, k):
            i, s = O.merge_topk(list(idx.numpy()), list(scores.numpy()), k)
            return torch.from_numpy(s), torch.from_numpy(i)

    shard, lo = bench.strong_shard(n_total, dim, rank, world, dev)
    return CpuIndex(shard, lo, group)


def _args():
    import argparse

    return argparse.Namespace(steps=2, warmup=1, scan_depth=2)


def _worker(rank, port, out_dir, world):
    import bench

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cpu")
    made = {}

    def make_index(r, w, d):
        made["ix"] = _double_index(N_TOTAL, DIM, r, w, d, dist.group.WORLD)
        return made["ix"]

    line = bench.run_scan_strong(_args(), rank, world, dev, N_TOTAL, "bf16", NQ, DIM, K,
                                 make_index=make_index, reps=2)
    gq = torch.Generator().manual_seed(7)
    allq = torch.nn.functional.normalize(torch.randn(NQ, DIM, generator=gq)).bfloat16()
    myq = allq[rank * NQ // world:(rank + 1) * NQ // world]
    s, i = made["ix"].search(myq, K, equal_counts=True)
    np.save(os.path.join(out_dir, f"idx{rank}.npy"), i.numpy())
    np.save(os.path.join(out_dir, f"sc{rank}.npy"), s.numpy())
    np.save(os.path.join(out_dir, f"shard{rank}.npy"), made["ix"].docs.float().numpy())
    if rank == 0:
        with open(os.path.join(out_dir, "line.json"), "w") as f:
            json.dump({"retrieval_strong_cpu_rehearsal": line}, f)
    dist.destroy_process_group()


def test_strong_scaling_leg_gloo_ws2(tmp_path):
    import bench

    world = 2
    mp.start_processes(_worker, args=(_free_port(), str(tmp_path), world), nprocs=world,
                       join=True, start_method="spawn")
    line = json.load(open(tmp_path / "line.json"))["retrieval_strong_cpu_rehearsal"]
    assert line["scaling"] == "strong" and line["ranks"] == 2 and line["backend"] == "gloo"
    assert line["docs_total"] == N_TOTAL and line["docs_per_rank"] == [1500, 1500]
    assert line["queries"] == NQ and line["queries_per_rank"] == NQ // 2
    assert line["result_shape"] == [NQ, K] and line["value"] > 0
    assert set(line["phases"]) == {"query_allgather_us", "local_scan_us",
                                   "list_allgather_merge_us"}
    assert all(v > 0 for v in line["phases"].values())
    # the two shards are the one-rank corpus, split
    full, lo = bench.strong_shard(N_TOTAL, DIM, 0, 1, torch.device("cpu"))
    assert lo == 0
    both = np.concatenate([np.load(tmp_path / "shard0.npy"), np.load(tmp_path / "shard1.npy")])
    assert np.array_equal(both, full.float().numpy())
    # the merged global top-k of the gathered queries = the oracle over the whole corpus
    gq = torch.Generator().manual_seed(7)
    allq = torch.nn.functional.normalize(torch.randn(NQ, DIM, generator=gq)).bfloat16()
    ri, rs = O.scan_topk(allq.float().numpy(), full.float().numpy(), K, 0)
    for r in range(world):
        assert np.array_equal(np.load(tmp_path / f"idx{r}.npy"), ri)
        assert np.array_equal(np.load(tmp_path / f"sc{r}.npy"), rs)


def test_strong_shard_same_corpus_any_world():
    import bench

    cpu = torch.device("cpu")
    full, _ = bench.strong_shard(1000, 8, 0, 1, cpu)
    for world in (2, 4, 8):
        parts = [bench.strong_shard(1000, 8, r, world, cpu) for r in range(world)]
        assert [lo for _, lo in parts] == [r * 1000 // world for r in range(world)]
        assert torch.equal(torch.cat([p for p, _ in parts]), full)
