"""Benchmark of the contrastive-training + dense-retrieval hot path on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--part scan|train|all]

For N>1 the driver launches one process per GPU with torch.distributed.run; each
rank reads RANK/LOCAL_RANK/WORLD_SIZE from the environment and RCCL (backend
"nccl") carries the collectives.  Rank 0 prints ONE JSON line.

Retrieval leg: each rank keeps a 100k-doc shard (D=768 bf16,
unit-norm Gaussian, seed 2024+rank) resident in HBM; one step = one batch of
Q=256 query embeddings all-gathered to every rank, scanned against the local
shard and reduced to the global top-100 (scaling: weak -- the per-GPU shard is
fixed, the global corpus grows with N).
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "information-retrieval-with-contrastive-learning_amd")
for _p in (ROOT, PKG):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X spec (MI355X_MICROARCH.md chip table)
BF16_PEAK_TFS = 2500.0  # dense bf16 MFMA spec

SCAN_N_PER_GPU = 100_000
SCAN_Q = 256
SCAN_D = 768
SCAN_K = 100


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor()


def _blas_threads():
    try:
        from threadpoolctl import threadpool_info

        return max((i.get("num_threads", 1) for i in threadpool_info()), default=1)
    except Exception:
        return int(os.environ.get("OMP_NUM_THREADS", "1"))


def _pmc_traffic(kernel_tag: str):
    """HBM bytes per launch from a committed rocprofv3 --pmc summary, if present
    (profiles/pmc_<tag>.json, written by tools/pmc_summary.py)."""
    p = os.path.join(ROOT, "profiles", f"pmc_{kernel_tag}.json")
    if not os.path.exists(p):
        return None
    try:
        with open(p) as f:
            return float(json.load(f)["hbm_bytes_per_launch"])
    except Exception:
        return None


def _prof_query(lib, name):
    tot = ctypes.c_double(0)
    cnt = ctypes.c_int64(0)
    lib.irc_prof_query(name.encode(), ctypes.byref(tot), ctypes.byref(cnt))
    return tot.value, cnt.value


def run_scan(args, rank, world, dev):
    from irc_amd import _lib, retrieval

    lib = _lib.load()
    g = torch.Generator().manual_seed(2024 + rank)
    shard = torch.nn.functional.normalize(torch.randn(SCAN_N_PER_GPU, SCAN_D, generator=g))
    shard = shard.bfloat16().to(dev)
    gq = torch.Generator().manual_seed(7)
    allq = torch.nn.functional.normalize(torch.randn(SCAN_Q, SCAN_D, generator=gq)).bfloat16()
    lo = rank * SCAN_Q // world
    hi = (rank + 1) * SCAN_Q // world
    myq = allq[lo:hi].to(dev)
    index = retrieval.ShardedDenseIndex(shard, doc_offset=rank * SCAN_N_PER_GPU,
                                        group=dist.group.WORLD if world > 1 else None)
    for _ in range(args.warmup):
        index.search(myq, SCAN_K)
    torch.cuda.synchronize()
    lib.irc_prof_reset()
    lib.irc_prof_enable(1)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        index.search(myq, SCAN_K)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    lib.irc_prof_enable(0)
    ktot, kcnt = _prof_query(lib, "scan_filter")
    if world > 1:
        t = torch.tensor([dt], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    kavg_s = (ktot / 1e3) / max(kcnt, 1)
    # algorithmic bytes of one filter-scan launch: the shard once + the queries once
    alg_bytes = SCAN_N_PER_GPU * SCAN_D * 2 + SCAN_Q * SCAN_D * 2
    achieved = alg_bytes / kavg_s / 1e9 if kcnt else None
    traffic = _pmc_traffic("scan_filter")
    res = {
        "qps": SCAN_Q * args.steps / dt,
        "ms_per_step": dt * 1e3 / args.steps,
        "kernel_avg_us": kavg_s * 1e6,
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": (achieved / HBM_PEAK_GBS) if achieved else None,
                     "traffic": traffic, "kernel": "scan_tile_kernel<768,4,KEYS> (filter pass)",
                     "alg_bytes_per_launch": alg_bytes,
                     "mfma_tflops": 2 * SCAN_Q * SCAN_N_PER_GPU * SCAN_D / kavg_s / 1e12
                     if kcnt else None},
    }
    return res


def cpu_baseline_scan(budget_s: float = 10.0):
    """The oracle's fp32 scan (reference CPU arithmetic: q @ d.T + closest_docs
    selection) on the host cores, full C2 shape, repeated for ~budget_s."""
    from oracle import irc_oracle as O

    g = torch.Generator().manual_seed(2024)
    d = torch.nn.functional.normalize(torch.randn(SCAN_N_PER_GPU, SCAN_D, generator=g))
    d = d.bfloat16().float().numpy()
    gq = torch.Generator().manual_seed(7)
    q = torch.nn.functional.normalize(torch.randn(SCAN_Q, SCAN_D, generator=gq))
    q = q.bfloat16().float().numpy()
    O.scan_topk_fast_f32(q[:8], d[:20000], SCAN_K)  # warm BLAS
    reps, t0 = 0, time.perf_counter()
    while True:
        O.scan_topk_fast_f32(q, d, SCAN_K)
        reps += 1
        if time.perf_counter() - t0 >= budget_s:
            break
    dt = time.perf_counter() - t0
    return {"value": SCAN_Q * reps / dt, "unit": "queries/s", "cores": _blas_threads(),
            "kind": "port", "cpu_model": _cpu_model(),
            "sample": f"{reps} x full C2 batch (Q={SCAN_Q}, N={SCAN_N_PER_GPU}, D={SCAN_D}, "
                      f"k={SCAN_K}), numpy fp32 BLAS + exact top-k"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--part", default="scan", choices=["scan"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=10.0)
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", device_id=dev)

    scan = run_scan(args, rank, world, dev)
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline_scan(args.cpu_budget)
    if rank == 0:
        line = {
            "metric": "query-doc pairs/sec (train) + queries/sec @ top-k over N docs, 1/2/4/8 GPU",
            "value": scan["qps"],
            "unit": "queries/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": scan["ms_per_step"],
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic (unit-norm Gaussian embeddings, seed 2024+rank)",
            "config": {"workload": "retrieval: corpus scan + top-k (C2: BERT-base d=768, "
                                   "100k docs per GPU, 256-query batch, k=100)",
                       "docs_per_gpu": SCAN_N_PER_GPU, "queries": SCAN_Q, "dim": SCAN_D,
                       "k": SCAN_K, "parallelism": f"corpus-sharded x{world}"},
            "roofline": scan["roofline"],
            "cpu_baseline": cpu,
            "kernel_avg_us": scan["kernel_avg_us"],
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
