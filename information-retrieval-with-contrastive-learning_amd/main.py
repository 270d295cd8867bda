"""Drop-in for the reference main.py (same flags; main.py:14-112).

    python main.py [--config config.yaml] [--data doc|fever] [--gpu 0] [--ckpt X]
                   [--model LSTM|BERT] [--loss InfoNCE] [--opt adam] [--sample uniform|tf_idf]
                   [--seed 1337] [--logdir log] [--ckptdir ckpt] [--retrieval sparse|dense]

Multi-GPU (one process per GPU):
    torchrun --nproc-per-node N --master-addr 127.0.0.1 main.py [same flags]
When the launcher sets WORLD_SIZE > 1, the process group is initialised over RCCL
(backend "nccl") on cuda:LOCAL_RANK before any other GPU call; training is data
parallel (each rank a disjoint slice of the pairs, global in-batch negatives,
gradient all-reduce; logging and checkpoints on rank 0) and ``--retrieval dense``
shards the evidence corpus over the ranks.  IRC_DIST_BACKEND=gloo selects gloo
(tests that share one GPU between ranks).

--data doc trains (src.train.train); --data fever runs src.evaluation.predict:
the reference's sparse candidate filter per claim (default) or, with
``--retrieval dense``, the bi-encoder's exact top-k over the evidence corpus.  The compute runs on the MI355X HIP kernels only:
``--gpu -1`` (CPU) is rejected -- there is no CPU fallback in this build.
"""
import argparse
import os
import random
import sys

import numpy as np
import torch
import yaml

HERE = os.path.dirname(os.path.abspath(__file__))
if HERE not in sys.path:
    sys.path.insert(0, HERE)


def get_args(argv=None):
    p = argparse.ArgumentParser(description="Argument Parser.")
    p.add_argument("--config", type=str, default=os.path.join(HERE, "config.yaml"),
                   help="Path to experiment configuration.")
    p.add_argument("--log", action="store_true", default=False,
                   help="Recording loss and metric scores.")
    p.add_argument("--logdir", default="log", type=str, help="Directory for logging.")
    p.add_argument("--data", default="doc", type=str, help="doc: train, fever: retrieve")
    p.add_argument("--ckptdir", default="ckpt", type=str, help="Checkpoint directory.")
    p.add_argument("--seed", default=1337, type=int, help="Random seed.")
    p.add_argument("--gpu", default="0", type=str, help="GPU id (-1: CPU, not supported)")
    p.add_argument("--ckpt", type=str, help="Path to load target pretrain model")
    p.add_argument("--model", default="LSTM", type=str, choices=["LSTM", "BERT"],
                   help="LSTM: frozen BERT + BiLSTM head (reference); BERT: trainable "
                        "BERT bi-encoder (superset)")
    p.add_argument("--loss", default="InfoNCE", type=str,
                   choices=["InfoNCE", "ProtoNCE", "HProtoNCE"])
    p.add_argument("--opt", default="adam", type=str, choices=["adam", "sgd"])
    p.add_argument("--sample", default="uniform", type=str, choices=["uniform", "tf_idf"])
    p.add_argument("--retrieval", default="sparse", type=str, choices=["sparse", "dense"],
                   help="--data fever: sparse n-gram filter as the reference (default) or "
                        "dense bi-encoder top-k (superset)")
    return p.parse_args(argv)


def resolve_device(gpu: str) -> torch.device:
    first = int(gpu.split(",")[0])
    if first < 0:
        raise SystemExit("this build runs on MI355X (HIP) only: --gpu -1 (CPU) has no kernels")
    return torch.device(f"cuda:{first}")


def init_distributed():
    """(group, rank, world, local_rank, created) from the launcher's environment
    (torch.distributed.run / torchrun: WORLD_SIZE, RANK, LOCAL_RANK, MASTER_*), or
    (None, 0, 1, None, False) for a single process; created: this call initialised
    the default process group (main() then also destroys it).  Runs before any other GPU call:
    RCCL's communicator is bound to cuda:LOCAL_RANK (device_id)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world <= 1:
        return None, 0, 1, None, False
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    backend = os.environ.get("IRC_DIST_BACKEND", "nccl")
    created = not dist.is_initialized()
    if created:
        if backend == "nccl":
            dev = torch.device("cuda", local % max(torch.cuda.device_count(), 1))
            torch.cuda.set_device(dev)
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    return dist.group.WORLD, dist.get_rank(), dist.get_world_size(), local, created


def main(argv=None):
    args = get_args(argv)
    group, rank, world, local, created = init_distributed()
    args.dist_group, args.rank, args.world_size = group, rank, world
    torch.cuda.manual_seed(args.seed)
    torch.manual_seed(args.seed)
    np.random.seed(args.seed)
    random.seed(args.seed)
    with open(args.config, "r") as f:
        args.config = yaml.safe_load(f)
    prec = (args.config.get("bert") or {}).get("precision")
    if prec:
        from irc_amd.precision import set_precision

        set_precision(prec)
    args.device = resolve_device(args.gpu)
    if local is not None:  # one GPU per rank: cuda:LOCAL_RANK (wrapped on a shared box)
        args.device = torch.device("cuda", local % max(torch.cuda.device_count(), 1))
    if args.data == "doc":
        from src.train import train

        train(args)
    elif args.data == "fever":
        from src.evaluation import predict

        predict(args)
    else:
        raise SystemExit(f"unknown --data {args.data!r}")
    if created:
        import torch.distributed as dist

        dist.barrier(group)
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
