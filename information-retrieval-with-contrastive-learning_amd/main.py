"""Drop-in for the reference main.py (same flags; main.py:14-112).

    python main.py [--config config.yaml] [--data doc|fever] [--gpu 0] [--ckpt X]
                   [--model LSTM|BERT] [--loss InfoNCE] [--opt adam] [--sample uniform|tf_idf]
                   [--seed 1337] [--logdir log] [--ckptdir ckpt] [--retrieval sparse|dense]

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


def main(argv=None):
    args = get_args(argv)
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
    if args.data == "doc":
        from src.train import train

        train(args)
    elif args.data == "fever":
        from src.evaluation import predict

        predict(args)
    else:
        raise SystemExit(f"unknown --data {args.data!r}")


if __name__ == "__main__":
    main()
