"""The device-corpus input path's host half (src/dataset.py PairSampler): the
sentence pairs it selects, batch by batch, are exactly the strings the
reference-style DataLoader(DocDataset) yields with n_jobs = 0 from the same
seeds (uniform sampling: np.random.choice without replacement over a document's
sentences; the DataLoader's shuffled, drop_last batches)."""
import argparse
import pickle
import random

import numpy as np
import torch

from src.dataset import DocDataset, PairSampler, get_dataloader


def _args(tmp_path, n_docs=57, bsz=8):
    rnd = random.Random(1)
    docs = [[f"d{d} s{s} " + " ".join(f"w{rnd.randrange(50)}" for _ in range(rnd.randrange(2, 9)))
             for s in range(rnd.randrange(2, 7))] for d in range(n_docs)]
    with open(tmp_path / "docs.pkl", "wb") as f:
        pickle.dump(docs, f)
    cfg = {"dataset": {"docs_sentence": str(tmp_path / "docs.pkl")},
           "train": {"batch_size": bsz, "n_jobs": 0}, "eval": {"batch_size": bsz, "n_jobs": 0}}
    return argparse.Namespace(config=cfg, data="doc", sample="uniform", seed=3), docs


def _seed(s):
    torch.manual_seed(s)
    np.random.seed(s)
    random.seed(s)


def test_pair_sampler_replays_dataloader_pairs(tmp_path):
    args, docs = _args(tmp_path)
    flat = [s for d in docs for s in d]
    _seed(11)
    ref = []
    for _ in range(2):  # two epochs
        for idx, a, p in get_dataloader(args, train=True):
            ref.append((idx.view(-1).tolist(), list(a), list(p)))
    _seed(11)
    ps = PairSampler(args)
    got = []
    for _ in range(2):
        for idx, sel in ps:
            B = idx.shape[0]
            got.append((idx.view(-1).tolist(), [flat[i] for i in sel[:B]],
                        [flat[i] for i in sel[B:]]))
    assert len(ps) == len(get_dataloader(args, train=True))
    assert got == ref
