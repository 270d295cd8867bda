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


def test_pairs_uniform_equals_np_random_choice_and_state(tmp_path):
    """irc_pair_sample (C restatement of np.random.choice(n, 2, replace=False) on the
    legacy global MT19937) against the per-call numpy draws, over documents of 2 to
    700 sentences: the same pairs and the same RNG state afterwards, across the
    624-word regeneration boundary."""
    args, _ = _args(tmp_path)
    ps = PairSampler(args)
    rng = np.random.default_rng(4)
    lens = np.concatenate([rng.integers(2, 9, 3000), [2, 64, 65, 700, 333, 1024]])
    ps.doc_start = np.zeros(len(lens) + 1, np.int64)
    np.cumsum(lens, out=ps.doc_start[1:])
    docs = rng.integers(0, len(lens), 5000)
    docs[:6] = np.arange(len(lens) - 6, len(lens))
    np.random.seed(77)
    ref = [np.random.choice(int(lens[d]), size=2, replace=False) for d in docs]
    ref_state = np.random.get_state()
    np.random.seed(77)
    a, b = ps.pairs_uniform(docs)
    st = np.random.get_state()
    assert np.array_equal(a - ps.doc_start[docs], [r[0] for r in ref])
    assert np.array_equal(b - ps.doc_start[docs], [r[1] for r in ref])
    assert np.array_equal(st[1], ref_state[1]) and st[2] == ref_state[2]
    assert np.random.random() == (np.random.set_state(ref_state), np.random.random())[1]
