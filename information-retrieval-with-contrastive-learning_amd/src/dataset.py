"""Drop-in for src/dataset.py: document-pair and FEVER datasets (host side).

Same on-disk formats and sampling as the reference (src/dataset.py:21-182):
``docs_sentence.pkl`` is a list of documents, each a list of sentence strings;
a training item is (LongTensor([idx]), sent1, sent2) with two distinct
sentences of the same document drawn uniformly (np.random.choice, no
replacement) or from the top 10% TF-IDF-similar pairs.  These files are the
user's own data (written by the reference's preprocessing scripts).
"""
import json
import math
import pickle
import random
from unicodedata import normalize

import numpy as np
import torch
from torch.utils.data import Dataset


def process_wiki(fname):
    with open(fname, "r") as f:
        wiki = json.load(f)
    for datum in wiki.values():
        datum["lines"] = [" ".join(line.split("\t")[1:]) for line in datum["lines"].split("\n")]
    return wiki


def process_jsonl(fname):
    out = []
    with open(fname, "r", encoding="utf-8") as f:
        for line in f:
            dic = json.loads(line)
            ev = {}
            for evidences in dic["evidence"]:
                for evidence in evidences:
                    if evidence[2] is not None:
                        doc_id = normalize("NFKD", evidence[2])
                        ev[doc_id] = ev.get(doc_id, []) + [evidence[3]]
            out.append({"id": dic["id"], "claim": dic["claim"], "label": dic["label"],
                        "evidences": ev})
    return out


class DocDataset(Dataset):
    def __init__(self, args):
        super().__init__()
        with open(args.config["dataset"]["docs_sentence"], "rb") as f:
            self.data = pickle.load(f)
        self.sample_method = args.sample
        if self.sample_method == "tf_idf":
            with open(args.config["dataset"]["full_docs_sentence_similarity"], "rb") as f:
                self.docs_sents_similarity = pickle.load(f)
            self.ratio = 0.1

    def __len__(self):
        return len(self.data)

    def __getitem__(self, idx):
        doc = self.data[idx]
        if self.sample_method == "uniform":
            sent1, sent2 = np.random.choice(doc, size=2, replace=False)
        elif self.sample_method == "tf_idf":
            sims = self.docs_sents_similarity[idx]
            k = math.ceil(len(sims) * self.ratio)
            (i, j), _ = random.choice(sims[:k])
            sent1, sent2 = doc[i], doc[j]
        else:
            raise ValueError(self.sample_method)
        return torch.LongTensor([idx]), sent1, sent2


class FeverDataset(Dataset):
    def __init__(self, args):
        super().__init__()
        self.wiki = process_wiki(args.config["dataset"]["small_wiki"])
        fever = self.process(process_jsonl(args.config["dataset"]["dev_data"]))
        self.label_map = {"SUPPORTS": 1, "REFUTES": 0}
        self.data = [{"id": d["id"], "label": self.label_map[d["label"]], "claim": d["claim"],
                      "evidences": d["evidences"]} for d in fever if d["label"] != "NOT ENOUGH INFO"]

    def __len__(self):
        return len(self.data)

    def __getitem__(self, idx):
        return self.data[idx]

    def process(self, data):
        for datum in data:
            datum["evidences"] = [{"title": doc_id, "document": self.wiki[doc_id]["lines"],
                                   "sent_idx": sent_ids}
                                  for doc_id, sent_ids in datum["evidences"].items()]
        return data

    def collate_fn(self, data):
        return data


def get_dataloader(args, train=True, distributed=None):
    """dataset.py:159-182.  Under data parallelism (``args.dist_group`` set by
    main.py from the launcher's WORLD_SIZE / RANK) each rank reads a disjoint
    slice of the dataset through a DistributedSampler (shuffled per epoch with
    ``args.seed``; ``set_epoch`` is called by the training loop), so the global
    batch is ``batch_size * world`` distinct pairs.  ``distributed=False`` keeps
    the whole dataset on every rank (the ProtoNCE feature pass, whose clustering
    must be identical on every rank)."""
    bsz = args.config["train"]["batch_size"] if train else args.config["eval"]["batch_size"]
    n_jobs = args.config["train"]["n_jobs"] if train else args.config["eval"]["n_jobs"]
    if args.data == "doc":
        dataset, collate_fn = DocDataset(args), None
    elif args.data == "fever":
        dataset = FeverDataset(args)
        collate_fn = dataset.collate_fn
    else:
        raise ValueError(args.data)
    group = getattr(args, "dist_group", None)
    if distributed is None:
        distributed = train
    sampler = None
    if distributed and group is not None:
        import torch.distributed as dist

        sampler = torch.utils.data.distributed.DistributedSampler(
            dataset, num_replicas=dist.get_world_size(group), rank=dist.get_rank(group),
            shuffle=train, seed=int(getattr(args, "seed", 0)), drop_last=train)
    return torch.utils.data.DataLoader(dataset, batch_size=bsz,
                                       shuffle=train if sampler is None else False,
                                       sampler=sampler, num_workers=n_jobs, drop_last=train,
                                       pin_memory=torch.cuda.is_available(),
                                       collate_fn=collate_fn)


class PairSampler:
    """The training DataLoader's iteration (shuffle, batch_size, drop_last; a
    DistributedSampler slice under data parallelism) with each item's sentence
    pair drawn exactly as DocDataset.__getitem__ draws it -- uniform:
    np.random.choice over the document's sentences without replacement (the same
    RNG consumption as choosing from the sentence list); tf_idf: random.choice
    over the top 10% similar pairs -- in the main process (the reference's
    n_jobs = 0 order).  Yields (indexes LongTensor [B, 1], sentence indices int64
    [2B]: the anchors, then the positives) into a DeviceCorpus's numbering
    (doc_start[d] + s), so no string ever leaves the host."""

    def __init__(self, args, dataset=None):
        self.dataset = dataset if dataset is not None else DocDataset(args)
        docs = self.dataset.data
        self.doc_start = np.zeros(len(docs) + 1, np.int64)
        np.cumsum([len(d) for d in docs], out=self.doc_start[1:])
        self.bsz = int(args.config["train"]["batch_size"])
        group = getattr(args, "dist_group", None)
        if group is not None:
            import torch.distributed as dist

            self.sampler = torch.utils.data.distributed.DistributedSampler(
                self.dataset, num_replicas=dist.get_world_size(group), rank=dist.get_rank(group),
                shuffle=True, seed=int(getattr(args, "seed", 0)), drop_last=True)
        else:
            self.sampler = torch.utils.data.RandomSampler(self.dataset)

    def __len__(self):
        return len(self.sampler) // self.bsz

    def pair(self, idx):
        ds = self.dataset
        doc = ds.data[idx]
        if ds.sample_method == "uniform":
            i, j = np.random.choice(len(doc), size=2, replace=False)
        elif ds.sample_method == "tf_idf":
            sims = ds.docs_sents_similarity[idx]
            k = math.ceil(len(sims) * ds.ratio)
            (i, j), _ = random.choice(sims[:k])
        else:
            raise ValueError(ds.sample_method)
        return int(self.doc_start[idx] + i), int(self.doc_start[idx] + j)

    def pairs_uniform(self, batch):
        """pair() for a whole batch of documents in the uniform mode: the same draws
        from numpy's global RandomState (irc_pair_sample restates
        np.random.choice(n, 2, replace=False) on its MT19937 state and hands the
        advanced state back), ~0.1 us per pair instead of ~20 us of Python each --
        at B = 256 the per-call form cost ~5 ms of host time per step."""
        from irc_amd import _lib

        st = np.random.get_state()
        key = np.array(st[1], dtype=np.uint32)
        pos = np.array([st[2]], dtype=np.int32)
        docs = np.ascontiguousarray(batch, dtype=np.int64)
        a = np.empty(docs.shape[0], np.int64)
        b = np.empty(docs.shape[0], np.int64)
        _lib.call("irc_pair_sample", key.ctypes.data, pos.ctypes.data, self.doc_start.ctypes.data,
                  docs.ctypes.data, docs.shape[0], a.ctypes.data, b.ctypes.data)
        np.random.set_state(("MT19937", key, int(pos[0]), st[3], st[4]))
        return a, b

    def __iter__(self):
        # a DataLoader iterator draws its workers' base seed from torch's default
        # generator before the sampler draws its permutation seed: draw it too, so
        # the permutation (and so the pairs) are the DataLoader's
        torch.empty((), dtype=torch.int64).random_()
        batch = []
        for idx in self.sampler:
            batch.append(int(idx))
            if len(batch) == self.bsz:
                if self.dataset.sample_method == "uniform":
                    a, b = self.pairs_uniform(batch)
                    sel = np.concatenate([a, b])
                else:
                    pairs = [self.pair(i) for i in batch]
                    sel = np.array([a for a, _ in pairs] + [b for _, b in pairs], np.int64)
                yield torch.LongTensor(batch).view(-1, 1), sel
                batch = []
