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
