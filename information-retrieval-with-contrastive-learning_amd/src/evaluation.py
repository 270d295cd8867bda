"""Drop-in for src/evaluation.py: claim -> evidence retrieval.

``predict`` (src/evaluation.py:86-116) keeps the reference's behaviour by
default (``args.retrieval`` "sparse", main.py ``--retrieval``): per claim the
hashed n-gram candidate filter ``documents_filtering`` (here on the GPU,
irc_amd.sparse) with its latency and ``len(docs)`` printed, as the reference
prints them.  ``--retrieval dense`` (superset) runs the dense path the reference
sketches in its commented-out tail (:110-115): ``ctx2vec`` embeddings
(contrastive_module.py:96-100) of the evidence corpus sharded into HBM and each
claim batch scored against all of them with the exact top-k scan
(irc_amd.retrieval, closest_docs ordering, tfidf_doc_ranker.py:60-75), then
evidence recall@k printed.
"""
import pickle
import time

import torch
from tqdm import tqdm

from irc_amd.retrieval import ShardedDenseIndex
from irc_amd.sparse import SparseIndex, load_sparse_csr
from src.dataset import get_dataloader
from src.model import load_model


_SPARSE_CACHE = {}


def _sparse_index(count_matrix, metadata, device):
    """The inverted count matrix resident in HBM, built once per matrix object."""
    key = (id(count_matrix), str(device))
    idx = _SPARSE_CACHE.get(key)
    if idx is None:
        idx = _SPARSE_CACHE[key] = SparseIndex(count_matrix, ngram=metadata["ngram"],
                                               device=device)
    return idx


def documents_filtering(claim, args, count_matrix, metadata, full_doc_dict, bigram_only=True):
    """src/evaluation.py:57-81: {doc_id: doc} of the docs sharing a hashed n-gram
    with the claim.  Tokenisation and hashing on the host (irc_amd.sparse, the
    reference's SimpleTokenizer / filter_ngram / murmurhash3); the row union over
    the inverted count matrix on the GPU (irc_csr_union_*)."""
    if metadata.get("tokenizer", "simple") != "simple":
        raise ValueError("only the DrQA 'simple' tokenizer is supported on this path")
    device = getattr(args, "device", None) or torch.device("cuda")
    index = _sparse_index(count_matrix, metadata, device)
    doc_ids = metadata["doc_dict"][1]
    docs = {}
    for i in index.documents_filtering([claim], bigram_only)[0]:
        doc_id = doc_ids[int(i)]
        if doc_id in full_doc_dict:  # the reference skips ids missing from the dict
            docs[doc_id] = full_doc_dict[doc_id]
    return docs


@torch.no_grad()
def encode_corpus(model, texts, device, batch_size=256):
    embs = []
    for i in range(0, len(texts), batch_size):
        embs.append(model.ctx2vec(texts[i:i + batch_size], device))
    return torch.cat(embs, 0) if embs else torch.empty(0, model.loss_config["dim"], device=device)


@torch.no_grad()
def predict(args, k=100):
    """evaluation.py:86-108: load the checkpoint, then per claim the sparse filter
    (latency and candidate count printed); ``args.retrieval == "dense"``:
    predict_dense.  Returns the per-claim candidate counts (sparse) or recall@k."""
    if getattr(args, "retrieval", "sparse") == "dense":
        return predict_dense(args, k)
    assert args.ckpt is not None
    _, model, _, _ = load_model(args.ckpt)
    model = model.to(args.device)
    # data parallel: each rank filters a disjoint share of the claim batches
    fever_loader = get_dataloader(args, train=False,
                                  distributed=getattr(args, "dist_group", None) is not None)
    ds = args.config["dataset"]
    _, metadata = load_sparse_csr(ds["tfidf"])
    count_matrix, _ = load_sparse_csr(ds["inverted_file"])
    with open(ds["full_docs_dict"], "rb") as f:  # the user's own preprocessing output
        full_docs_dict = pickle.load(f)
    counts = []
    for batch in tqdm(fever_loader, desc="Iteration"):
        claim = [data["claim"] for data in batch]
        s = time.time()
        docs = documents_filtering(claim[0], args, count_matrix, metadata, full_docs_dict, False)
        e = time.time()
        print(e - s)
        print(len(docs))
        counts.append(len(docs))
    return counts


@torch.no_grad()
def predict_dense(args, k=100):
    """Dense claim -> evidence-line retrieval with the trained bi-encoder: prints
    each batch's latency and the evidence recall@k; returns recall@k.

    Under data parallelism (``args.dist_group``, main.py under torchrun) the
    evidence corpus is sharded: rank r encodes and keeps only its contiguous
    slice (irc_amd.retrieval.shard_bounds) in HBM, each claim batch is split over
    the ranks, and ShardedDenseIndex.search all-gathers the claim embeddings,
    scans every shard and merges the per-shard top-k -- every rank receives the
    global result for the whole batch."""
    from irc_amd.retrieval import shard_bounds

    assert args.ckpt is not None
    _, model, _, _ = load_model(args.ckpt)
    model = model.to(args.device).eval()
    loader = get_dataloader(args, train=False, distributed=False)
    group = getattr(args, "dist_group", None)
    world = int(getattr(args, "world_size", 1)) if group is not None else 1
    rank = int(getattr(args, "rank", 0)) if group is not None else 0
    # evidence corpus = every evidence document line of the dev set's wiki pages
    titles, texts = [], []
    for title, page in loader.dataset.wiki.items():
        for line in page["lines"]:
            if line.strip():
                titles.append(title)
                texts.append(line)
    lo, hi = shard_bounds(len(texts), world, rank)
    index = ShardedDenseIndex(encode_corpus(model, texts[lo:hi], args.device), doc_offset=lo,
                              group=group)
    dim = model.loss_config["dim"]
    hits = total = 0
    for batch in tqdm(loader, desc="Iteration", disable=rank != 0):
        claims = [d["claim"] for d in batch]
        s = time.time()
        c0, c1 = shard_bounds(len(claims), world, rank)
        mine = claims[c0:c1]
        q = model.ctx2vec(mine, args.device) if mine else \
            torch.empty((0, dim), dtype=torch.float32, device=args.device)
        scores, idx = index.search(q, k)  # rows: the whole batch, in order
        torch.cuda.synchronize()
        if rank == 0:
            print(f"batch of {len(claims)} claims: {time.time() - s:.4f}s")
        idx = idx.cpu().tolist()
        for d, row in zip(batch, idx):
            gold = {e["title"] for e in d["evidences"]}
            hits += int(any(titles[j] in gold for j in row if j >= 0))
            total += 1
    if rank == 0:
        print(f"evidence recall@{k}: {hits / max(total, 1):.4f}")
    return hits / max(total, 1)
