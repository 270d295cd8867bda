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
    fever_loader = get_dataloader(args, train=False)
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
    each batch's latency and the evidence recall@k; returns recall@k."""
    assert args.ckpt is not None
    _, model, _, _ = load_model(args.ckpt)
    model = model.to(args.device).eval()
    loader = get_dataloader(args, train=False)
    # evidence corpus = every evidence document line of the dev set's wiki pages
    titles, texts = [], []
    for title, page in loader.dataset.wiki.items():
        for line in page["lines"]:
            if line.strip():
                titles.append(title)
                texts.append(line)
    index = ShardedDenseIndex(encode_corpus(model, texts, args.device))
    hits = total = 0
    for batch in tqdm(loader, desc="Iteration"):
        claims = [d["claim"] for d in batch]
        s = time.time()
        q = model.ctx2vec(claims, args.device)
        scores, idx = index.search(q, k)
        torch.cuda.synchronize()
        print(f"batch of {len(claims)} claims: {time.time() - s:.4f}s")
        idx = idx.cpu().tolist()
        for d, row in zip(batch, idx):
            gold = {e["title"] for e in d["evidences"]}
            hits += int(any(titles[j] in gold for j in row if j >= 0))
            total += 1
    print(f"evidence recall@{k}: {hits / max(total, 1):.4f}")
    return hits / max(total, 1)
