"""Drop-in for src/evaluation.py: dense retrieval with the trained bi-encoder.

The reference's ``predict`` (src/evaluation.py:86-116) runs a sparse hashed
n-gram candidate filter and leaves the dense claim/evidence cosine commented
out (:110-115).  Here ``predict`` does the dense path the reference sketches:
``ctx2vec`` embeddings (contrastive_module.py:96-100) of the evidence corpus are
sharded into HBM and each claim batch is scored against all of them with the
exact top-k scan (irc_amd.retrieval, closest_docs ordering,
tfidf_doc_ranker.py:60-75).  ``documents_filtering`` (the sparse filter) is the
"next" row of SURVEY.md 8f and raises until it is built.
"""
import time

import torch
from tqdm import tqdm

from irc_amd.retrieval import ShardedDenseIndex
from src.dataset import get_dataloader
from src.model import load_model


def documents_filtering(claim, args, count_matrix, metadata, full_doc_dict, bigram_only=True):
    raise NotImplementedError("sparse hashed-ngram candidate filter: SURVEY.md 8f row 2")


@torch.no_grad()
def encode_corpus(model, texts, device, batch_size=256):
    embs = []
    for i in range(0, len(texts), batch_size):
        embs.append(model.ctx2vec(texts[i:i + batch_size], device))
    return torch.cat(embs, 0) if embs else torch.empty(0, model.loss_config["dim"], device=device)


@torch.no_grad()
def predict(args, k=100):
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
