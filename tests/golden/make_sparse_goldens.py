"""Golden fixtures for the sparse (hashed n-gram TF-IDF) retrieval path, made by
RUNNING the reference's own code on a small synthetic corpus.

  python tests/golden/make_sparse_goldens.py

Runs only in the build container (it imports /root/reference read-only, with the
never-called stand-ins of make_goldens.py for pexpect & co).  It builds the
inverted count matrix with the reference's tokenizer / n-gram filter / feature
hash exactly as preprocessing/drqa/build_tfidf.py:63-121 does (without its
sqlite DocDB and process pool), the TF-IDF matrix with build_tfidf.py's
get_tfidf_matrix (:128-152), and then records:
  * the reference's documents_filtering (src/evaluation.py:57-81) candidate doc
    indices per claim (all n-grams and bigram_only);
  * TfidfDocRanker.closest_docs (preprocessing/drqa/retriever/
    tfidf_doc_ranker.py:60-75) doc indices and fp64 scores per claim;
  * the hashed n-gram ids of every claim (TfidfDocRanker.parse + utils.hash);
  * sha256 digests of both CSR matrices (data / indices / indptr) and of the
    stop-word list, so the product's restatement can be checked without them.
Only these numbers and the synthetic texts are saved (sparse.npz).
"""
from __future__ import annotations

import hashlib
import os
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_goldens import _import_ref  # noqa: E402

HASH_SIZE = 2 ** 16
NGRAM = 2


def synthetic_corpus(rng, n_docs=300):
    words = [f"term{i}" for i in range(160)] + [
        "the", "of", "and", "in", "to", "a", "is", "was", "for", "on", "with", "by", "as",
        "café", "naïve", "Zürich", "São", "Ångström", "2019", "1.5", "U.S.", "don't", "it's",
        "élan", "co-operate", "x86-64", "e-mail", "U2", "façade"]
    punct = [",", ".", ";", ":", "(", ")", "\"", "'", "-", "--", "!", "?"]
    docs = []
    for _ in range(n_docs):
        n = int(rng.integers(8, 60))
        toks = []
        for _ in range(n):
            if rng.random() < 0.12:
                toks.append(str(rng.choice(punct)))
            else:
                w = str(rng.choice(words))
                toks.append(w.capitalize() if rng.random() < 0.2 else w)
        docs.append(" ".join(toks))
    claims = []
    for i in range(24):
        d = docs[int(rng.integers(0, n_docs))].split()
        s = int(rng.integers(0, max(1, len(d) - 6)))
        claims.append(" ".join(d[s:s + int(rng.integers(3, 9))]))
    claims.append("term3 term7 café")   # short, accented
    claims.append("the of and ,")        # stopwords / punctuation only
    return docs, claims


def digest(*arrays):
    h = hashlib.sha256()
    for a in arrays:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


def main():
    _import_ref()
    import scipy.sparse as sp
    from collections import Counter

    from preprocessing.drqa import tokenizers
    from preprocessing.drqa.retriever import utils
    from preprocessing.drqa.retriever.tfidf_doc_ranker import TfidfDocRanker
    import src.evaluation as ev

    rng = np.random.default_rng(2024)
    docs, claims = synthetic_corpus(rng)
    tok = tokenizers.get_class("simple")()
    doc_ids = [f"doc_{i}" for i in range(len(docs))]
    doc2idx = {d: i for i, d in enumerate(doc_ids)}

    # build_tfidf.py:63-121 (count + get_count_matrix), in-process
    row, col, data = [], [], []
    for doc_id, text in zip(doc_ids, docs):
        tokens = tok.tokenize(utils.normalize(text))
        ngrams = tokens.ngrams(n=NGRAM, uncased=True, filter_fn=utils.filter_ngram)
        counts = Counter([utils.hash(g, HASH_SIZE) for g in ngrams])
        row.extend(counts.keys())
        col.extend([doc2idx[doc_id]] * len(counts))
        data.extend(counts.values())
    count_matrix = sp.csr_matrix((data, (row, col)), shape=(HASH_SIZE, len(doc_ids)))
    count_matrix.sum_duplicates()
    # build_tfidf.py:128-152
    from preprocessing.drqa import build_tfidf
    tfidf = build_tfidf.get_tfidf_matrix(count_matrix)
    freqs = build_tfidf.get_doc_freqs(count_matrix)
    tfidf = sp.csr_matrix(tfidf)
    metadata = {"doc_freqs": freqs, "tokenizer": "simple", "hash_size": HASH_SIZE,
                "ngram": NGRAM, "doc_dict": (doc2idx, doc_ids)}

    stop_digest = hashlib.sha256("\n".join(sorted(utils.STOPWORDS)).encode()).hexdigest()
    out = {"docs": np.array(docs), "claims": np.array(claims),
           "stop_digest": np.array(stop_digest),
           "cfg": np.array([HASH_SIZE, NGRAM, len(docs)], np.int64),
           "count_digest": np.array(digest(count_matrix.data.astype(np.float64),
                                           count_matrix.indices.astype(np.int64),
                                           count_matrix.indptr.astype(np.int64))),
           "tfidf_digest": np.array(digest(tfidf.data.astype(np.float64),
                                           tfidf.indices.astype(np.int64),
                                           tfidf.indptr.astype(np.int64))),
           "doc_freqs": freqs.astype(np.int64)}

    with tempfile.TemporaryDirectory() as td:
        path = os.path.join(td, "tfidf.npz")
        utils.save_sparse_csr(path, tfidf, metadata)
        ranker = TfidfDocRanker(tfidf_path=path, strict=False)
        full_docs = {d: t for d, t in zip(doc_ids, docs)}
        k = 10
        for c, claim in enumerate(claims):
            wids = [utils.hash(w, HASH_SIZE) for w in ranker.parse(utils.normalize(claim))]
            out[f"wids_{c}"] = np.array(wids, np.int64)
            for tag, bigram_only in (("all", False), ("bi", True)):
                cand = ev.documents_filtering(claim, None, count_matrix, metadata, full_docs,
                                              bigram_only)
                out[f"cand_{tag}_{c}"] = np.array(sorted(doc2idx[d] for d in cand), np.int64)
            ids, scores = ranker.closest_docs(claim, k)
            out[f"top_idx_{c}"] = np.array([doc2idx[d] for d in ids], np.int64)
            out[f"top_score_{c}"] = np.asarray(scores, np.float64)
    np.savez_compressed(os.path.join(HERE, "sparse.npz"), **out)
    print("wrote", os.path.join(HERE, "sparse.npz"), len(claims), "claims")


if __name__ == "__main__":
    main()
