"""GPU sparse TF-IDF path (irc_csr_union_*, irc_csr_spmv_f64, irc_topk_f64) against
the reference's own outputs (tests/golden/sparse.npz, make_sparse_goldens.py):

* documents_filtering candidates: bit-exact doc index lists (all n-grams and
  bigram_only);
* closest_docs: fp64 scores bit-identical to the reference's scipy product; the
  ranking equals the reference's except inside groups of exactly equal scores,
  where this build puts the lower doc index first (numpy's argpartition leaves
  it unspecified) -- checked against the full scipy score row.
"""
import numpy as np
import pytest

from conftest import load_golden

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def corpus(gpu):
    from irc_amd import sparse

    g = load_golden("sparse.npz")
    hash_size, n, _ = (int(x) for x in g["cfg"])
    counts = sparse.build_count_matrix([str(t) for t in g["docs"]], hash_size, n)
    tfidf = sparse.tfidf_matrix(counts)
    return g, counts, tfidf, sparse.doc_freqs(counts)


@pytest.mark.parametrize("bigram_only", [False, True])
def test_documents_filtering_matches_reference(gpu, corpus, bigram_only):
    from irc_amd import sparse

    g, counts, _, _ = corpus
    index = sparse.SparseIndex(counts, ngram=int(g["cfg"][1]), device=gpu)
    claims = [str(c) for c in g["claims"]]
    got = index.documents_filtering(claims, bigram_only=bigram_only)
    tag = "bi" if bigram_only else "all"
    for c in range(len(claims)):
        np.testing.assert_array_equal(got[c], g[f"cand_{tag}_{c}"], err_msg=claims[c])


def test_closest_docs_matches_reference(gpu, corpus):
    from irc_amd import sparse

    g, counts, tfidf, freqs = corpus
    index = sparse.SparseIndex(tfidf, ngram=int(g["cfg"][1]), doc_freqs_=freqs, device=gpu)
    claims = [str(c) for c in g["claims"]]
    k = 10
    got = index.batch_closest_docs(claims, k)
    for c, (idx, sc) in enumerate(got):
        ref_idx, ref_sc = g[f"top_idx_{c}"], g[f"top_score_{c}"]
        # scores bit-identical to the reference's (same fp64 order of operations)
        np.testing.assert_array_equal(sc, ref_sc, err_msg=claims[c])
        # full scipy row -> the expected order under the (score desc, idx asc) rule
        wids, w = index.text2spvec(claims[c])
        row = np.zeros(tfidf.shape[1])
        for h, x in zip(wids, w):
            lo, hi = tfidf.indptr[h], tfidf.indptr[h + 1]
            row[tfidf.indices[lo:hi]] += x * tfidf.data[lo:hi]
        nz = np.nonzero(row)[0]
        order = nz[np.lexsort((nz, -row[nz]))][:k]
        np.testing.assert_array_equal(idx, order, err_msg=claims[c])
        # same set as the reference outside exact-tie groups at the boundary
        for d in set(idx.tolist()) ^ set(ref_idx.tolist()):
            assert row[d] == sc[-1]


def test_union_large_random(gpu):
    """Many long rows, docs beyond one compaction chunk, several queries."""
    import scipy.sparse as sp

    from irc_amd import sparse

    rng = np.random.default_rng(3)
    n_docs, hash_size, nnz = 600_000, 4096, 2_000_000
    m = sp.csr_matrix((np.ones(nnz), (rng.integers(0, hash_size, nnz),
                                      rng.integers(0, n_docs, nnz))), shape=(hash_size, n_docs))
    m.sum_duplicates()
    index = sparse.SparseIndex(m, device=gpu)
    rows = [np.unique(rng.integers(0, hash_size, int(r))) for r in (1, 7, 40, 0, 300)]
    idx, off = index.union(rows)
    idx, off = idx.cpu().numpy(), off.cpu().numpy()
    for q, r in enumerate(rows):
        want = np.unique(m[r].nonzero()[1]) if len(r) else np.zeros(0, np.int64)
        np.testing.assert_array_equal(idx[off[q]:off[q + 1]], want)


def test_reference_api_dropins(gpu, corpus, tmp_path):
    """src.evaluation.documents_filtering and TfidfDocRanker (loaded from a
    build_tfidf-format .npz) with the reference's signatures and return types."""
    import argparse

    import numpy as np

    from irc_amd import sparse
    from src.evaluation import documents_filtering

    g, counts, tfidf, freqs = corpus
    n_docs = int(g["cfg"][2])
    doc_ids = [f"doc_{i}" for i in range(n_docs)]
    metadata = {"doc_freqs": freqs, "tokenizer": "simple", "hash_size": int(g["cfg"][0]),
                "ngram": int(g["cfg"][1]), "doc_dict": ({d: i for i, d in enumerate(doc_ids)},
                                                        doc_ids)}
    full = {d: str(t) for d, t in zip(doc_ids, g["docs"])}
    args = argparse.Namespace(device=gpu)
    claim = str(g["claims"][0])
    docs = documents_filtering(claim, args, counts, metadata, full, False)
    assert sorted(metadata["doc_dict"][0][d] for d in docs) == g["cand_all_0"].tolist()
    path = str(tmp_path / "tfidf.npz")
    np.savez(path, data=tfidf.data, indices=tfidf.indices, indptr=tfidf.indptr,
             shape=tfidf.shape, metadata=metadata)
    ranker = sparse.TfidfDocRanker(path, strict=False, device=gpu)
    ids, scores = ranker.closest_docs(claim, 10)
    np.testing.assert_array_equal(scores, g["top_score_0"])
    assert ids[0] == doc_ids[int(g["top_idx_0"][0])]


def test_dense_rows_union_and_topk_ties(gpu):
    """Zipf-head-like rows covering most docs (runs of equal bitmap words within a
    wave, merged before the atomic) and small-integer data (many exact score ties
    at the k-th boundary, candidate counts far above one workgroup's threads)."""
    import scipy.sparse as sp

    from irc_amd import sparse

    rng = np.random.default_rng(11)
    n_docs, hash_size = 70_001, 64
    dens = [0.9, 0.6, 0.3, 0.05, 0.002] + [0.01] * (hash_size - 5)
    rr, cc = [], []
    for r, p in enumerate(dens):
        docs = np.nonzero(rng.random(n_docs) < p)[0]
        rr.append(np.full(len(docs), r))
        cc.append(docs)
    rr, cc = np.concatenate(rr), np.concatenate(cc)
    m = sp.csr_matrix((rng.integers(1, 4, len(rr)).astype(np.float64), (rr, cc)),
                      shape=(hash_size, n_docs))
    m.sort_indices()
    index = sparse.SparseIndex(m, device=gpu)
    rows = [np.array([0]), np.array([1, 2]), np.array([0, 3, 4, 9]), np.array([4]),
            np.array([2, 5, 6, 7, 8])]
    idx, off = index.union(rows)
    idx, off = idx.cpu().numpy(), off.cpu().numpy()
    for q, r in enumerate(rows):
        np.testing.assert_array_equal(idx[off[q]:off[q + 1]], np.unique(m[r].nonzero()[1]))
    weights = [np.ones(len(r)) * (1.0 + 0.5 * q) for q, r in enumerate(rows)]
    for mode in ("union", "all", "auto"):  # gathered through the union / whole row
        for k in (1, 100, 1024):
            got = index.topk_rows(rows, weights, k, candidates=mode)
            for q, (r, w) in enumerate(zip(rows, weights)):
                row = np.asarray(m[r].T @ w).ravel()
                nz = np.nonzero(row)[0]
                order = nz[np.lexsort((nz, -row[nz]))][:k]
                np.testing.assert_array_equal(got[q][0], order, err_msg=f"{mode} q={q} k={k}")
                np.testing.assert_array_equal(got[q][1], row[order])
