"""Host side of the sparse TF-IDF path (irc_amd.sparse) against the fixtures the
reference itself produced (tests/golden/make_sparse_goldens.py): tokenisation,
n-gram filtering and feature hashing per claim, and the rebuilt count / TF-IDF
matrices (sha256 of data, indices, indptr)."""
import hashlib

import numpy as np

from conftest import load_golden


def _digest(*arrays):
    h = hashlib.sha256()
    for a in arrays:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


def test_stopwords_match_reference():
    from irc_amd import sparse

    g = load_golden("sparse.npz")
    assert hashlib.sha256("\n".join(sorted(sparse.STOPWORDS)).encode()).hexdigest() == \
        str(g["stop_digest"])


def test_claim_ngram_ids_match_reference():
    from irc_amd import sparse

    g = load_golden("sparse.npz")
    hash_size, n, _ = (int(x) for x in g["cfg"])
    for c, claim in enumerate(g["claims"]):
        ids = sparse.text_ngram_ids(str(claim), n, hash_size)
        np.testing.assert_array_equal(np.array(ids, np.int64), g[f"wids_{c}"], err_msg=str(claim))


def test_rebuilt_matrices_match_reference():
    from irc_amd import sparse

    g = load_golden("sparse.npz")
    hash_size, n, _ = (int(x) for x in g["cfg"])
    counts = sparse.build_count_matrix([str(t) for t in g["docs"]], hash_size, n)
    assert _digest(counts.data.astype(np.float64), counts.indices.astype(np.int64),
                   counts.indptr.astype(np.int64)) == str(g["count_digest"])
    np.testing.assert_array_equal(sparse.doc_freqs(counts), g["doc_freqs"])
    tfidf = sparse.tfidf_matrix(counts)
    assert _digest(tfidf.data.astype(np.float64), tfidf.indices.astype(np.int64),
                   tfidf.indptr.astype(np.int64)) == str(g["tfidf_digest"])
