"""Hashed n-gram TF-IDF retrieval -- the reference's actual ``predict`` path
 with the sparse products on the GPU.

Host side (text -> hashed n-gram ids, the offline matrix build) restates the
reference's DrQA pieces; the corpus matrices live in HBM and every per-query
product runs in HIP kernels (csrc/sparse.hip) behind the C ABI:

* ``SparseIndex.documents_filtering`` = src/evaluation.py:57-81 (the docs
  sharing any hashed n-gram with the claim), on ``irc_csr_union_*``;
* ``SparseIndex.closest_docs`` / ``batch_closest_docs`` =
  preprocessing/drqa/retriever/tfidf_doc_ranker.py:60-83 (tf-idf sparse dot +
  top-k), on ``irc_csr_spmv_f64`` (bit-identical fp64 scores) + ``irc_topk_f64``.

Third-party arithmetic the reference calls: ``regex`` (SimpleTokenizer's
Unicode classes) and scikit-learn's ``murmurhash3_32`` (utils.hash), used as-is.
"""
from __future__ import annotations

import unicodedata
from collections import Counter

import numpy as np
import regex
import torch

from . import _lib
from ._torch import ptr, stream_ptr

# preprocessing/drqa/tokenizers/simple_tokenizer.py:18-29: alphanumeric runs or
# single non-whitespace characters, case-insensitive Unicode matching
_TOKEN_RE = regex.compile(r"([\p{L}\p{N}\p{M}]+)|([^\p{Z}\p{C}])",
                          flags=regex.IGNORECASE + regex.UNICODE + regex.MULTILINE)
_PUNCT_RE = regex.compile(r"^\p{P}+$")

# preprocessing/drqa/retriever/utils.py:52-71: the NLTK English stop words plus
# contraction fragments (data, listed alphabetically here)
STOPWORDS = frozenset("""
'd 'll 'm 're 's 've '' `` a about above after again against ain all am an and any are aren
as at be because been before being below between both but by can couldn d did didn do does
doesn doing don down during each few for from further had hadn has hasn have haven having he
her here hers herself him himself his how i if in into is isn it its itself just ll m ma me
mightn more most mustn my myself n't needn no nor not now o of off on once only or other our
ours ourselves out over own re s same shan she should shouldn so some such t than that the
their theirs them themselves then there these they this those through to too under until up
ve very was wasn we were weren what when where which while who whom why will with won
wouldn y you your yours yourself yourselves
""".split())


def normalize(text: str) -> str:
    """utils.py:60-62 (NFD)."""
    return unicodedata.normalize("NFD", text)


def tokenize(text: str) -> list[str]:
    """SimpleTokenizer.tokenize (simple_tokenizer.py:31-54): the token texts."""
    return [m.group() for m in _TOKEN_RE.finditer(text)]


def filter_word(text: str) -> bool:
    """utils.py:65-72: punctuation-only tokens and stop words."""
    text = normalize(text)
    return bool(_PUNCT_RE.match(text)) or text.lower() in STOPWORDS


def filter_ngram(gram) -> bool:
    """utils.py:75-94, mode 'any'."""
    return any(filter_word(w) for w in gram)


def ngrams(words: list[str], n: int, uncased: bool = True) -> list[str]:
    """Tokens.ngrams (tokenizers/tokenizer.py:79-103) with filter_ngram."""
    if uncased:
        words = [w.lower() for w in words]
    return [" ".join(words[s:e + 1]) for s in range(len(words))
            for e in range(s, min(s + n, len(words))) if not filter_ngram(words[s:e + 1])]


def feature_hash(token: str, num_buckets: int) -> int:
    """utils.py:43-45: unsigned 32-bit MurmurHash3 (scikit-learn) mod buckets."""
    from sklearn.utils import murmurhash3_32

    return murmurhash3_32(token, positive=True) % num_buckets


def text_ngram_ids(text: str, n: int, hash_size: int) -> list[int]:
    """TfidfDocRanker.parse + hashing (tfidf_doc_ranker.py:85-98) of one text."""
    return [feature_hash(g, hash_size) for g in ngrams(tokenize(normalize(text)), n)]


def build_count_matrix(texts, hash_size: int, n: int = 2):
    """build_tfidf.py:63-121 (count + get_count_matrix), in-process: scipy CSR
    [hash_size, n_docs] of hashed n-gram counts (offline preprocessing, host)."""
    import scipy.sparse as sp

    row, col, data = [], [], []
    for j, t in enumerate(texts):
        c = Counter(text_ngram_ids(t, n, hash_size))
        row.extend(c.keys())
        col.extend([j] * len(c))
        data.extend(c.values())
    m = sp.csr_matrix((data, (row, col)), shape=(hash_size, len(texts)))
    m.sum_duplicates()
    return m


def doc_freqs(counts) -> np.ndarray:
    """build_tfidf.py:155-159: docs per hashed n-gram."""
    return np.asarray((counts > 0).astype(int).sum(1)).squeeze()


def tfidf_matrix(counts):
    """build_tfidf.py:128-152: log1p(tf) * max(0, log((N - Nt + .5) / (Nt + .5)))."""
    import scipy.sparse as sp

    ns = doc_freqs(counts)
    idfs = np.log((counts.shape[1] - ns + 0.5) / (ns + 0.5))
    idfs[idfs < 0] = 0
    return sp.csr_matrix(sp.diags(idfs, 0).dot(counts.log1p()))


class SparseIndex:
    """A CSR matrix [hash_size, n_docs] resident in HBM plus the metadata the
    reference keeps beside it (``ngram``, ``hash_size``, ``doc_freqs``)."""

    def __init__(self, matrix, ngram: int = 2, doc_freqs_=None, device=None):
        device = torch.device(device or "cuda")
        m = matrix.tocsr()
        if not m.has_sorted_indices:  # the doc-range split of irc_csr_spmv_f64 needs them
            m = m.sorted_indices()
        self.hash_size, self.n_docs = m.shape
        self.ngram = int(ngram)
        self._row_len = np.diff(m.indptr).astype(np.int64)  # host: union-size bounds
        self.indptr = torch.from_numpy(m.indptr.astype(np.int64)).to(device)
        self.indices = torch.from_numpy(m.indices.astype(np.int32)).to(device)
        self.data = torch.from_numpy(m.data.astype(np.float64)).to(device)
        self.doc_freqs = None if doc_freqs_ is None else np.asarray(doc_freqs_).squeeze()
        self.device = device

    # ---------------------------------------------------------------- queries
    def _pack(self, row_lists, weights=None):
        off = np.zeros(len(row_lists) + 1, np.int64)
        off[1:] = np.cumsum([len(r) for r in row_lists])
        rows = np.concatenate([np.asarray(r, np.int64) for r in row_lists]) if off[-1] \
            else np.zeros(0, np.int64)
        dev = self.device
        t_off = torch.from_numpy(off).to(dev)
        t_rows = torch.from_numpy(rows).to(dev)
        t_w = None
        if weights is not None:
            w = np.concatenate([np.asarray(x, np.float64) for x in weights]) if off[-1] \
                else np.zeros(0, np.float64)
            t_w = torch.from_numpy(w).to(dev)
        return t_off, t_rows, t_w, int(off[-1])

    def union(self, row_lists):
        """Sorted unique docs with a nonzero in any row of each list (device)."""
        Q = len(row_lists)
        t_off, t_rows, _, n_pairs = self._pack(row_lists)
        words = (self.n_docs + 31) // 32
        nchunks = int(_lib.fn("irc_csr_union_chunks")(self.n_docs))
        bitmaps = torch.empty((max(Q * words, 1),), dtype=torch.int32, device=self.device)
        chunk_sums = torch.empty((max(Q * nchunks, 1),), dtype=torch.int64, device=self.device)
        st = stream_ptr(self.device)
        _lib.call("irc_csr_union_count", ptr(self.indptr), ptr(self.indices), self.n_docs,
                  ptr(t_off), ptr(t_rows), Q, n_pairs, ptr(bitmaps), ptr(chunk_sums), st)
        counts = chunk_sums[:Q * nchunks].view(Q, nchunks).sum(1) if nchunks else \
            torch.zeros(Q, dtype=torch.int64, device=self.device)
        out_off = torch.zeros(Q + 1, dtype=torch.int64, device=self.device)
        out_off[1:] = torch.cumsum(counts, 0)
        total = int(out_off[-1].item())
        out = torch.empty((max(total, 1),), dtype=torch.int32, device=self.device)
        _lib.call("irc_csr_union_emit", ptr(bitmaps), self.n_docs, Q, ptr(chunk_sums),
                  ptr(out_off), ptr(out), st)
        return out[:total], out_off

    def documents_filtering(self, claims, bigram_only: bool = True):
        """src/evaluation.py:57-81 for a batch of claims: per claim the sorted doc
        indices sharing a hashed n-gram (bigrams only when bigram_only)."""
        row_lists = []
        for c in claims:
            grams = ngrams(tokenize(c), self.ngram)
            if bigram_only:
                grams = [g for g in grams if len(g.split()) > 1]
            row_lists.append(np.unique([feature_hash(g, self.hash_size) for g in grams]))
        idx, off = self.union(row_lists)
        idx, off = idx.cpu().numpy(), off.cpu().numpy()
        return [idx[off[i]:off[i + 1]].astype(np.int64) for i in range(len(claims))]

    def text2spvec(self, query: str):
        """tfidf_doc_ranker.py:100-126: (unique hashed ids ascending, fp64 weights)."""
        wids = text_ngram_ids(query, self.ngram, self.hash_size)
        if not wids:
            return np.zeros(0, np.int64), np.zeros(0, np.float64)
        uniq, cnt = np.unique(wids, return_counts=True)
        tfs = np.log1p(cnt)
        ns = self.doc_freqs[uniq]
        idfs = np.log((self.n_docs - ns + 0.5) / (ns + 0.5))
        idfs[idfs < 0] = 0
        return uniq.astype(np.int64), np.multiply(tfs, idfs)

    def batch_closest_docs(self, queries, k: int = 1):
        """closest_docs for each query: [(doc indices, fp64 scores)] by descending
        score (equal scores: lower index first); queries with no valid n-gram
        return empty lists (the reference's strict=False behaviour)."""
        if self.doc_freqs is None:
            raise ValueError("closest_docs needs doc_freqs (build with doc_freqs(counts))")
        vecs = [self.text2spvec(q) for q in queries]
        return self.topk_rows([v[0] for v in vecs], [v[1] for v in vecs], k)

    def topk_rows(self, rows, weights, k: int, candidates: str = "auto"):
        """Top-k docs of sum_r w_r * A[r] per query (rows ascending, fp64 weights):
        [(doc indices, fp64 scores)], (score desc, index asc), nonzero scores only.

        candidates: "union" gathers each query's scores through its row union;
        "all" scans the whole score row contiguously (same result: the buffer is
        zero outside the union); "auto" takes "all" when the rows' total length,
        an upper bound of the union, averages >= n_docs / 8 per query."""
        Q = len(rows)
        t_off, t_rows, t_w, _ = self._pack(rows, weights)
        dense = torch.zeros((Q, self.n_docs), dtype=torch.float64, device=self.device)
        st = stream_ptr(self.device)
        _lib.call("irc_csr_spmv_f64", ptr(self.indptr), ptr(self.indices), ptr(self.data),
                  self.n_docs, ptr(t_off), ptr(t_rows), ptr(t_w), Q, ptr(dense), st)
        if candidates == "auto":
            bound = sum(min(int(self._row_len[np.asarray(r, np.int64)].sum()), self.n_docs)
                        for r in rows)
            candidates = "all" if Q and bound * 8 >= Q * self.n_docs else "union"
        if candidates == "all":
            cand_p = cand_off_p = None
        elif candidates == "union":
            cand, cand_off = self.union(rows)
            cand_p, cand_off_p = ptr(cand), ptr(cand_off)
        else:
            raise ValueError(f"candidates must be 'auto', 'union' or 'all', not {candidates!r}")
        out_s = torch.empty((Q, k), dtype=torch.float64, device=self.device)
        out_i = torch.empty((Q, k), dtype=torch.int64, device=self.device)
        out_n = torch.empty((Q,), dtype=torch.int32, device=self.device)
        _lib.call("irc_topk_f64", ptr(dense), self.n_docs, cand_p, cand_off_p, Q, k,
                  ptr(out_s), ptr(out_i), ptr(out_n), st)
        s, i, n = out_s.cpu().numpy(), out_i.cpu().numpy(), out_n.cpu().numpy()
        return [(i[r, :n[r]], s[r, :n[r]]) for r in range(Q)]

    def closest_docs(self, query: str, k: int = 1):
        return self.batch_closest_docs([query], k)[0]


def load_sparse_csr(filename):
    """utils.py:33-37: (csr matrix, metadata dict) from a build_tfidf .npz.  The
    metadata is a pickled dict, so this is for files the user built, never for
    files shipped by others."""
    import scipy.sparse as sp

    loader = np.load(filename, allow_pickle=True)
    matrix = sp.csr_matrix((loader["data"], loader["indices"], loader["indptr"]),
                           shape=loader["shape"])
    return matrix, loader["metadata"].item(0) if "metadata" in loader else None


class TfidfDocRanker:
    """Drop-in for preprocessing/drqa/retriever/tfidf_doc_ranker.py:28-126 with the
    sparse products on the GPU (SparseIndex); returns doc ids as the reference."""

    def __init__(self, tfidf_path, strict=True, device=None):
        matrix, metadata = load_sparse_csr(tfidf_path)
        if metadata.get("tokenizer", "simple") != "simple":
            raise ValueError("only the DrQA 'simple' tokenizer is supported")
        self.ngrams = metadata["ngram"]
        self.hash_size = metadata["hash_size"]
        self.doc_freqs = np.asarray(metadata["doc_freqs"]).squeeze()
        self.doc_dict = metadata["doc_dict"]
        self.num_docs = len(self.doc_dict[0])
        self.strict = strict
        self.index = SparseIndex(matrix, ngram=self.ngrams, doc_freqs_=self.doc_freqs,
                                 device=device)

    def get_doc_index(self, doc_id):
        return self.doc_dict[0][doc_id]

    def get_doc_id(self, doc_index):
        return self.doc_dict[1][doc_index]

    def parse(self, query):
        return ngrams(tokenize(query), self.ngrams)

    def text2spvec(self, query):
        wids, w = self.index.text2spvec(query)
        if len(wids) == 0 and self.strict:
            raise RuntimeError("No valid word in: %s" % query)
        return wids, w

    def batch_closest_docs(self, queries, k=1, num_workers=None):
        if self.strict:
            for q in queries:
                self.text2spvec(q)
        out = self.index.batch_closest_docs(queries, k)
        return [([self.get_doc_id(int(i)) for i in idx], sc) for idx, sc in out]

    def closest_docs(self, query, k=1):
        return self.batch_closest_docs([query], k)[0]
