"""CPU oracle for the contrastive-training + dense-retrieval hot path.

TEST INFRASTRUCTURE ONLY.  This module is a plain-numpy restatement of the
reference algorithm (PM25/Information-Retrieval-with-Contrastive-Learning,
mounted read-only at /root/reference).  Only ``tests/``, ``__graft_entry__.smoke()``
and ``bench.py``'s ``cpu_baseline`` leg may import it, and only as the checker or
the timed CPU baseline -- never as a product code path.  The MI355X product path
(``irc_amd``) never imports it and fails loudly when the HIP library is missing.

Parity pinning: every function here is checked in ``tests/test_oracle_golden.py``
against golden vectors that ``tests/golden/make_goldens.py`` produced by importing
and running the reference itself (torch 2.10 CPU / transformers 5.15 in this
container; the reference pins torch 1.7.1 / transformers 4.6.1, whose arithmetic
for these ops is the same up to fp32 rounding order).

Citations are ``file:line`` relative to the reference root.
"""
from __future__ import annotations

import numpy as np

try:  # exact-erf GELU as HF BERT uses (hidden_act="gelu")
    from scipy.special import erf as _erf
except Exception:  # pragma: no cover - scipy is in the image
    import math

    _erf = np.vectorize(math.erf)

F32 = np.float32
F64 = np.float64

# ---------------------------------------------------------------------------
# Dense retrieval: scores = <e_q, e_n>, per-query top-k by (score desc, idx asc)
# ---------------------------------------------------------------------------
# Semantics: src/evaluation.py:110-112 (cosine of L2-normalised ctx2vec outputs,
# i.e. a plain dot product) + preprocessing/drqa/retriever/tfidf_doc_ranker.py:60-75
# (closest_docs: argpartition(-s, k)[:k] then argsort(-s[o]) -> ids by descending
# score).  numpy leaves the order of tied scores unspecified there; this build
# defines it: equal scores -> lower global doc index first.


def canon_scores(s: np.ndarray) -> np.ndarray:
    """fp32 scores with -0.0 folded to +0.0 and NaN mapped to -inf.

    The HIP kernel encodes (score, index) into one distinct 64-bit key; this is
    the same canonicalisation it applies before encoding.
    """
    s = np.asarray(s, dtype=F32).copy()
    s[s == 0] = 0.0
    s[np.isnan(s)] = -np.inf
    return s


def topk_rows(scores: np.ndarray, k: int, idx_base: int = 0):
    """Exact per-row top-k of an fp32 score matrix with the (desc, idx asc) rule.

    Returns (idx int64 [Q, k], score fp32 [Q, k]); rows with fewer than k
    columns are padded with (-1, -inf).
    """
    scores = canon_scores(scores)
    q, n = scores.shape
    out_i = np.full((q, k), -1, dtype=np.int64)
    out_s = np.full((q, k), -np.inf, dtype=F32)
    kk = min(k, n)
    if kk == 0 or q == 0:
        return out_i, out_s
    # k-th largest value per row, then strictly-greater + lowest-index ties.
    kth = -np.partition(-scores, kk - 1, axis=1)[:, kk - 1]
    for r in range(q):
        row = scores[r]
        gt = np.flatnonzero(row > kth[r])
        eq = np.flatnonzero(row == kth[r])[: kk - gt.size]
        sel = np.concatenate([gt, eq])
        order = np.lexsort((sel, -row[sel]))  # primary: score desc, then idx asc
        sel = sel[order]
        out_i[r, :kk] = sel + idx_base
        out_s[r, :kk] = row[sel]
    return out_i, out_s


def scan_scores(queries: np.ndarray, docs: np.ndarray) -> np.ndarray:
    """fp32 dot products, accumulated in fp64 then rounded once.

    For the integer-grid fixtures (values m/2^7, |m| <= 127, D <= 768) every
    product and partial sum is exact in fp32, so this equals the GPU result
    bit for bit whatever the MFMA accumulation order.
    """
    return (np.asarray(queries, F64) @ np.asarray(docs, F64).T).astype(F32)


def scan_topk(queries: np.ndarray, docs: np.ndarray, k: int, doc_offset: int = 0,
              chunk: int = 65536):
    """Corpus scan + top-k, chunked over docs with a running exact merge."""
    q = np.asarray(queries)
    best_i = np.full((q.shape[0], 0), -1, dtype=np.int64)
    best_s = np.full((q.shape[0], 0), -np.inf, dtype=F32)
    for c0 in range(0, docs.shape[0], chunk):
        s = scan_scores(q, docs[c0:c0 + chunk])
        ci, cs = topk_rows(s, k, doc_offset + c0)
        best_i, best_s = merge_topk([best_i, ci], [best_s, cs], k)
    if best_i.shape[1] < k:
        pad = k - best_i.shape[1]
        best_i = np.pad(best_i, ((0, 0), (0, pad)), constant_values=-1)
        best_s = np.pad(best_s, ((0, 0), (0, pad)), constant_values=-np.inf)
    return best_i, best_s


# ---------------------------------------------------------------------------
# fp8 corpus (BASELINE.json config C5): OCP e4m3fn quantisation
# ---------------------------------------------------------------------------
# Not in the reference (which scores fp32 embeddings, src/evaluation.py:110-112);
# this restates the published OCP 8-bit floating point spec (E4M3, "fn": no
# infinities, S.1111.111 = NaN, max 448, subnormals m * 2^-9) with
# round-to-nearest-even, and saturation to +-448 as the build applies before
# converting.  Pinned against torch's float8_e4m3fn cast in
# tests/test_oracle_golden.py (a second, independent implementation of the spec).


def e4m3_decode_table() -> np.ndarray:
    """float32 value of each of the 256 e4m3fn codes (NaN for S.1111.111)."""
    c = np.arange(256)
    sign = np.where(c >> 7, -1.0, 1.0)
    e = (c >> 3) & 15
    m = c & 7
    mag = np.where(e == 0, m * 2.0 ** -9, (1.0 + m / 8.0) * 2.0 ** (e - 7.0))
    v = sign * mag
    v[(e == 15) & (m == 7)] = np.nan
    return v.astype(F32)


def quantize_e4m3(x: np.ndarray, scale: float = 1.0) -> np.ndarray:
    """uint8 e4m3fn codes of RNE(x * scale) (fp32 arithmetic), saturated to +-448."""
    a = np.asarray(x, dtype=F32) * F32(scale)
    nan = np.isnan(a)
    neg = np.signbit(a)
    mag = np.minimum(np.abs(np.where(nan, 0, a)).astype(F64), 448.0)
    # quantum: 2^(E-3) in the normal range (a = 1.f * 2^E, E >= -6), 2^-9 below
    _, e2 = np.frexp(mag)
    E = np.maximum(e2.astype(np.int64) - 1, -6)
    quantum = np.ldexp(1.0, E - 3)
    qv = np.rint(mag / quantum) * quantum  # round half to even, exact in fp64
    # encode the (representable) quantised magnitude
    table = e4m3_decode_table()[:127].astype(F64)  # codes 0x00..0x7e, ascending
    code = np.searchsorted(table, qv).astype(np.uint8)
    code = np.where(neg, code | 0x80, code).astype(np.uint8)
    return np.where(nan, np.uint8(0x7F), code).astype(np.uint8)


def quantize_rows_e4m3(x: np.ndarray):
    """Per-row e4m3 (BASELINE config C5 fp8 encoder weights; not in the reference,
    which runs BERT in fp32): scale = amax|row| / 448 (1 for a zero row), codes =
    RNE(row * (448 / amax)) in fp32 -- returns (codes uint8, scales float32)."""
    x = np.asarray(x, dtype=F32)
    amax = np.max(np.abs(x), axis=1).astype(F32)
    inv = np.where(amax > 0, F32(448.0) / np.where(amax > 0, amax, F32(1)), F32(1)).astype(F32)
    codes = np.stack([quantize_e4m3(x[i], inv[i]) for i in range(x.shape[0])]) if len(x) else \
        np.zeros(x.shape, np.uint8)
    scale = np.where(amax > 0, amax / F32(448.0), F32(1)).astype(F32)
    return codes, scale


def mx_pad(rows: int) -> int:
    return (int(rows) + 255) // 256 * 256


def mx_scale_index(row, col, mpad):
    """Byte offset of (row, column)'s E8M0 scale in the MX layout (csrc/mx.h):
    per 128-column K-tile one record of mpad * 4 bytes; within it per 256-row block
    1 KB ordered [row bit 7][k-block = col bits 5-6][row bits 0-3][row bits 4-6]."""
    row = np.asarray(row, dtype=np.int64)
    col = np.asarray(col, dtype=np.int64)
    return ((col >> 7) * mpad * 4 + (row >> 8) * 1024 + ((row >> 7) & 1) * 512 +
            ((col >> 5) & 3) * 128 + (row & 15) * 8 + ((row >> 4) & 7))


def mx_exponent(amax: np.ndarray) -> np.ndarray:
    """Smallest p with amax / 2^p <= 448 (0 for amax == 0), clamped to [-127, 127]."""
    amax = np.asarray(amax, dtype=F64)
    p = np.zeros(amax.shape, np.int64)
    nz = amax > 0
    e = np.ceil(np.log2(np.where(nz, amax, 1.0) / 448.0)).astype(np.int64)
    e = np.where(np.ldexp(448.0, e - 1) >= amax, e - 1, e)  # exact checks in fp64
    e = np.where(np.ldexp(448.0, e) < amax, e + 1, e)
    p[nz] = e[nz]
    return np.clip(p, -127, 127)


def quantize_mx_e4m3(x: np.ndarray):
    """MX-fp8 of x [M, K] (K % 128 == 0; config C5's CDNA4 block-scaled MFMA operand,
    not in the reference): per 32 consecutive values of a row the power-of-two scale
    2^p of mx_exponent(block max), codes e4m3(RNE(x / 2^p)).  Returns (codes uint8
    [M, K], scales uint8 in the MX layout with mpad = mx_pad(M) rows, E8M0 = p + 127)."""
    x = np.asarray(x, dtype=F32)
    M, K = x.shape
    blk = x.reshape(M, K // 32, 32)
    p = mx_exponent(np.max(np.abs(blk), axis=2))                  # [M, K/32]
    scaled = (blk.astype(F64) * np.ldexp(1.0, -p)[..., None]).astype(F32)  # exact (power of 2)
    codes = quantize_e4m3(scaled.reshape(M, K))
    mp = mx_pad(M)
    scales = np.zeros((K // 128) * mp * 4, np.uint8)
    rows, kb = np.meshgrid(np.arange(M), np.arange(K // 32), indexing="ij")
    scales[mx_scale_index(rows, kb * 32, mp)] = (p + 127).astype(np.uint8)
    return codes, scales


def dequantize_mx_e4m3(codes: np.ndarray, scales: np.ndarray) -> np.ndarray:
    """float64 values of an MX-fp8 matrix (codes [M, K], scales in the MX layout)."""
    M, K = codes.shape
    mp = mx_pad(M)
    rows, kb = np.meshgrid(np.arange(M), np.arange(K // 32), indexing="ij")
    p = scales[mx_scale_index(rows, kb * 32, mp)].astype(np.int64) - 127
    v = e4m3_decode_table()[codes].astype(F64).reshape(M, K // 32, 32)
    return (v * np.ldexp(1.0, p)[..., None]).reshape(M, K)


def dequantize_e4m3(codes: np.ndarray) -> np.ndarray:
    return e4m3_decode_table()[np.asarray(codes, dtype=np.uint8)]


def scan_topk_fp8(q_codes: np.ndarray, d_codes: np.ndarray, k: int, doc_offset: int = 0,
                  score_scale: float = 1.0):
    """The fp8 scan's result: top-k of the quantised embeddings' dot products,
    times the (power-of-two) score_scale."""
    idx, sc = scan_topk(dequantize_e4m3(q_codes), dequantize_e4m3(d_codes), k, doc_offset)
    return idx, (sc * F32(score_scale)).astype(F32)


def scan_topk_fast_f32(queries: np.ndarray, docs: np.ndarray, k: int,
                       doc_offset: int = 0, chunk: int = 65536):
    """Same as scan_topk but with fp32 BLAS matmul (the timed CPU baseline).

    This is the reference's CPU arithmetic (torch/numpy fp32 ``q @ d.T``) plus the
    closest_docs selection; used by bench.py's cpu_baseline leg.
    """
    q = np.ascontiguousarray(queries, dtype=F32)
    best_i = np.full((q.shape[0], 0), -1, dtype=np.int64)
    best_s = np.full((q.shape[0], 0), -np.inf, dtype=F32)
    for c0 in range(0, docs.shape[0], chunk):
        d = np.asarray(docs[c0:c0 + chunk], dtype=F32)
        s = q @ d.T
        ci, cs = topk_rows(s, k, doc_offset + c0)
        best_i, best_s = merge_topk([best_i, ci], [best_s, cs], k)
    return best_i, best_s


def merge_topk(idx_list, score_list, k: int):
    """Merge per-shard top-k lists (global indices) with the (desc, idx asc) rule.

    Mirrors the multi-GPU reduce: each shard's list is exact for its shard, so
    the merge of the lists is exact for the union.  Entries with idx < 0 are
    padding and dropped.
    """
    idx = np.concatenate([np.asarray(i, np.int64) for i in idx_list], axis=1)
    sc = np.concatenate([canon_scores(s) for s in score_list], axis=1)
    q = idx.shape[0]
    out_i = np.full((q, k), -1, dtype=np.int64)
    out_s = np.full((q, k), -np.inf, dtype=F32)
    for r in range(q):
        valid = idx[r] >= 0
        ii, ss = idx[r][valid], sc[r][valid]
        order = np.lexsort((ii, -ss))[:k]
        out_i[r, :order.size] = ii[order]
        out_s[r, :order.size] = ss[order]
    return out_i, out_s


# ---------------------------------------------------------------------------
# NT-Xent / InfoNCE with MoCo queue -- src/contrastor/contrastive_loss.py:56-93
# ---------------------------------------------------------------------------

def _logsumexp(x: np.ndarray, axis: int = -1) -> np.ndarray:
    m = np.max(x, axis=axis, keepdims=True)
    return (m + np.log(np.sum(np.exp(x - m), axis=axis, keepdims=True))).squeeze(axis)


def nce_info_loss(q: np.ndarray, k: np.ndarray, queue: np.ndarray | None, T: float,
                  want_grad: bool = True, want_dk: bool = False):
    """Loss and dL/dq of ``NCELoss._compute_info_loss`` (fp64 internally).

    * F = cat[q; k] (2N x D), S = F F^T (contrastive_loss.py:61-62);
    * the diagonal is dropped (:65-68); row i's positive is column (i+N) mod 2N
      (:57-58, :71); the other 2N-2 columns are negatives (:74-75);
    * with a queue, rows N..2N-1 REUSE q's queue logits: (q @ queue).repeat(2, 1)
      (:79-80) -- a reference quirk reproduced here;
    * CrossEntropy(sum) with target 0, divided by 2 (:51, :91-92).
    Gradient flows into q only (k comes from the no-grad momentum encoder,
    contrastive_module.py:82-83, 109-110).  ``want_dk``: also return dL/dk, the
    use_momentum False case where k = seq2vec(positive) through encoder_q with
    autograd (contrastive_module.py:82-83); the queue logits use q only.
    """
    q = np.asarray(q, F64)
    k = np.asarray(k, F64)
    n = q.shape[0]
    F = np.concatenate([q, k], axis=0)
    S = F @ F.T
    rows = np.arange(2 * n)
    pos = (rows + n) % (2 * n)
    L = S / T
    Lm = L.copy()
    Lm[rows, rows] = -np.inf  # drop diagonal
    if queue is not None and queue.shape[1] > 0:
        Qlog = (q @ np.asarray(queue, F64)) / T  # [n, K]
        Qrep = np.concatenate([Qlog, Qlog], axis=0)  # .repeat(2, 1)
        full = np.concatenate([Lm, Qrep], axis=1)
    else:
        Qrep = None
        full = Lm
    lse = _logsumexp(full, axis=1)
    loss = 0.5 * np.sum(lse - L[rows, pos])
    if not want_grad:
        return loss, None
    P = np.exp(full - lse[:, None])  # softmax over each row's logits
    G = P[:, : 2 * n].copy()  # dLoss/dL_ij (before the 1/2 and 1/T)
    G[rows, pos] -= 1.0
    G[rows, rows] = 0.0
    G *= 0.5 / T
    dF = (G + G.T) @ F
    dq = dF[:n].copy()
    if Qrep is not None:
        GQ = P[:, 2 * n:] * (0.5 / T)
        dq += (GQ[:n] + GQ[n:]) @ np.asarray(queue, F64).T
    if want_dk:
        return loss, dq, dF[n:].copy()
    return loss, dq


# ---------------------------------------------------------------------------
# BiLSTM head + Linear + mean-pool + L2 norm  (src/model.py:7-41,
# src/contrastor/contrastive_module.py:102-112)
# ---------------------------------------------------------------------------

def _sigmoid(x):
    return 1.0 / (1.0 + np.exp(-x))


def lstm_layer_dir_fwd(x, w_ih, w_hh, b_ih, b_hh, reverse: bool):
    """One direction of one torch nn.LSTM layer (gate order i, f, g, o).

    x: [B, L, In].  Zero initial state; no packing, so the reverse direction
    starts on the last (possibly PAD) position (model.py:39 passes the padded
    tensor straight in).  Returns h [B, L, H] and a cache for BPTT.
    """
    B, Lx, _ = x.shape
    H = w_hh.shape[1]
    xp = x @ w_ih.T + b_ih + b_hh  # [B, L, 4H]
    h = np.zeros((B, H), x.dtype)
    c = np.zeros((B, H), x.dtype)
    hs = np.zeros((B, Lx, H), x.dtype)
    cache = []
    ts = range(Lx - 1, -1, -1) if reverse else range(Lx)
    for t in ts:
        g = xp[:, t] + h @ w_hh.T
        i_, f_, g_, o_ = np.split(g, 4, axis=1)
        i_, f_, o_ = _sigmoid(i_), _sigmoid(f_), _sigmoid(o_)
        g_ = np.tanh(g_)
        c_prev, h_prev = c, h
        c = f_ * c + i_ * g_
        tc = np.tanh(c)
        h = o_ * tc
        hs[:, t] = h
        cache.append((t, i_, f_, g_, o_, c_prev, h_prev, tc))
    return hs, cache


def lstm_layer_dir_bwd(dhs, x, w_ih, w_hh, cache):
    """BPTT for lstm_layer_dir_fwd.  Returns dx, dW_ih, dW_hh, db (= db_ih = db_hh)."""
    B, Lx, H = dhs.shape
    dxp = np.zeros((B, Lx, 4 * H), dhs.dtype)
    dh_next = np.zeros((B, H), dhs.dtype)
    dc_next = np.zeros((B, H), dhs.dtype)
    dW_hh = np.zeros_like(w_hh)
    for (t, i_, f_, g_, o_, c_prev, h_prev, tc) in reversed(cache):
        dh = dhs[:, t] + dh_next
        do = dh * tc
        dc = dh * o_ * (1.0 - tc * tc) + dc_next
        di = dc * g_
        dg = dc * i_
        df = dc * c_prev
        dc_next = dc * f_
        dgates = np.concatenate([di * i_ * (1 - i_), df * f_ * (1 - f_),
                                 dg * (1 - g_ * g_), do * o_ * (1 - o_)], axis=1)
        dxp[:, t] = dgates
        dW_hh += dgates.T @ h_prev
        dh_next = dgates @ w_hh
    dx = dxp @ w_ih
    dW_ih = np.einsum("blg,bli->gi", dxp, x)
    db = dxp.sum(axis=(0, 1))
    return dx, dW_ih, dW_hh, db


def lstm_param_names(num_layers: int, bidirectional: bool):
    dirs = ["", "_reverse"] if bidirectional else [""]
    out = []
    for l in range(num_layers):
        for d in dirs:
            out.append((l, d))
    return out


_SELU = (1.0507009873554804934193349852946, 1.6732632423543772848170429916717)


def _softplus(u):
    return np.where(u > 20.0, u, np.log1p(np.exp(np.minimum(u, 20.0))))


def act_fwd(name: str, u):
    """``eval(f"nn.{act}()")`` (model.py:25) with torch's default arguments."""
    if name == "Identity":
        return u
    sg = 1.0 / (1.0 + np.exp(-u))
    return {
        "ReLU": lambda: np.maximum(u, 0.0),
        "ReLU6": lambda: np.clip(u, 0.0, 6.0),
        "LeakyReLU": lambda: np.where(u > 0, u, 0.01 * u),
        "ELU": lambda: np.where(u > 0, u, np.expm1(np.minimum(u, 0.0))),
        "CELU": lambda: np.where(u > 0, u, np.expm1(np.minimum(u, 0.0))),
        "SELU": lambda: _SELU[0] * np.where(u > 0, u, _SELU[1] * np.expm1(np.minimum(u, 0.0))),
        "GELU": lambda: gelu(u),
        "SiLU": lambda: u * sg,
        "Mish": lambda: u * np.tanh(_softplus(u)),
        "Sigmoid": lambda: sg,
        "Tanh": lambda: np.tanh(u),
        "Softplus": lambda: _softplus(u),
        "Softsign": lambda: u / (1.0 + np.abs(u)),
        "Hardtanh": lambda: np.clip(u, -1.0, 1.0),
        "Hardsigmoid": lambda: np.clip(u + 3.0, 0.0, 6.0) / 6.0,
        "Hardswish": lambda: u * np.clip(u + 3.0, 0.0, 6.0) / 6.0,
        "Tanhshrink": lambda: u - np.tanh(u),
    }[name]()


def act_grad(name: str, u):
    """d act / du (torch autograd's values at the kinks)."""
    if name == "Identity":
        return np.ones_like(u)
    sg = 1.0 / (1.0 + np.exp(-u))
    t = np.tanh(u)
    return {
        "ReLU": lambda: (u > 0).astype(u.dtype),
        "ReLU6": lambda: ((u > 0) & (u < 6)).astype(u.dtype),
        "LeakyReLU": lambda: np.where(u > 0, 1.0, 0.01),
        "ELU": lambda: np.where(u > 0, 1.0, np.exp(np.minimum(u, 0.0))),
        "CELU": lambda: np.where(u > 0, 1.0, np.exp(np.minimum(u, 0.0))),
        "SELU": lambda: np.where(u > 0, _SELU[0], _SELU[0] * _SELU[1] * np.exp(np.minimum(u, 0.0))),
        "GELU": lambda: 0.5 * (1.0 + _erf(u / np.sqrt(2.0))) + u * np.exp(-0.5 * u * u) / np.sqrt(2 * np.pi),
        "SiLU": lambda: sg * (1.0 + u * (1.0 - sg)),
        "Mish": lambda: np.tanh(_softplus(u)) + u * (1.0 - np.tanh(_softplus(u)) ** 2) * sg,
        "Sigmoid": lambda: sg * (1.0 - sg),
        "Tanh": lambda: 1.0 - t * t,
        "Softplus": lambda: np.where(u > 20.0, 1.0, sg),
        "Softsign": lambda: 1.0 / (1.0 + np.abs(u)) ** 2,
        "Hardtanh": lambda: ((u > -1) & (u < 1)).astype(u.dtype),
        "Hardsigmoid": lambda: np.where((u > -3) & (u < 3), 1.0 / 6.0, 0.0),
        "Hardswish": lambda: np.where(u <= -3, 0.0, np.where(u < 3, u / 3.0 + 0.5, 1.0)),
        "Tanhshrink": lambda: t * t,
    }[name]()


def lstm_head_fwd(features, p, num_layers: int, bidirectional: bool = True, act="Identity"):
    """``LSTM.forward`` (model.py:38-41): nn.LSTM then Linear + the activation (:23-26)."""
    x = np.asarray(features)
    caches = []
    for l in range(num_layers):
        outs = []
        lc = []
        for d in (["", "_reverse"] if bidirectional else [""]):
            sfx = f"l{l}{d}"
            hs, cache = lstm_layer_dir_fwd(
                x, p[f"lstm.weight_ih_{sfx}"], p[f"lstm.weight_hh_{sfx}"],
                p[f"lstm.bias_ih_{sfx}"], p[f"lstm.bias_hh_{sfx}"], reverse=(d != ""))
            outs.append(hs)
            lc.append(cache)
        caches.append((x, lc))
        x = np.concatenate(outs, axis=2)
    u = x @ p["scaling_layer.0.weight"].T + p["scaling_layer.0.bias"]
    return act_fwd(act, u), (caches, x, u, act)


def lstm_head_bwd(dy, p, cache, num_layers: int, bidirectional: bool = True):
    caches, xlast, u, act = cache
    dy = dy * act_grad(act, u)
    grads = {}
    grads["scaling_layer.0.weight"] = np.einsum("blo,bli->oi", dy, xlast)
    grads["scaling_layer.0.bias"] = dy.sum(axis=(0, 1))
    dx = dy @ p["scaling_layer.0.weight"]
    for l in range(num_layers - 1, -1, -1):
        x, lc = caches[l]
        H = p[f"lstm.weight_hh_l{l}"].shape[1]
        dsum = np.zeros_like(x)
        for di, d in enumerate(["", "_reverse"] if bidirectional else [""]):
            sfx = f"l{l}{d}"
            dhs = dx[:, :, di * H:(di + 1) * H]
            dxi, dwi, dwh, db = lstm_layer_dir_bwd(
                np.ascontiguousarray(dhs), x, p[f"lstm.weight_ih_{sfx}"],
                p[f"lstm.weight_hh_{sfx}"], lc[di])
            dsum += dxi
            grads[f"lstm.weight_ih_{sfx}"] = dwi
            grads[f"lstm.weight_hh_{sfx}"] = dwh
            grads[f"lstm.bias_ih_{sfx}"] = db
            grads[f"lstm.bias_hh_{sfx}"] = db.copy()
        dx = dsum
    return grads


def l2_normalize(x, eps: float = 1e-12):
    """torch.nn.functional.normalize(x, dim=1): x / max(||x||_2, eps)."""
    n = np.sqrt(np.sum(x * x, axis=1, keepdims=True))
    return x / np.maximum(n, eps)


def seq2vec(features, p, num_layers: int, bidirectional: bool = True, act="Identity"):
    """``seq2vec`` (contrastive_module.py:102-112): head -> mean over ALL L
    positions (PAD included) -> L2 normalise."""
    y, cache = lstm_head_fwd(features, p, num_layers, bidirectional, act)
    m = y.mean(axis=1)
    return l2_normalize(m), (y, m, cache)


def seq2vec_bwd(demb, p, cache, num_layers: int, bidirectional: bool = True):
    y, m, hc = cache
    nrm = np.sqrt(np.sum(m * m, axis=1, keepdims=True))
    nrm_c = np.maximum(nrm, 1e-12)
    e = m / nrm_c
    # d(m/||m||) = (I - e e^T) / ||m||  (for ||m|| > eps)
    dm = (demb - e * np.sum(demb * e, axis=1, keepdims=True)) / nrm_c
    L = y.shape[1]
    dy = np.repeat(dm[:, None, :] / L, L, axis=1)
    return lstm_head_bwd(dy, p, hc, num_layers, bidirectional)


# ---------------------------------------------------------------------------
# Frozen BERT encoder (contrastive_module.py:36-41 -> HF BertModel)
# ---------------------------------------------------------------------------

def layer_norm(x, g, b, eps: float = 1e-12):
    mu = x.mean(axis=-1, keepdims=True)
    var = ((x - mu) ** 2).mean(axis=-1, keepdims=True)
    return (x - mu) / np.sqrt(var + eps) * g + b


def gelu(x):
    return 0.5 * x * (1.0 + _erf(x / np.sqrt(2.0)))


def bert_forward(input_ids, attention_mask, w: dict, num_layers: int, num_heads: int,
                 eps: float = 1e-12, dtype=F32):
    """``BertModel(...).last_hidden_state`` in eval mode (no dropout).

    embeddings = LN(word[ids] + type[0] + pos[arange(L)]); per layer
    LN(x + Wo Attn(x)) then LN(h + W2 gelu(W1 h)); attention scores scaled by
    d_head^-1/2 with an additive key mask.  PAD query rows are computed and kept.
    Weight names are HF's state_dict keys without the ``bert_model.`` prefix.
    """
    ids = np.asarray(input_ids)
    mask = np.asarray(attention_mask).astype(dtype)
    B, L = ids.shape
    W = {kk: np.asarray(v, dtype) for kk, v in w.items()}
    x = (W["embeddings.word_embeddings.weight"][ids]
         + W["embeddings.token_type_embeddings.weight"][0]
         + W["embeddings.position_embeddings.weight"][:L][None])
    x = layer_norm(x, W["embeddings.LayerNorm.weight"], W["embeddings.LayerNorm.bias"], eps)
    H = x.shape[-1]
    dh = H // num_heads
    addmask = (1.0 - mask)[:, None, None, :] * np.finfo(dtype).min
    for l in range(num_layers):
        pre = f"encoder.layer.{l}."

        def lin(t, name):
            return t @ W[pre + name + ".weight"].T + W[pre + name + ".bias"]

        qh = lin(x, "attention.self.query").reshape(B, L, num_heads, dh).transpose(0, 2, 1, 3)
        kh = lin(x, "attention.self.key").reshape(B, L, num_heads, dh).transpose(0, 2, 1, 3)
        vh = lin(x, "attention.self.value").reshape(B, L, num_heads, dh).transpose(0, 2, 1, 3)
        s = qh @ kh.transpose(0, 1, 3, 2) * (dh ** -0.5) + addmask
        s = s - s.max(axis=-1, keepdims=True)
        pr = np.exp(s)
        pr /= pr.sum(axis=-1, keepdims=True)
        ctx = (pr @ vh).transpose(0, 2, 1, 3).reshape(B, L, H)
        a = layer_norm(lin(ctx, "attention.output.dense") + x,
                       W[pre + "attention.output.LayerNorm.weight"],
                       W[pre + "attention.output.LayerNorm.bias"], eps)
        h1 = gelu(lin(a, "intermediate.dense"))
        x = layer_norm(lin(h1, "output.dense") + a, W[pre + "output.LayerNorm.weight"],
                       W[pre + "output.LayerNorm.bias"], eps)
    return x


# ---------------------------------------------------------------------------
# Optimizer-side pieces (src/train.py:150-175, contrastive_module.py:43-68)
# ---------------------------------------------------------------------------

def clip_grad_norm(grads: dict, max_norm: float):
    """torch.nn.utils.clip_grad_norm_ (train.py:157-159): returns total norm and
    scales the grads in place by min(1, max_norm / (norm + 1e-6))."""
    tot = np.sqrt(sum(float(np.sum(np.asarray(g, F64) ** 2)) for g in grads.values()))
    coef = min(1.0, max_norm / (tot + 1e-6))
    for kk in grads:
        grads[kk] = grads[kk] * coef
    return tot


def adam_step(p, g, m, v, step: int, lr: float, b1: float, b2: float, eps: float = 1e-8):
    """torch.optim.Adam (model.py:52-57), default eps/weight_decay, one tensor."""
    m = b1 * m + (1 - b1) * g
    v = b2 * v + (1 - b2) * g * g
    bc1 = 1 - b1 ** step
    bc2 = 1 - b2 ** step
    denom = np.sqrt(v) / np.sqrt(bc2) + eps
    p = p - (lr / bc1) * m / denom
    return p, m, v


def sgd_step(p, g, buf, lr: float, momentum: float, weight_decay: float):
    """torch.optim.SGD (model.py:45-51), dampening 0, nesterov False, one tensor;
    buf None on the first step (torch: buf = d.clone())."""
    d = g + weight_decay * p
    buf = d.copy() if buf is None else momentum * buf + d
    return p - lr * buf, buf


def cosine_lr(lr0: float, steps: int, total_steps: int) -> float:
    """adjust_learning_rate (src/train.py:18-23)."""
    return lr0 * 0.5 * (1.0 + np.cos(np.pi * steps / total_steps))


def momentum_update(pk, pq, m: float):
    """_momentum_update_key_encoder (contrastive_module.py:48-51)."""
    return pk * m + pq * (1.0 - m)


def dequeue_and_enqueue(queue, ptr: int, keys):
    """_dequeue_and_enqueue (contrastive_module.py:55-68): only when
    queue_size % B == 0 (so B=1024/2048 never update the queue)."""
    K = queue.shape[1]
    B = keys.shape[0]
    queue = queue.copy()
    if K % B == 0:
        queue[:, ptr:ptr + B] = np.asarray(keys).T
        ptr = (ptr + B) % K
    return queue, ptr
