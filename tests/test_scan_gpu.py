"""Parity of the HIP corpus scan + top-k (irc_scan_topk) with the CPU oracle.

Bit-exact on integer-grid embeddings (every fp32 dot product is exact in any
accumulation order) and on the reference-generated golden fixtures; margin-aware
on Gaussian data; size-independent properties at the full C2 size.
"""
import numpy as np
import pytest
import torch

from conftest import load_golden
from oracle import irc_oracle as O

pytestmark = pytest.mark.gpu


class _single_pass:
    """Enable the single-pass GEMM filter (off by default) for Q > 64 inside a test."""

    def __init__(self, on=True):
        self.on = on

    def __enter__(self):
        from irc_amd import retrieval

        self.prev = retrieval.set_single_pass_min_q(65 if self.on else 1 << 30)

    def __exit__(self, *exc):
        from irc_amd import retrieval

        torch.cuda.synchronize()
        retrieval.set_single_pass_min_q(self.prev)


def _grid(rng, shape, lim=127):
    return rng.integers(-lim, lim + 1, shape).astype(np.float32) / 128


def _dev(x, dev):
    return torch.from_numpy(np.ascontiguousarray(x)).to(dev)


@pytest.mark.parametrize("D", [64, 128, 256, 384, 512, 768, 1024])
def test_scores_exact_on_grid(gpu, D):
    from irc_amd import retrieval

    rng = np.random.default_rng(D)
    q = _grid(rng, (70, D))
    d = _grid(rng, (517, D))
    s = retrieval.scan_scores(_dev(q, gpu), _dev(d, gpu)).cpu().numpy()
    np.testing.assert_array_equal(s, O.scan_scores(q, d))


def test_golden_grid_reference_order(gpu):
    from irc_amd import retrieval

    g = load_golden("scan.npz")
    q = g["grid_q"].astype(np.float32) / 128
    d = g["grid_d"].astype(np.float32) / 128
    s, i = retrieval.scan_topk(_dev(q, gpu), _dev(d, gpu), int(g["grid_k"]))
    np.testing.assert_array_equal(i.cpu().numpy(), g["grid_idx"])
    np.testing.assert_array_equal(s.cpu().numpy(), g["grid_score"])


def test_golden_ties(gpu):
    from irc_amd import retrieval

    g = load_golden("scan.npz")
    q = g["tie_q"].astype(np.float32) / 128
    d = g["tie_d"].astype(np.float32) / 128
    k = int(g["tie_k"])
    s, i = retrieval.scan_topk(_dev(q, gpu), _dev(d, gpu), k)
    ri, rs = O.scan_topk(q, d, k)
    np.testing.assert_array_equal(s.cpu().numpy(), g["tie_score"])
    np.testing.assert_array_equal(i.cpu().numpy(), ri)


@pytest.mark.parametrize("Q,N,D,k,off", [
    (1, 1, 128, 1, 0),          # single doc
    (3, 5, 128, 8, 11),         # k > N -> padded
    (33, 31, 64, 10, 0),        # partial tile, Q not a multiple of 32
    (257, 4099, 128, 100, 5),   # two query blocks, ragged tail
    (16, 60000, 128, 100, 0),   # two-phase (sampled threshold) path
    (64, 40000, 768, 1024, 3),  # maximum k
    (8, 20000, 128, 1, 0),      # k = 1
    # single-pass scan with four k-slices (D = 768 / 1024, Q <= 64): one and two
    # 32-query groups, merged half-lane lists, ragged tails, k up to 256
    (1, 50011, 768, 100, 0),
    (33, 40000, 768, 100, 2),
    (64, 30007, 768, 256, 4),
    (7, 20000, 1024, 200, 5),
    (40, 25000, 1024, 64, 0),
    # Q >= 128: filter on the ping-pong GEMM kernel (regions = 256-doc tiles)
    (128, 60000, 768, 100, 0),  # two-phase, C2 dims
    (200, 30000, 256, 1024, 7),  # maximum k, ragged Q
    (384, 9000, 64, 50, 0),     # two query tiles, D = 64 (one K-tile)
    (1024, 12000, 128, 100, 9),  # four query tiles sharing each doc tile (C3-style batch)
])
def test_topk_exact_vs_oracle(gpu, Q, N, D, k, off):
    from irc_amd import retrieval

    rng = np.random.default_rng(Q * 7 + N)
    q = _grid(rng, (Q, D), 3)  # small range -> many exact ties
    d = _grid(rng, (N, D), 3)
    s, i = retrieval.scan_topk(_dev(q, gpu), _dev(d, gpu), k, off)
    ri, rs = O.scan_topk(q, d, k, doc_offset=off)
    np.testing.assert_array_equal(i.cpu().numpy(), ri)
    np.testing.assert_array_equal(s.cpu().numpy(), rs)


@pytest.mark.parametrize("Q,N,D,k,off", [(128, 60000, 768, 100, 0), (256, 50000, 128, 256, 5),
                                         (100, 9000, 512, 50, 1), (256, 4099, 64, 100, 2)])
def test_topk_exact_vs_oracle_single_pass(gpu, Q, N, D, k, off):
    """The single-pass GEMM filter (4-key lists per 256-doc tile + select_dense with
    rescans), enabled explicitly (off by default), bit-exact against the oracle on
    integer grids with many exact ties."""
    from irc_amd import retrieval

    rng = np.random.default_rng(Q * 11 + N)
    q = _grid(rng, (Q, D), 3)
    d = _grid(rng, (N, D), 3)
    with _single_pass():
        s, i = retrieval.scan_topk(_dev(q, gpu), _dev(d, gpu), k, off)
    ri, rs = O.scan_topk(q, d, k, doc_offset=off)
    np.testing.assert_array_equal(i.cpu().numpy(), ri)
    np.testing.assert_array_equal(s.cpu().numpy(), rs)


def test_adversarial_sorted_corpus(gpu):
    """Later docs strictly better than the sample: nearly every doc survives the
    threshold, the selection must still be exact."""
    N, D, k = 50000, 128, 100
    q = np.zeros((4, D), np.float32)
    q[:, 0] = 1.0
    _check_sorted_corpus(gpu, q, N, D, k)


def test_adversarial_sorted_corpus_gemm_filter(gpu):
    """Same with Q = 160 (the GEMM-kernel filter): whole 256-doc regions survive."""
    N, D, k = 50000, 128, 100
    q = np.zeros((160, D), np.float32)
    q[:, 0] = 1.0
    q[::2, 1] = 0.5
    _check_sorted_corpus(gpu, q, N, D, k)


def test_adversarial_sorted_corpus_gemm_sample(gpu):
    """Q = 300 (two query tiles): the sampled pipeline with its threshold sample on the
    GEMM kernel (4-key lists per 256-doc sample tile, k-th of the lists): whole
    regions survive the threshold, the selection must still be exact."""
    N, D, k = 50000, 128, 100
    q = np.zeros((300, D), np.float32)
    q[:, 0] = 1.0
    q[::3, 1] = 0.5
    _check_sorted_corpus(gpu, q, N, D, k)


def _check_sorted_corpus(gpu, q, N, D, k):
    from irc_amd import retrieval

    d = np.zeros((N, D), np.float32)
    d[:, 0] = (np.arange(N) % 256) / 128.0 - 1.0  # ramp, repeated -> huge tie groups
    s, i = retrieval.scan_topk(_dev(q, gpu), _dev(d, gpu), k)
    ri, rs = O.scan_topk(q, d, k)
    np.testing.assert_array_equal(i.cpu().numpy(), ri)
    np.testing.assert_array_equal(s.cpu().numpy(), rs)


@pytest.mark.parametrize("Q", [64, 256])
def test_gaussian_margin_aware(gpu, Q):
    from irc_amd import retrieval

    torch.manual_seed(2024)
    N, D, k = 30000, 768, 100
    q = torch.nn.functional.normalize(torch.randn(Q, D)).bfloat16()
    d = torch.nn.functional.normalize(torch.randn(N, D)).bfloat16()
    s, i = retrieval.scan_topk(q.to(gpu), d.to(gpu), k)
    s, i = s.cpu().numpy(), i.cpu().numpy()
    full = O.scan_scores(q.float().numpy(), d.float().numpy())
    ri, rs = O.topk_rows(full, k)
    tol = 1e-5  # fp32 accumulation-order difference on unit vectors, D=768
    for r in range(Q):
        # returned scores are the true scores of the returned docs (to fp32 rounding)
        np.testing.assert_allclose(s[r], full[r, i[r]], atol=tol)
        # same set except where the oracle's boundary score is within tol
        diff = set(i[r]) ^ set(ri[r])
        for doc in diff:
            assert abs(full[r, doc] - rs[r, -1]) <= 2 * tol
        assert np.all(np.diff(s[r]) <= 0)


def test_merge_matches_unsharded(gpu):
    from irc_amd import retrieval

    rng = np.random.default_rng(3)
    q = _grid(rng, (40, 128), 2)
    d = _grid(rng, (7001, 128), 2)
    k = 64
    bounds = [retrieval.shard_bounds(7001, 3, r) for r in range(3)]
    parts = [retrieval.scan_topk(_dev(q, gpu), _dev(d[a:b], gpu), k, a) for a, b in bounds]
    ms, mi = retrieval.topk_merge(torch.stack([p[0] for p in parts]),
                                  torch.stack([p[1] for p in parts]), k)
    ri, rs = O.scan_topk(q, d, k)
    np.testing.assert_array_equal(mi.cpu().numpy(), ri)
    np.testing.assert_array_equal(ms.cpu().numpy(), rs)


def test_full_c2_size_properties(gpu):
    """C2: Q=256, N=100k, D=768, k=100 -- properties that do not need the oracle."""
    from irc_amd import retrieval

    g = torch.Generator(device="cpu").manual_seed(2024)
    Q, N, D, k = 256, 100_000, 768, 100
    d = torch.nn.functional.normalize(torch.randn(N, D, generator=g)).bfloat16().to(gpu)
    q = torch.nn.functional.normalize(torch.randn(Q, D, generator=g)).bfloat16().to(gpu)
    s, i = retrieval.scan_topk(q, d, k)
    full = retrieval.scan_scores(q, d)  # same MFMA arithmetic
    assert bool((i >= 0).all()) and bool((i < N).all())
    assert torch.equal(s, torch.gather(full, 1, i))  # scores belong to their docs, bit-exact
    assert bool((s[:, 1:] <= s[:, :-1]).all())
    # completeness: nothing outside the list beats the k-th entry
    masked = full.clone()
    masked.scatter_(1, i, float("-inf"))
    assert bool((masked.max(dim=1).values <= s[:, -1]).all())
    # idempotence: a second call returns the same bits
    s2, i2 = retrieval.scan_topk(q, d, k)
    assert torch.equal(i, i2) and torch.equal(s, s2)
    # the oracle at full size, margin-aware, on 6 rows spread over the query batch:
    # the fp32 restatement of closest_docs (O.scan_topk, evaluation.py:110-112) over the
    # same bf16 embeddings; the lists agree except where two docs' true scores are
    # within the accumulation-order tolerance of the oracle's k-th score
    rows = [0, 1, 97, 128, 200, 255]
    dn = d.float().cpu().numpy()
    qn = q[rows].float().cpu().numpy()
    ri, rs = O.scan_topk(qn, dn, k)
    exact = qn.astype(np.float64) @ dn.astype(np.float64).T
    tol = 1e-5  # fp32 accumulation-order difference on unit vectors, D = 768
    sc, ic = s[rows].cpu().numpy(), i[rows].cpu().numpy()
    for t in range(len(rows)):
        np.testing.assert_allclose(sc[t], exact[t, ic[t]], atol=tol)
        for doc in set(ic[t].tolist()) ^ set(ri[t].tolist()):
            assert abs(exact[t, doc] - rs[t, -1]) <= 2 * tol, (rows[t], doc)


@pytest.mark.parametrize("Q,D,fp8", [(1, 768, False), (16, 768, False), (64, 256, False),
                                      (40, 768, True), (128, 768, False), (256, 768, False),
                                      (200, 768, True)])
def test_clustered_corpus_rescan_properties(gpu, Q, D, fp8):
    """A block of 600 consecutive docs aligned with the queries: ~25 winners per
    worker there, so the single-pass scan's 4-key lists overflow and
    select_dense must rescan those workers.  Scores bit-exact with the scan's
    own MFMA scores, complete, sorted, ties to the lower index."""
    from irc_amd import retrieval

    g = torch.Generator().manual_seed(7)
    N, k = 40_000, 100
    unit = lambda x: torch.nn.functional.normalize(x, dim=-1)  # noqa: E731
    base = unit(torch.randn(D, generator=g))
    q = unit(base + 0.5 * unit(torch.randn(Q, D, generator=g)))
    d = unit(torch.randn(N, D, generator=g))
    d[17_000:17_600] = unit(base + 0.5 * unit(torch.randn(600, D, generator=g)))
    with _single_pass(Q > 64):  # Q > 64: the single-pass GEMM filter and its rescans
        if fp8:
            qq = retrieval.quantize_fp8(q.to(gpu))
            dd = retrieval.quantize_fp8(d.to(gpu))
            s, i = retrieval.scan_topk_fp8(qq, dd, k, 0, 1.0 / 256)
            full = retrieval.scan_scores_fp8(qq, dd) * (1.0 / 256)
        else:
            qq, dd = q.bfloat16().to(gpu), d.bfloat16().to(gpu)
            s, i = retrieval.scan_topk(qq, dd, k)
            full = retrieval.scan_scores(qq, dd)
    assert bool((i >= 0).all()) and bool((i < N).all())
    assert bool(((i >= 17_000) & (i < 17_600)).all())  # the block wins
    assert torch.equal(s, torch.gather(full, 1, i))
    assert bool((s[:, 1:] <= s[:, :-1]).all())
    tie = s[:, 1:] == s[:, :-1]
    assert bool((i[:, 1:][tie] > i[:, :-1][tie]).all())
    masked = full.clone()
    masked.scatter_(1, i, float("-inf"))
    assert bool((masked.max(dim=1).values <= s[:, -1]).all())


def test_search_many_equals_serial_search(gpu):
    """Pipelined batches (search_many, 2 / 3 streams, own workspaces) return exactly
    what serial search() calls return."""
    from irc_amd import retrieval

    rng = np.random.default_rng(8)
    d = _dev(_grid(rng, (30000, 256), 3), gpu)
    index = retrieval.ShardedDenseIndex(d)
    batches = [_dev(_grid(rng, (q, 256), 3), gpu) for q in (256, 1, 300, 64, 256, 256, 17)]
    for depth in (2, 3):
        many = index.search_many(batches, 50, depth=depth)
        for q, (s, i) in zip(batches, many):
            s0, i0 = index.search(q, 50)
            assert torch.equal(s, s0) and torch.equal(i, i0)


@pytest.mark.parametrize("q,nb,depth", [(256, 7, 3), (64, 5, 2), (1, 4, 3), (200, 2, 3),
                                        (300, 1, 3)])
def test_native_search_many_equals_serial_search(gpu, q, nb, depth):
    """Batches of one shape take the one-call loop (irc_scan_topk_many): the GEMM filter
    (Q >= 192), the single pass (Q <= 64), fewer batches than streams; exactly what serial
    search() calls return, and ready on the current stream."""
    from irc_amd import retrieval

    rng = np.random.default_rng(q + nb)
    d = _dev(_grid(rng, (30000, 256), 3), gpu)
    index = retrieval.ShardedDenseIndex(d, doc_offset=11)
    batches = [_dev(_grid(rng, (q, 256), 3), gpu) for _ in range(nb)]
    many = index.search_many(batches, 50, depth=depth)
    assert len(many) == nb
    for qb, (s, i) in zip(batches, many):
        s0, i0 = index.search(qb, 50)
        assert torch.equal(s, s0) and torch.equal(i, i0)


def test_graphed_search_many_equals_serial_search(gpu):
    """HIP-graph replays of the whole local search (one graph per stream) return
    exactly what serial search() calls return, for bf16 and fp8 shards."""
    from irc_amd import retrieval

    rng = np.random.default_rng(9)
    d = _dev(_grid(rng, (20000, 256), 3), gpu)
    for dtype in ("bf16", "fp8"):
        index = retrieval.ShardedDenseIndex(d, doc_offset=5, dtype=dtype)
        batches = [_dev(_grid(rng, (256, 256), 3), gpu) for _ in range(5)]
        many = index.search_many(batches, 40, depth=2, graphs=True)
        for q, (s, i) in zip(batches, many):
            s0, i0 = index.search(q, 40)
            assert torch.equal(s, s0) and torch.equal(i, i0), dtype


def test_graphed_search_many_survives_workspace_growth(gpu):
    """a captured graph must keep its own scan workspace.  The
    sequence Q=64 -> Q=256 (bigger workspace) -> Q=64 on one index, then a second
    index with a larger shard and a bigger k, then the first index's Q=64 graphs
    again, and finally the shard tensor replaced in place of the attribute: every
    replay equals a serial search() on the current shard."""
    from irc_amd import retrieval

    rng = np.random.default_rng(13)
    small = retrieval.ShardedDenseIndex(_dev(_grid(rng, (9000, 256), 3), gpu), doc_offset=1)
    big = retrieval.ShardedDenseIndex(_dev(_grid(rng, (60000, 256), 3), gpu), doc_offset=2)

    def check(index, q, k):
        many = index.search_many([q, q, q], k, depth=2, graphs=True)
        s0, i0 = index.search(q, k)
        for s, i in many:
            assert torch.equal(s, s0) and torch.equal(i, i0)

    q64 = _dev(_grid(rng, (64, 256), 3), gpu)
    q256 = _dev(_grid(rng, (256, 256), 3), gpu)
    check(small, q64, 30)
    check(small, q256, 30)
    check(small, q64, 30)
    check(big, q256, 120)
    check(big, q64, 120)
    check(small, q64, 30)  # the first graphs replay after every growth above
    small.docs = _dev(_grid(rng, (9000, 256), 3), gpu).to(torch.bfloat16)
    check(small, q64, 30)  # new shard tensor: captured anew, not the old pointer


@pytest.mark.parametrize("Q,D,fp8", [(1, 768, False), (16, 768, False), (64, 1024, False),
                                      (32, 768, True), (128, 768, False), (256, 768, False),
                                      (256, 1024, False), (200, 768, True)])
def test_rescan_bit_exact_vs_oracle_on_grid(gpu, Q, D, fp8):
    """the single-pass scan's rescan path pinned to
    the oracle.  Integer-grid corpus (every score exact in fp32 in any order) with
    a block of 600 consecutive docs aligned with the queries: all k = 100 winners
    sit in a few workers, whose 4-key lists provably overflow, so select_dense
    must rescan.  The rescan counter proves it happened; indices and scores are
    compared bit for bit with the oracle (ties: lower index first).  D >= 512:
    the single-pass path's lists must fit one select stage (at D = 256 on 40k
    docs the worker count is too high and the sampled pipeline runs instead)."""
    from irc_amd import retrieval

    rng = np.random.default_rng(100 + Q)
    N, k, lo = 40_000, 100, 17_000
    lim, step = (7, 16) if fp8 else (40, 128)  # fp8: e4m3-exact values m/16, |m| <= 15
    base = rng.integers(-lim, lim + 1, D)
    docs = rng.integers(-2, 3, (N, D))
    docs[lo:lo + 600] = base + rng.integers(-3, 4, (600, D))
    qs = base + rng.integers(-3, 4, (Q, D))
    # Q > 64: the single-pass GEMM filter (4-key lists per 256-doc tile, rescans
    # with its own 16x16x32 MFMA sequence)
    d = (docs / step).astype(np.float32)
    q = (qs / step).astype(np.float32)
    retrieval.rescan_stats(reset=True)
    with _single_pass(Q > 64):
        if fp8:
            q8, d8 = O.quantize_e4m3(q), O.quantize_e4m3(d)
            assert np.array_equal(O.dequantize_e4m3(d8), d)  # the grid is e4m3-exact
            s, i = retrieval.scan_topk_fp8(_dev(q8, gpu), _dev(d8, gpu), k, 3, 1.0 / 256)
            ri, rs = O.scan_topk_fp8(q8, d8, k, doc_offset=3, score_scale=1.0 / 256)
        else:
            s, i = retrieval.scan_topk(_dev(q, gpu), _dev(d, gpu), k, 3)
            ri, rs = O.scan_topk(q, d, k, doc_offset=3)
        nq, nw = retrieval.rescan_stats(reset=True)
    print(f"Q={Q} D={D} fp8={fp8}: {nq} queries rescanned, {nw} workers")
    assert nq >= 1 and nw >= nq  # the block's truncated lists forced rescans
    np.testing.assert_array_equal(i.cpu().numpy(), ri)
    np.testing.assert_array_equal(s.cpu().numpy(), rs)
    assert ((ri >= lo + 3) & (ri < lo + 603)).all()


@pytest.mark.parametrize("Q,fp8", [(192, False), (256, False), (256, True)])
def test_single_pass_gemm_filter_equals_sampled_pipeline(gpu, Q, fp8):
    """Q >= 192 runs the GEMM filter either way: the single-pass form (lists + select
    with rescans) and the sampled-threshold form (sample pass, threshold select,
    threshold epilogue, region select) score with the same MFMAs, so their results
    are equal bit for bit -- on a Gaussian corpus and on the adversarial sorted one
    (huge tie groups: every tile's list truncated)."""
    from irc_amd import retrieval

    g = torch.Generator().manual_seed(Q)
    N, D, k = 50_000, 768, 100
    q = torch.nn.functional.normalize(torch.randn(Q, D, generator=g))
    d = torch.nn.functional.normalize(torch.randn(N, D, generator=g))
    ds = torch.zeros(N, D)
    ds[:, 0] = (torch.arange(N) % 256) / 128.0 - 1.0
    qs = torch.zeros(Q, D)
    qs[:, 0] = 1.0
    qs[::2, 1] = 0.5
    for qq, dd in ((q, d), (qs, ds)):
        outs = []
        prev = retrieval.set_single_pass_min_q(65)
        try:
            for mq in (65, 1 << 20):
                retrieval.set_single_pass_min_q(mq)
                if fp8:
                    q8 = retrieval.quantize_fp8(qq.to(gpu))
                    d8 = retrieval.quantize_fp8(dd.to(gpu))
                    outs.append(retrieval.scan_topk_fp8(q8, d8, k, 11, 1.0 / 256))
                else:
                    outs.append(retrieval.scan_topk(qq.bfloat16().to(gpu),
                                                    dd.bfloat16().to(gpu), k, 11))
            torch.cuda.synchronize()
        finally:
            retrieval.set_single_pass_min_q(prev)
        assert torch.equal(outs[0][1], outs[1][1]) and torch.equal(outs[0][0], outs[1][0])


@pytest.mark.parametrize("dtype", ["bf16", "fp8"])
def test_shard_beyond_one_pass_is_chunked_exact(gpu, dtype):
    """A shard of more 256-doc tiles than the GEMM filter's select handles in one pass
    (4096 tiles = 1,048,576 docs) at Q >= 192: scanned as two doc chunks plus a merge
    (scan_topk.hip chunk_docs).  Integer grid with many ties across the chunk boundary:
    bit-exact against the oracle (the first queries) and, for every query, against the
    same queries below the GEMM-filter threshold (Q = 191: one unchunked pass)."""
    from irc_amd import retrieval

    rng = np.random.default_rng(41)
    N, D, k = (1 << 20) + 3000, 128, 100
    d = _grid(rng, (N, D), lim=3 if dtype == "bf16" else 2)
    q = _grid(rng, (192, D), lim=3 if dtype == "bf16" else 2)
    if dtype == "fp8":
        d8, q8 = O.quantize_e4m3(d * 16), O.quantize_e4m3(q * 16)
        run = lambda qq: retrieval.scan_topk_fp8(_dev(qq, gpu), _dev(d8, gpu), k, 5,  # noqa
                                                 1.0 / 256)
        qsrc = q8
    else:
        run = lambda qq: retrieval.scan_topk(_dev(qq, gpu), _dev(d, gpu), k, 5)  # noqa: E731
        qsrc = q
    s, i = (t.cpu().numpy() for t in run(qsrc))
    s1, i1 = (t.cpu().numpy() for t in run(qsrc[:191]))
    np.testing.assert_array_equal(i[:191], i1)
    np.testing.assert_array_equal(s[:191], s1)
    if dtype == "fp8":
        ri, rs = O.scan_topk_fp8(q8[:6], d8, k, 5, 1.0 / 256)
    else:
        ri, rs = O.scan_topk(q[:6], d, k, 5)
    np.testing.assert_array_equal(i[:6], ri)
    np.testing.assert_array_equal(s[:6], rs)
    assert (i[:, 1:] != i[:, :-1]).all()
