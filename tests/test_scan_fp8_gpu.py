"""fp8 (e4m3fn) corpus scan -- BASELINE config C5 -- against the CPU oracle.

The quantiser is bit-exact against the oracle's OCP e4m3fn restatement (itself
pinned to torch's float8 cast in test_oracle_golden.py).  Scores of e4m3 values
m/16 (|m| <= 15) are exact in fp32 whatever the accumulation order, so the top-k
is checked bit-exact on such grids; Gaussian embeddings quantised on the GPU are
checked margin-aware like the bf16 scan.
"""
import numpy as np
import pytest
import torch

from oracle import irc_oracle as O

pytestmark = pytest.mark.gpu


def _grid_codes(rng, shape):
    # m/16 with |m| <= 15: exactly representable in e4m3 (4 significant bits)
    return O.quantize_e4m3(rng.integers(-15, 16, shape).astype(np.float32) / 16)


def _dev(x, dev):
    return torch.from_numpy(np.ascontiguousarray(x)).to(dev)


@pytest.mark.parametrize("src_dtype", [torch.float32, torch.bfloat16])
def test_quantize_bit_exact(gpu, src_dtype):
    from irc_amd import retrieval

    rng = np.random.default_rng(1)
    mags = rng.choice(np.array([1e-3, 1e-2, 0.1, 1, 10, 30], np.float32), 50_001)
    x = torch.from_numpy(rng.standard_normal(50_001).astype(np.float32) * mags).to(src_dtype)
    x[:6] = torch.tensor([0.0, -0.0, 2**-13, 3 * 2**-14, 60.0, -100.0]).to(src_dtype)
    got = retrieval.quantize_fp8(x.to(gpu), 16.0).cpu().numpy()
    want = O.quantize_e4m3(x.float().numpy(), 16.0)
    np.testing.assert_array_equal(got, want)


@pytest.mark.parametrize("Q,D", [(70, 64), (70, 128), (70, 256), (70, 512), (70, 768),
                                 (70, 1024),
                                 # Q >= 192, D % 128 == 0: the ping-pong GEMM kernel on
                                 # v_mfma_scale_f32_16x16x128_f8f6f4
                                 (256, 768), (300, 128), (192, 1024)])
def test_scores_exact_on_grid(gpu, Q, D):
    from irc_amd import retrieval

    rng = np.random.default_rng(D + Q)
    q, d = _grid_codes(rng, (Q, D)), _grid_codes(rng, (517, D))
    s = retrieval.scan_scores_fp8(_dev(q, gpu), _dev(d, gpu)).cpu().numpy()
    np.testing.assert_array_equal(s, O.scan_scores(O.dequantize_e4m3(q), O.dequantize_e4m3(d)))


@pytest.mark.parametrize("Q,N,D,k,off", [
    (1, 1, 128, 1, 0),           # single doc
    (3, 5, 128, 8, 11),          # k > N -> padded
    (33, 31, 64, 10, 0),         # partial tile, Q not a multiple of 32
    (1, 100_000, 768, 100, 0),   # C5 shape, one query, two-phase
    (16, 60_000, 768, 100, 5),   # two-phase
    (64, 40_000, 768, 1024, 3),  # maximum k
    (257, 20_000, 128, 100, 0),  # several query blocks
    (200, 30_000, 1024, 50, 7),  # D = 1024, GEMM-kernel filter (scaled fp8 MFMA)
    (256, 100_000, 768, 100, 0),  # C5 dims, GEMM-kernel filter
    (384, 9_000, 384, 1024, 0),  # two query tiles, D = 384 (3 K-tiles), max k
    (1024, 12_000, 256, 100, 9),  # four query tiles sharing each doc tile
])
def test_topk_exact_vs_oracle(gpu, Q, N, D, k, off):
    from irc_amd import retrieval

    rng = np.random.default_rng(Q * 7 + N)
    q, d = _grid_codes(rng, (Q, D)), _grid_codes(rng, (N, D))
    s, i = retrieval.scan_topk_fp8(_dev(q, gpu), _dev(d, gpu), k, off, 1.0 / 256)
    ri, rs = O.scan_topk_fp8(q, d, k, doc_offset=off, score_scale=1.0 / 256)
    np.testing.assert_array_equal(i.cpu().numpy(), ri)
    np.testing.assert_array_equal(s.cpu().numpy(), rs)


def test_index_fp8_gaussian_margin_aware(gpu):
    """ShardedDenseIndex(dtype="fp8") on unit-norm Gaussian embeddings: the ranking
    of the quantised embeddings (same codes as the oracle's quantiser)."""
    from irc_amd import retrieval

    torch.manual_seed(7)
    Q, N, D, k = 48, 30_000, 768, 100
    q = torch.nn.functional.normalize(torch.randn(Q, D))
    d = torch.nn.functional.normalize(torch.randn(N, D))
    index = retrieval.ShardedDenseIndex(d.to(gpu), dtype="fp8")
    s, i = index.search(q.to(gpu), k)
    s, i = s.cpu().numpy(), i.cpu().numpy()
    qc, dc = O.quantize_e4m3(q.numpy(), 16.0), O.quantize_e4m3(d.numpy(), 16.0)
    np.testing.assert_array_equal(index.docs.cpu().numpy(), dc)
    full = O.scan_scores(O.dequantize_e4m3(qc), O.dequantize_e4m3(dc)) / np.float32(256)
    ri, rs = O.topk_rows(full, k)
    tol = 1e-5  # fp32 accumulation order on D = 768 products of e4m3 values
    for r in range(Q):
        np.testing.assert_allclose(s[r], full[r, i[r]], atol=tol)
        for doc in set(i[r]) ^ set(ri[r]):
            assert abs(full[r, doc] - rs[r, -1]) <= 2 * tol
        assert np.all(np.diff(s[r]) <= 0)


def test_fp8_full_c5_shard_properties(gpu):
    """A C5 shard (5M docs / 8 GPUs = 625k x 768 e4m3, 256 queries): properties."""
    from irc_amd import retrieval

    g = torch.Generator(device="cpu").manual_seed(5)
    Q, N, D, k = 256, 625_000, 768, 100
    d8 = retrieval.quantize_fp8(
        torch.nn.functional.normalize(torch.randn(N, D, generator=g)).to(gpu))
    q8 = retrieval.quantize_fp8(
        torch.nn.functional.normalize(torch.randn(Q, D, generator=g)).to(gpu))
    s, i = retrieval.scan_topk_fp8(q8, d8, k)
    assert bool((i >= 0).all()) and bool((i < N).all())
    full = retrieval.scan_scores_fp8(q8, d8)
    assert torch.equal(s, torch.gather(full, 1, i))
    assert bool((s[:, 1:] <= s[:, :-1]).all())
    masked = full.clone()
    masked.scatter_(1, i, float("-inf"))
    assert bool((masked.max(dim=1).values <= s[:, -1]).all())


@pytest.mark.parametrize("dtype", ["bf16", "fp8"])
def test_index_save_load_roundtrip(gpu, tmp_path, dtype):
    """On-disk corpus shard + doc-id map: the reloaded index holds the same bytes
    and returns the same top-k bits."""
    from irc_amd import retrieval

    torch.manual_seed(3)
    d = torch.nn.functional.normalize(torch.randn(5000, 256)).to(gpu)
    q = torch.nn.functional.normalize(torch.randn(20, 256)).to(gpu)
    idx = retrieval.ShardedDenseIndex(d, doc_offset=11, dtype=dtype)
    ids = [f"page_{i}" for i in range(5011)]
    idx.save(str(tmp_path), rank=0, doc_ids=ids)
    back, doc_dict = retrieval.ShardedDenseIndex.load(str(tmp_path), 0, gpu)
    assert back.dtype == dtype and back.doc_offset == 11
    assert torch.equal(back.docs.view(torch.uint8), idx.docs.view(torch.uint8))
    s0, i0 = idx.search(q, 50)
    s1, i1 = back.search(q, 50)
    assert torch.equal(s0, s1) and torch.equal(i0, i1)
    assert doc_dict[1] == ids and doc_dict[0]["page_7"] == 7
