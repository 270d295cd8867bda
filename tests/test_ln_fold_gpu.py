"""irc_gemm_ln -- the BERT encoder's LayerNorm fold -- vs plain PyTorch fp32 references.

The fold rewrites LN(h) . W^T + b (HF BertSelfOutput / BertOutput LayerNorm feeding
the next nn.Linear, contrastive_module.py:39 -> modeling_bert) as
r (h . W'^T) - r mu s + t with W' = bf16(W diag(gamma)), s = colsum(W'), t = b + W beta,
the statistics (mu, r) coming from the producing GEMM's epilogue as per-row
(sum, sum of squares) partials.  Shapes cover both kernels that run it: the 256 x 256
ping-pong kernel (and its small-shape fallback) and the 256 x 384 big-tile kernel
(M = 32768 - 68 rows with N = 768: whole waves of big tiles, ragged last tile).

Tolerances: bf16 operands and outputs; the fold's error is held to within 1.5x
(+ a small floor) of the explicit LayerNorm -> GEMM path's error against the same
fp32 reference, i.e. the fold may not be measurably less accurate."""
import pytest
import torch

pytestmark = pytest.mark.gpu

# (M, N, K): pp (4096 x 768), big (32700 x 768, ragged last row tile), pp fallback
# below both kernels' tile-count heuristics (1000 x 768), wide pp (4096 x 3072)
SHAPES = [(4096, 768, 768), (32700, 768, 768), (1000, 768, 256), (4096, 3072, 768)]


def _producer(gpu, M, N, K, seed):
    """h = a . b^T + bias + residual (bf16) with its LN statistics; rows carry an offset
    and a scale so the fold's mean subtraction and 1/sigma are exercised."""
    from irc_amd import ops

    g = torch.Generator().manual_seed(seed)
    a = (torch.randn(M, K, generator=g) * 0.5).bfloat16().to(gpu)
    b = (torch.randn(N, K, generator=g) * 0.05).bfloat16().to(gpu)
    bias = (torch.randn(N, generator=g) * 0.1).to(gpu)
    off = torch.randn(M, 1, generator=g) * 2.0
    scl = torch.rand(M, 1, generator=g) * 3.0 + 0.25
    res = (torch.randn(M, N, generator=g) * scl + off).bfloat16().to(gpu)
    h, st = ops.gemm_ln(a, b, bias, epilogue=ops.EPI_BIAS_RESID, residual=res, want_stats=True)
    ref = a.float() @ b.float().T + bias + res.float()
    return h, st, ref


@pytest.mark.parametrize("M,N,K", SHAPES)
def test_producer_and_stats(gpu, M, N, K):
    h, st, ref = _producer(gpu, M, N, K, M + N)
    assert st.t.shape == (M, st.nt, 2) and st.h == N
    err = (h.float() - ref).abs().max().item()
    assert err <= 1e-2 * ref.abs().max().item()
    # the statistics are those of the stored bf16 values (fp32 partial sums)
    hf = h.float()
    s = st.t.sum(1)
    assert torch.allclose(s[:, 0], hf.sum(1), rtol=1e-4, atol=1e-2)
    assert torch.allclose(s[:, 1], (hf * hf).sum(1), rtol=1e-4, atol=1e-2)


def _ln_params(gpu, H, seed):
    g = torch.Generator().manual_seed(seed)
    gamma = (1.0 + 0.3 * torch.randn(H, generator=g)).to(gpu)
    beta = (0.2 * torch.randn(H, generator=g)).to(gpu)
    return gamma, beta


@pytest.mark.parametrize("epi", [1, 2])
@pytest.mark.parametrize("M,H,N", [(4096, 768, 3072), (32700, 768, 2304), (1000, 768, 768),
                                   (32700, 768, 768)])
def test_fold(gpu, epi, M, H, N):
    from irc_amd import ops

    eps = 1e-12
    h, st, _ = _producer(gpu, M, H, 256, 7 * M + N)
    gamma, beta = _ln_params(gpu, H, N)
    g = torch.Generator().manual_seed(M - N)
    W = (torch.randn(N, H, generator=g) * 0.05).to(gpu)
    bias = (torch.randn(N, generator=g) * 0.1).to(gpu)
    wf = (W * gamma[None]).bfloat16()
    s = wf.float().sum(1).contiguous()
    t = (bias + W @ beta).contiguous()
    y = ops.gemm_ln(h, wf, t, epilogue=epi, stats=st, eps=eps, colsum=s)
    # fp32 reference and the explicit LayerNorm kernel -> GEMM path
    ln = torch.nn.functional.layer_norm(h.float(), (H,), gamma, beta, eps)
    ref = ln @ W.T + bias
    if epi == 2:
        ref = torch.nn.functional.gelu(ref)
    x = ops.layernorm(h, gamma, beta, eps)
    y0 = ops.gemm(x, W.bfloat16(), bias=bias, epilogue=epi)
    err = (y.float() - ref).abs().max().item()
    err0 = (y0.float() - ref).abs().max().item()
    assert err <= 1.5 * err0 + 2e-3 * ref.abs().max().item(), (err, err0)
    rel = (y.float() - ref).norm().item() / ref.norm().item()
    assert rel < 1e-2


@pytest.mark.parametrize("M,N,K", [(4096, 768, 3072), (32700, 768, 3072), (1000, 768, 768)])
def test_residual_layernorm(gpu, M, N, K):
    """FFN2 / out-projection form: out = u . W^T + b + bf16(LN(h)), LN(h) recomputed
    from h and its statistics exactly as irc_layernorm writes it; plus the output's
    own statistics for the next fold."""
    from irc_amd import ops

    eps = 1e-12
    h, st, _ = _producer(gpu, M, N, 256, M + K)
    gamma, beta = _ln_params(gpu, N, K)
    g = torch.Generator().manual_seed(K)
    u = (torch.randn(M, K, generator=g) * 0.5).bfloat16().to(gpu)
    W = (torch.randn(N, K, generator=g) * 0.03).bfloat16().to(gpu)
    bias = (torch.randn(N, generator=g) * 0.1).to(gpu)
    y, st2 = ops.gemm_ln(u, W, bias, epilogue=ops.EPI_BIAS_RESID, residual=h, stats=st,
                         gamma=gamma, beta=beta, eps=eps, want_stats=True)
    x = ops.layernorm(h, gamma, beta, eps)  # the LN kernel's bf16 output
    y0 = ops.gemm(u, W, bias=bias, epilogue=ops.EPI_BIAS_RESID, residual=x)
    ref = u.float() @ W.float().T + bias + x.float()
    err = (y.float() - ref).abs().max().item()
    err0 = (y0.float() - ref).abs().max().item()
    assert err <= 1.5 * err0 + 2e-3 * ref.abs().max().item(), (err, err0)
    yf = y.float()
    s = st2.t.sum(1)
    assert torch.allclose(s[:, 0], yf.sum(1), rtol=1e-4, atol=1e-2)
    assert torch.allclose(s[:, 1], (yf * yf).sum(1), rtol=1e-4, atol=1e-2)


def test_gemm_ln_rejects_bad_inputs(gpu):
    from irc_amd import ops

    a = torch.zeros(256, 768, dtype=torch.bfloat16, device=gpu)
    b = torch.zeros(768, 768, dtype=torch.bfloat16, device=gpu)
    bias = torch.zeros(768, device=gpu)
    with pytest.raises(TypeError):
        ops.gemm_ln(a.float(), b, bias, epilogue=ops.EPI_BIAS_RESID, residual=a)
    with pytest.raises(ops.IRCError):  # the fold without statistics
        ops.gemm_ln(a, b, bias, epilogue=ops.EPI_BIAS)
    with pytest.raises(ops.IRCError):  # K % 64
        ops.gemm_ln(a[:, :700], b[:, :700], bias, epilogue=ops.EPI_BIAS_RESID, residual=a)


@pytest.mark.parametrize("B,L,layers", [(4, 128, 3), (256, 128, 2)])
def test_bert_encode_folded(gpu, B, L, layers):
    """The folded encoder vs the explicit one and the fp32 reference (tests/bert_ref.py),
    random LayerNorm parameters; B = 256 x L = 128 routes the N = 768 GEMMs to the
    big-tile kernel, B = 4 to the 256 x 256 fallback."""
    import dataclasses

    import bert_ref
    from irc_amd.bert import BERT_BASE, BertModel

    cfg = dataclasses.replace(BERT_BASE, num_hidden_layers=layers)
    m = BertModel(cfg, seed=3)
    g = torch.Generator().manual_seed(11)
    with torch.no_grad():
        for n, p in m.named_parameters():
            if n.endswith("LayerNorm.weight"):
                p.copy_(1.0 + 0.2 * torch.randn(p.shape, generator=g))
            elif n.endswith("LayerNorm.bias") or n.endswith(".bias"):
                p.copy_(0.1 * torch.randn(p.shape, generator=g))
    m = m.to(gpu)
    ids = torch.randint(1, cfg.vocab_size, (B, L), generator=g)
    mask = torch.ones(B, L, dtype=torch.int64)
    mask[: B // 2, L // 2:] = 0
    ids[mask == 0] = 0
    ids, mask = ids.to(gpu), mask.to(gpu)
    m.ln_fold = False
    y0 = m.encode(ids, mask).float()
    m.ln_fold = True
    y1 = m.encode(ids, mask).float()
    P = {k: v.float() for k, v in m.state_dict().items()}
    ref = bert_ref.bert_hidden(P, ids, mask, layers, cfg.num_attention_heads, cfg.layer_norm_eps)
    e0 = (y0 - ref).norm().item() / ref.norm().item()
    e1 = (y1 - ref).norm().item() / ref.norm().item()
    assert e1 < 1.5 * e0 + 1e-3, (e1, e0)
    assert e1 < 2e-2
