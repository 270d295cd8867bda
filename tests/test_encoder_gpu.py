"""irc_layernorm vs a plain PyTorch fp32 reference of the same op (HF BertSelfOutput /
BertOutput LayerNorm, eps 1e-12, reached from contrastive_module.py:39).

bf16 rows with H in {512, 768, 1024} take the vectorised half-wave kernel, other
shapes the one-wave-per-row kernel.  Tolerance: bf16 output rounding
(1e-3 + 4e-3 |y|); fp32 1e-5."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dtype,rows,H", [(torch.bfloat16, 1000, 768), (torch.bfloat16, 7, 1024),
                                          (torch.bfloat16, 33, 512), (torch.bfloat16, 9, 300),
                                          (torch.float32, 65, 768)])
def test_layernorm(gpu, dtype, rows, H):
    from irc_amd import ops

    g = torch.Generator().manual_seed(rows + H)
    x = (torch.randn((rows, H), generator=g) * 3 + 1).to(dtype)
    gamma = torch.rand((H,), generator=g) + 0.5
    beta = torch.randn((H,), generator=g)
    y = ops.layernorm(x.to(gpu), gamma.to(gpu), beta.to(gpu), eps=1e-12)
    ref = torch.nn.functional.layer_norm(x.float(), (H,), gamma, beta, eps=1e-12)
    # bf16: one output rounding (half-ulp = 2^-9 |y|) plus fp32 statistics
    tol = (1e-3 + 4e-3 * ref.abs()) if dtype == torch.bfloat16 else 1e-5
    assert ((y.float().cpu() - ref).abs() <= tol).all()


@pytest.mark.parametrize("H,rows,L", [(768, 1000, 50), (1024, 64, 64), (96, 37, 37)])
def test_embed_ln(gpu, H, rows, L):
    """irc_embed_ln (HF BertEmbeddings: word[ids] + token_type[0] + position[l], then
    LayerNorm, contrastive_module.py:39) vs a plain fp32 reference; H = 768 / 1024 take the
    vectorised half-wave kernel, H = 96 the one-wave-per-row one.  Tolerance: bf16 output
    rounding of the table sums and the LN output."""
    from irc_amd import ops

    g = torch.Generator().manual_seed(H + rows)
    V = 300
    word = (torch.randn(V, H, generator=g) * 0.5).bfloat16()
    pos = (torch.randn(128, H, generator=g) * 0.2).bfloat16()
    type0 = (torch.randn(H, generator=g) * 0.1).bfloat16()
    gamma = torch.rand(H, generator=g) + 0.5
    beta = torch.randn(H, generator=g) * 0.1
    B = rows // L
    ids = torch.randint(0, V, (B, L), generator=g)
    y = ops.embed_ln(ids.to(gpu), word.to(gpu), pos.to(gpu), type0.to(gpu), gamma.to(gpu),
                     beta.to(gpu), 1e-12)
    e = (word.float()[ids] + type0.float()) + pos.float()[:L][None]
    ref = torch.nn.functional.layer_norm(e, (H,), gamma, beta, eps=1e-12).reshape(B * L, H)
    tol = 1e-3 + 8e-3 * ref.abs()
    assert ((y.float().cpu() - ref).abs() <= tol).all()
