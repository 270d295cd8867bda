"""irc_gemm (bf16 and exact-fp32 MFMA) vs a plain PyTorch fp32 reference of the same op."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _ref(a, b, trans_a, b_is_nk, bias, epi, res, alpha):
    A = a.float().cpu()
    B = b.float().cpu()
    A = A.t() if trans_a else A
    B = B.t() if b_is_nk else B
    y = alpha * (A @ B)
    if bias is not None:
        y = y + bias.cpu()
    if epi == 2:
        y = torch.nn.functional.gelu(y)
    if res is not None:
        y = y + res.float().cpu()
    return y


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("trans_a,b_is_nk", [(False, True), (False, False), (True, True),
                                             (True, False)])
@pytest.mark.parametrize("M,N,K", [(1, 1, 8), (37, 70, 24), (200, 300, 136), (256, 128, 768)])
def test_layouts(gpu, dtype, trans_a, b_is_nk, M, N, K):
    from irc_amd import ops

    g = torch.Generator().manual_seed(M * 1000 + N + K)
    a = torch.randn((K, M) if trans_a else (M, K), generator=g).to(dtype)
    b = torch.randn((N, K) if b_is_nk else (K, N), generator=g).to(dtype)
    out = ops.gemm(a.to(gpu), b.to(gpu), trans_a=trans_a, b_is_nk=b_is_nk,
                   out_dtype=torch.float32)
    ref = _ref(a, b, trans_a, b_is_nk, None, 0, None, 1.0)
    tol = 1e-4 * K if dtype == torch.float32 else 2e-2 * K ** 0.5
    assert (out.cpu() - ref).abs().max().item() <= tol


@pytest.mark.parametrize("epi", [1, 2, 3, 4])
@pytest.mark.parametrize("odt", [torch.bfloat16, torch.float32])
def test_epilogues(gpu, epi, odt):
    from irc_amd import ops

    g = torch.Generator().manual_seed(epi)
    M, N, K = 300, 260, 192
    a = torch.randn(M, K, generator=g).bfloat16()
    b = torch.randn(N, K, generator=g).bfloat16()
    bias = torch.randn(N, generator=g) if epi in (1, 2, 3) else None
    res = torch.randn(M, N, generator=g).to(odt) if epi in (3, 4) else None
    out = ops.gemm(a.to(gpu), b.to(gpu), bias=None if bias is None else bias.to(gpu),
                   epilogue=epi, residual=None if res is None else res.to(gpu), out_dtype=odt,
                   alpha=0.5)
    ref = _ref(a, b, False, True, bias, epi, res, 0.5)
    rel = (out.float().cpu() - ref).abs().max().item() / ref.abs().max().item()
    assert rel < (1e-2 if odt == torch.bfloat16 else 2e-3)


def test_fp32_accumulate(gpu):
    from irc_amd import ops

    g = torch.Generator().manual_seed(9)
    a = torch.randn(64, 96, generator=g)
    b = torch.randn(80, 96, generator=g)
    c0 = torch.randn(64, 80, generator=g)
    c = c0.clone().to(gpu)
    ops.gemm(a.to(gpu), b.to(gpu), out=c, accumulate=True)
    torch.testing.assert_close(c.cpu(), c0 + a @ b.t(), rtol=1e-5, atol=1e-4)


def test_fp32_mfma_is_exact_on_integers(gpu):
    """exact fp32 products: integer operands give the exact integer result."""
    from irc_amd import ops

    g = torch.Generator().manual_seed(3)
    a = torch.randint(-50, 50, (129, 64), generator=g).float()
    b = torch.randint(-50, 50, (33, 64), generator=g).float()
    out = ops.gemm(a.to(gpu), b.to(gpu)).cpu()
    assert torch.equal(out, a @ b.t())
