"""Small training-path kernels vs plain PyTorch fp32 references of the same op:
column sums (bias gradients; bf16 vector path and scalar path, deterministic),
and the transposing bf16 cast of weights."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("R,C,dtype", [(16384, 2048, torch.bfloat16), (1000, 520, torch.bfloat16),
                                       (777, 30, torch.bfloat16), (300, 64, torch.float32)])
def test_colsum(gpu, R, C, dtype):
    from irc_amd import ops

    g = torch.Generator().manual_seed(R + C)
    x = torch.randn((R, C), generator=g).to(dtype)
    out = ops.colsum(x.to(gpu))
    ref = x.double().sum(0)
    assert ((out.cpu().double() - ref).abs() <= 1e-4 * R ** 0.5).all()
    acc = torch.ones(C, device=gpu)
    ops.colsum(x.to(gpu), out=acc, accumulate=True)
    assert torch.equal(acc.cpu(), (out + 1).cpu())  # same fixed order -> identical


@pytest.mark.parametrize("R,C", [(2048, 768), (2048, 512), (33, 70)])
def test_cast_bf16_t(gpu, R, C):
    from irc_amd import ops

    x = torch.randn(R, C)
    y = ops.cast_bf16_t(x.to(gpu))
    assert y.shape == (C, R)
    assert torch.equal(y.cpu(), x.t().contiguous().to(torch.bfloat16))
