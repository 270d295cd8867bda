"""Small training-path kernels vs plain PyTorch fp32 references of the same op:
column sums (bias gradients; bf16 vector path and scalar path, deterministic),
the transposing bf16 cast of weights, the head activations (src/model.py:25,
`eval(f"nn.{act}()")`) forward and backward against torch autograd, and the fused
SGD step against torch.optim.SGD (src/model.py:45-51)."""
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


ACTS = ["Identity", "ReLU", "ReLU6", "LeakyReLU", "ELU", "CELU", "SELU", "GELU", "SiLU", "Mish",
        "Sigmoid", "Tanh", "Softplus", "Softsign", "Hardtanh", "Hardsigmoid", "Hardswish",
        "Tanhshrink"]


@pytest.mark.parametrize("name", ACTS)
def test_activation_fwd_bwd(gpu, name):
    """Tolerance: fp32 transcendental ulps, 2e-6 relative + 1e-6 absolute."""
    from irc_amd import ops

    g = torch.Generator().manual_seed(len(name))
    u = torch.cat([torch.randn(5000, generator=g) * 4,
                   torch.tensor([-25., -6., -3., -1., 0., 1., 3., 6., 19.9, 20.1, 25.])])
    ur = u.clone().requires_grad_(True)
    y = getattr(torch.nn, name)()(ur)
    gy = torch.randn(u.shape, generator=g)
    y.backward(gy)
    kind = ops.ACTIVATIONS[name]
    yd = ops.activation(kind, u.to(gpu))
    torch.testing.assert_close(yd.cpu(), y.detach(), rtol=2e-6, atol=1e-6)
    gd = ops.activation_bwd(kind, u.to(gpu), gy.to(gpu).clone())
    torch.testing.assert_close(gd.cpu(), ur.grad, rtol=2e-6, atol=1e-6)


@pytest.mark.parametrize("clip", [None, 0.5])
def test_sgd_step_matches_torch(gpu, clip):
    """Three steps of the fused SGD (momentum 0.9, weight decay 1e-2, the clip
    coefficient applied to the gradient) against torch.optim.SGD after
    clip_grad_norm_; within 1e-6 relative (one fma difference per update)."""
    from irc_amd import ops

    n = 10007
    g0 = torch.Generator().manual_seed(9)
    p = torch.randn(n, generator=g0)
    pr = p.clone().requires_grad_(True)
    opt = torch.optim.SGD([pr], lr=0.05, momentum=0.9, weight_decay=1e-2)
    pd = p.to(gpu)
    buf = torch.zeros(n, device=gpu)
    for it in range(3):
        grad = torch.randn(n, generator=g0)
        pr.grad = grad.clone()
        if clip is not None:
            torch.nn.utils.clip_grad_norm_([pr], clip)
        opt.step()
        gd = grad.to(gpu)
        coef = ops.grad_norm_clip(gd, clip if clip is not None else float("inf"))
        ops.sgd_step(pd, gd, buf, coef, 0.05, 0.9, 1e-2, it == 0)
    torch.testing.assert_close(pd.cpu(), pr.detach(), rtol=1e-6, atol=1e-7)
    torch.testing.assert_close(buf.cpu(), opt.state[pr]["momentum_buffer"], rtol=1e-5, atol=1e-7)
