"""Trainable BERT bi-encoder (`--model BERT`): backward kernels and whole-encoder
gradients vs plain PyTorch fp32 references with autograd (tests/bert_ref.py, pinned
to the reference's HF output by test_bert_ref_matches_golden).

Tolerances (written per test): fp32 parity mode (exact-fp32 MFMA, VALU attention)
1e-4 relative Frobenius on gradients; bf16 production mode 3e-2 relative
Frobenius (bf16 operands / activation gradients, fp32 accumulation), 2e-2 on
single kernels.
"""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from bert_ref import bert_seq2vec

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def _mask(B, L, g, full_first=True):
    lens = torch.randint(1, L + 1, (B,), generator=g)
    if full_first:
        lens[0] = L
    return (torch.arange(L)[None] < lens[:, None]).long()


# ---------------------------------------------------------------- single kernels
def _attn_ref(qkv, mask, B, L, H, heads):
    dh = H // heads
    x = qkv.view(B, L, 3, heads, dh)
    q, k, v = (x[:, :, i].permute(0, 2, 1, 3) for i in range(3))
    s = q @ k.transpose(-1, -2) / math.sqrt(dh)
    bias = (1.0 - mask.float())[:, None, None, :] * torch.finfo(torch.float32).min
    p = torch.softmax(s + bias, dim=-1)
    return (p @ v).permute(0, 2, 1, 3).reshape(B * L, H)


@pytest.mark.parametrize("dtype,L,H,heads", [(torch.bfloat16, 64, 768, 12),
                                             (torch.bfloat16, 32, 128, 2),
                                             (torch.bfloat16, 128, 256, 4),
                                             (torch.float32, 64, 128, 2),
                                             (torch.float32, 24, 96, 3),
                                             (torch.bfloat16, 40, 128, 2),
                                             (torch.bfloat16, 93, 768, 12),
                                             (torch.bfloat16, 100, 256, 4),
                                             (torch.bfloat16, 129, 256, 4),
                                             (torch.bfloat16, 200, 256, 4),
                                             (torch.bfloat16, 317, 128, 2),
                                             (torch.bfloat16, 318, 128, 2),
                                             (torch.bfloat16, 400, 128, 2),
                                             (torch.bfloat16, 512, 768, 12),
                                             (torch.float32, 300, 128, 2),
                                             (torch.float32, 512, 32, 2),
                                             (torch.bfloat16, 65, 768, 12),
                                             (torch.bfloat16, 72, 256, 4),
                                             (torch.bfloat16, 2, 128, 2),
                                             (torch.bfloat16, 17, 256, 4),
                                             (torch.bfloat16, 127, 256, 4)])
def test_attention_bwd(gpu, dtype, L, H, heads):
    from irc_amd import ops

    B = 4
    g = torch.Generator().manual_seed(L * 7 + H)
    qkv = torch.randn((B * L, 3 * H), generator=g).to(dtype)
    mask = _mask(B, L, g)
    dctx = torch.randn((B * L, H), generator=g).to(dtype)
    q32 = qkv.float().requires_grad_(True)
    ref_ctx = _attn_ref(q32, mask, B, L, H, heads)
    ref_ctx.backward(dctx.float())
    ctx = ops.attention(qkv.to(gpu), mask.to(gpu), B, L, H, heads)
    dqkv = ops.attention_bwd(qkv.to(gpu), mask.to(gpu), ctx, dctx.to(gpu), B, L, H, heads)
    tol = 1e-4 if dtype == torch.float32 else 2e-2
    for part in range(3):  # dQ, dK, dV separately
        sl = slice(part * H, (part + 1) * H)
        r = _rel(dqkv.float()[:, sl], q32.grad[:, sl])
        assert r <= tol, f"part {part}: rel {r:.3g}"


@pytest.mark.parametrize("dtype,H,bcast", [(torch.bfloat16, 768, 0), (torch.bfloat16, 1024, 0),
                                           (torch.bfloat16, 768, 16), (torch.float32, 128, 0),
                                           (torch.float32, 96, 8), (torch.bfloat16, 200, 0)])
def test_layernorm_bwd(gpu, dtype, H, bcast):
    from irc_amd import ops

    rows = 16 * 37 if bcast == 0 else 16 * 12
    g = torch.Generator().manual_seed(H + bcast)
    x = (torch.randn((rows, H), generator=g) * 3 + 1).to(dtype)
    gamma = torch.randn(H, generator=g)
    beta = torch.randn(H, generator=g)
    dy_rows = rows // bcast if bcast else rows
    dy = torch.randn((dy_rows, H), generator=g)
    dy_in = dy if bcast else dy.to(dtype)
    scale = 1.0 / bcast if bcast else 1.0
    xr = x.float().requires_grad_(True)
    gr, br = gamma.clone().requires_grad_(True), beta.clone().requires_grad_(True)
    y = F.layer_norm(xr, (H,), gr, br, 1e-12)
    dyr = dy.repeat_interleave(bcast, 0) * scale if bcast else dy_in.float()
    y.backward(dyr)
    dg = torch.full((H,), 0.5, device=gpu)
    db = torch.full((H,), -0.25, device=gpu)
    dx = ops.layernorm_bwd(dy_in.to(gpu), x.to(gpu), gamma.to(gpu), dg, db, 1e-12,
                           bcast_L=bcast, dy_scale=scale)
    tol = 1e-5 if dtype == torch.float32 else 1e-2
    assert _rel(dx.float(), xr.grad) <= tol
    assert _rel(dg - 0.5, gr.grad) <= 1e-4
    assert _rel(db + 0.25, br.grad) <= 1e-4


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("M,N,K", [(512, 384, 256), (200, 136, 72)])
def test_gemm_gelu_epilogues(gpu, dtype, M, N, K):
    from irc_amd import ops

    g = torch.Generator().manual_seed(M + N + K)
    a = torch.randn((M, K), generator=g).to(dtype)
    w = (torch.randn((N, K), generator=g) / math.sqrt(K)).to(dtype)
    b = torch.randn(N, generator=g)
    out, pre = ops.gemm_gelu_save(a.to(gpu), w.to(gpu), b.to(gpu))
    u = a.float() @ w.float().T + b
    tol = 1e-5 if dtype == torch.float32 else 2e-2
    assert _rel(pre.float(), u) <= tol
    assert _rel(out.float(), F.gelu(u)) <= tol
    # epilogue 5: C = (dY W) * gelu'(u) with the saved pre-activation
    dY = torch.randn((M, K), generator=g).to(dtype)
    wk = (torch.randn((K, N), generator=g) / math.sqrt(K)).to(dtype)  # [K][N]
    du = ops.gemm(dY.to(gpu), wk.to(gpu), b_is_nk=False, epilogue=ops.EPI_DGELU, residual=pre)
    ur = pre.float().cpu().requires_grad_(True)
    F.gelu(ur).backward(dY.float() @ wk.float())
    assert _rel(du.float(), ur.grad) <= (1e-5 if dtype == torch.float32 else 2e-2)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_embed_bwd(gpu, dtype):
    from irc_amd import ops

    B, L, H, V = 6, 20, 64, 50
    g = torch.Generator().manual_seed(3)
    ids = torch.randint(0, V, (B, L), generator=g)
    ids[:, -3:] = 0  # PAD rows: no word-table gradient
    dx = torch.randn((B * L, H), generator=g).to(dtype)
    dword = torch.zeros((V, H), device=gpu)
    dpos = torch.ones((L + 4, H), device=gpu)
    dtype0 = torch.zeros((H,), device=gpu)
    ops.embed_bwd(dx.to(gpu), ids.to(gpu), dword, dpos[:L], dtype0, pad_id=0)
    dxf = dx.float()
    ref_w = torch.zeros((V, H)).index_add_(0, ids.flatten(), dxf)
    ref_w[0] = 0
    assert _rel(dword, ref_w) <= 1e-6
    assert _rel(dpos[:L] - 1, dxf.view(B, L, H).sum(0)) <= 1e-6
    assert torch.all(dpos[L:] == 1)
    assert _rel(dtype0, dxf.sum(0)) <= 1e-6


# ---------------------------------------------------------------- whole encoder
def _tiny_cfg(H=128, layers=2, heads=2, inter=256, vocab=300, maxpos=64):
    from irc_amd.bert import BertConfig

    return BertConfig(vocab_size=vocab, hidden_size=H, num_hidden_layers=layers,
                      num_attention_heads=heads, intermediate_size=inter,
                      max_position_embeddings=maxpos)


def _ids(B, L, V, seed):
    g = torch.Generator().manual_seed(seed)
    mask = _mask(B, L, g)
    ids = torch.randint(5, V, (B, L), generator=g)
    ids = torch.where(mask.bool(), ids, torch.zeros_like(ids))
    return ids, mask


def _encoder_grads(gpu, precision, cfg, B, L, seed):
    from irc_amd import precision as prec
    from irc_amd.bert_train import BertEncoder, seq2vec_ids

    prec.set_precision(precision)
    try:
        enc = BertEncoder(cfg, seed=seed).to(gpu)
        # non-trivial LN / bias values so every gradient path is exercised
        with torch.no_grad():
            gg = torch.Generator().manual_seed(seed + 1)
            for n, shp in enc.specs:
                if n.endswith("bias") or "LayerNorm" in n:
                    enc.view(n).add_(0.1 * torch.randn(shp, generator=gg).to(gpu))
        enc.invalidate_shadow()
        ids, mask = _ids(B, L, cfg.vocab_size, seed)
        r = torch.randn((B, cfg.hidden_size), generator=torch.Generator().manual_seed(seed + 2))
        enc.flat_grad.zero_()
        emb = seq2vec_ids(enc, ids.to(gpu), mask.to(gpu), grad=True)
        (emb * r.to(gpu)).sum().backward()
        torch.cuda.synchronize()
        P = {n: enc.view(n).detach().cpu().clone().requires_grad_(True) for n, _ in enc.specs}
        ref = bert_seq2vec(P, ids, mask, cfg.num_hidden_layers, cfg.num_attention_heads)
        (ref * r).sum().backward()
        return enc, emb, ref, P
    finally:
        prec.set_precision("bf16")


@pytest.mark.parametrize("precision,L,tol", [("fp32", 32, 1e-4), ("fp32", 20, 1e-4),
                                             ("bf16", 64, 3e-2), ("bf16", 32, 3e-2),
                                             ("bf16", 93, 3e-2), ("bf16", 100, 3e-2),
                                             ("bf16", 129, 3e-2), ("bf16", 318, 3e-2),
                                             ("bf16", 512, 3e-2), ("fp32", 200, 1e-4)])
def test_bert_encoder_grads(gpu, precision, L, tol):
    """Whole-encoder gradients at the lengths a joint-padded batch can take (the
    reference pads to the longest of 2B sentences and truncates at 512,
    contrastive_module.py:38): L > 128 runs the streamed attention forward and the
    block-looped attention backward."""
    cfg = _tiny_cfg(maxpos=max(64, L))
    enc, emb, ref, P = _encoder_grads(gpu, precision, cfg, B=6, L=L, seed=L)
    emb_tol = 1e-5 if precision == "fp32" else 2e-2
    assert (emb.cpu() - ref.detach()).abs().max().item() <= emb_tol
    bad = []
    for n, _ in enc.specs:
        if n.startswith("pooler."):
            assert enc.view(n, enc.flat_grad).abs().max().item() == 0.0
            continue
        got = enc.view(n, enc.flat_grad)
        if n.endswith("key.bias"):
            # exactly zero in real arithmetic (softmax is invariant to q.b_k, the same
            # shift for every key of a row): compare against the value-bias scale
            scale = P[n.replace("key.bias", "value.bias")].grad.norm().item()
            if got.norm().item() > tol * scale:
                bad.append((n, got.norm().item() / scale))
            continue
        rel = _rel(got, P[n].grad)
        if rel > tol:
            bad.append((n, rel))
    assert not bad, bad


def test_bert_encoder_grads_base_width(gpu):
    """H = 768 / 12 heads (the BERT-base layer shapes: big-tile GEMMs, vector LN
    backward, MFMA attention backward), 1 layer, bf16."""
    cfg = _tiny_cfg(H=768, layers=1, heads=12, inter=3072, vocab=500, maxpos=64)
    enc, emb, ref, P = _encoder_grads(gpu, "bf16", cfg, B=8, L=64, seed=5)
    assert (emb.cpu() - ref.detach()).abs().max().item() <= 2e-2
    for n, _ in enc.specs:
        if n.startswith("pooler."):
            continue
        got = enc.view(n, enc.flat_grad)
        if n.endswith("key.bias"):  # zero in real arithmetic (see above)
            scale = P[n.replace("key.bias", "value.bias")].grad.norm().item()
            assert got.norm().item() <= 3e-2 * scale, n
            continue
        rel = _rel(got, P[n].grad)
        assert rel <= 3e-2, (n, rel)


# ---------------------------------------------------------------- training step
def _bert_args(cfg_bert, B, queue_size=None):
    import argparse
    import os

    import yaml

    from conftest import PKG

    with open(os.path.join(PKG, "config.yaml")) as f:
        cfg = yaml.safe_load(f)
    cfg["model"]["BERT"] = {"config": cfg_bert}
    cfg["train"].update(batch_size=B, acml_batch_size=B)
    if queue_size:
        cfg["loss"]["InfoNCE"]["queue_size"] = queue_size
    return argparse.Namespace(config=cfg, loss="InfoNCE", model="BERT", opt="adam",
                              sample="uniform")


def test_bert_mode_train_step_matches_reference(gpu):
    """Two full fp32 training steps in --model BERT mode (loss with the queue,
    backward, clip + Adam, momentum update, enqueue) vs the same steps in plain
    PyTorch fp32 (torch.optim.Adam, clip_grad_norm_, the reference NCELoss math)."""
    from irc_amd import precision as prec
    from src.model import build_model, get_optimizer
    from src.train import TrainState

    cfgb = {"vocab_size": 300, "hidden_size": 128, "num_hidden_layers": 2,
            "num_attention_heads": 2, "intermediate_size": 256, "max_position_embeddings": 64}
    B, L = 8, 32
    prec.set_precision("fp32")
    try:
        args = _bert_args(cfgb, B, queue_size=32)
        torch.manual_seed(0)
        model = build_model(args).to(gpu).train()
        assert model.bert_model is None and model.loss_config["dim"] == 128
        model.add_queue_to_loss = True
        opt = get_optimizer(args, model)
        st = TrainState(args, model, opt)
        # reference state
        P = {n: model.encoder_q.view(n).cpu().clone().requires_grad_(True)
             for n, _ in model.encoder_q.specs if not n.startswith("pooler.")}
        Pk = {n: model.encoder_k.view(n).cpu().clone() for n in P}
        queue = model.queue.cpu().clone()
        ropt = torch.optim.Adam(list(P.values()), lr=2.5e-4, betas=(0.9, 0.999))
        losses, rlosses = [], []
        for step in range(2):
            ids, mask = _ids(2 * B, L, 300, 100 + step)
            loss, stepped = st.micro_batch(B, lambda: model.forward_ids(
                ids.to(gpu), mask.to(gpu), B))
            assert stepped
            losses.append(float(st.loss_record[-1]))
            # reference step
            q = bert_seq2vec(P, ids[:B], mask[:B], 2, 2)
            with torch.no_grad():
                k = bert_seq2vec(Pk, ids[B:], mask[B:], 2, 2)
            Fm = torch.cat([q, k])
            S = Fm @ Fm.T
            n2 = 2 * B
            keep = ~torch.eye(n2, dtype=torch.bool)
            S = S[keep].view(n2, n2 - 1)
            pos_col = torch.tensor([(i + B) % n2 - (1 if (i + B) % n2 > i else 0)
                                    for i in range(n2)])
            pos = S[torch.arange(n2), pos_col]
            neg = torch.stack([torch.cat([S[i, :pos_col[i]], S[i, pos_col[i] + 1:]])
                               for i in range(n2)])
            lq = (q @ queue).repeat(2, 1)
            logits = torch.cat([pos[:, None], neg, lq], 1) / 0.05
            rl = F.cross_entropy(logits, torch.zeros(n2, dtype=torch.long),
                                 reduction="sum") / 2 / B
            ropt.zero_grad()
            rl.backward()
            torch.nn.utils.clip_grad_norm_(list(P.values()), 1.0)
            ropt.step()
            with torch.no_grad():
                for n in P:
                    Pk[n] = Pk[n] * 0.9 + P[n].detach() * 0.1
                queue[:, (step * B) % 32:(step * B) % 32 + B] = k.T
            rlosses.append(rl.item())
        np.testing.assert_allclose(losses, rlosses, rtol=1e-4)
        # Adam's early steps move each element by ~lr * sign(g): an element whose
        # gradient is at rounding-noise level (e.g. every key bias, whose gradient
        # is zero in real arithmetic) may move either way on the two sides.  So:
        # every element within Adam's bound (2 steps x 2 lr), and >= 99% of the
        # elements of each tensor equal to 1e-6 (the momentum copy likewise).
        lim = 2 * 2 * 2.5e-4
        for n in P:
            for got, want in ((model.encoder_q.view(n).cpu(), P[n].detach()),
                              (model.encoder_k.view(n).cpu(), Pk[n])):
                d = (got - want).abs()
                assert d.max().item() <= lim, n
                assert (d > 1e-6).float().mean().item() <= 0.01, n
        assert _rel(model.queue, queue) <= 1e-5
    finally:
        prec.set_precision("bf16")


def test_bert_mode_bf16_steps_finite_and_shadow_current(gpu):
    """bf16 production mode: steps run, the loss is finite and decreasing on a fixed
    batch, and the bf16 operand shadows track the fp32 master weights after Adam /
    the momentum update."""
    from src.model import build_model, get_optimizer
    from src.train import TrainState

    cfgb = {"vocab_size": 300, "hidden_size": 128, "num_hidden_layers": 2,
            "num_attention_heads": 2, "intermediate_size": 256, "max_position_embeddings": 64}
    B, L = 16, 64
    args = _bert_args(cfgb, B, queue_size=64)
    torch.manual_seed(0)
    model = build_model(args).to(gpu).train()
    opt = get_optimizer(args, model)
    st = TrainState(args, model, opt)
    ids, mask = _ids(2 * B, L, 300, 7)
    ids, mask = ids.to(gpu), mask.to(gpu)
    for _ in range(6):
        st.micro_batch(B, lambda: model.forward_ids(ids, mask, B))
    losses = [float(x) for x in st.loss_record]
    assert all(math.isfinite(x) for x in losses)
    assert losses[-1] < losses[0]
    for enc in (model.encoder_q, model.encoder_k):
        sh = enc.shadow()
        assert torch.equal(sh, enc.flat.detach().to(torch.bfloat16))
    sT = model.encoder_q.shadow_t()
    n = "encoder.layer.1.intermediate.dense.weight"
    assert torch.equal(sT[n], model.encoder_q.view(n).to(torch.bfloat16).T.contiguous())


@pytest.mark.parametrize("dtype,R,C", [(torch.bfloat16, 16384, 768), (torch.bfloat16, 1000, 3072),
                                       (torch.float32, 700, 136)])
def test_colsum_batched(gpu, dtype, R, C):
    from irc_amd import ops

    nb = 3
    g = torch.Generator().manual_seed(R + C)
    x = torch.randn((nb, R, C), generator=g).to(dtype)
    stride = C + 40
    out = torch.ones((nb * stride,), device=gpu)
    ops.colsum_batched(x.to(gpu), out, stride, accumulate=True)
    ref = x.float().sum(1)
    got = out.view(nb, stride)[:, :C].cpu() - 1
    assert _rel(got, ref) <= 1e-5
    assert torch.all(out.view(nb, stride)[:, C:] == 1)
