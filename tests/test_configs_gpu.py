"""Parity at the BASELINE configs the bench times (configs_untested).

* C2 loss: NCELoss at N=256, K=12544, D=128/768 against the reference's values
  (tests/golden/nce_c2.npz, inputs regenerated from tests/synth_inputs.py).
* C2 encoder: 12-layer BERT-base (H=768) against HF's last_hidden_state
  (tests/golden/bert_base.npz), fp32 parity mode and bf16 production mode.
* C2 training step at full size: BERT-base frozen bf16, B=256, L=64, K=12544,
  3-layer BiLSTM 768->256x2->128 -- bf16 against fp32 mode (loss within
  north_star's 1e-3, gradients), queue / queue_ptr update rule, finite step.
* C3 / C4 retrieval shards at full size (250k x 768, Q=1024; 625k x 1024,
  Q=2048 on the GEMM-kernel filter) on integer-grid embeddings, where every
  score is exact in fp32 in any order: bit-exact against the oracle on sampled
  queries and, for every query, the exact (score desc, index asc) rule against
  the full score matrix; plus an adversarial shard where EVERY doc survives
  the threshold at Q=2048.
"""
import argparse

import numpy as np
import pytest
import torch

import synth_inputs as SI
from conftest import load_golden
from oracle import irc_oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture
def fp32_mode():
    from irc_amd.precision import get_precision, set_precision

    old = get_precision()
    set_precision("fp32")
    yield
    set_precision(old)


# ------------------------------------------------------------------ C2 loss
@pytest.mark.parametrize("case", [0, 1])
@pytest.mark.parametrize("with_q", [False, True])
def test_nce_c2_shapes_vs_reference(gpu, case, with_q):
    from irc_amd.nce import info_nce

    g = load_golden("nce_c2.npz")
    n, d, kq, seed = SI.NCE_C2_CASES[case]
    q, k, queue = SI.nce_c2_inputs(n, d, kq, seed)
    tag = f"n{n}_d{d}_k{kq}_{'q' if with_q else 'noq'}"
    qq = torch.from_numpy(q).to(gpu).requires_grad_(True)
    loss = info_nce(qq, torch.from_numpy(k).to(gpu),
                    torch.from_numpy(queue).to(gpu) if with_q else None, 0.05)
    loss.backward()
    dq = qq.grad.cpu().numpy().astype(np.float64)
    ref = float(g[f"{tag}_loss"])
    rel = abs(loss.item() - ref) / abs(ref)
    print(f"{tag}: loss {loss.item():.6f} vs reference {ref:.6f} (rel {rel:.2e})")
    assert rel <= 1e-5  # exact-fp32 MFMA GEMMs + fp32 row LSE
    np.testing.assert_allclose(dq[:16], g[f"{tag}_dq_head"], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(dq[-16:], g[f"{tag}_dq_tail"], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(np.linalg.norm(dq, axis=1), g[f"{tag}_dq_rownorm"], rtol=1e-4)
    np.testing.assert_allclose(dq.sum(axis=0), g[f"{tag}_dq_colsum"], rtol=1e-3, atol=1e-4)


# ------------------------------------------------------------------ C2 encoder
def _bert_base(dev):
    from irc_amd.bert import BertConfig, BertModel

    m = BertModel(BertConfig(**SI.BERT_BASE))
    sd = {n: torch.from_numpy(SI.bert_param(n, tuple(v.shape)))
          for n, v in m.state_dict().items() if "position_ids" not in n}
    missing = m.load_state_dict(sd, strict=False).missing_keys
    assert not [n for n in missing if "position_ids" not in n]
    return m.to(dev)


def _bert_base_out(gpu):
    g = load_golden("bert_base.npz")
    m = _bert_base(gpu)
    out = m.encode(torch.from_numpy(g["input_ids"]).to(gpu),
                   torch.from_numpy(g["attention_mask"]).to(gpu)).float().cpu().numpy()
    return g, out


def test_bert_base_12_layers_fp32(gpu, fp32_mode):
    g, out = _bert_base_out(gpu)
    err = np.abs(out - g["last_hidden_state"]).max()
    print(f"BERT-base fp32 mode: max abs err {err:.2e}")
    np.testing.assert_allclose(out, g["last_hidden_state"], rtol=1e-4, atol=3e-4)


def test_bert_base_12_layers_bf16(gpu):
    """Production precision (bf16 operands, fp32 accumulation / LN statistics).
    LN outputs are O(1); the error of 12 bf16 layers is stated and bounded, and
    the pooled seq2vec direction (what the loss and the scan consume) is held to
    cosine >= 0.9999 of the reference's."""
    g, out = _bert_base_out(gpu)
    err = np.abs(out - g["last_hidden_state"]).max()
    rms = np.sqrt(np.mean((out - g["last_hidden_state"]) ** 2))
    pooled = out.astype(np.float64).mean(axis=1)
    pooled /= np.linalg.norm(pooled, axis=1, keepdims=True)
    cos = (pooled * g["seq2vec"]).sum(axis=1)
    print(f"BERT-base bf16: max abs err {err:.3e}, rms {rms:.3e}, pooled cosine {cos.min():.6f}")
    assert err <= 0.15 and rms <= 0.02
    assert cos.min() >= 0.9999


# ------------------------------------------------------------------ C2 train step
def _c2_step(gpu, precision, weights="bf16", B=256):
    from bench import c2_config, synthetic_batch
    from irc_amd.precision import get_precision, set_precision
    from src.model import build_model, get_optimizer

    old = get_precision()
    set_precision(precision)
    try:
        cfg = c2_config()
        cfg["train"].update(batch_size=B, acml_batch_size=B)
        ns = argparse.Namespace(config=cfg, loss="InfoNCE", model="LSTM", opt="adam",
                                sample="uniform")
        torch.manual_seed(1337)
        model = build_model(ns).to(gpu).train()
        model.bert_model.set_weight_format(weights)
        model.add_queue_to_loss = True
        opt = get_optimizer(ns, model)
        ids, mask = synthetic_batch(2 * B, 64, 1337)
        ids, mask = ids.to(gpu), mask.to(gpu)
        queue0 = model.queue.clone()
        a, p = model.bert_extract_ids(ids, mask, B)
        with torch.no_grad():
            emb_k = model.seq2vec(p, query=False)
        loss = model.forward_features(a, p)  # heads, loss, enqueue
        loss.backward()
        grad = model.encoder_q.flat_grad.clone()
        coef = opt.clip_and_step(1.0)
        model._momentum_update_key_encoder()
        torch.cuda.synchronize()
        return (loss.item(), grad, coef.cpu(), emb_k, queue0, model)
    finally:
        set_precision(old)


def test_c2_train_step_full_size(gpu):
    l16, g16, c16, k16, q0, m16 = _c2_step(gpu, "bf16")
    l32, g32, c32, _, _, _ = _c2_step(gpu, "fp32")
    rel = abs(l16 - l32) / abs(l32)
    grel = ((g16 - g32).norm() / g32.norm()).item()
    print(f"C2 step: loss bf16 {l16:.6f} vs fp32 {l32:.6f} (rel {rel:.2e}); "
          f"grad rel {grel:.2e}; grad norm {c16[0].item():.4f} / {c32[0].item():.4f}")
    assert np.isfinite(l16) and np.isfinite(l32)
    assert rel <= 1e-3  # north_star: InfoNCE loss within 1e-3 (bf16)
    assert grel <= 5e-2
    assert torch.isfinite(m16.encoder_q.flat).all() and torch.isfinite(m16.encoder_k.flat).all()
    # enqueue rule (contrastive_module.py:55-68): 12544 % 256 == 0 -> keys at [0, 256)
    assert int(m16.queue_ptr.item()) == 256
    assert torch.equal(m16.queue[:, 256:], q0[:, 256:])
    np.testing.assert_allclose(m16.queue[:, :256].T.cpu().numpy(), k16.cpu().numpy(), atol=1e-6)


def test_c5_fp8_step_loss_vs_fp32(gpu):
    """C5: the C2 step with every frozen-encoder nn.Linear on MX-fp8 (irc_gemm_mx: e4m3
    codes with one E8M0 scale per 32 consecutive k of a row, for weights and inputs;
    inputs quantised by their producing LayerNorm / attention / GELU epilogues,
    irc_amd/bert.py set_weight_format("fp8")).  Its InfoNCE loss against the fp32-mode step
    on the same inputs and initial weights: the fp8 quantisation of 72 GEMM inputs
    perturbs the features (pooled cosine ~0.998, tests/test_fp8_encoder_gpu.py), so
    the bound is looser than bf16's 1e-3; the measured delta is printed."""
    l8, g8, _, _, _, m8 = _c2_step(gpu, "bf16", weights="fp8")
    l32, g32, _, _, _, _ = _c2_step(gpu, "fp32")
    rel = abs(l8 - l32) / abs(l32)
    grel = ((g8 - g32).norm() / g32.norm()).item()
    print(f"C5 fp8 step: loss {l8:.6f} vs fp32 {l32:.6f} (rel {rel:.2e}); grad rel {grel:.2e}")
    assert np.isfinite(l8)
    assert rel <= 5e-3
    assert grel <= 0.25
    assert torch.isfinite(m8.encoder_q.flat).all()


@pytest.mark.parametrize("case", [0, 1])
@pytest.mark.parametrize("with_q", [False, True])
def test_nce_c34_global_batch_vs_reference(gpu, case, with_q):
    """C3 / C4 global batches: NCELoss at N = 1024 and 2048 (D = 128, K = 12544)
    against the reference's values (tests/golden/nce_c34.npz)."""
    from irc_amd.nce import info_nce

    g = load_golden("nce_c34.npz")
    n, d, kq, seed = SI.NCE_C34_CASES[case]
    q, k, queue = SI.nce_c2_inputs(n, d, kq, seed)
    tag = f"n{n}_d{d}_k{kq}_{'q' if with_q else 'noq'}"
    qq = torch.from_numpy(q).to(gpu).requires_grad_(True)
    loss = info_nce(qq, torch.from_numpy(k).to(gpu),
                    torch.from_numpy(queue).to(gpu) if with_q else None, 0.05)
    loss.backward()
    dq = qq.grad.cpu().numpy().astype(np.float64)
    ref = float(g[f"{tag}_loss"])
    rel = abs(loss.item() - ref) / abs(ref)
    print(f"{tag}: loss {loss.item():.4f} vs reference {ref:.4f} (rel {rel:.2e})")
    assert rel <= 1e-5
    np.testing.assert_allclose(dq[:16], g[f"{tag}_dq_head"], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(dq[-16:], g[f"{tag}_dq_tail"], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(np.linalg.norm(dq, axis=1), g[f"{tag}_dq_rownorm"], rtol=1e-4)
    np.testing.assert_allclose(dq.sum(axis=0), g[f"{tag}_dq_colsum"], rtol=1e-3, atol=1e-4)


def test_c3_global_batch_step_never_enqueues(gpu):
    """One full training step at global B = 1024 (C3) on one GPU: 12544 % 1024 != 0,
    so the reference never enqueues (contrastive_module.py:59; nce_c34.npz holds
    the reference's own behaviour) -- queue and queue_ptr stay bit-identical."""
    g = load_golden("nce_c34.npz")
    assert int(g["enq_b1024_k12544_ptr"]) == 0
    loss, grad, coef, _, q0, m = _c2_step(gpu, "bf16", B=1024)
    print(f"C3 step B=1024: loss {loss:.4f}, grad norm {coef[0].item():.4f}")
    assert np.isfinite(loss) and torch.isfinite(grad).all()
    assert int(m.queue_ptr.item()) == 0
    assert torch.equal(m.queue, q0)


# ------------------------------------------------------------------ C4 encoder
def _bert_large_out(gpu):
    from irc_amd.bert import BertConfig, BertModel

    g = load_golden("bert_large.npz")
    m = BertModel(BertConfig(**SI.BERT_LARGE))
    sd = {n: torch.from_numpy(SI.bert_param(n, tuple(v.shape)))
          for n, v in m.state_dict().items() if "position_ids" not in n}
    missing = m.load_state_dict(sd, strict=False).missing_keys
    assert not [n for n in missing if "position_ids" not in n]
    m = m.to(gpu)
    out = m.encode(torch.from_numpy(g["input_ids"]).to(gpu),
                   torch.from_numpy(g["attention_mask"]).to(gpu)).float().cpu().numpy()
    return g, out


def test_bert_large_24_layers_fp32(gpu, fp32_mode):
    """C4 encoder: BERT-large (24 layers, H=1024, A=16, I=4096) in fp32 parity
    mode against HF's last_hidden_state."""
    g, out = _bert_large_out(gpu)
    err = np.abs(out - g["last_hidden_state"]).max()
    print(f"BERT-large fp32 mode: max abs err {err:.2e}")
    np.testing.assert_allclose(out, g["last_hidden_state"], rtol=1e-4, atol=3e-4)


def test_bert_large_24_layers_bf16(gpu):
    """C4 encoder in production precision: error stated, pooled direction held to
    cosine >= 0.9999 of the reference's."""
    g, out = _bert_large_out(gpu)
    err = np.abs(out - g["last_hidden_state"]).max()
    rms = np.sqrt(np.mean((out - g["last_hidden_state"]) ** 2))
    pooled = out.astype(np.float64).mean(axis=1)
    pooled /= np.linalg.norm(pooled, axis=1, keepdims=True)
    cos = (pooled * g["seq2vec"]).sum(axis=1)
    print(f"BERT-large bf16: max abs err {err:.3e}, rms {rms:.3e}, pooled cosine {cos.min():.6f}")
    assert err <= 0.25 and rms <= 0.03
    assert cos.min() >= 0.9999


# ------------------------------------------------------------------ C3 / C4 shards
def _grid_gpu(gen, shape, lim, dev):
    m = torch.randint(-lim, lim + 1, shape, generator=gen, device=dev, dtype=torch.int32)
    return (m.float() / 128).bfloat16()  # exact in bf16 (|m| <= 127)


def _check_exact_rule(s, i, full, k):
    """(score desc, index asc) top-k of the exact score matrix, checked without
    sorting it: membership, order, completeness and the boundary-tie rule."""
    Q, N = full.shape
    assert bool((i >= 0).all()) and bool((i < N).all())
    assert torch.equal(s, torch.gather(full, 1, i))
    assert bool((s[:, 1:] <= s[:, :-1]).all())
    same = s[:, 1:] == s[:, :-1]
    assert bool((i[:, 1:][same] > i[:, :-1][same]).all())  # equal scores: lower index first
    masked = full.scatter(1, i, float("-inf"))
    bnd = s[:, -1:]
    assert bool((masked <= bnd).all())  # nothing outside beats the k-th score
    ar = torch.arange(N, device=full.device).expand(Q, N)
    tie_min = torch.where(masked == bnd, ar, N).min(dim=1).values
    ret_max = torch.where(s == bnd, i, -1).max(dim=1).values
    assert bool((tie_min > ret_max).all())  # boundary ties went to the lower indices


def _full_shard(gpu, Q, N, D, k, lim, seed, n_oracle=6):
    from irc_amd import retrieval

    gen = torch.Generator(device=gpu).manual_seed(seed)
    d = _grid_gpu(gen, (N, D), lim, gpu)
    q = _grid_gpu(gen, (Q, D), lim, gpu)
    s, i = retrieval.scan_topk(q, d, k)
    full = retrieval.scan_scores(q, d)  # exact on the grid
    _check_exact_rule(s, i, full, k)
    del full
    rows = np.r_[0:n_oracle // 2, Q - n_oracle // 2:Q]
    ri, rs = O.scan_topk(q[rows].float().cpu().numpy(), d.float().cpu().numpy(), k)
    np.testing.assert_array_equal(i[rows].cpu().numpy(), ri)
    np.testing.assert_array_equal(s[rows].cpu().numpy(), rs)
    return s, i


def test_c3_shard_full_size(gpu):
    """C3: 1M docs over 4 GPUs = 250k x 768 per shard, 1024 queries, top-100."""
    _full_shard(gpu, 1024, 250_000, 768, 100, 127, 31)


@pytest.mark.parametrize("lim", [127, 3])
def test_c4_shard_full_size(gpu, lim):
    """C4: 5M docs over 8 GPUs = 625k x 1024 per shard, 2048 queries, top-100
    (lim 3: values in {-3..3}/128 -> huge exact tie groups at the boundary)."""
    _full_shard(gpu, 2048, 625_000, 1024, 100, lim, 41 + lim)


def test_every_doc_survives_at_q2048(gpu):
    """Adversarial: identical docs, so every doc ties with every other for every
    query and every doc passes the threshold -- each 256-doc region is full, the
    select sees the whole shard; the answer is the k lowest indices."""
    from irc_amd import retrieval

    Q, N, D, k = 2048, 200_000, 128, 100
    gen = torch.Generator(device=gpu).manual_seed(5)
    q = _grid_gpu(gen, (Q, D), 127, gpu)
    d = _grid_gpu(gen, (1, D), 127, gpu).expand(N, D).contiguous()
    s, i = retrieval.scan_topk(q, d, k, 17)
    want_i = torch.arange(17, 17 + k, device=gpu).expand(Q, k)
    assert torch.equal(i, want_i)
    ref = retrieval.scan_scores(q, d[:1])
    assert torch.equal(s, ref.expand(Q, k))


@pytest.mark.parametrize("case", [0, 1])
def test_nce_fused_matches_unfused_and_times(gpu, case, monkeypatch):
    """The fused InfoNCE (csrc/nce_fused.hip; S and LQ never in HBM) against the
    unfused GEMM path at the C3 / C4 global batches: same loss (fp32 exact MFMA in
    both, different summation order) and dq; both timed (forward + backward, HIP
    events), the fused one expected no slower."""
    from irc_amd import nce

    n, d, kq, seed = SI.NCE_C34_CASES[case]
    q, k, queue = SI.nce_c2_inputs(n, d, kq, seed)
    out = {}
    for fused in ("1", "0"):
        monkeypatch.setenv("IRC_NCE_FUSED", fused)
        qq = torch.from_numpy(q).to(gpu).requires_grad_(True)
        kk, qu = torch.from_numpy(k).to(gpu), torch.from_numpy(queue).to(gpu)

        def run():
            qq.grad = None
            loss = nce.info_nce(qq, kk, qu, 0.05)
            loss.backward()
            return loss

        for _ in range(3):
            run()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            loss = run()
        e1.record()
        torch.cuda.synchronize()
        out[fused] = (loss.item(), qq.grad.clone(), e0.elapsed_time(e1) / 10 * 1e3)
    (lf, gf, tf), (lu, gu, tu) = out["1"], out["0"]
    print(f"N={n} K={kq}: fused {tf:.1f} us, unfused {tu:.1f} us (fwd+bwd); loss {lf:.4f} / {lu:.4f}")
    assert abs(lf - lu) <= 1e-5 * abs(lu)
    assert ((gf - gu).norm() / gu.norm()).item() <= 1e-5
