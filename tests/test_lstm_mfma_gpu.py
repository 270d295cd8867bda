"""MFMA BiLSTM recurrences at the production head width H = 256 -- the multi-CU
cluster kernels (csrc/lstm_coop.hip, the default) and the single-CU kernels
(csrc/lstm_mfma.hip) -- vs the numpy oracle (oracle/irc_oracle.py lstm_head_fwd / seq2vec /
seq2vec_bwd, which restate nn.LSTM, src/model.py:16-41, and seq2vec,
contrastive_module.py:102-112) and vs the VALU recurrences at the same precision.

bf16 production mode: W_ih, W_hh and h are bf16 operands, gates / c / accumulation
fp32.  Tolerances (stated per check): embeddings within 2e-2 absolute (unit
vectors), per-position head outputs within 3e-2 relative to their max, each
parameter gradient within 4e-2 relative Frobenius error of the fp64 oracle.
"""
import numpy as np
import pytest
import torch

from oracle import irc_oracle as O

pytestmark = pytest.mark.gpu

H = 256


def _head(In, layers, out, dev, seed=0):
    from irc_amd.lstm_head import LSTMHead

    torch.manual_seed(seed)
    cfg = {"model": {"LSTM": {"num_layers": layers, "bidirectional": True, "input_size": In,
                              "hidden_size": H, "output_size": out,
                              "activation": "Identity"}}}
    h = LSTMHead(cfg).to(dev)
    p = {n: v.detach().cpu().numpy().astype(np.float64) for n, v in h.named_flat_params()}
    return h, p


def _rel(a, b):
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


@pytest.fixture(params=["coop", "mfma"])
def rec(request, monkeypatch):
    monkeypatch.setenv("IRC_LSTM_RECURRENCE", request.param)
    return request.param


@pytest.fixture
def bf16_mode():
    from irc_amd.precision import get_precision, set_precision

    old = get_precision()
    set_precision("bf16")
    yield
    set_precision(old)


@pytest.mark.parametrize("B,L,In,layers", [(40, 9, 64, 2), (5, 1, 32, 1), (64, 16, 128, 1),
                                           (600, 3, 32, 1)])
def test_mfma_forward_vs_oracle(gpu, bf16_mode, rec, B, L, In, layers):
    from irc_amd import ops

    assert ops.lstm_mfma_supported(H)
    h, p = _head(In, layers, 48, gpu)
    assert h._recurrence(torch.bfloat16) == rec
    rng = np.random.default_rng(1)
    x = rng.standard_normal((B, L, In)).astype(np.float32)
    xd = torch.from_numpy(x).to(gpu)
    y = h(xd).cpu().numpy()
    y_ref, _ = O.lstm_head_fwd(x.astype(np.float64), p, layers)
    assert np.abs(y - y_ref).max() <= 3e-2 * np.abs(y_ref).max()
    emb, _ = h.forward_compute(xd, save=False)
    e_ref, _ = O.seq2vec(x.astype(np.float64), p, layers)
    np.testing.assert_allclose(emb.cpu().numpy(), e_ref, atol=2e-2)


@pytest.mark.parametrize("B,L,In,layers", [(40, 9, 64, 2), (33, 4, 96, 1), (530, 2, 32, 1)])
def test_mfma_grads_vs_oracle(gpu, bf16_mode, rec, B, L, In, layers):
    h, p = _head(In, layers, 32, gpu, seed=3)
    rng = np.random.default_rng(2)
    x = rng.standard_normal((B, L, In)).astype(np.float32)
    demb = rng.standard_normal((B, 32)).astype(np.float32)
    emb, saved = h.forward_compute(torch.from_numpy(x).to(gpu), save=True)
    h.flat_grad.zero_()
    h.backward_compute(saved, torch.from_numpy(demb).to(gpu))
    _, cache = O.seq2vec(x.astype(np.float64), p, layers)
    ref = O.seq2vec_bwd(demb.astype(np.float64), p, cache, layers)
    for name, _ in h.specs:
        got = h.view(name, h.flat_grad).cpu().numpy()
        assert _rel(got, ref[name]) <= 4e-2, (name, _rel(got, ref[name]))


def test_mfma_matches_valu_same_precision(gpu, bf16_mode, rec, monkeypatch):
    """Both recurrences see bf16 W and h; they differ only in accumulation order
    (and hence occasional 1-ulp bf16 roundings of h)."""
    h, _ = _head(64, 2, 32, gpu, seed=5)
    rng = np.random.default_rng(4)
    x = torch.from_numpy(rng.standard_normal((48, 12, 64)).astype(np.float32)).to(gpu)
    demb = torch.from_numpy(rng.standard_normal((48, 32)).astype(np.float32)).to(gpu)

    def run():
        e, s = h.forward_compute(x, save=True)
        h.flat_grad.zero_()
        h.backward_compute(s, demb)
        return e.cpu().numpy(), h.flat_grad.cpu().numpy().copy()

    e_m, g_m = run()
    monkeypatch.setenv("IRC_LSTM_RECURRENCE", "valu")
    e_v, g_v = run()
    np.testing.assert_allclose(e_m, e_v, atol=5e-3)
    assert _rel(g_m, g_v) <= 2e-2


def test_mfma_rejects_unsupported_width(gpu):
    from irc_amd import _lib, ops

    assert not ops.lstm_mfma_supported(128)
    w = torch.zeros(8 * 128 * 16, device=gpu)
    with pytest.raises(_lib.IRCError):
        ops.lstm_pack(w[:8 * 128 * 16].view(8 * 128, 16), w[:1024], w[:1024],
                      w[:8 * 128 * 128 // 8].view(-1), 128, 2)


@pytest.mark.parametrize("B,L", [(40, 7), (520, 5)])
def test_coop_matches_single_cu_and_no_timeout(gpu, B, L):
    """The cluster recurrence against the single-CU one on identical packed inputs
    (bf16 h on both sides; they differ only in MFMA shape / summation order), and
    the cluster timeout word stays clear (every member saw every hand-off)."""
    from irc_amd import ops

    torch.manual_seed(9)
    nd = 2
    whh = (torch.randn(nd * 4 * H, H) * 0.06).to(gpu)
    wih = (torch.randn(nd * 4 * H, 64) * 0.1).to(gpu)
    bih = torch.zeros(nd * 4 * H, device=gpu)
    x = torch.randn(B * L, 64, device=gpu).to(torch.bfloat16)
    wp, bp, w, wT = ops.lstm_pack(wih, bih, bih, whh, H, nd)
    xp = ops.gemm(x, wp, bias=bp, epilogue=ops.EPI_BIAS, out_dtype=torch.float32)
    wf, wb = ops.lstm_coop_pack(whh, H, nd)
    h_c, g_c, c_c, hp_c, sync = ops.lstm_fwd_coop(xp, wf, B, L, H, nd, save=True)
    h_m, g_m, c_m, hp_m = ops.lstm_fwd_mfma(xp, w, B, L, H, nd, save=True)
    assert not ops.lstm_coop_timed_out(sync, B, nd)
    assert (h_c.float() - h_m.float()).abs().max().item() <= 2e-2
    assert (hp_c.float() - hp_m.float()).abs().max().item() <= 2e-2
    # hprev written by the recurrence == the separate shift pass over its own hout
    from irc_amd import _lib
    from irc_amd._torch import ptr, stream_ptr

    hp_ref = torch.full_like(hp_c, 7.0)
    _lib.call("irc_lstm_hprev", ptr(h_c), ptr(hp_ref), B, L, H, nd, stream_ptr(gpu))
    assert torch.equal(hp_c, hp_ref)
    dy = torch.randn(B * L, nd * H, device=gpu) * 0.1
    dg_c, sync_b = ops.lstm_bwd_coop(dy, wb, g_c, c_c, B, L, H, nd)
    dg_m = ops.lstm_bwd_mfma(dy, wT, g_m, c_m, B, L, H, nd)
    assert not ops.lstm_coop_timed_out(sync_b, B, nd)
    err = (dg_c.float() - dg_m.float()).norm() / dg_m.float().norm()
    assert err.item() <= 2e-2
    # bitwise reproducible (fixed member summation order)
    dg_c2, _ = ops.lstm_bwd_coop(dy, wb, g_c, c_c, B, L, H, nd)
    assert torch.equal(dg_c, dg_c2)


@pytest.fixture
def forced_coop_timeout():
    """IRC_LSTM_COOP_SPIN_MAX=0 (read per call by the library): the first cross-CU
    wait of every workgroup times out, whether its data has arrived or not -- the
    debug path that must never yield numbers."""
    import os

    os.environ["IRC_LSTM_COOP_SPIN_MAX"] = "0"
    yield
    del os.environ["IRC_LSTM_COOP_SPIN_MAX"]


def test_coop_forced_timeout_poisons_outputs(gpu, forced_coop_timeout, bf16_mode):
    """A timed-out cluster call NaN-poisons its own output on the device and sets
    the sticky fault word -- whatever the caller does with the sync word."""
    from irc_amd import ops

    torch.manual_seed(3)
    B, L, nd = 64, 9, 2
    whh = (torch.randn(nd * 4 * H, H) * 0.06).to(gpu)
    xp = torch.randn(B * L, nd * 4 * H, device=gpu)
    wf, wb = ops.lstm_coop_pack(whh, H, nd)
    fault = torch.zeros(1, dtype=torch.int32, device=gpu)
    h, g, c, hp, sync = ops.lstm_fwd_coop(xp, wf, B, L, H, nd, save=True)
    ops.lstm_coop_fault(sync, B, nd, fault)
    assert ops.lstm_coop_timed_out(sync, B, nd)
    assert int(fault.item()) != 0
    assert bool(torch.isnan(h.float()).all())
    assert bool(torch.isnan(hp.float()).all())
    dg, sync_b = ops.lstm_bwd_coop(torch.randn(B * L, nd * H, device=gpu), wb, g, c, B, L, H, nd)
    assert ops.lstm_coop_timed_out(sync_b, B, nd)
    assert bool(torch.isnan(dg.float()).all())


def test_coop_forced_timeout_raises_in_train_step(gpu, forced_coop_timeout, bf16_mode):
    """The production step (H = 256 BiLSTM head on the cluster recurrence) raises
    at its next sync point instead of training on stale state."""
    import argparse

    import yaml

    from conftest import PKG
    from irc_amd._lib import IRCError
    from src.model import build_model, get_optimizer
    from src.train import TrainState

    with open(f"{PKG}/config.yaml") as f:
        cfg = yaml.safe_load(f)
    cfg["bert"] = {"name": "tiny", "config": {"vocab_size": 200, "hidden_size": 64,
                                              "num_hidden_layers": 1, "num_attention_heads": 2,
                                              "intermediate_size": 128,
                                              "max_position_embeddings": 64}}
    cfg["model"]["LSTM"].update(input_size=64, hidden_size=H, num_layers=2, output_size=32)
    cfg["loss"]["InfoNCE"].update(queue_size=64)
    cfg["train"].update(batch_size=32, acml_batch_size=32)
    args = argparse.Namespace(config=cfg, loss="InfoNCE", model="LSTM", opt="adam",
                              sample="uniform")
    torch.manual_seed(0)
    model = build_model(args).to(gpu).train()
    st = TrainState(args, model, get_optimizer(args, model))
    ids = torch.randint(5, 200, (64, 16), device=gpu)
    mask = torch.ones_like(ids)
    with pytest.raises(IRCError, match="timed out"):
        st.micro_batch(32, lambda: model.forward_features(*model.bert_extract_ids(ids, mask, 32)))


def test_coop_forced_timeout_step_changes_no_parameter(gpu, forced_coop_timeout, bf16_mode):
    """between a timeout and the raise at log_step the loop
    takes steps without syncing; the fault word gates Adam and the momentum update
    on the device, so those steps change no parameter, moment or key-encoder
    weight (and nothing turns NaN)."""
    import argparse

    import yaml

    from conftest import PKG
    from src.model import build_model, get_optimizer
    from src.train import TrainState

    with open(f"{PKG}/config.yaml") as f:
        cfg = yaml.safe_load(f)
    cfg["bert"] = {"name": "tiny", "config": {"vocab_size": 200, "hidden_size": 64,
                                              "num_hidden_layers": 1, "num_attention_heads": 2,
                                              "intermediate_size": 128,
                                              "max_position_embeddings": 64}}
    cfg["model"]["LSTM"].update(input_size=64, hidden_size=H, num_layers=2, output_size=32)
    cfg["loss"]["InfoNCE"].update(queue_size=64)
    cfg["train"].update(batch_size=32, acml_batch_size=32)
    args = argparse.Namespace(config=cfg, loss="InfoNCE", model="LSTM", opt="adam",
                              sample="uniform")
    torch.manual_seed(0)
    model = build_model(args).to(gpu).train()
    opt = get_optimizer(args, model)
    st = TrainState(args, model, opt)
    q0, k0 = model.encoder_q.flat.detach().clone(), model.encoder_k.flat.detach().clone()
    ids = torch.randint(5, 200, (64, 16), device=gpu)
    mask = torch.ones_like(ids)
    for _ in range(2):  # sync_loss=False: the production loop's no-sync micro-batches
        _, stepped = st.micro_batch(
            32, lambda: model.forward_features(*model.bert_extract_ids(ids, mask, 32)),
            sync_loss=False)
        assert stepped
    torch.cuda.synchronize()
    assert int(model.encoder_q.coop_fault.item()) != 0
    assert float(st.grad_norm[2].item()) == 1.0  # gated
    assert torch.equal(model.encoder_q.flat.detach(), q0)
    assert torch.equal(model.encoder_k.flat.detach(), k0)
    assert torch.isfinite(opt.exp_avg).all() and not opt.exp_avg.any()
