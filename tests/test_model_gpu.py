"""Encoder, BiLSTM head, seq2vec and InfoNCE on the HIP kernels vs the goldens
that running the reference produced (tests/golden/make_goldens.py).

fp32 parity mode (exact-fp32 MFMA) is held to fp32 tolerances; the bf16
production mode to bf16 tolerances (stated per test).
"""
import numpy as np
import pytest
import torch

from conftest import bf16_ulps, load_golden

pytestmark = pytest.mark.gpu


@pytest.fixture
def fp32_mode():
    from irc_amd.precision import get_precision, set_precision

    old = get_precision()
    set_precision("fp32")
    yield
    set_precision(old)


def _bert_from_golden(g, dev):
    from irc_amd.bert import BertConfig, BertModel

    vocab, hid, nl, nh, inter, maxpos = (int(x) for x in g["cfg"])
    m = BertModel(BertConfig(vocab_size=vocab, hidden_size=hid, num_hidden_layers=nl,
                             num_attention_heads=nh, intermediate_size=inter,
                             max_position_embeddings=maxpos))
    st = {k[2:]: torch.from_numpy(v) for k, v in g.items() if k.startswith("w_")}
    res = m.load_state_dict(st, strict=False)
    assert not [k for k in res.missing_keys if "position_ids" not in k]
    return m.to(dev)


def test_bert_tiny_fp32(gpu, fp32_mode):
    g = load_golden("bert_tiny.npz")
    m = _bert_from_golden(g, gpu)
    out = m.encode(torch.from_numpy(g["input_ids"]).to(gpu),
                   torch.from_numpy(g["attention_mask"]).to(gpu))
    np.testing.assert_allclose(out.float().cpu().numpy(), g["last_hidden_state"], rtol=1e-4,
                               atol=2e-4)


def test_bert_tiny_bf16(gpu):
    g = load_golden("bert_tiny.npz")
    m = _bert_from_golden(g, gpu)
    out = m.encode(torch.from_numpy(g["input_ids"]).to(gpu),
                   torch.from_numpy(g["attention_mask"]).to(gpu))
    # bf16 operands: LN outputs are O(1); tolerance 6e-2 absolute
    np.testing.assert_allclose(out.float().cpu().numpy(), g["last_hidden_state"], atol=6e-2)


@pytest.mark.parametrize("mode,atol", [("fp32", 3e-4), ("bf16", 8.0)])  # bf16: 4.79 ulps measured
def test_bert_long_512_matches_reference(gpu, mode, atol):
    """The reference's own bert_extract at the 512-token truncation
    (tests/golden/bert_long.npz, a 600-word sentence in the joint batch): L = 512
    runs the streamed MFMA attention (bf16) / the key-tiled kernel (fp32)."""
    from irc_amd.precision import get_precision, set_precision

    g = load_golden("bert_long.npz")
    old = get_precision()
    set_precision(mode)
    try:
        m = _bert_from_golden(g, gpu)
        out = m.encode(torch.from_numpy(g["input_ids"]).to(gpu),
                       torch.from_numpy(g["attention_mask"]).to(gpu))
    finally:
        set_precision(old)
    ref = np.concatenate([g["anchor_hs"], g["positive_hs"]])
    if mode == "fp32":
        np.testing.assert_allclose(out.float().cpu().numpy(), ref, atol=atol, rtol=1e-4)
    else:
        # bf16 hidden states (LayerNorm outputs, |x| up to ~7): within `atol` bf16 ulps of
        # the reference value, the ulp taken at max(|ref|, 1) (conftest.bf16_ulps)
        e = bf16_ulps(out.float().cpu().numpy(), ref, 1.0)
        print(f"bert_long bf16: {e:.2f} ulps")
        assert e <= atol, f"{e:.2f} bf16 ulps"


def test_ctx2vec_long_matches_reference(gpu):
    """The reference's ctx2vec at L = 502 (bert_long.npz): GPU WordPiece + joint
    padding token-exact against the reference tokenizer, then BERT -> BiLSTM head ->
    mean over all 502 positions (PAD included) -> L2 norm, bf16 (tolerance 2e-2 on
    unit vectors)."""
    from irc_amd.lstm_head import LSTMHead, seq2vec
    from irc_amd.tokenizer import load_tokenizer, synthetic_vocab_file
    from irc_amd.wordpiece import GpuWordPiece

    g = load_golden("bert_long.npz")
    vocab = int(g["cfg"][0])
    wp = GpuWordPiece(load_tokenizer(synthetic_vocab_file(vocab), vocab), gpu)
    ids, mask = wp(list(g["d2"]))
    assert torch.equal(ids.cpu(), torch.from_numpy(g["ctx_input_ids"]))
    assert torch.equal(mask.cpu(), torch.from_numpy(g["ctx_attention_mask"]))
    ids_j, mask_j = wp(list(g["d1"]) + list(g["d2"]))
    assert torch.equal(ids_j.cpu(), torch.from_numpy(g["input_ids"]))
    m = _bert_from_golden(g, gpu)
    inp, hid, layers, outd = (int(x) for x in g["head_dims"])
    h = LSTMHead({"model": {"LSTM": {"num_layers": layers, "bidirectional": True,
                                     "input_size": inp, "hidden_size": hid,
                                     "output_size": outd, "activation": "Identity"}}},
                 init=False)
    h.load_state_dict({k[2:]: torch.from_numpy(v) for k, v in g.items() if k.startswith("h_")})
    h = h.to(gpu)
    with torch.no_grad():
        emb = seq2vec(h, m.encode(ids, mask), grad=False)
    assert (emb.float().cpu() - torch.from_numpy(g["ctx2vec"])).abs().max().item() <= 2e-2


def _head_from_golden(g, tag, dev):
    from irc_amd.lstm_head import LSTMHead

    B, L, inp, hid, layers, outd, kq = (int(x) for x in g[f"{tag}_dims"])
    cfg = {"model": {"LSTM": {"num_layers": layers, "bidirectional": True, "input_size": inp,
                              "hidden_size": hid, "output_size": outd,
                              "activation": "Identity"}}}
    h = LSTMHead(cfg, init=False)
    pre = f"{tag}_param_"
    h.load_state_dict({k[len(pre):]: torch.from_numpy(v) for k, v in g.items()
                       if k.startswith(pre)})
    return h.to(dev), (B, L, inp, hid, layers, outd, kq)


@pytest.mark.parametrize("tag", ["a", "b"])
def test_head_forward_fp32(gpu, fp32_mode, tag):
    g = load_golden("seq2vec.npz")
    h, dims = _head_from_golden(g, tag, gpu)
    y = h(torch.from_numpy(g[f"{tag}_anchor"]).to(gpu))
    np.testing.assert_allclose(y.cpu().numpy(), g[f"{tag}_head_out"], rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("tag", ["a", "b"])
def test_seq2vec_loss_and_grads_fp32(gpu, fp32_mode, tag):
    from irc_amd.lstm_head import seq2vec
    from irc_amd.nce import info_nce

    g = load_golden("seq2vec.npz")
    h, dims = _head_from_golden(g, tag, gpu)
    a = torch.from_numpy(g[f"{tag}_anchor"]).to(gpu)
    p = torch.from_numpy(g[f"{tag}_positive"]).to(gpu)
    queue = torch.from_numpy(g[f"{tag}_queue"]).to(gpu)
    eq = seq2vec(h, a, grad=True)
    ek = seq2vec(h, p, grad=False)
    np.testing.assert_allclose(eq.detach().cpu().numpy(), g[f"{tag}_emb_q"], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(ek.cpu().numpy(), g[f"{tag}_emb_k"], rtol=1e-4, atol=1e-5)
    loss = info_nce(eq, ek, queue, 0.05)
    assert abs(loss.item() - float(g[f"{tag}_loss"])) <= 1e-4 * abs(float(g[f"{tag}_loss"]))
    h.flat_grad.zero_()
    loss.backward()
    for name, _ in h.specs:
        ref = g[f"{tag}_grad_{name}"]
        got = h.view(name, h.flat_grad).cpu().numpy()
        np.testing.assert_allclose(got, ref, rtol=2e-3, atol=2e-5 * max(1.0, np.abs(ref).max()),
                                   err_msg=name)


@pytest.mark.parametrize("tag", ["n4_d8_k16_noq", "n4_d8_k16_q", "n32_d128_k0_noq",
                                 "n32_d128_k512_q", "n64_d128_k1024_q", "n8_d32_k64_q"])
def test_infonce_loss_and_dq(gpu, tag):
    from irc_amd.nce import info_nce

    g = load_golden("nce.npz")
    q = torch.from_numpy(g[f"{tag}_q"]).to(gpu).requires_grad_(True)
    k = torch.from_numpy(g[f"{tag}_k"]).to(gpu)
    queue = torch.from_numpy(g[f"{tag}_queue"]).to(gpu) if f"{tag}_queue" in g else None
    loss = info_nce(q, k, queue, 0.05)
    ref = float(g[f"{tag}_loss"])
    # north-star tolerance: 1e-3 (bf16); fp32 MFMA logits land within 1e-5 relative
    assert abs(loss.item() - ref) <= 1e-5 * abs(ref) + 1e-5
    (loss * 0.25).backward()
    np.testing.assert_allclose(q.grad.cpu().numpy(), 0.25 * g[f"{tag}_dq"], rtol=1e-4, atol=1e-6)


def test_optimizer_ops_vs_oracle(gpu):
    from irc_amd import ops
    from oracle import irc_oracle as O

    rng = np.random.default_rng(0)
    n = 10_001
    p = rng.standard_normal(n).astype(np.float32)
    gr = rng.standard_normal(n).astype(np.float32) * 3
    pt, gt = torch.from_numpy(p).to(gpu), torch.from_numpy(gr).to(gpu)
    m, v = torch.zeros_like(pt), torch.zeros_like(pt)
    coef = ops.grad_norm_clip(gt, 1.0)
    grads = {"g": gr.astype(np.float64)}
    tot = O.clip_grad_norm(grads, 1.0)
    assert abs(coef[0].item() - tot) <= 1e-5 * tot
    ops.adam_step(pt, gt, m, v, coef, 0.9, 0.999, 2.5e-4 / (1 - 0.9), (1 - 0.999) ** 0.5, 1e-8)
    rp, _, _ = O.adam_step(p.astype(np.float64), grads["g"], 0, 0, 1, 2.5e-4, 0.9, 0.999)
    np.testing.assert_allclose(pt.cpu().numpy(), rp, rtol=1e-6, atol=1e-7)
    pk = torch.from_numpy(rng.standard_normal(n).astype(np.float32)).to(gpu)
    ref = O.momentum_update(pk.cpu().numpy(), p, 0.9)
    ops.momentum_update(pk, torch.from_numpy(p).to(gpu), 0.9)
    np.testing.assert_allclose(pk.cpu().numpy(), ref, rtol=1e-6, atol=1e-6)


def test_enqueue_device_pointer(gpu):
    from irc_amd import ops
    from oracle import irc_oracle as O

    D, K, B = 8, 32, 8
    q0 = np.zeros((D, K), np.float32)
    queue = torch.zeros(D, K, device=gpu)
    ptr = torch.zeros(1, dtype=torch.int64, device=gpu)
    ref, rptr = q0, 0
    for i in range(5):
        keys = np.full((B, D), i + 1, np.float32)
        keys[:, 0] = np.arange(B)
        ops.enqueue(queue, torch.from_numpy(keys).to(gpu), ptr)
        ref, rptr = O.dequeue_and_enqueue(ref, rptr, keys)
    np.testing.assert_array_equal(queue.cpu().numpy(), ref)
    assert int(ptr.item()) == rptr
