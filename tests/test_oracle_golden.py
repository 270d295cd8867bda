"""Pin the CPU oracle against golden vectors produced by running the reference.

CPU-only (no GPU): these tests are what makes the oracle trustworthy as the
parity checker for the HIP kernels.
"""
import numpy as np
import pytest

from conftest import load_golden
from oracle import irc_oracle as O
from oracle import train_oracle


def test_nce_known_answers():
    g = load_golden("nce.npz")
    # SURVEY.md 8c known answers (reference run, torch.manual_seed(0), N=4 C=8 K=16)
    assert abs(float(g["n4_d8_k16_noq_loss"]) - 48.34416198730469) < 1e-9
    assert abs(float(g["n4_d8_k16_q_loss"]) - 64.79255676269531) < 1e-9


@pytest.mark.parametrize("tag", ["n4_d8_k16_noq", "n4_d8_k16_q", "n32_d128_k0_noq",
                                 "n32_d128_k512_noq", "n32_d128_k512_q", "n64_d128_k1024_q",
                                 "n64_d128_k1024_noq", "n8_d32_k64_q"])
def test_nce_loss_and_grad(tag):
    g = load_golden("nce.npz")
    queue = g.get(f"{tag}_queue")
    loss, dq = O.nce_info_loss(g[f"{tag}_q"], g[f"{tag}_k"], queue, 0.05)
    ref = float(g[f"{tag}_loss"])
    assert abs(loss - ref) <= 2e-6 * abs(ref) + 1e-5
    np.testing.assert_allclose(dq, g[f"{tag}_dq"], rtol=1e-4, atol=2e-5)


def _lstm_params(g, tag):
    pre = f"{tag}_param_"
    return {k[len(pre):]: np.asarray(v, np.float64) for k, v in g.items() if k.startswith(pre)}


@pytest.mark.parametrize("tag", ["a", "b"])
def test_seq2vec_and_head_grads(tag):
    g = load_golden("seq2vec.npz")
    B, L, inp, hid, layers, outd, kq = (int(x) for x in g[f"{tag}_dims"])
    p = _lstm_params(g, tag)
    a = np.asarray(g[f"{tag}_anchor"], np.float64)
    pos = np.asarray(g[f"{tag}_positive"], np.float64)
    y, _ = O.lstm_head_fwd(a, p, layers)
    np.testing.assert_allclose(y, g[f"{tag}_head_out"], rtol=1e-4, atol=1e-5)
    eq, cache = O.seq2vec(a, p, layers)
    ek, _ = O.seq2vec(pos, p, layers)  # encoder_k == encoder_q at init
    np.testing.assert_allclose(eq, g[f"{tag}_emb_q"], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(ek, g[f"{tag}_emb_k"], rtol=1e-4, atol=1e-5)
    loss, dq = O.nce_info_loss(eq, ek, g[f"{tag}_queue"], 0.05)
    assert abs(loss - float(g[f"{tag}_loss"])) < 1e-4
    grads = O.seq2vec_bwd(dq, p, cache, layers)
    for name, gv in grads.items():
        ref = g[f"{tag}_grad_{name}"]
        np.testing.assert_allclose(gv, ref, rtol=2e-3, atol=2e-5 * max(1.0, np.abs(ref).max()),
                                   err_msg=name)


def test_bert_forward():
    g = load_golden("bert_tiny.npz")
    w = {k[2:]: v for k, v in g.items() if k.startswith("w_")}
    vocab, hid, nl, nh, inter, maxpos = (int(x) for x in g["cfg"])
    out = O.bert_forward(g["input_ids"], g["attention_mask"], w, nl, nh)
    np.testing.assert_allclose(out, g["last_hidden_state"], rtol=1e-4, atol=1e-4)


def test_bert_long_matches_reference_at_512():
    """The reference's bert_extract / ctx2vec at the 512-token truncation
    (tests/golden/bert_long.npz): the oracle reproduces both, and the host tokenizer
    (irc_amd.tokenizer, bert-base-uncased's model_max_length) cuts the joint batch at
    the same 512 tokens."""
    g = load_golden("bert_long.npz")
    w = {k[2:]: v for k, v in g.items() if k.startswith("w_")}
    vocab, hid, nl, nh, inter, maxpos = (int(x) for x in g["cfg"])
    ids, mask = g["input_ids"], g["attention_mask"]
    assert ids.shape == (6, 512) and maxpos == 512
    out = O.bert_forward(ids, mask, w, nl, nh)
    np.testing.assert_allclose(out, np.concatenate([g["anchor_hs"], g["positive_hs"]]),
                               rtol=1e-4, atol=1e-4)
    hidden = O.bert_forward(g["ctx_input_ids"], g["ctx_attention_mask"], w, nl, nh)
    p = {k[2:]: v.astype(np.float64) for k, v in g.items() if k.startswith("h_")}
    emb, _ = O.seq2vec(hidden.astype(np.float64), p, int(g["head_dims"][2]))
    np.testing.assert_allclose(emb, g["ctx2vec"], rtol=1e-4, atol=1e-5)

    from irc_amd.tokenizer import load_tokenizer, synthetic_vocab_file

    tok = load_tokenizer(synthetic_vocab_file(vocab), vocab)
    t = tok(list(g["d1"]) + list(g["d2"]), padding=True, truncation=True, return_tensors="np")
    np.testing.assert_array_equal(t["input_ids"], ids)
    np.testing.assert_array_equal(t["attention_mask"], mask)


def test_bert_ref_matches_golden():
    """The torch fp32 BERT used as the trainable encoder's gradient reference
    (tests/bert_ref.py) reproduces the reference's own HF last_hidden_state."""
    import torch

    from bert_ref import bert_hidden

    g = load_golden("bert_tiny.npz")
    P = {k[2:]: torch.from_numpy(v).float() for k, v in g.items() if k.startswith("w_")}
    vocab, hid, nl, nh, inter, maxpos = (int(x) for x in g["cfg"])
    out = bert_hidden(P, torch.from_numpy(g["input_ids"]).long(),
                      torch.from_numpy(g["attention_mask"]).long(), nl, nh)
    np.testing.assert_allclose(out.numpy(), g["last_hidden_state"], rtol=1e-4, atol=1e-4)


def test_scan_grid_matches_reference_closest_docs():
    g = load_golden("scan.npz")
    q = g["grid_q"].astype(np.float32) / 128
    d = g["grid_d"].astype(np.float32) / 128
    k = int(g["grid_k"])
    idx, sc = O.scan_topk(q, d, k)
    np.testing.assert_array_equal(idx, g["grid_idx"])
    np.testing.assert_array_equal(sc, g["grid_score"])


def test_scan_ties_rule():
    g = load_golden("scan.npz")
    q = g["tie_q"].astype(np.float32) / 128
    d = g["tie_d"].astype(np.float32) / 128
    k = int(g["tie_k"])
    idx, sc = O.scan_topk(q, d, k, chunk=700)  # chunked merge must not change ties
    np.testing.assert_array_equal(sc, g["tie_score"])  # reference's score multiset/order
    full = O.scan_scores(q, d)
    for r in range(q.shape[0]):
        assert np.all(full[r, idx[r]] == sc[r])
        # tie rule: equal scores -> ascending index
        for j in range(k - 1):
            assert sc[r, j] > sc[r, j + 1] or idx[r, j] < idx[r, j + 1]
        # completeness at the boundary: no excluded doc beats the last one
        rest = np.setdiff1d(np.arange(d.shape[0]), idx[r])
        last_s, last_i = sc[r, -1], idx[r, -1]
        assert not np.any((full[r, rest] > last_s) | ((full[r, rest] == last_s) & (rest < last_i)))


def test_scan_edge_cases():
    rng = np.random.default_rng(0)
    q = rng.integers(-3, 4, (3, 128)).astype(np.float32) / 128
    d = rng.integers(-3, 4, (5, 128)).astype(np.float32) / 128
    idx, sc = O.scan_topk(q, d, 8, doc_offset=100)  # k > N: padded
    assert (idx[:, 5:] == -1).all() and np.isneginf(sc[:, 5:]).all()
    assert set(idx[0, :5]) == set(range(100, 105))
    idx0, _ = O.scan_topk(q, d[:0], 4)
    assert (idx0 == -1).all()


def test_merge_equals_global():
    rng = np.random.default_rng(1)
    q = rng.integers(-2, 3, (4, 128)).astype(np.float32) / 128
    d = rng.integers(-2, 3, (999, 128)).astype(np.float32) / 128
    full_i, full_s = O.scan_topk(q, d, 50)
    parts = [(0, 250), (250, 600), (600, 999)]
    li, ls = zip(*[O.scan_topk(q, d[a:b], 50, doc_offset=a) for a, b in parts])
    mi, ms = O.merge_topk(li, ls, 50)
    np.testing.assert_array_equal(mi, full_i)
    np.testing.assert_array_equal(ms, full_s)


@pytest.mark.parametrize("fixture", ["train_traj.npz", "train_traj_nomom.npz",
                                     "train_traj_sgd.npz"])
def test_train_trajectory_matches_reference(fixture):
    fx = load_golden(fixture)
    losses, final = train_oracle.run_trajectory(fx)
    np.testing.assert_allclose(losses, fx["mb_loss"], rtol=2e-5, atol=1e-4)
    for k, v in final.items():
        ref = fx["final_" + k]
        np.testing.assert_allclose(np.asarray(v).reshape(ref.shape), ref, rtol=1e-4, atol=2e-6,
                                   err_msg=k)


def test_enqueue_rule():
    queue = np.zeros((4, 12))
    q2, ptr = O.dequeue_and_enqueue(queue, 8, np.ones((4, 4)))
    assert ptr == 0 and (q2[:, 8:] == 1).all()
    q3, ptr = O.dequeue_and_enqueue(queue, 0, np.ones((5, 4)))  # 12 % 5 != 0: no update
    assert ptr == 0 and (q3 == 0).all()


def test_lstm_head_init_matches_reference_rng_order():
    """irc_amd.lstm_head.LSTMHead(config) after torch.manual_seed(s) starts from the
    exact parameters the reference's LSTM(config) gets (host-side init)."""
    import torch

    from irc_amd.lstm_head import LSTMHead

    g = load_golden("lstm_init.npz")
    for tag in ("s", "m"):
        inp, hid, layers, outd, seed = (int(x) for x in g[f"{tag}_dims"])
        cfg = {"model": {"LSTM": {"num_layers": layers, "bidirectional": True,
                                  "input_size": inp, "hidden_size": hid, "output_size": outd,
                                  "activation": "Identity"}}}
        torch.manual_seed(seed)
        h = LSTMHead(cfg)
        sd = h.state_dict()
        for name, _ in h.specs:
            np.testing.assert_array_equal(sd[name].numpy(), g[f"{tag}_{name}"], err_msg=name)


def test_e4m3_quantiser_matches_torch_cast():
    """The oracle's OCP e4m3fn RNE quantiser (fp8 corpus, config C5) agrees code for
    code with torch's float8_e4m3fn cast, an independent implementation of the spec
    (inputs clamped to +-448 as the build saturates)."""
    import torch

    rng = np.random.default_rng(0)
    mags = rng.choice(np.array([1e-3, 1e-2, 0.1, 1, 10, 100, 500], np.float32), 100_000)
    x = np.concatenate([
        rng.standard_normal(100_000).astype(np.float32) * mags,
        np.array([0.0, -0.0, 2**-10, 2**-9, 1.5 * 2**-9, 2.5 * 2**-9, 3 * 2**-10, 447, 448,
                  449, 460, 464, 465, 1e4, -1e4, 2**-6], np.float32)])
    codes = O.quantize_e4m3(x)
    ref = torch.from_numpy(np.clip(x, -448, 448)).to(torch.float8_e4m3fn).view(torch.uint8).numpy()
    np.testing.assert_array_equal(codes, ref)
    # decode table: max, min normal, min subnormal
    np.testing.assert_array_equal(O.dequantize_e4m3(np.array([0x7E, 0x08, 0x01], np.uint8)),
                                  np.array([448.0, 2**-6, 2**-9], np.float32))


@pytest.mark.parametrize("case", [0, 1])
def test_nce_c2_shapes_match_reference(case):
    """NCELoss at the C2 shapes (N=256, K=12544, D=128/768), inputs regenerated
    from tests/synth_inputs.py, against the reference's own values."""
    import synth_inputs as SI

    g = load_golden("nce_c2.npz")
    n, d, kq, seed = SI.NCE_C2_CASES[case]
    q, k, queue = SI.nce_c2_inputs(n, d, kq, seed)
    for with_q in (False, True):
        tag = f"n{n}_d{d}_k{kq}_{'q' if with_q else 'noq'}"
        np.testing.assert_array_equal(
            g[f"{tag}_in_sums"], [q.astype(np.float64).sum(), k.astype(np.float64).sum(),
                                  queue.astype(np.float64).sum()])  # inputs regenerate
        loss, dq = O.nce_info_loss(q, k, queue if with_q else None, 0.05)
        assert abs(loss - g[f"{tag}_loss"]) <= 1e-5 * abs(g[f"{tag}_loss"])
        np.testing.assert_allclose(dq[:16], g[f"{tag}_dq_head"], rtol=1e-4, atol=1e-6)
        np.testing.assert_allclose(dq[-16:], g[f"{tag}_dq_tail"], rtol=1e-4, atol=1e-6)
        np.testing.assert_allclose(np.linalg.norm(dq, axis=1), g[f"{tag}_dq_rownorm"], rtol=1e-5)
        np.testing.assert_allclose(dq.sum(axis=0), g[f"{tag}_dq_colsum"], rtol=1e-4, atol=1e-5)


def _bert_shapes(cfg):
    names = ["embeddings.word_embeddings.weight", "embeddings.position_embeddings.weight",
             "embeddings.token_type_embeddings.weight", "embeddings.LayerNorm.weight",
             "embeddings.LayerNorm.bias"]
    H, I = cfg["hidden_size"], cfg["intermediate_size"]
    shapes = {names[0]: (cfg["vocab_size"], H), names[1]: (cfg["max_position_embeddings"], H),
              names[2]: (2, H), names[3]: (H,), names[4]: (H,)}
    for l in range(cfg["num_hidden_layers"]):
        p = f"encoder.layer.{l}."
        for n, s in (("attention.self.query", (H, H)), ("attention.self.key", (H, H)),
                     ("attention.self.value", (H, H)), ("attention.output.dense", (H, H)),
                     ("intermediate.dense", (I, H)), ("output.dense", (H, I))):
            shapes[p + n + ".weight"], shapes[p + n + ".bias"] = s, (s[0],)
        for n in ("attention.output.LayerNorm", "output.LayerNorm"):
            shapes[p + n + ".weight"] = shapes[p + n + ".bias"] = (H,)
    return shapes


@pytest.mark.parametrize("size", ["base", "large"])
def test_bert_matches_reference(size):
    """The oracle's BERT against HF's last_hidden_state (the reference's frozen
    encoder): BERT-base (12 layers, H=768; padded B=4, L=64) and BERT-large
    (config C4: 24 layers, H=1024, A=16, I=4096; padded B=2, L=64)."""
    import synth_inputs as SI

    g = load_golden(f"bert_{size}.npz")
    cfg = SI.BERT_BASE if size == "base" else SI.BERT_LARGE
    w = {n: SI.bert_param(n, s) for n, s in _bert_shapes(cfg).items()}
    hs = O.bert_forward(g["input_ids"], g["attention_mask"], w, cfg["num_hidden_layers"],
                        cfg["num_attention_heads"])
    np.testing.assert_allclose(hs, g["last_hidden_state"], rtol=1e-4, atol=2e-4)


@pytest.mark.parametrize("case", [0, 1])
def test_nce_c34_global_batch_matches_reference(case):
    """NCELoss at the C3 / C4 global batches (N = 1024 / 2048, D = 128, K = 12544)
    against the reference's values, and the reference's enqueue rule at those B:
    12544 % B != 0, so the queue and its pointer stay untouched (the golden holds
    what the reference's own _dequeue_and_enqueue did)."""
    import synth_inputs as SI

    g = load_golden("nce_c34.npz")
    n, d, kq, seed = SI.NCE_C34_CASES[case]
    q, k, queue = SI.nce_c2_inputs(n, d, kq, seed)
    for with_q in (False, True):
        tag = f"n{n}_d{d}_k{kq}_{'q' if with_q else 'noq'}"
        loss, dq = O.nce_info_loss(q, k, queue if with_q else None, 0.05)
        assert abs(loss - g[f"{tag}_loss"]) <= 1e-5 * abs(g[f"{tag}_loss"])
        np.testing.assert_allclose(dq[:16], g[f"{tag}_dq_head"], rtol=1e-4, atol=1e-6)
        np.testing.assert_allclose(dq[-16:], g[f"{tag}_dq_tail"], rtol=1e-4, atol=1e-6)
        np.testing.assert_allclose(np.linalg.norm(dq, axis=1), g[f"{tag}_dq_rownorm"], rtol=1e-5)
        np.testing.assert_allclose(dq.sum(axis=0), g[f"{tag}_dq_colsum"], rtol=1e-4, atol=1e-5)
    for b in (n, 256):
        q2, ptr = O.dequeue_and_enqueue(queue, 0, k[:b])
        assert ptr == int(g[f"enq_b{b}_k{kq}_ptr"])
        assert int((q2 != queue).any(axis=0).sum()) == int(g[f"enq_b{b}_k{kq}_changed_cols"])
    assert int(g[f"enq_b{n}_k{kq}_ptr"]) == 0 and int(g[f"enq_b{n}_k{kq}_changed_cols"]) == 0


def test_torch_cpu_baseline_restatement_matches_reference():
    """The timed torch-CPU baseline (oracle/torch_cpu_step.py) computes the
    reference's numbers: BERT vs the HF golden, NCELoss vs the reference golden."""
    import torch

    from oracle import torch_cpu_step as T

    g = load_golden("bert_tiny.npz")
    w = {k[2:]: torch.from_numpy(v) for k, v in g.items() if k.startswith("w_")}
    hs = T.bert_forward(w, torch.from_numpy(g["input_ids"]), torch.from_numpy(g["attention_mask"]),
                        int(g["cfg"][2]), int(g["cfg"][3]))
    np.testing.assert_allclose(hs.numpy(), g["last_hidden_state"], rtol=1e-4, atol=1e-5)
    n = load_golden("nce.npz")
    tag = "n32_d128_k512_q"
    loss = T.nce_loss(torch.from_numpy(n[f"{tag}_q"]), torch.from_numpy(n[f"{tag}_k"]),
                      torch.from_numpy(n[f"{tag}_queue"]), 0.05)
    assert abs(loss.item() - float(n[f"{tag}_loss"])) <= 1e-5 * float(n[f"{tag}_loss"])


def test_activation_oracle_matches_torch():
    """oracle.act_fwd / act_grad (the head activation, model.py:25) against torch's
    modules and autograd, kinks included."""
    import torch

    u = np.concatenate([np.random.default_rng(0).standard_normal(2000) * 4,
                        [-25., -6., -3., -1., 0., 1., 3., 6., 19.9, 20.1, 25.]])
    for name in ["Identity", "ReLU", "ReLU6", "LeakyReLU", "ELU", "CELU", "SELU", "GELU", "SiLU",
                 "Mish", "Sigmoid", "Tanh", "Softplus", "Softsign", "Hardtanh", "Hardsigmoid",
                 "Hardswish", "Tanhshrink"]:
        ut = torch.tensor(u, requires_grad=True)
        y = getattr(torch.nn, name)()(ut)
        y.sum().backward()
        np.testing.assert_allclose(O.act_fwd(name, u), y.detach().numpy(), rtol=1e-12,
                                   atol=1e-12, err_msg=name)
        np.testing.assert_allclose(O.act_grad(name, u), ut.grad.numpy(), rtol=1e-7,
                                   atol=1e-12, err_msg=name)
