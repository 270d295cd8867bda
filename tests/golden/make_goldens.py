"""Generate the committed golden fixtures by RUNNING the reference.

Runs only in the build container (it needs /root/reference, which never travels
to the GPU box).  It imports the reference modules from their read-only location
-- nothing of the reference is copied into this repository; only the numeric
inputs/outputs are saved as small .npz fixtures next to this script.

  python tests/golden/make_goldens.py

Offline substitutions (the reference fetches bert-base-uncased by name,
contrastive_module.py:32-33, which cannot work without network):
  * BertModel.from_pretrained   -> BertModel(BertConfig(tiny)) after manual_seed(0)
  * BertTokenizer.from_pretrained -> BertTokenizer(<synthetic local vocab.txt>)
  * faiss / fastcluster / pexpect / torch.utils.tensorboard -> empty stand-in
    modules (never called on the InfoNCE path; needed only for imports).
"""
from __future__ import annotations

import argparse
import os
import pickle
import random
import sys
import tempfile
import types

import numpy as np
import torch

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))


def _stub_modules():
    for name in ("faiss", "fastcluster", "pexpect"):
        if name not in sys.modules:
            sys.modules[name] = types.ModuleType(name)
    tb = types.ModuleType("torch.utils.tensorboard")

    class SummaryWriter:  # minimal stand-in: records scalars
        def __init__(self, *a, **k):
            self.scalars = []

        def add_scalar(self, tag, val, step):
            self.scalars.append((tag, float(val), int(step)))

        def close(self):
            pass

    tb.SummaryWriter = SummaryWriter
    sys.modules["torch.utils.tensorboard"] = tb


def _import_ref():
    if not os.path.isdir(REF):
        raise SystemExit("reference not present; fixtures are already committed")
    if REF not in sys.path:
        sys.path.insert(0, REF)
    _stub_modules()


TINY_BERT = dict(vocab_size=200, hidden_size=32, num_hidden_layers=2, num_attention_heads=2,
                 intermediate_size=64, max_position_embeddings=64)


def _write_vocab(path, vocab_size):
    toks = ["[PAD]", "[UNK]", "[CLS]", "[SEP]", "[MASK]"]
    toks += [f"w{i}" for i in range(vocab_size - len(toks))]
    with open(path, "w") as f:
        f.write("\n".join(toks) + "\n")


def _install_bert_shims(vocab_path, bert_kw, tok_kw=None):
    from transformers import BertConfig, BertModel, BertTokenizer
    import src.contrastor.contrastive_module as cm
    tok_kw = tok_kw or {}

    class _Model:
        @staticmethod
        def from_pretrained(name, *a, **k):
            torch.manual_seed(0)
            return BertModel(BertConfig(**bert_kw))

    class _Tok:
        @staticmethod
        def from_pretrained(name, *a, **k):
            return BertTokenizer(vocab_path, **tok_kw)

    cm.BertModel = _Model
    cm.BertTokenizer = _Tok


def _np(t):
    return t.detach().cpu().numpy()


# ---------------------------------------------------------------------------
def gen_nce(out):
    """NCELoss._compute_info_loss values + autograd dL/dq (contrastive_loss.py:56-93)."""
    from src.contrastor.contrastive_loss import NCELoss

    cases = [(4, 8, 16, 0), (32, 128, 0, 1), (32, 128, 512, 2), (64, 128, 1024, 3),
             (8, 32, 64, 4)]
    res = {}
    for (n, d, kq, seed) in cases:
        torch.manual_seed(seed)
        q = torch.nn.functional.normalize(torch.randn(n, d))
        k = torch.nn.functional.normalize(torch.randn(n, d))
        queue = torch.nn.functional.normalize(torch.randn(d, max(kq, 1)), dim=0)
        crit = NCELoss({"temperature": 0.05})
        for with_q in (False, True):
            if with_q and kq == 0:
                continue
            qq = q.clone().requires_grad_(True)
            loss = crit(qq, k, queue if with_q else None)
            loss.backward()
            tag = f"n{n}_d{d}_k{kq}_{'q' if with_q else 'noq'}"
            res[f"{tag}_q"] = _np(q)
            res[f"{tag}_k"] = _np(k)
            if with_q:
                res[f"{tag}_queue"] = _np(queue)
            res[f"{tag}_loss"] = np.float64(loss.item())
            res[f"{tag}_dq"] = _np(qq.grad)
    np.savez_compressed(os.path.join(out, "nce.npz"), **res)
    print("nce:", len(res), "arrays; known answers",
          res["n4_d8_k16_noq_loss"], res["n4_d8_k16_q_loss"])


def gen_nce_c2(out):
    """NCELoss at the C2 shapes (N = 256, K = 12544, D = 128 and
    768), with and without the queue.  Inputs are regenerated from numpy streams
    (tests/synth_inputs.py); the fixture holds the loss, dL/dq's first / last 16
    rows, every row norm and every column sum of dL/dq."""
    sys.path.insert(0, os.path.dirname(HERE))
    import synth_inputs as SI
    from src.contrastor.contrastive_loss import NCELoss

    res = {}
    for (n, d, kq, seed) in SI.NCE_C2_CASES:
        q, k, queue = SI.nce_c2_inputs(n, d, kq, seed)
        crit = NCELoss({"temperature": 0.05})
        for with_q in (False, True):
            qq = torch.from_numpy(q).clone().requires_grad_(True)
            loss = crit(qq, torch.from_numpy(k), torch.from_numpy(queue) if with_q else None)
            loss.backward()
            dq = _np(qq.grad)
            tag = f"n{n}_d{d}_k{kq}_{'q' if with_q else 'noq'}"
            res[f"{tag}_loss"] = np.float64(loss.item())
            res[f"{tag}_dq_head"] = dq[:16]
            res[f"{tag}_dq_tail"] = dq[-16:]
            res[f"{tag}_dq_rownorm"] = np.linalg.norm(dq.astype(np.float64), axis=1)
            res[f"{tag}_dq_colsum"] = dq.astype(np.float64).sum(axis=0)
            res[f"{tag}_in_sums"] = np.array([q.astype(np.float64).sum(),
                                              k.astype(np.float64).sum(),
                                              queue.astype(np.float64).sum()])
    np.savez_compressed(os.path.join(out, "nce_c2.npz"), **res)
    print("nce_c2:", {k: v for k, v in res.items() if k.endswith("_loss")})


def gen_nce_c34(out):
    """NCELoss at the C3 / C4 global batches (N = 1024 and 2048, D = 128,
    K = 12544), with and without the queue: the same fixture layout as nce_c2.
    Plus the reference's enqueue rule at these batch sizes: 12544 % B != 0, so
    _dequeue_and_enqueue (contrastive_module.py:55-68) leaves queue and queue_ptr
    untouched -- recorded from the reference method itself."""
    import types as _types

    sys.path.insert(0, os.path.dirname(HERE))
    import synth_inputs as SI
    from src.contrastor.contrastive_loss import NCELoss
    from src.contrastor.contrastive_module import RetrievalModelWrapper

    res = {}
    for (n, d, kq, seed) in SI.NCE_C34_CASES:
        q, k, queue = SI.nce_c2_inputs(n, d, kq, seed)
        crit = NCELoss({"temperature": 0.05})
        for with_q in (False, True):
            qq = torch.from_numpy(q).clone().requires_grad_(True)
            loss = crit(qq, torch.from_numpy(k), torch.from_numpy(queue) if with_q else None)
            loss.backward()
            dq = _np(qq.grad)
            tag = f"n{n}_d{d}_k{kq}_{'q' if with_q else 'noq'}"
            res[f"{tag}_loss"] = np.float64(loss.item())
            res[f"{tag}_dq_head"] = dq[:16]
            res[f"{tag}_dq_tail"] = dq[-16:]
            res[f"{tag}_dq_rownorm"] = np.linalg.norm(dq.astype(np.float64), axis=1)
            res[f"{tag}_dq_colsum"] = dq.astype(np.float64).sum(axis=0)
        # the reference's enqueue at B = n (and at B = 256 for contrast)
        for b in (n, 256):
            me = _types.SimpleNamespace(
                queue=torch.from_numpy(queue.copy()), queue_ptr=torch.zeros(1, dtype=torch.long),
                loss_config={"queue_size": kq})
            RetrievalModelWrapper._dequeue_and_enqueue(me, torch.from_numpy(k[:b]))
            res[f"enq_b{b}_k{kq}_ptr"] = np.int64(int(me.queue_ptr[0]))
            res[f"enq_b{b}_k{kq}_changed_cols"] = np.int64(
                int((me.queue.numpy() != queue).any(axis=0).sum()))
    np.savez_compressed(os.path.join(out, "nce_c34.npz"), **res)
    print("nce_c34:", {k: v for k, v in res.items() if k.endswith("_loss") or "enq" in k})


def gen_bert_large(out):
    """HF BertModel at BERT-large size (24 layers, H = 1024, A = 16, I = 4096),
    the frozen encoder of config C4, B = 2, L = 64 with padding; weights from the
    same per-parameter numpy streams as gen_bert_base."""
    sys.path.insert(0, os.path.dirname(HERE))
    import synth_inputs as SI
    from transformers import BertConfig, BertModel

    m = BertModel(BertConfig(**SI.BERT_LARGE)).eval()
    sd = {n: torch.from_numpy(SI.bert_param(n, tuple(v.shape)))
          for n, v in m.state_dict().items() if "position_ids" not in n}
    missing = m.load_state_dict(sd, strict=False).missing_keys
    assert not [n for n in missing if "position_ids" not in n], missing
    ids, mask = SI.bert_base_batch(seed=8, lens=SI.BERT_LARGE_LENS)
    with torch.no_grad():
        hs = m(input_ids=torch.from_numpy(ids), attention_mask=torch.from_numpy(mask))
    hs = _np(hs.last_hidden_state)
    pooled = hs.astype(np.float64).mean(axis=1)
    np.savez_compressed(os.path.join(out, "bert_large.npz"), input_ids=ids, attention_mask=mask,
                        last_hidden_state=hs,
                        seq2vec=(pooled / np.linalg.norm(pooled, axis=1, keepdims=True)))
    print("bert_large:", hs.shape, float(np.abs(hs).mean()))


def gen_bert_base(out):
    """HF BertModel at BERT-base size (12 layers, H = 768, A = 12, I = 3072) with
    padding, B = 4, L = 64 -- the frozen encoder of config C2 as the reference
    calls it (contrastive_module.py:36-41).  Weights from per-parameter numpy
    streams (tests/synth_inputs.py), so only the output is committed."""
    sys.path.insert(0, os.path.dirname(HERE))
    import synth_inputs as SI
    from transformers import BertConfig, BertModel

    m = BertModel(BertConfig(**SI.BERT_BASE)).eval()
    sd = {n: torch.from_numpy(SI.bert_param(n, tuple(v.shape)))
          for n, v in m.state_dict().items() if "position_ids" not in n}
    missing = m.load_state_dict(sd, strict=False).missing_keys
    assert not [n for n in missing if "position_ids" not in n], missing
    ids, mask = SI.bert_base_batch()
    with torch.no_grad():
        hs = m(input_ids=torch.from_numpy(ids), attention_mask=torch.from_numpy(mask))
    hs = _np(hs.last_hidden_state)
    pooled = hs.astype(np.float64).mean(axis=1)
    np.savez_compressed(os.path.join(out, "bert_base.npz"), input_ids=ids, attention_mask=mask,
                        last_hidden_state=hs,
                        seq2vec=(pooled / np.linalg.norm(pooled, axis=1, keepdims=True)))
    print("bert_base:", hs.shape, float(np.abs(hs).mean()))


def _lstm_cfg(inp, hid, layers, outd):
    return {"model": {"LSTM": {"num_layers": layers, "bidirectional": True, "input_size": inp,
                               "hidden_size": hid, "output_size": outd,
                               "activation": "Identity"}}}


def gen_seq2vec(out, tmp):
    """LSTM head + seq2vec + loss backward through encoder_q (model.py:7-41,
    contrastive_module.py:102-112)."""
    from src.model import LSTM
    from src.contrastor.contrastive_module import RetrievalModelWrapper
    from src.contrastor.contrastive_loss import NCELoss

    vocab = os.path.join(tmp, "vocab.txt")
    _write_vocab(vocab, TINY_BERT["vocab_size"])
    _install_bert_shims(vocab, TINY_BERT)
    res = {}
    for tag, (B, L, inp, hid, layers, outd, kq, seed) in {
        "a": (4, 7, 24, 16, 3, 12, 8, 11),
        "b": (6, 5, 32, 8, 2, 8, 12, 12),
    }.items():
        torch.manual_seed(seed)
        cfg = _lstm_cfg(inp, hid, layers, outd)
        enc = LSTM(cfg)
        lc = {"temperature": 0.05, "use_momentum": True, "momentum": 0.9, "use_queue": True,
              "queue_size": kq, "dim": outd}
        model = RetrievalModelWrapper(enc, NCELoss(lc), lc)
        a = torch.randn(B, L, inp)
        p = torch.randn(B, L, inp)
        emb_q = model.seq2vec(a)
        emb_k = model.seq2vec(p, query=False)
        loss = model.criterion(emb_q, emb_k, model.queue)
        loss.backward()
        res[f"{tag}_anchor"] = _np(a)
        res[f"{tag}_positive"] = _np(p)
        res[f"{tag}_queue"] = _np(model.queue)
        res[f"{tag}_emb_q"] = _np(emb_q)
        res[f"{tag}_emb_k"] = _np(emb_k)
        res[f"{tag}_loss"] = np.float64(loss.item())
        res[f"{tag}_head_out"] = _np(model.encoder_q(features=a))
        res[f"{tag}_dims"] = np.array([B, L, inp, hid, layers, outd, kq])
        for name, prm in model.encoder_q.named_parameters():
            res[f"{tag}_param_{name}"] = _np(prm)
            res[f"{tag}_grad_{name}"] = _np(prm.grad)
    np.savez_compressed(os.path.join(out, "seq2vec.npz"), **res)
    print("seq2vec:", len(res), "arrays")


def gen_lstm_init(out):
    """Initial parameters of the reference LSTM head for fixed seeds (model.py:8-36):
    pins the RNG-consumption order of nn.LSTM + Linear + init_weights."""
    from src.model import LSTM

    res = {}
    for tag, (inp, hid, layers, outd, seed) in {"s": (24, 16, 2, 8, 1337),
                                                 "m": (64, 32, 3, 16, 7)}.items():
        torch.manual_seed(seed)
        m = LSTM(_lstm_cfg(inp, hid, layers, outd))
        res[f"{tag}_dims"] = np.array([inp, hid, layers, outd, seed])
        for name, prm in m.named_parameters():
            res[f"{tag}_{name}"] = _np(prm)
    np.savez_compressed(os.path.join(out, "lstm_init.npz"), **res)
    print("lstm init:", len(res), "arrays")


def gen_bert(out, tmp):
    """HF BertModel last_hidden_state with padding (contrastive_module.py:36-41)."""
    from transformers import BertConfig, BertModel

    torch.manual_seed(0)
    m = BertModel(BertConfig(**TINY_BERT)).eval()
    g = torch.Generator().manual_seed(7)
    B, L = 5, 13
    ids = torch.randint(5, TINY_BERT["vocab_size"], (B, L), generator=g)
    lens = torch.tensor([13, 9, 4, 13, 2])
    mask = (torch.arange(L)[None] < lens[:, None]).long()
    ids[:, 0] = 2
    ids = torch.where(mask.bool(), ids, torch.zeros_like(ids))
    for b in range(B):
        ids[b, lens[b] - 1] = 3
    with torch.no_grad():
        hs = m(input_ids=ids, attention_mask=mask).last_hidden_state
    res = {"input_ids": _np(ids), "attention_mask": _np(mask), "last_hidden_state": _np(hs)}
    for kname, v in m.state_dict().items():
        res["w_" + kname] = _np(v)
    res["cfg"] = np.array([TINY_BERT[k] for k in ("vocab_size", "hidden_size",
                                                  "num_hidden_layers", "num_attention_heads",
                                                  "intermediate_size",
                                                  "max_position_embeddings")])
    np.savez_compressed(os.path.join(out, "bert_tiny.npz"), **res)
    print("bert:", hs.shape)


LONG_BERT = dict(vocab_size=300, hidden_size=128, num_hidden_layers=2, num_attention_heads=2,
                 intermediate_size=256, max_position_embeddings=512)


def gen_bert_long(out, tmp):
    """The reference's own bert_extract and ctx2vec (contrastive_module.py:36-41,
    96-112) on sentences long enough that the joint padding reaches the 512-token
    truncation: d1 + d2 holds a 600-word sentence, so the batch is cut to L = 512;
    ctx2vec(d2) pads to its longest, 500 words + [CLS] / [SEP] = 502.  The tokenizer
    carries bert-base-uncased's model_max_length (512), which `truncation=True` reads.
    Local 2-layer config with head dim 64 (the MFMA attention path) and
    max_position_embeddings = 512; a 2-layer BiLSTM head 128 -> 16 -> 8."""
    from src.model import LSTM
    from src.contrastor.contrastive_module import RetrievalModelWrapper
    from src.contrastor.contrastive_loss import NCELoss

    vocab = os.path.join(tmp, "vocab_long.txt")
    _write_vocab(vocab, LONG_BERT["vocab_size"])
    _install_bert_shims(vocab, LONG_BERT, {"model_max_length": 512})
    torch.manual_seed(3)
    enc = LSTM(_lstm_cfg(128, 16, 2, 8))
    lc = {"temperature": 0.05, "use_momentum": True, "momentum": 0.9, "use_queue": True,
          "queue_size": 12, "dim": 8}
    model = RetrievalModelWrapper(enc, NCELoss(lc), lc)
    rng = np.random.default_rng(512)

    def sent(n):
        return " ".join(f"w{i}" for i in rng.integers(0, LONG_BERT["vocab_size"] - 5, n))

    d1 = [sent(600), sent(3), sent(40)]
    d2 = [sent(250), sent(500), sent(1)]
    t = model.bert_tokenizer(d1 + d2, padding=True, truncation=True, return_tensors="pt")
    a, p = model.bert_extract(d1, d2, "cpu")
    with torch.no_grad():
        c2v = model.ctx2vec(d2, "cpu")
    tc = model.bert_tokenizer(d2, padding=True, truncation=True, return_tensors="pt")
    res = {"d1": np.array(d1), "d2": np.array(d2), "input_ids": _np(t["input_ids"]),
           "attention_mask": _np(t["attention_mask"]), "anchor_hs": _np(a), "positive_hs": _np(p),
           "ctx_input_ids": _np(tc["input_ids"]), "ctx_attention_mask": _np(tc["attention_mask"]),
           "ctx2vec": _np(c2v),
           "cfg": np.array([LONG_BERT[k] for k in ("vocab_size", "hidden_size",
                                                   "num_hidden_layers", "num_attention_heads",
                                                   "intermediate_size",
                                                   "max_position_embeddings")]),
           "head_dims": np.array([128, 16, 2, 8])}
    for kname, v in model.bert_model.state_dict().items():
        res["w_" + kname] = _np(v)
    for kname, v in model.encoder_q.state_dict().items():
        res["h_" + kname] = _np(v)
    np.savez_compressed(os.path.join(out, "bert_long.npz"), **res)
    print("bert_long:", tuple(t["input_ids"].shape), tuple(tc["input_ids"].shape))


def _ref_ranker(docs_f64):
    """The reference's TfidfDocRanker.closest_docs ranking over a dense corpus.

    The ranker object is created without its file-loading __init__; doc_mat is
    the [D x N] corpus as a scipy sparse matrix so ``spvec * self.doc_mat`` is
    the plain dot product (tfidf_doc_ranker.py:60-75)."""
    import scipy.sparse as sp
    from preprocessing.drqa.retriever.tfidf_doc_ranker import TfidfDocRanker

    r = object.__new__(TfidfDocRanker)
    r.doc_mat = sp.csr_matrix(docs_f64.T)
    r.doc_dict = (None, list(range(docs_f64.shape[0])))
    return r


def gen_scan(out):
    """Integer-grid scan fixtures; ordering from the reference's closest_docs."""
    import scipy.sparse as sp

    res = {}
    rng = np.random.default_rng(2024)
    # (a) tie-free integer grid: expected order straight from closest_docs.
    Q, N, D, k = 8, 2000, 128, 100
    while True:
        qm = rng.integers(-127, 128, size=(Q, D))
        dm = rng.integers(-127, 128, size=(N, D))
        s = (qm @ dm.T)
        top = -np.sort(-s, axis=1)[:, : k + 1]
        ok = all(len(np.unique(row)) == k + 1 for row in top)
        if ok:
            break
    qv = qm / 128.0
    dv = dm / 128.0
    ranker = _ref_ranker(dv)
    ids = np.zeros((Q, k), np.int64)
    scs = np.zeros((Q, k), np.float64)
    for i in range(Q):
        ranker.text2spvec = (lambda vec: (lambda _q: sp.csr_matrix(vec[None])))(qv[i])
        di, ds = ranker.closest_docs(None, k=k)
        ids[i], scs[i] = di, ds
    res.update(grid_q=qm.astype(np.int8), grid_d=dm.astype(np.int8), grid_k=np.int64(k),
               grid_idx=ids, grid_score=scs.astype(np.float32))
    # (b) heavy ties: values in {-1,0,1}/128.  closest_docs returns the right
    # multiset of scores; the order among equal scores is the build's rule
    # (lower index first), so only the score list is taken from the reference.
    Q, N, D, k = 6, 3000, 128, 64
    qm = rng.integers(-1, 2, size=(Q, D))
    dm = rng.integers(-1, 2, size=(N, D))
    dv = dm / 128.0
    ranker = _ref_ranker(dv)
    scs = np.zeros((Q, k), np.float64)
    for i in range(Q):
        ranker.text2spvec = (lambda vec: (lambda _q: sp.csr_matrix(vec[None])))(qm[i] / 128.0)
        _, ds = ranker.closest_docs(None, k=k)
        scs[i] = ds
    res.update(tie_q=qm.astype(np.int8), tie_d=dm.astype(np.int8), tie_k=np.int64(k),
               tie_score=scs.astype(np.float32))
    np.savez_compressed(os.path.join(out, "scan.npz"), **res)
    print("scan: grid + tie fixtures")


# ---------------------------------------------------------------------------
def gen_train_traj_nomom(out, tmp):
    """The same run with loss.use_momentum False: keys come from encoder_q with
    autograd (contrastive_module.py:82-83), no encoder_k, no momentum update."""
    gen_train_traj(out, tmp, use_momentum=False, fname="train_traj_nomom.npz")


def gen_train_traj_sgd(out, tmp):
    """The same run with --opt sgd (torch.optim.SGD with momentum and weight decay,
    model.py:45-51) over two passes of the data, so the per-pass cosine
    adjust_learning_rate (train.py:18-23, 90-91) changes the rate, and a Tanh head
    activation (model.py:25, eval(f"nn.{act}()"))."""
    gen_train_traj(out, tmp, fname="train_traj_sgd.npz", opt="sgd", act="Tanh", total_steps=6)


def gen_train_traj(out, tmp, use_momentum=True, fname="train_traj.npz", opt="adam",
                   act="Identity", total_steps=4):
    """Run the reference train() loop on a tiny config; record the trajectory."""
    import yaml
    import src.contrastor.contrastive_module as cm
    import src.train as rtrain
    from src.train import train

    vocab = os.path.join(tmp, "vocab.txt")
    _write_vocab(vocab, TINY_BERT["vocab_size"])
    _install_bert_shims(vocab, TINY_BERT)

    # synthetic docs_sentence.pkl: list of docs, each a list of 3-8 sentences
    rs = np.random.RandomState(99)
    docs = []
    for _ in range(64):
        nsent = rs.randint(3, 9)
        docs.append([" ".join(f"w{rs.randint(0, 150)}" for _ in range(rs.randint(3, 12)))
                     for _ in range(nsent)])
    dpath = os.path.join(tmp, "docs_sentence.pkl")
    with open(dpath, "wb") as f:
        pickle.dump(docs, f)

    with open(os.path.join(REF, "config.yaml")) as f:
        cfg = yaml.load(f, Loader=yaml.FullLoader)
    cfg["model"]["LSTM"].update(input_size=TINY_BERT["hidden_size"], hidden_size=16,
                                num_layers=2, output_size=8, activation=act)
    cfg["loss"]["InfoNCE"].update(queue_size=32, queue_start_steps=2, use_momentum=use_momentum)
    cfg["train"].update(batch_size=8, acml_batch_size=16, total_steps=total_steps, log_step=2,
                        n_jobs=0)
    cfg["dataset"]["docs_sentence"] = dpath
    if opt == "sgd":  # a rate large enough to move the tiny head visibly
        cfg["optimizer"]["SGD"].update(learning_rate="0.05", momentum=0.9, weight_decay="1e-2")

    args = argparse.Namespace(config=cfg, log=False, logdir=os.path.join(tmp, "log"), data="doc",
                              ckptdir=os.path.join(tmp, "ckpt"), seed=1337, gpu="-1", ckpt=None,
                              model="LSTM", loss="InfoNCE", opt=opt, sample="uniform")
    args.device = torch.device("cpu")
    torch.manual_seed(1337)
    np.random.seed(1337)
    random.seed(1337)

    rec = {"ids": [], "mask": [], "loss": [], "B": []}
    init_state = {}
    orig_extract = cm.RetrievalModelWrapper.bert_extract
    orig_forward = cm.RetrievalModelWrapper.forward

    def bert_extract(self, d1, d2, device):
        t = self.bert_tokenizer(d1 + d2, padding=True, truncation=True, return_tensors="pt")
        rec["ids"].append(_np(t["input_ids"]))
        rec["mask"].append(_np(t["attention_mask"]))
        rec["B"].append(len(d1))
        if not init_state:
            for kname, v in self.state_dict().items():
                init_state[kname] = _np(v).copy()
            init_state["__add_queue__"] = np.int64(self.add_queue_to_loss)
        return orig_extract(self, d1, d2, device)

    def forward(self, *a, **k):
        loss = orig_forward(self, *a, **k)
        rec["loss"].append(float(loss.item()))
        rec.setdefault("addq", []).append(int(self.add_queue_to_loss))
        return loss

    orig_adjust = rtrain.adjust_learning_rate

    def adjust(optimizer, steps, config):  # records where each pass starts
        rec.setdefault("epoch_mb", []).append((len(rec["loss"]), int(steps)))
        return orig_adjust(optimizer, steps, config)

    cm.RetrievalModelWrapper.bert_extract = bert_extract
    cm.RetrievalModelWrapper.forward = forward
    rtrain.adjust_learning_rate = adjust
    try:
        train(args)
    finally:
        cm.RetrievalModelWrapper.bert_extract = orig_extract
        cm.RetrievalModelWrapper.forward = orig_forward
        rtrain.adjust_learning_rate = orig_adjust

    ck_path = os.path.join(args.ckptdir, f"uniform_InfoNCE_LSTM_{total_steps}.pth")
    if use_momentum and opt == "adam":  # the reference-written checkpoint: load_model fixture
        import shutil

        shutil.copyfile(ck_path, os.path.join(out, "ref_ckpt_InfoNCE_LSTM_4.pth"))
    ck = torch.load(ck_path, map_location="cpu",
                    weights_only=False)  # our own freshly written file
    final = ck["Model"]
    res = {}
    for kname, v in init_state.items():
        res["init_" + kname] = v
    for kname, v in final.items():
        res["final_" + kname] = _np(v)
    Lmax = max(x.shape[1] for x in rec["ids"])
    nmb = len(rec["ids"])
    ids = np.zeros((nmb, 16, Lmax), np.int64)
    mask = np.zeros((nmb, 16, Lmax), np.int64)
    lens = np.zeros((nmb,), np.int64)
    for i in range(nmb):
        r, c = rec["ids"][i].shape
        ids[i, :r, :c] = rec["ids"][i]
        mask[i, :r, :c] = rec["mask"][i]
        lens[i] = c
    res.update(mb_ids=ids, mb_mask=mask, mb_len=lens, mb_B=np.array(rec["B"]),
               mb_loss=np.array(rec["loss"]), mb_addq=np.array(rec["addq"]),
               lstm_cfg=np.array([TINY_BERT["hidden_size"], 16, 2, 8]),
               loss_cfg=np.array([0.05, 0.9, 32, 2]),
               train_cfg=np.array([8, 16, total_steps, 2]),
               adam=np.array([2.5e-4, 0.9, 0.999, 1.0]))
    if opt == "sgd":
        c = cfg["optimizer"]["SGD"]
        res.update(sgd=np.array([float(c["learning_rate"]), float(c["momentum"]),
                                 float(c["weight_decay"]), 1.0]),
                   sgd_epoch_mb=np.array(rec["epoch_mb"], np.int64))
    if act != "Identity":
        res["activation"] = np.array(act)
    if not use_momentum:
        res["use_momentum"] = np.int64(0)
    np.savez_compressed(os.path.join(out, fname), **res)
    print("train traj: micro-batch losses", rec["loss"])


def main():
    _import_ref()
    with tempfile.TemporaryDirectory() as tmp:
        if len(sys.argv) > 1:  # regenerate selected fixtures only
            for name in sys.argv[1:]:
                fn = globals()[f"gen_{name}"]
                fn(HERE, tmp) if "tmp" in fn.__code__.co_varnames[:fn.__code__.co_argcount] \
                    else fn(HERE)
            return
        gen_nce(HERE)
        gen_nce_c2(HERE)
        gen_nce_c34(HERE)
        gen_bert_base(HERE)
        gen_bert_large(HERE)
        gen_lstm_init(HERE)
        gen_seq2vec(HERE, tmp)
        gen_bert(HERE, tmp)
        gen_bert_long(HERE, tmp)
        gen_scan(HERE)
        gen_train_traj(HERE, tmp)
        gen_train_traj_nomom(HERE, tmp)
        gen_train_traj_sgd(HERE, tmp)


if __name__ == "__main__":
    main()
