"""`main.py --data fever` end to end on a tiny synthetic FEVER set, and ctx2vec
parity (reference src/evaluation.py:86-116,
contrastive_module.py:96-100).

* predict (default, the reference's behaviour): per claim the sparse n-gram
  filter; its candidate counts equal the reference arithmetic
  (count_matrix[unique hashed n-grams].nonzero() -> np.unique, evaluation.py:57-83)
  computed here on the host with scipy.
* predict --retrieval dense: ctx2vec corpus + exact top-k; recall@k returned.
* ctx2vec against the oracle's tokenize -> BERT -> seq2vec on the reference
  run's initial weights (train_traj.npz), fp32 parity mode.
"""
import argparse
import json
import os
import pickle

import numpy as np
import pytest
import torch
import yaml

from conftest import PKG, load_golden
from oracle import irc_oracle as O

pytestmark = pytest.mark.gpu


def _fever_files(tmp_path, hash_size=1 << 16):
    import scipy.sparse as sp

    from irc_amd import sparse

    rnd = np.random.RandomState(5)
    words = [f"tok{i}" for i in range(120)]
    wiki, texts, titles = {}, [], []
    for p in range(30):
        lines = [" ".join(rnd.choice(words, rnd.randint(5, 12))) for _ in range(rnd.randint(2, 5))]
        title = f"Page_{p}"
        wiki[title] = {"lines": "\n".join(f"{i}\t{l}" for i, l in enumerate(lines))}
        texts.append(" ".join(lines))
        titles.append(title)
    claims = []
    for c in range(12):
        p = rnd.randint(30)
        line = wiki[titles[p]]["lines"].split("\n")[0].split("\t")[1].split()
        claim = " ".join(line[:4] + list(rnd.choice(words, 3)))
        claims.append({"id": c, "claim": claim, "label": ["SUPPORTS", "REFUTES"][c % 2],
                       "evidence": [[[0, c, titles[p], 0]]]})
    claims.append({"id": 99, "claim": "tok1 tok2", "label": "NOT ENOUGH INFO",
                   "evidence": [[[0, 99, None, None]]]})
    (tmp_path / "wiki.json").write_text(json.dumps(wiki))
    with open(tmp_path / "dev.jsonl", "w") as f:
        for c in claims:
            f.write(json.dumps(c) + "\n")
    counts = sparse.build_count_matrix(texts, hash_size, 2)
    meta = {"doc_dict": ({t: i for i, t in enumerate(titles)}, titles), "ngram": 2,
            "hash_size": hash_size, "tokenizer": "simple",
            "doc_freqs": sparse.doc_freqs(counts)}
    for name, m in (("count_matrix.npz", counts), ("tfidf.npz", sparse.tfidf_matrix(counts))):
        m = sp.csr_matrix(m)
        np.savez(tmp_path / name, data=m.data, indices=m.indices, indptr=m.indptr,
                 shape=m.shape, metadata=meta)
    with open(tmp_path / "full_docs_dict.pkl", "wb") as f:
        pickle.dump({t: x for t, x in zip(titles[:25], texts[:25])}, f)  # 5 ids missing
    return claims, counts, titles


def _config(tmp_path):
    with open(os.path.join(PKG, "config.yaml")) as f:
        cfg = yaml.safe_load(f)
    ds = cfg["dataset"]
    ds.update(small_wiki=str(tmp_path / "wiki.json"), dev_data=str(tmp_path / "dev.jsonl"),
              tfidf=str(tmp_path / "tfidf.npz"), inverted_file=str(tmp_path / "count_matrix.npz"),
              full_docs_dict=str(tmp_path / "full_docs_dict.pkl"))
    cfg["bert"] = {"name": "tiny", "seed": 0, "config": {
        "vocab_size": 300, "hidden_size": 64, "num_hidden_layers": 2, "num_attention_heads": 2,
        "intermediate_size": 128, "max_position_embeddings": 64}}
    cfg["model"]["LSTM"].update(num_layers=2, input_size=64, hidden_size=32, output_size=64)
    cfg["eval"].update(batch_size=1, n_jobs=0)
    path = tmp_path / "config.yaml"
    with open(path, "w") as f:
        yaml.safe_dump(cfg, f)
    return cfg, str(path)


def _checkpoint(tmp_path, cfg):
    from src.model import build_model, get_optimizer, save_model

    args = argparse.Namespace(config=cfg, loss="InfoNCE", model="LSTM", opt="adam",
                              sample="uniform", ckptdir=str(tmp_path))
    torch.manual_seed(0)
    model = build_model(args)
    save_model(model, get_optimizer(args, model), args, 0)
    return str(tmp_path / "uniform_InfoNCE_LSTM_0.pth")


def test_predict_sparse_matches_reference_counts(gpu, tmp_path, capsys):
    import main as entry
    from irc_amd import sparse

    claims, counts, titles = _fever_files(tmp_path)
    cfg, cfg_path = _config(tmp_path)
    ckpt = _checkpoint(tmp_path, cfg)
    entry.main(["--data", "fever", "--config", cfg_path, "--ckpt", ckpt, "--gpu", "0"])
    out = capsys.readouterr().out.split("\n")
    printed = [int(x) for x in out if x.strip().isdigit()]
    kept = set(titles[:25])
    expect = []
    for c in claims:
        if c["label"] == "NOT ENOUGH INFO":
            continue  # FeverDataset drops NEI claims (dataset.py:108)
        wids = np.unique([sparse.feature_hash(g, counts.shape[0])
                          for g in sparse.ngrams(sparse.tokenize(c["claim"]), 2)])
        _, idx = counts[wids].nonzero()
        expect.append(sum(titles[i] in kept for i in np.unique(idx)))
    assert printed == expect


def test_predict_dense_recall(gpu, tmp_path):
    from src.evaluation import predict

    _fever_files(tmp_path)
    cfg, _ = _config(tmp_path)
    ckpt = _checkpoint(tmp_path, cfg)
    cfg["eval"]["batch_size"] = 4
    args = argparse.Namespace(config=cfg, data="fever", ckpt=ckpt, device=gpu,
                              retrieval="dense")
    r = predict(args, k=5)
    assert 0.0 <= r <= 1.0


def test_ctx2vec_matches_oracle(gpu):
    from irc_amd.precision import get_precision, set_precision
    from src.model import build_model
    from test_train_gpu import _args_from_golden

    fx = load_golden("train_traj.npz")
    init = {k[5:]: torch.from_numpy(v) for k, v in fx.items()
            if k.startswith("init_") and not k.startswith("init___")}
    texts = ["w1 w2 w3", "w10 w20 w30 w40 w50 w60 w7", "w5", "w100 w101 w3 w3 w3"]
    old = get_precision()
    set_precision("fp32")
    try:
        model = build_model(_args_from_golden(fx))
        model.load_state_dict(init, strict=False)
        model = model.to(gpu).eval()
        with torch.no_grad():
            got = model.ctx2vec(texts, gpu).cpu().numpy()
    finally:
        set_precision(old)
    t = model.bert_tokenizer(texts, padding=True, truncation=True, return_tensors="np")
    bert_w = {k[len("bert_model."):]: v.numpy() for k, v in init.items()
              if k.startswith("bert_model.")}
    feats = O.bert_forward(t["input_ids"], t["attention_mask"], bert_w, 2, 2)
    pq = {k[len("encoder_q."):]: v.numpy().astype(np.float64) for k, v in init.items()
          if k.startswith("encoder_q.")}
    ref, _ = O.seq2vec(feats.astype(np.float64), pq, int(fx["lstm_cfg"][2]))
    assert got.shape == ref.shape
    np.testing.assert_allclose(got, ref, atol=2e-5)
