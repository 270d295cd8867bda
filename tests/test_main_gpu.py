"""End-to-end drop-in run: the package's main.py / src.train.train loop on a tiny
synthetic docs_sentence.pkl (C1-shaped: 2-layer BERT H=128, 2-layer BiLSTM head),
for InfoNCE and for ProtoNCE with re-clustering -- exercises the dataset,
tokenizer, frozen-BERT prefetch pipeline, clustering, loss, optimizer and the
checkpoint writer together (the numbers themselves are pinned elsewhere)."""
import os
import pickle

import pytest
import yaml

from conftest import PKG

pytestmark = pytest.mark.gpu


def _write_inputs(tmp_path, loss):
    import random

    rnd = random.Random(0)
    docs = [[" ".join(f"w{rnd.randrange(900)}" for _ in range(rnd.randrange(4, 12)))
             for _ in range(rnd.randrange(3, 7))] for _ in range(200)]
    data = tmp_path / "docs_sentence.pkl"
    with open(data, "wb") as f:
        pickle.dump(docs, f)
    with open(os.path.join(PKG, "config.yaml")) as f:
        cfg = yaml.safe_load(f)
    cfg["dataset"]["docs_sentence"] = str(data)
    cfg["bert"] = {"name": "tiny", "vocab": None, "seed": 0, "precision": "bf16",
                   "config": {"vocab_size": 1000, "hidden_size": 128, "num_hidden_layers": 2,
                              "num_attention_heads": 2, "intermediate_size": 512,
                              "max_position_embeddings": 64}}
    cfg["model"]["LSTM"].update(num_layers=2, input_size=128, hidden_size=64, output_size=32)
    cfg["train"].update(batch_size=16, acml_batch_size=32, total_steps=4, log_step=2, n_jobs=0)
    cfg["eval"].update(batch_size=32, n_jobs=0)
    for name in ("InfoNCE", "ProtoNCE"):
        cfg["loss"][name].update(queue_size=64, queue_start_steps=2)
    cfg["loss"]["ProtoNCE"].update(cluster_start_steps=1)
    cfg["loss"]["ProtoNCE"]["cluster"].update(update_steps=2, num_cluster=[40, 48],
                                              num_neg_proto=4, niter=3, nredo=1)
    path = tmp_path / "config.yaml"
    with open(path, "w") as f:
        yaml.safe_dump(cfg, f)
    return str(path)


@pytest.mark.parametrize("loss", ["InfoNCE", "ProtoNCE"])
def test_main_train_end_to_end(gpu, tmp_path, loss):
    import main as entry

    cfg = _write_inputs(tmp_path, loss)
    entry.main(["--config", cfg, "--loss", loss, "--gpu", "0", "--logdir",
                str(tmp_path / "log"), "--ckptdir", str(tmp_path / "ckpt")])
    ckpts = sorted(os.listdir(tmp_path / "ckpt"))
    assert ckpts == [f"uniform_{loss}_LSTM_2.pth", f"uniform_{loss}_LSTM_4.pth"], ckpts


@pytest.mark.parametrize("model", ["LSTM", "BERT"])
def test_main_train_long_sentences(gpu, tmp_path, model):
    """A ragged corpus in which every document holds one long sentence (130 to 600
    words), so the jointly padded batches reach L = 512 through the reference's
    truncation (contrastive_module.py:38): main.py trains through them, frozen BERT +
    BiLSTM and --model BERT (trainable encoder, attention backward at long L)."""
    import random

    import main as entry

    rnd = random.Random(1)
    docs = []
    for d in range(40):
        sents = [" ".join(f"w{rnd.randrange(900)}" for _ in range(rnd.randrange(4, 12)))
                 for _ in range(2)]
        sents.append(" ".join(f"w{rnd.randrange(900)}" for _ in range((130, 300, 500, 600)[d % 4])))
        rnd.shuffle(sents)
        docs.append(sents)
    data = tmp_path / "docs_sentence.pkl"
    with open(data, "wb") as f:
        pickle.dump(docs, f)
    with open(os.path.join(PKG, "config.yaml")) as f:
        cfg = yaml.safe_load(f)
    cfg["dataset"]["docs_sentence"] = str(data)
    bert = {"vocab_size": 1000, "hidden_size": 128, "num_hidden_layers": 2,
            "num_attention_heads": 2, "intermediate_size": 512, "max_position_embeddings": 512}
    cfg["bert"] = {"name": "tiny", "vocab": None, "seed": 0, "precision": "bf16", "config": bert}
    cfg["model"]["BERT"] = {"config": bert}
    cfg["model"]["LSTM"].update(num_layers=2, input_size=128, hidden_size=64, output_size=32)
    cfg["train"].update(batch_size=8, acml_batch_size=8, total_steps=4, log_step=2, n_jobs=0)
    cfg["loss"]["InfoNCE"].update(queue_size=64, queue_start_steps=2)
    path = tmp_path / "config.yaml"
    with open(path, "w") as f:
        yaml.safe_dump(cfg, f)
    entry.main(["--config", str(path), "--model", model, "--gpu", "0", "--logdir",
                str(tmp_path / "log"), "--ckptdir", str(tmp_path / "ckpt")])
    ckpts = sorted(os.listdir(tmp_path / "ckpt"))
    assert ckpts == [f"uniform_InfoNCE_{model}_2.pth", f"uniform_InfoNCE_{model}_4.pth"], ckpts


def _dist_worker(rank, port, cfg, out_dir):
    os.environ.update(WORLD_SIZE="2", RANK=str(rank), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), IRC_DIST_BACKEND="gloo")
    import main as entry

    entry.main(["--config", cfg, "--gpu", "0", "--logdir", os.path.join(out_dir, "log"),
                "--ckptdir", os.path.join(out_dir, "ckpt")])


def test_main_train_two_ranks(gpu, tmp_path):
    """main.py as torchrun starts it, two ranks sharing the test box's GPU (gloo:
    RCCL needs a device per rank): data-parallel InfoNCE training end to end
    through the HIP path; rank 0 writes the checkpoints, and the saved replica
    equals what every rank holds (loaded back weights-only)."""
    import socket

    import torch
    import torch.multiprocessing as mp

    from src.model import load_model

    cfg = _write_inputs(tmp_path, "InfoNCE")
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mp.start_processes(_dist_worker, args=(port, cfg, str(tmp_path)), nprocs=2, join=True,
                       start_method="spawn")
    ckpts = sorted(os.listdir(tmp_path / "ckpt"))
    assert ckpts == ["uniform_InfoNCE_LSTM_2.pth", "uniform_InfoNCE_LSTM_4.pth"], ckpts
    args, model, _, step = load_model(str(tmp_path / "ckpt" / ckpts[-1]))
    assert step == 4 and not hasattr(args, "dist_group") and args.world_size == 2
    assert torch.isfinite(model.encoder_q.flat).all()
