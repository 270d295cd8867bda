"""The drop-in entrypoint under a launcher (VERDICT r2 missing #2): main.main()
in two gloo ranks, as torchrun would start it (WORLD_SIZE / RANK / LOCAL_RANK /
MASTER_* in the environment), with the model and optimizer replaced by CPU test
doubles (the HIP model is covered by tests/test_dist_gpu.py and
tests/test_main_gpu.py).  Checks what main.py / src.train own under data
parallelism:

* init_distributed brings the process group up from the environment and
  TrainState.set_process_group is wired (the model's dist_group is set);
* each rank reads a disjoint slice of the documents (DistributedSampler);
* the loss is the global batch's (embeddings all-gathered) and the gradients
  are all-reduced: after several optimizer steps both replicas are bit-identical
  although their data differ;
* scalars and checkpoints come from rank 0 only.
"""
import os
import pickle
import socket

import numpy as np
import torch
import torch.multiprocessing as mp
import yaml

from conftest import PKG

WORLD = 2
FEAT, DIM, VOCAB = 12, 8, 60


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class _Enc(torch.nn.Module):
    def __init__(self):
        super().__init__()
        g = torch.Generator().manual_seed(3)
        self.flat = torch.nn.Parameter(torch.randn(FEAT * DIM, generator=g, dtype=torch.float64))
        self.flat.grad = torch.zeros_like(self.flat)

    @property
    def flat_grad(self):
        return self.flat.grad


class _DoubleModel(torch.nn.Module):
    """Stands in for RetrievalModelWrapper: bag-of-words features -> linear encoder
    -> unit embeddings; keys without grad (momentum-encoder style); the global
    InfoNCE over gathered embeddings (tests/test_dist_cpu.py's torch restatement of
    contrastive_loss.py:56-93)."""

    def __init__(self, out_dir, rank):
        super().__init__()
        self.encoder_q = _Enc()
        g = torch.Generator().manual_seed(4)
        self.table = torch.randn(VOCAB, FEAT, generator=g, dtype=torch.float64)
        self.use_LSTM, self.use_momentum, self.use_queue = False, False, False
        self.dist_group = None
        self.seen, self.losses = [], []
        self.out_dir, self.rank = out_dir, rank

    def to(self, *a, **k):  # nominal cuda device: nothing moves on the CPU test host
        return self

    def _feat(self, sents):
        return torch.stack([self.table[[int(w[1:]) for w in s.split()]].mean(0) for s in sents])

    def forward(self, anchor, positive, device, cluster_result=None, indexes=None):
        from irc_amd.dist import gather_rows
        from test_dist_cpu import _nce_torch

        assert self.dist_group is not None, "TrainState.set_process_group was not wired"
        self.seen.extend(int(i) for i in indexes.view(-1))
        W = self.encoder_q.flat.view(FEAT, DIM)
        q = torch.nn.functional.normalize(self._feat(anchor) @ W, dim=1)
        with torch.no_grad():
            k = torch.nn.functional.normalize(self._feat(positive) @ W, dim=1)
        q, k = gather_rows(q, self.dist_group), gather_rows(k, self.dist_group)
        loss = _nce_torch(q, k, None, 0.05)
        self.losses.append(loss.item())
        return loss


class _DoubleOpt:
    def __init__(self, model):
        self.p = model.encoder_q.flat

    def to(self, device):
        return self

    def clip_and_step(self, max_norm):
        n = torch.nn.utils.clip_grad_norm_([self.p], max_norm)
        with torch.no_grad():
            self.p -= 0.1 * self.p.grad
        return n.reshape(1)

    def zero_grad(self):
        self.p.grad.zero_()

    def state_dict(self):
        return {}


def _worker(rank, port, cfg_path, out_dir):
    os.environ.update(WORLD_SIZE=str(WORLD), RANK=str(rank), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), IRC_DIST_BACKEND="gloo")
    import main as entry
    import src.train as T

    made = {}

    def build_model(args):
        made["m"] = _DoubleModel(out_dir, rank)
        return made["m"]

    saves = []
    T.build_model = build_model
    T.get_optimizer = lambda args, model: _DoubleOpt(model)
    T.save_model = lambda model, opt, args, step: saves.append(step)
    entry.main(["--config", cfg_path, "--gpu", "0", "--logdir", os.path.join(out_dir, "log"),
                "--ckptdir", os.path.join(out_dir, "ckpt")])
    m = made["m"]
    np.savez(os.path.join(out_dir, f"r{rank}.npz"), seen=np.array(m.seen),
             losses=np.array(m.losses), w=m.encoder_q.flat.detach().numpy(),
             saves=np.array(saves, dtype=np.int64))


def test_main_under_two_gloo_ranks(tmp_path):
    import random

    rnd = random.Random(0)
    docs = [[" ".join(f"w{rnd.randrange(VOCAB)}" for _ in range(rnd.randrange(3, 8)))
             for _ in range(rnd.randrange(3, 6))] for _ in range(40)]
    with open(tmp_path / "docs.pkl", "wb") as f:
        pickle.dump(docs, f)
    with open(os.path.join(PKG, "config.yaml")) as f:
        cfg = yaml.safe_load(f)
    cfg["dataset"]["docs_sentence"] = str(tmp_path / "docs.pkl")
    cfg["train"].update(batch_size=4, acml_batch_size=4, total_steps=4, log_step=2, n_jobs=0)
    cfg_path = tmp_path / "config.yaml"
    with open(cfg_path, "w") as f:
        yaml.safe_dump(cfg, f)
    mp.start_processes(_worker, args=(_free_port(), str(cfg_path), str(tmp_path)), nprocs=WORLD,
                       join=True, start_method="spawn")
    r0, r1 = np.load(tmp_path / "r0.npz"), np.load(tmp_path / "r1.npz")
    # 4 steps x 4 pairs per rank out of 40 docs: one epoch, disjoint slices
    assert len(r0["seen"]) == len(r1["seen"]) == 16
    assert not set(r0["seen"].tolist()) & set(r1["seen"].tolist())
    # global loss on both ranks, and identical replicas after 4 all-reduced steps
    np.testing.assert_array_equal(r0["losses"], r1["losses"])
    np.testing.assert_array_equal(r0["w"], r1["w"])
    assert not np.array_equal(r0["w"], _Enc().flat.detach().numpy())
    # checkpoints / scalars on rank 0 only
    assert r0["saves"].tolist() == [2, 4] and r1["saves"].tolist() == []
    assert os.path.isdir(tmp_path / "log" / "InfoNCE_LSTM")
