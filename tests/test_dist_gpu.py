"""Data-parallel training on the real model classes, two ranks
sharing the one GPU of the test box (gloo carries the collectives; RCCL needs one
device per rank): each rank runs TrainState.set_process_group with its half of a
micro-batch through the HIP path -- frozen BERT, BiLSTM head, global in-batch
negatives via gather_rows, the flat-gradient
all-reduce, fused clip + Adam, momentum update, enqueue of the gathered keys --
and must reproduce the single-process step over the whole micro-batch (fp32
parity mode: same math, different reduction splits)."""
import argparse
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

WORLD, B, L, STEPS = 2, 64, 24, 2


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _args(b, model="LSTM"):
    import yaml

    from conftest import PKG

    with open(f"{PKG}/config.yaml") as f:
        cfg = yaml.safe_load(f)
    cfg["bert"] = {"name": "tiny", "seed": 3, "config": {
        "vocab_size": 500, "hidden_size": 128, "num_hidden_layers": 2, "num_attention_heads": 2,
        "intermediate_size": 256, "max_position_embeddings": 64}}
    cfg["model"]["LSTM"].update(input_size=128, hidden_size=256, num_layers=2, output_size=64)
    cfg["model"]["BERT"] = {"name": "tiny", "seed": 5, "config": {
        "vocab_size": 500, "hidden_size": 64, "num_hidden_layers": 5, "num_attention_heads": 2,
        "intermediate_size": 128, "max_position_embeddings": 64}}
    cfg["loss"]["InfoNCE"].update(queue_size=256, queue_start_steps=1)
    cfg["train"].update(batch_size=b, acml_batch_size=b)
    return argparse.Namespace(config=cfg, loss="InfoNCE", model=model, opt="adam",
                              sample="uniform")


def _batches():
    g = torch.Generator().manual_seed(11)
    out = []
    for _ in range(STEPS):
        ids = torch.randint(5, 500, (2 * B, L), generator=g)
        mask = torch.ones_like(ids)
        mask[:, L - 5:] = (torch.rand(2 * B, 5, generator=g) < 0.5).long()
        out.append((ids * mask, mask))
    return out


def _run(rank, world, dev, out_dir, model_kind="LSTM"):
    from irc_amd.precision import set_precision
    from src.model import build_model, get_optimizer
    from src.train import TrainState

    set_precision("fp32")
    b = B // world
    args = _args(b, model_kind)
    torch.manual_seed(1337)
    model = build_model(args).to(dev).train()
    if model_kind == "BERT":
        model.encoder_q.reduce_bucket_layers = 2  # 3 buckets over 5 layers
    st = TrainState(args, model, get_optimizer(args, model))
    if world > 1:
        st.set_process_group(dist.group.WORLD)
    losses = []
    for ids, mask in _batches():
        a = slice(rank * b, (rank + 1) * b)
        p = slice(B + rank * b, B + (rank + 1) * b)
        ids_r = torch.cat([ids[a], ids[p]]).to(dev)
        mask_r = torch.cat([mask[a], mask[p]]).to(dev)
        if model_kind == "BERT":
            fwd = lambda: model.forward_ids(ids_r, mask_r, b)  # noqa: E731
        else:
            fwd = lambda: model.forward_features(*model.bert_extract_ids(ids_r, mask_r, b))  # noqa: E731
        loss, stepped = st.micro_batch(b, fwd)
        assert stepped
        losses.append(loss.item())
    sd = {k: v.cpu().numpy() for k, v in model.state_dict().items()
          if k.startswith(("encoder_q", "encoder_k", "queue"))}
    np.savez(os.path.join(out_dir, f"{model_kind}_r{rank}_w{world}.npz"),
             losses=np.array(losses), **sd)


def _worker(rank, port, out_dir, model_kind):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        _run(rank, WORLD, torch.device("cuda:0"), out_dir, model_kind)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("model_kind", ["LSTM", "BERT"])
def test_dp_two_ranks_match_single_process(gpu, tmp_path, model_kind):
    """LSTM: frozen BERT + BiLSTM heads (one all-reduce after backward).  BERT: the
    trainable encoder, whose gradient is all-reduced in 3 buckets DURING its
    backward (BertEncoder.set_grad_reduce) -- same numbers either way."""
    mp.start_processes(_worker, args=(_free_port(), str(tmp_path), model_kind), nprocs=WORLD,
                       join=True, start_method="spawn")
    from irc_amd.precision import get_precision, set_precision

    old = get_precision()
    try:
        _run(0, 1, gpu, str(tmp_path), model_kind)
    finally:
        set_precision(old)
    ref = np.load(tmp_path / f"{model_kind}_r0_w1.npz")
    for r in range(WORLD):
        got = np.load(tmp_path / f"{model_kind}_r{r}_w{WORLD}.npz")
        # global batch loss on every rank = single-process loss (same logits rows)
        np.testing.assert_allclose(got["losses"], ref["losses"], rtol=2e-5)
        # parameters after STEPS Adam steps: Adam normalises each coordinate (g /
        # sqrt(v)), so a coordinate whose gradient is ~0 can move by up to lr on a
        # rounding difference of the split reductions -> atol = lr / 2 per step
        for k in ref.files:
            if k != "losses":
                np.testing.assert_allclose(got[k], ref[k], rtol=1e-4, atol=1.25e-4 * STEPS,
                                           err_msg=k)
    a = np.load(tmp_path / f"{model_kind}_r0_w2.npz")
    b = np.load(tmp_path / f"{model_kind}_r1_w2.npz")
    for k in a.files:  # replicas stay bit-identical across ranks
        if k != "losses":
            np.testing.assert_array_equal(a[k], b[k], err_msg=k)
