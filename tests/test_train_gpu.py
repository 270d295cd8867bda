"""End-to-end training parity: replay the reference's own 4-step train() run
(tests/golden/train_traj.npz: tiny BERT + 2-layer BiLSTM head, B=8, acml=16,
queue 32 switched on at step 2) through the HIP path and compare every
micro-batch loss and the final encoder_q / encoder_k / queue state.
"""
import argparse

import numpy as np
import pytest
import torch

from conftest import load_golden

pytestmark = pytest.mark.gpu


def _args_from_golden(fx):
    import yaml

    from conftest import PKG

    with open(f"{PKG}/config.yaml") as f:
        cfg = yaml.safe_load(f)
    in_dim, hsz, nlayers, outd = (int(x) for x in fx["lstm_cfg"])
    T, mom, qsize, qstart = fx["loss_cfg"]
    B, acml, total, log_step = (int(x) for x in fx["train_cfg"])
    cfg["model"]["LSTM"].update(input_size=in_dim, hidden_size=hsz, num_layers=nlayers,
                                output_size=outd,
                                activation=str(fx["activation"]) if "activation" in fx
                                else "Identity")
    opt = "adam"
    if "sgd" in fx:
        opt = "sgd"
        lr, m, wd, _ = (float(x) for x in fx["sgd"])
        cfg["optimizer"]["SGD"].update(learning_rate=lr, momentum=m, weight_decay=wd)
    cfg["loss"]["InfoNCE"].update(temperature=float(T), momentum=float(mom),
                                  queue_size=int(qsize), queue_start_steps=int(qstart),
                                  use_momentum=bool(int(fx["use_momentum"]))
                                  if "use_momentum" in fx else True)
    cfg["train"].update(batch_size=B, acml_batch_size=acml, total_steps=total, log_step=log_step)
    init = {k[len("init_bert_model."):]: v for k, v in fx.items()
            if k.startswith("init_bert_model.")}
    vocab, hid = init["embeddings.word_embeddings.weight"].shape
    nl = 1 + max(int(k.split(".")[2]) for k in init if k.startswith("encoder.layer."))
    cfg["bert"] = {"name": "tiny", "config": {
        "vocab_size": int(vocab), "hidden_size": int(hid), "num_hidden_layers": nl,
        "num_attention_heads": 2, "intermediate_size": int(
            init["encoder.layer.0.intermediate.dense.weight"].shape[0]),
        "max_position_embeddings": int(init["embeddings.position_embeddings.weight"].shape[0])}}
    return argparse.Namespace(config=cfg, loss="InfoNCE", model="LSTM", opt=opt,
                              sample="uniform")


def _replay(gpu, precision, pipelined=False, fixture="train_traj.npz"):
    from irc_amd.precision import get_precision, set_precision
    from src.model import build_model, get_optimizer
    from src.train import TrainState, adjust_learning_rate

    fx = load_golden(fixture)
    old = get_precision()
    set_precision(precision)
    try:
        args = _args_from_golden(fx)
        model = build_model(args)
        init = {k[5:]: torch.from_numpy(v) for k, v in fx.items()
                if k.startswith("init_") and not k.startswith("init___")}
        res = model.load_state_dict(init, strict=False)
        assert not [k for k in res.missing_keys if "position_ids" not in k], res.missing_keys
        model = model.to(gpu).train()
        opt = get_optimizer(args, model)
        st = TrainState(args, model, opt)
        losses = []
        total = int(fx["train_cfg"][2])
        acml = int(fx["train_cfg"][1])
        n_mb = fx["mb_len"].shape[0]

        def batch(i):
            L, nb = int(fx["mb_len"][i]), int(fx["mb_B"][i])
            ids = torch.from_numpy(fx["mb_ids"][i, :2 * nb, :L]).to(gpu)
            mask = torch.from_numpy(fx["mb_mask"][i, :2 * nb, :L]).to(gpu)
            return nb, ids, mask

        pending = None
        if pipelined:  # src/train.py's loop: BERT of micro-batch i+1 overlaps heads of i
            nb0, ids0, mask0 = batch(0)
            pending = model.bert_extract_async(ids0, mask0, nb0)
        epoch_at = {int(a): int(b) for a, b in fx["sgd_epoch_mb"]} if "sgd_epoch_mb" in fx \
            else {}
        for i in range(n_mb):
            if i in epoch_at:  # src/train.py: the cosine rate, once per pass (--opt sgd)
                assert st.step_sum == epoch_at[i]
                adjust_learning_rate(opt, st.step_sum, args.config)
            nb, ids, mask = batch(i)
            if pipelined:
                handle = pending
                if i + 1 < n_mb:
                    nb1, ids1, mask1 = batch(i + 1)
                    if pipelined == "ready":  # resident inputs: no wait on the heads' work
                        torch.cuda.current_stream(gpu).synchronize()
                        pending = model.bert_extract_async(ids1, mask1, nb1, inputs_ready=True)
                    else:
                        pending = model.bert_extract_async(ids1, mask1, nb1)
                loss, _ = st.micro_batch(
                    nb, lambda: model.forward_features(*model.features_ready(handle)))
            else:
                loss, _ = st.micro_batch(
                    nb, lambda: model.forward_features(*model.bert_extract_ids(ids, mask, nb)))
            losses.append(loss.item() * acml)
            if st.step_sum >= total:
                break
        return fx, np.array(losses), model
    finally:
        set_precision(old)


@pytest.mark.parametrize("fixture", ["train_traj.npz", "train_traj_nomom.npz",
                                     "train_traj_sgd.npz"])
def test_train_trajectory_fp32(gpu, fixture):
    """fixture train_traj_nomom: loss.use_momentum False -- no encoder_k, the keys
    come from encoder_q with autograd, so the InfoNCE backward feeds dk too.
    train_traj_sgd: --opt sgd (momentum + weight decay, the per-pass cosine rate over
    two passes) with a Tanh head activation (src/model.py:25,45-51)."""
    fx, losses, model = _replay(gpu, "fp32", fixture=fixture)
    np.testing.assert_allclose(losses, fx["mb_loss"], rtol=2e-4, atol=1e-4)
    sd = model.state_dict()
    for k in ("queue", "queue_ptr"):
        np.testing.assert_allclose(sd[k].cpu().numpy(), fx["final_" + k], rtol=1e-4, atol=1e-5)
    for k in fx:
        if k.startswith("final_encoder_"):
            name = k[len("final_"):]
            np.testing.assert_allclose(sd[name].cpu().numpy(), fx[k], rtol=1e-3, atol=2e-6,
                                       err_msg=name)


@pytest.mark.parametrize("fixture", ["train_traj.npz", "train_traj_sgd.npz"])
def test_train_trajectory_bf16(gpu, fixture):
    """Production precision: bf16 BERT/LSTM operands, fp32 state/loss/optimizer.
    Micro-batch losses (~25-45) within 5e-3 relative of the reference's fp32 run
    (achieved <= 2.7e-3 on MI355X: a 2-layer H=32 BERT, where one bf16 rounding is
    a larger share of each feature; at the C2 shapes the bf16 step's loss is
    within 1.2e-5 of fp32 mode, tests/test_configs_gpu.py)."""
    fx, losses, model = _replay(gpu, "bf16", fixture=fixture)
    rel = np.abs(losses - fx["mb_loss"]) / np.abs(fx["mb_loss"])
    print("bf16 trajectory: per-micro-batch loss rel err", " ".join(f"{r:.1e}" for r in rel))
    np.testing.assert_allclose(losses, fx["mb_loss"], rtol=5e-3)


@pytest.mark.parametrize("mode", [True, "ready"])
def test_train_pipelined_bert_prefetch_matches_sequential(gpu, mode):
    """bert_extract_async (the next micro-batch's frozen-BERT features on a side
    stream, as src/train.py and bench.py run it) changes only the overlap, never
    the numbers: losses and final parameters bit-identical to the sequential loop."""
    fx, seq_losses, seq_model = _replay(gpu, "bf16")
    _, pipe_losses, pipe_model = _replay(gpu, "bf16", pipelined=mode)
    np.testing.assert_array_equal(pipe_losses, seq_losses)
    a, b = seq_model.state_dict(), pipe_model.state_dict()
    for k in a:
        if k.startswith(("encoder_q", "encoder_k", "queue")):
            assert torch.equal(a[k], b[k]), k
