"""Checkpoint compatibility (reference src/model.py:76-99,
src/train.py:47-48): a checkpoint the REFERENCE wrote (tests/golden/
ref_ckpt_InfoNCE_LSTM_4.pth, the step-4 file of the run behind train_traj.npz)
loads through the drop-in load_model -- weights-only, Args allow-listed -- into
the same parameters, queue and Adam moments; and save -> load_model -> resume
continues the trajectory bit-identically on the GPU."""
import argparse
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN, load_golden

REF_CKPT = os.path.join(GOLDEN, "ref_ckpt_InfoNCE_LSTM_4.pth")
TINY_BERT = {"name": "tiny", "config": {"vocab_size": 200, "hidden_size": 32,
                                        "num_hidden_layers": 2, "num_attention_heads": 2,
                                        "intermediate_size": 64, "max_position_embeddings": 64}}


def test_load_reference_checkpoint_weights_only():
    from src.model import load_model

    fx = load_golden("train_traj.npz")
    args, model, opt, step = load_model(REF_CKPT, bert_config=TINY_BERT)
    assert step == 4 and args.model == "LSTM" and args.loss == "InfoNCE"
    sd = model.state_dict()
    for k in fx:
        if k.startswith("final_"):
            name = k[len("final_"):]
            np.testing.assert_array_equal(sd[name].cpu().numpy().reshape(fx[k].shape), fx[k],
                                          err_msg=name)
    # the reference's torch.optim.Adam moments (param indices 0.. = encoder_q in
    # nn.LSTM order) land in the fused optimizer's flat moments
    torch.serialization.add_safe_globals([argparse.Namespace])
    ref = torch.load(REF_CKPT, map_location="cpu", weights_only=True)["Optimizer"]
    head = model.encoder_q
    for i, (name, shape) in enumerate(head.specs):
        assert torch.equal(head.view(name, opt.exp_avg), ref["state"][i]["exp_avg"].reshape(shape))
        assert torch.equal(head.view(name, opt.exp_avg_sq),
                           ref["state"][i]["exp_avg_sq"].reshape(shape))
    assert opt.step_count == 4


def test_load_model_refuses_code_in_pickle(tmp_path):
    """A checkpoint whose pickle would run code is rejected, not executed."""
    from src.model import load_model

    class Evil:
        def __reduce__(self):
            return (os.system, ("echo pwned",))

    p = tmp_path / "evil.pth"
    torch.save({"Model": {}, "Optimizer": {}, "Current_step": 0, "Args": Evil()}, p)
    with pytest.raises(Exception, match="(?i)weights_only|unsupported|global"):
        load_model(str(p))


@pytest.mark.gpu
def test_save_load_resume_is_bit_identical(gpu, tmp_path):
    """fp32 parity mode: 2 steps, save_model, load_model, 2 more steps == 4 steps
    straight (losses, encoder_q/encoder_k, queue, queue_ptr)."""
    from irc_amd.precision import get_precision, set_precision
    from src.model import build_model, get_optimizer, load_model, save_model
    from src.train import TrainState
    from test_train_gpu import _args_from_golden

    fx = load_golden("train_traj.npz")
    init = {k[5:]: torch.from_numpy(v) for k, v in fx.items()
            if k.startswith("init_") and not k.startswith("init___")}

    def batches(i0, i1):
        for i in range(i0, i1):
            L, nb = int(fx["mb_len"][i]), int(fx["mb_B"][i])
            yield nb, torch.from_numpy(fx["mb_ids"][i, :2 * nb, :L]).to(gpu), \
                torch.from_numpy(fx["mb_mask"][i, :2 * nb, :L]).to(gpu)

    def run(st, model, i0, i1):
        out = []
        for nb, ids, mask in batches(i0, i1):
            loss, _ = st.micro_batch(
                nb, lambda: model.forward_features(*model.bert_extract_ids(ids, mask, nb)))
            out.append(loss.item())
        return out

    old = get_precision()
    set_precision("fp32")
    try:
        args = _args_from_golden(fx)
        args.ckptdir = str(tmp_path)
        model = build_model(args)
        model.load_state_dict(init, strict=False)
        model = model.to(gpu).train()
        opt = get_optimizer(args, model)
        st = TrainState(args, model, opt)
        straight = run(st, model, 0, 8)
        ref_sd = {k: v.clone() for k, v in model.state_dict().items()}

        model = build_model(args)
        model.load_state_dict(init, strict=False)
        model = model.to(gpu).train()
        opt = get_optimizer(args, model)
        st = TrainState(args, model, opt)
        first = run(st, model, 0, 4)
        assert st.step_sum == 2
        save_model(model, opt, args, st.step_sum)
        path = os.path.join(str(tmp_path), f"{args.sample}_{args.loss}_{args.model}_2.pth")
        args2, model2, opt2, step = load_model(path)
        assert step == 2
        model2 = model2.to(gpu).train()
        opt2.to(gpu)
        st2 = TrainState(args2, model2, opt2, init_step=step)
        second = run(st2, model2, 4, 8)
    finally:
        set_precision(old)
    assert first + second == straight
    sd = model2.state_dict()
    for k, v in ref_sd.items():
        if k.startswith(("encoder_q", "encoder_k", "queue")):
            assert torch.equal(sd[k], v), k
