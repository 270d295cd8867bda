"""Drop-in for src/model.py: LSTM head, build_model, get_optimizer, save/load.

``LSTM`` keeps the reference's config keys, parameter names and initialisation
(src/model.py:7-41) on the flat-buffer head of irc_amd.lstm_head.
``get_optimizer`` returns the fused SGD or Adam over encoder_q's flat buffer
(model.py:44-58 semantics); checkpoints keep the reference layout
{Model, Optimizer, Current_step, Args} and file name (model.py:76-99).
"""
import argparse

import torch

from irc_amd.bert_train import BertEncoder
from irc_amd.lstm_head import LSTMHead
from irc_amd.optim import FusedAdam, FusedSGD
from src.contrastor.contrastive_loss import NCELoss
from src.contrastor.contrastive_module import RetrievalModelWrapper


class LSTM(LSTMHead):
    """nn.LSTM(input, hidden, layers, batch_first, bidirectional) + Linear + the
    configured activation (``eval(f"nn.{act}()")``, model.py:23-26)."""


class BERT(BertEncoder):
    """``--model BERT``: the trainable BERT bi-encoder (mean-pool, D = hidden size).
    Architecture from config ``model.BERT`` ({name: preset, config: {...}, seed}) or,
    failing that, the ``bert`` section; bert-base-uncased by default."""

    def __init__(self, config, **kwargs):
        c = dict((config.get("model") or {}).get("BERT") or config.get("bert") or {})
        super().__init__(c.get("config"), name=c.get("name", "bert-base-uncased"),
                         seed=int(c.get("seed", 0)))


def get_optimizer(args, model):
    if args.opt == "sgd":
        c = args.config["optimizer"]["SGD"]
        return FusedSGD(model.encoder_q, lr=float(c["learning_rate"]),
                        momentum=float(c["momentum"]), weight_decay=float(c["weight_decay"]))
    if args.opt == "adam":
        return FusedAdam(model.encoder_q,
                         lr=float(args.config["optimizer"]["Adam"]["learning_rate"]),
                         betas=tuple(args.config["optimizer"]["Adam"]["betas"]))
    raise ValueError(f"unknown optimizer {args.opt!r} (sgd or adam)")


def build_model(args):
    print("[Runner] - Building contrastive model")
    loss_config = args.config["loss"][f"{args.loss}"]
    if args.model == "LSTM":
        bk_model = LSTM(args.config)
        loss_config["dim"] = args.config["model"]["LSTM"]["output_size"]
    elif args.model == "BERT":
        bk_model = BERT(args.config)
        loss_config["dim"] = bk_model.config.hidden_size
    else:
        raise ValueError(f"unknown model {args.model!r} (LSTM or BERT)")
    if args.loss in ["InfoNCE", "ProtoNCE", "HProtoNCE"]:
        criterion = NCELoss(loss_config)
    use_LSTM = isinstance(bk_model, LSTM)
    return RetrievalModelWrapper(bk_model, criterion, loss_config, use_LSTM=use_LSTM,
                                 bert_config=args.config.get("bert"))


def save_model(model, optimizer, args, current_step):
    path = f"{args.ckptdir}/{args.sample}_{args.loss}_{args.model}_{current_step}.pth"
    # the live process group is a handle of this run, not a setting: not stored
    saved_args = argparse.Namespace(**{k: v for k, v in vars(args).items() if k != "dist_group"})
    all_states = {
        "Model": model.state_dict(),
        "Optimizer": optimizer.state_dict(),
        "Current_step": current_step,
        "Args": saved_args,
    }
    torch.save(all_states, path)


def load_model(path, bert_config=None):
    """Reference load_model (model.py:87-99): (args, model, optimizer, step) from a
    checkpoint written by this package or by the reference itself.

    Loaded weights-only: the checkpoint's "Args" is an argparse.Namespace (config
    dict, strings, a torch.device), which is allow-listed; nothing in the file is
    executed.  ``bert_config`` (superset) replaces ``args.config['bert']`` -- for a
    reference checkpoint whose frozen BERT is not bert-base-uncased."""
    torch.serialization.add_safe_globals([argparse.Namespace])
    ckpt = torch.load(path, map_location="cpu", weights_only=True)
    args = ckpt["Args"]
    if bert_config is not None:
        args.config["bert"] = bert_config
    model = build_model(args)
    print("[Runner] - Loading model parameters")
    res = model.load_state_dict(ckpt["Model"], strict=False)
    missing = [k for k in res.missing_keys if not k.endswith("position_ids")]
    if missing:
        raise RuntimeError(f"checkpoint is missing {missing[:8]}")
    optimizer = get_optimizer(args, model)
    optimizer.load_state_dict(ckpt["Optimizer"])
    return args, model, optimizer, ckpt["Current_step"]
