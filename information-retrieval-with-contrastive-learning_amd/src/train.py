"""Drop-in for src/train.py: the contrastive training loop.

Same loop semantics as the reference (src/train.py:41-201): micro-batches of
``train.batch_size`` pairs, loss / acml_batch_size, gradient accumulation up to
``acml_batch_size`` (or a short last batch), clip_grad_norm_(gradient_clipping)
+ optimizer step + momentum update + zero_grad, queue switched on at
``queue_start_steps``, scalars + checkpoint every ``log_step``, and the OOM
catch-and-skip (matching "HIP out of memory" as well as the CUDA text).

Differences on purpose: the clip is fused into the optimizer step (no host
sync); TensorBoard is used when importable, else the scalars are printed.

Data parallel (main.py under torchrun sets ``args.dist_group``): every rank
steps its own disjoint micro-batches (DistributedSampler, reseeded per epoch),
the embeddings are all-gathered for global in-batch negatives and the head
gradient all-reduced (TrainState.set_process_group); the log directory, the
scalars, the progress bar and the checkpoints belong to rank 0.
"""
import math
import os
import shutil

import numpy as np
import torch
from tqdm import tqdm

from src.dataset import PairSampler, get_dataloader
from src.contrastor.utils import run_hierarchical_clustering, run_kmeans
from src.model import build_model, get_optimizer, load_model, save_model

OOM_MARKERS = ("CUDA out of memory", "HIP out of memory", "out of memory")


def adjust_learning_rate(optimizer, steps, config):
    """Cosine decay of the SGD learning rate (reference src/train.py:18-23), applied
    once per pass over the data when --opt sgd (train.py:90-91)."""
    lr = float(config["optimizer"]["SGD"]["learning_rate"])
    lr *= 0.5 * (1.0 + math.cos(math.pi * steps / config["train"]["total_steps"]))
    for param_group in optimizer.param_groups:
        param_group["lr"] = lr


class _NullWriter:
    def add_scalar(self, tag, value, step):
        pass

    def close(self):
        pass


class _PrintWriter:
    def __init__(self, logdir):
        self.logdir = logdir

    def add_scalar(self, tag, value, step):
        print(f"[{tag}] step {step}: {value:.6f}")

    def close(self):
        pass


def _writer(logdir):
    try:
        from torch.utils.tensorboard import SummaryWriter

        return SummaryWriter(logdir)
    except Exception:
        return _PrintWriter(logdir)


class TrainState:
    """One training run's mutable state, stepped one micro-batch at a time.

    Shared by ``train`` (below) and the parity tests / bench, which drive it with
    pre-tokenised batches."""

    def __init__(self, args, model, optimizer, init_step=0):
        self.args = args
        self.model = model
        self.optimizer = optimizer
        self.cfg = args.config
        self.acml = int(self.cfg["train"]["acml_batch_size"])
        self.bsz = int(self.cfg["train"]["batch_size"])
        assert self.acml % self.bsz == 0
        self.max_norm = float(self.cfg["optimizer"].get("gradient_clipping", 1.0))
        self.step_sum = init_step
        self.batch_size = 0
        self.loss_record = []
        self.loss_sum = 0.0
        self.grad_norm = None
        # Data parallel (one process per GPU): the flat encoder_q gradient is summed
        # over the group with one RCCL all-reduce before the fused clip + Adam, so
        # every rank applies the identical update.
        self.process_group = None
        self.world = 1

    def set_process_group(self, group):
        """Data-parallel training over ``group``: embeddings all-gathered for global
        in-batch negatives (model.dist_group) + head gradients all-reduced."""
        from irc_amd.dist import world_of

        self.process_group = group
        self.world = world_of(group)
        self.model.dist_group = group

    def check_faults(self):
        """Raise if a cluster recurrence of either encoder timed out since the last
        check (reads the heads' sticky device fault words: a host sync, so it runs
        only where the loop already syncs)."""
        for name in ("encoder_q", "encoder_k"):
            enc = getattr(self.model, name, None)
            if enc is not None and hasattr(enc, "check_fault"):
                enc.check_fault()

    def fault_words(self):
        """The heads' sticky device fault words (cluster recurrences), if any."""
        out = []
        for name in ("encoder_q", "encoder_k"):
            enc = getattr(self.model, name, None)
            w = getattr(enc, "coop_fault", None)
            if w is not None and w.is_cuda:
                out.append(w)
        return out

    def _maybe_enable_queue(self):
        m = self.model
        if m.use_queue and self.step_sum >= self.cfg["loss"][self.args.loss]["queue_start_steps"] \
                and not m.add_queue_to_loss:
            m.add_queue_to_loss = True

    def micro_batch(self, n_pairs, forward_fn, sync_loss=True):
        """forward_fn() -> loss tensor of this micro-batch (model(...) call)."""
        self._maybe_enable_queue()
        will_step = self.batch_size + n_pairs == self.acml or n_pairs != self.bsz
        enc = self.model.encoder_q
        # --model BERT under DP: the 110M-float gradient is all-reduced in buckets
        # DURING the encoder backward (overlapped); only when this micro-batch
        # steps and the encoder runs backward once (keys from the momentum encoder)
        overlap = self.process_group is not None and hasattr(enc, "set_grad_reduce") and \
            self.model.use_momentum and self.world > 1
        if overlap:
            enc.set_grad_reduce(self.process_group if will_step else None)
        self.batch_size += n_pairs
        # data parallel: the loss is the GLOBAL micro-batch's (gathered negatives),
        # so it is divided by the global accumulation size acml * world, as one
        # process stepping the whole global batch would (train.py:137-146)
        loss = forward_fn() / (self.acml * self.world)
        loss.backward()
        if sync_loss:
            self.loss_sum += loss.item()  # the reference logs every micro-batch (train.py:148)
            self.check_faults()
        else:
            self.loss_sum = self.loss_sum + loss.detach()
        stepped = False
        if self.batch_size == self.acml or n_pairs != self.bsz:
            if overlap:
                enc.wait_grad_reduce()
                enc.set_grad_reduce(None)
            elif self.process_group is not None:
                from irc_amd.dist import all_reduce_sum_

                all_reduce_sum_(self.model.encoder_q.flat_grad, self.process_group)
            faults = self.fault_words()
            if faults:  # a timed-out recurrence's step changes no parameter (no host sync)
                self.grad_norm = self.optimizer.clip_and_step(self.max_norm, faults=faults)
                if self.model.use_momentum:
                    self.model._momentum_update_key_encoder(gate=self.grad_norm)
            else:
                self.grad_norm = self.optimizer.clip_and_step(self.max_norm)
                if self.model.use_momentum:
                    self.model._momentum_update_key_encoder()
            self.optimizer.zero_grad()
            self.loss_record.append(self.loss_sum)
            self.step_sum += 1
            self.batch_size = 0
            self.loss_sum = 0.0
            stepped = True
        return loss, stepped


def _log_and_save(log, pbar, model, optimizer, args, step, loss_avg, grad_norm):
    """train.py:178-188 (rank 0 only under data parallelism)."""
    if math.isnan(grad_norm) or math.isinf(grad_norm):
        print(f"[Runner] - Error : grad norm is nan/inf at step {step}")
    log.add_scalar("train_loss", loss_avg, step)
    log.add_scalar("grad_norm", grad_norm, step)
    pbar.set_description("Train_Loss %.5f" % (loss_avg))
    print("Train_Loss %.5f" % (loss_avg))
    save_model(model, optimizer, args, step)


def train(args):
    if args.ckpt is None:
        model = build_model(args)
        optimizer = get_optimizer(args, model)
        init_step = 0
    else:
        _, model, optimizer, init_step = load_model(args.ckpt)
    model = model.to(args.device)
    optimizer.to(args.device)
    model.train()

    # LSTM heads on frozen BERT, on the GPU: the device-corpus input path (the corpus
    # tokenised once into HBM, micro-batches as sentence indices; the same pairs as
    # the DataLoader with n_jobs = 0) unless dataset.device_corpus is False
    prefetch = model.use_LSTM and args.device.type == "cuda"
    corpus = None
    if prefetch and args.config["dataset"].get("device_corpus", True) and args.data == "doc":
        from irc_amd.corpus import DeviceCorpus

        train_loader = PairSampler(args)
        corpus = DeviceCorpus(train_loader.dataset.data, model.bert_tokenizer, args.device)
    else:
        train_loader = get_dataloader(args, train=True)
    feat_loader = None
    if args.loss in ["ProtoNCE", "HProtoNCE"]:  # train.py:62-64
        feat_loader = get_dataloader(args, train=False)
    cluster_result = None

    def _maybe_recluster(cluster_result):
        """train.py:96-122: at the start of an accumulation, from cluster_start_steps
        on, every cluster.update_steps optimizer steps."""
        if feat_loader is None or st.batch_size != 0:
            return cluster_result
        cfg = args.config["loss"][args.loss]
        if st.step_sum >= cfg["cluster_start_steps"] and \
                st.step_sum % cfg["cluster"]["update_steps"] == 0:
            fn = run_kmeans if args.loss == "ProtoNCE" else run_hierarchical_clustering
            return fn(cfg, feat_loader, model, args.device)
        return cluster_result

    group = getattr(args, "dist_group", None)
    rank0 = int(getattr(args, "rank", 0)) == 0
    args.logdir = f"{args.logdir}/{args.loss}_{args.model}"
    if rank0:
        if os.path.isdir(args.logdir):
            shutil.rmtree(args.logdir)
        os.makedirs(args.logdir)
        os.makedirs(args.ckptdir, exist_ok=True)
    log = _writer(args.logdir) if rank0 else _NullWriter()

    st = TrainState(args, model, optimizer, init_step)
    if group is not None:
        st.set_process_group(group)
    total_steps = args.config["train"]["total_steps"]
    log_step = int(args.config["train"]["log_step"])
    if rank0:
        print("[Runner] - Start training")
    pbar = tqdm(initial=init_step, total=total_steps, dynamic_ncols=True, disable=not rank0)
    sampler = getattr(train_loader, "sampler", None)
    epoch = 0

    # LSTM heads on frozen BERT: the next micro-batch's BERT features are issued on
    # a side stream before this micro-batch's heads step (bert_extract_async), so
    # the two overlap; the loss values are those of the sequential loop.

    def _issue(b):
        if corpus is not None:
            idx, sel = b
            return idx, model.bert_extract_corpus_async(corpus, sel, idx.shape[0])
        idx, a, p = b
        return idx, model.bert_extract_texts_async(a, p, args.device)

    while st.step_sum < total_steps:
        if hasattr(sampler, "set_epoch"):  # DistributedSampler: a new permutation per pass
            sampler.set_epoch(epoch)
        epoch += 1
        if args.opt == "sgd":  # scheduler, once per pass (train.py:90-91)
            adjust_learning_rate(optimizer, st.step_sum, args.config)
        it = iter(train_loader)
        nxt = next(it, None)
        pending = _issue(nxt) if (prefetch and nxt is not None) else None
        while nxt is not None:
            batch, nxt = nxt, next(it, None)
            try:
                cluster_result = _maybe_recluster(cluster_result)
                if corpus is not None:
                    indexes = batch[0]
                else:
                    indexes, anchor_sample, positive_sample = batch
                if prefetch:
                    cur_idx, handle = pending
                    pending = _issue(nxt) if nxt is not None else None

                    def fwd(handle=handle, cur_idx=cur_idx):
                        a_feat, p_feat = model.features_ready(handle)
                        return model.forward_features(a_feat, p_feat, cluster_result,
                                                      cur_idx.view(-1))
                else:
                    def fwd(indexes=indexes, anchor_sample=anchor_sample,
                            positive_sample=positive_sample):
                        return model(anchor_sample, positive_sample, args.device,
                                     cluster_result, indexes)
                _, stepped = st.micro_batch(len(indexes), fwd, sync_loss=False)
                if stepped:
                    pbar.update(1)
                    if st.step_sum % log_step == 0:
                        # the per-micro-batch losses stay on the device until here (the
                        # reference syncs loss.item() every micro-batch, train.py:148;
                        # the logged mean is the same number)
                        loss_avg = float(np.mean([float(x) for x in st.loss_record]))
                        st.loss_record = []
                        grad_norm = float(st.grad_norm[0].item())
                        st.check_faults()
                        if rank0:
                            _log_and_save(log, pbar, model, optimizer, args, st.step_sum,
                                          loss_avg, grad_norm)
            except RuntimeError as e:
                if not any(m in str(e) for m in OOM_MARKERS):
                    raise
                print("[Runner] - HIP out of memory at step: ", st.step_sum)
                optimizer.zero_grad()
                torch.cuda.empty_cache()
            if st.step_sum >= total_steps:
                break

    pbar.close()
    log.close()
