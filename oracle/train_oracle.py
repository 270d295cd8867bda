"""CPU oracle for one full reference training step sequence (TEST INFRASTRUCTURE ONLY).

Restates src/train.py:86-175 (micro-batch loop, /acml_batch_size, gradient
accumulation, clip_grad_norm_(1.0), Adam or SGD with the per-pass cosine learning
rate, momentum update, queue switch-on at queue_start_steps, the head activation)
on top of the numpy pieces in ``irc_oracle``.  Used by the
CPU tests (pinned against tests/golden/train_traj.npz, which was produced by
running the reference's own ``train()``) and by bench.py's cpu_baseline leg.
"""
from __future__ import annotations

import numpy as np

from . import irc_oracle as O


def split_state(state: dict, prefix: str) -> dict:
    n = len(prefix)
    return {k[n:]: np.asarray(v, np.float64) for k, v in state.items() if k.startswith(prefix)}


def run_trajectory(fx: dict):
    """Replay the recorded micro-batches of train_traj.npz through the oracle.

    Returns (per-micro-batch raw losses, final state dict of encoder_q/encoder_k/queue).
    """
    init = {k[5:]: fx[k] for k in fx if k.startswith("init_")}
    bert_w = {k[len("bert_model."):]: init[k] for k in init if k.startswith("bert_model.")}
    nl_bert = 1 + max(int(k.split(".")[2]) for k in bert_w if k.startswith("encoder.layer."))
    hid = bert_w["embeddings.word_embeddings.weight"].shape[1]
    nheads = 2
    in_dim, hsz, nlayers, outd = (int(x) for x in fx["lstm_cfg"])
    T, mom, qsize, qstart = fx["loss_cfg"]
    use_mom = int(fx["use_momentum"]) if "use_momentum" in fx else 1
    B, acml, total, log_step = (int(x) for x in fx["train_cfg"])
    lr, b1, b2, clip = fx["adam"]
    act = str(fx["activation"]) if "activation" in fx else "Identity"
    sgd = fx["sgd"] if "sgd" in fx else None  # [lr0, momentum, weight_decay, clip]
    if sgd is not None:
        clip = sgd[3]
    # micro-batch index -> step count at which adjust_learning_rate ran (once per pass)
    lr_at = {int(i): int(st) for i, st in fx["sgd_epoch_mb"]} if sgd is not None else {}
    sgd_lr = float(sgd[0]) if sgd is not None else 0.0
    bufs = {k: None for k in split_state(init, "encoder_q.")}
    pq = split_state(init, "encoder_q.")
    pk = split_state(init, "encoder_k.")
    queue = np.asarray(init["queue"], np.float64)
    ptr = int(init["queue_ptr"][0])
    m_state = {k: np.zeros_like(v) for k, v in pq.items()}
    v_state = {k: np.zeros_like(v) for k, v in pq.items()}
    adam_t = 0
    grads = {k: np.zeros_like(v) for k, v in pq.items()}
    losses = []
    step, bs = 0, 0
    add_q = False
    for i in range(int(fx["mb_len"].shape[0])):
        if i in lr_at:
            sgd_lr = O.cosine_lr(float(sgd[0]), lr_at[i], total)
        L = int(fx["mb_len"][i])
        nb = int(fx["mb_B"][i])
        ids = fx["mb_ids"][i, :2 * nb, :L]
        mask = fx["mb_mask"][i, :2 * nb, :L]
        if step >= qstart and not add_q:
            add_q = True
        feats = O.bert_forward(ids, mask, bert_w, nl_bert, nheads).astype(np.float64)
        a, p = feats[:nb], feats[nb:]
        emb_q, cq = O.seq2vec(a, pq, nlayers, act=act)
        if use_mom:
            emb_k, _ = O.seq2vec(p, pk, nlayers, act=act)
            loss, dq = O.nce_info_loss(emb_q, emb_k, queue if add_q else None, float(T))
        else:  # keys through encoder_q with autograd (contrastive_module.py:82-83)
            emb_k, ck = O.seq2vec(p, pq, nlayers, act=act)
            loss, dq, dk = O.nce_info_loss(emb_q, emb_k, queue if add_q else None, float(T),
                                           want_dk=True)
            gk = O.seq2vec_bwd(dk / acml, pq, ck, nlayers)
            for k in grads:
                grads[k] += gk[k]
        losses.append(loss)
        g = O.seq2vec_bwd(dq / acml, pq, cq, nlayers)
        for k in grads:
            grads[k] += g[k]
        queue, ptr = O.dequeue_and_enqueue(queue, ptr, emb_k)
        bs += nb
        if bs == acml or nb != B:
            O.clip_grad_norm(grads, float(clip))
            adam_t += 1
            for k in pq:
                if sgd is not None:
                    pq[k], bufs[k] = O.sgd_step(pq[k], grads[k], bufs[k], sgd_lr,
                                                float(sgd[1]), float(sgd[2]))
                else:
                    pq[k], m_state[k], v_state[k] = O.adam_step(pq[k], grads[k], m_state[k],
                                                                v_state[k], adam_t, float(lr),
                                                                float(b1), float(b2))
            for k in pk:
                pk[k] = O.momentum_update(pk[k], pq[k], float(mom))
            grads = {k: np.zeros_like(v) for k, v in pq.items()}
            step += 1
            bs = 0
        if step >= total:
            break
    final = {"queue": queue, "queue_ptr": np.array([ptr])}
    final.update({"encoder_q." + k: v for k, v in pq.items()})
    final.update({"encoder_k." + k: v for k, v in pk.items()})
    return np.array(losses), final
