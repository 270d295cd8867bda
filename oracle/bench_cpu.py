"""CPU baselines for bench.py (TEST/BENCH INFRASTRUCTURE ONLY: the timed
reference-arithmetic leg, never a product path).

* train_step_baseline: one reference training micro-batch (frozen BERT forward,
  BiLSTM head q fwd+bwd and k fwd, NCELoss fwd+bwd, clip, Adam, momentum,
  enqueue) on the numpy oracle, for a bounded number of pairs.
* scan_baseline: the oracle's fp32 BLAS scan + exact top-k.
"""
from __future__ import annotations

import time

import numpy as np

from . import irc_oracle as O


def train_step_baseline(bert_w, nl_bert, nheads, head_p, nlayers, queue, ids, mask, T=0.05,
                        lr=2.5e-4, budget_s=10.0):
    """Repeats one micro-batch of len(ids)//2 pairs until budget_s; returns pairs/s."""
    n = ids.shape[0] // 2
    hp = {k: v.astype(np.float32) for k, v in head_p.items()}
    kp = {k: v.copy() for k, v in hp.items()}
    m_state = {k: np.zeros_like(v) for k, v in hp.items()}
    v_state = {k: np.zeros_like(v) for k, v in hp.items()}
    reps, t0 = 0, time.perf_counter()
    while True:
        feats = O.bert_forward(ids, mask, bert_w, nl_bert, nheads)
        eq, cache = O.seq2vec(feats[:n], hp, nlayers)
        ek, _ = O.seq2vec(feats[n:], kp, nlayers)
        loss, dq = O.nce_info_loss(eq, ek, queue, T)
        grads = O.seq2vec_bwd(dq, hp, cache, nlayers)
        O.clip_grad_norm(grads, 1.0)
        for k in hp:
            hp[k], m_state[k], v_state[k] = O.adam_step(hp[k], grads[k], m_state[k], v_state[k],
                                                        reps + 1, lr, 0.9, 0.999)
            kp[k] = O.momentum_update(kp[k], hp[k], 0.9)
        queue, _ = O.dequeue_and_enqueue(queue, 0, ek)
        reps += 1
        if time.perf_counter() - t0 >= budget_s:
            break
    dt = time.perf_counter() - t0
    return n * reps / dt, reps


def scan_baseline(q, d, k, budget_s=10.0):
    O.scan_topk_fast_f32(q[:8], d[:20000], k)  # warm BLAS
    reps, t0 = 0, time.perf_counter()
    while True:
        O.scan_topk_fast_f32(q, d, k)
        reps += 1
        if time.perf_counter() - t0 >= budget_s:
            break
    return q.shape[0] * reps / (time.perf_counter() - t0), reps
