"""torch-CPU restatement of the reference training step and dense scan (BENCH
INFRASTRUCTURE ONLY: the timed `cpu_baseline` legs of bench.py, never a product
path; SURVEY.md 8d asks for "the same torch CPU ops as the reference").

Training step = src/train.py:133-175 on the reference's modules:
  * frozen BERT forward (contrastive_module.py:36-41 -> HF BertModel math:
    embeddings + LN, per layer softmax(QK^T/sqrt(dh) + mask) V -> dense +
    residual -> LN -> erf-GELU FFN + residual -> LN), torch.no_grad;
  * encoder_q = nn.LSTM(768, 256, 3, batch_first, bidirectional) + Linear
    (src/model.py:7-41) with autograd, encoder_k the same under no_grad;
    seq2vec = mean over all L + F.normalize (contrastive_module.py:102-112);
  * NCELoss._compute_info_loss with the queue (contrastive_loss.py:56-93);
  * clip_grad_norm_(1.0), torch.optim.Adam, momentum update, enqueue
    (train.py:150-169, contrastive_module.py:43-68).
Dense scan = q @ d.T in 64k-doc chunks with a running exact top-k merge.
"""
from __future__ import annotations

import math
import time

import torch
import torch.nn as nn
import torch.nn.functional as F


def bert_forward(P, ids, mask, n_layers, heads, eps=1e-12):
    B, L = ids.shape
    x = F.embedding(ids, P["embeddings.word_embeddings.weight"])
    x = x + P["embeddings.token_type_embeddings.weight"][0]
    x = x + P["embeddings.position_embeddings.weight"][:L][None]
    H = x.shape[-1]
    x = F.layer_norm(x, (H,), P["embeddings.LayerNorm.weight"], P["embeddings.LayerNorm.bias"], eps)
    dh = H // heads
    bias = (1.0 - mask.float())[:, None, None, :] * torch.finfo(torch.float32).min
    for l in range(n_layers):
        p = f"encoder.layer.{l}."

        def lin(t, n):
            return F.linear(t, P[p + n + ".weight"], P[p + n + ".bias"])

        q, k, v = (lin(x, f"attention.self.{n}").view(B, L, heads, dh).transpose(1, 2)
                   for n in ("query", "key", "value"))
        s = q @ k.transpose(-1, -2) / math.sqrt(dh) + bias
        ctx = (torch.softmax(s, -1) @ v).transpose(1, 2).reshape(B, L, H)
        a = F.layer_norm(lin(ctx, "attention.output.dense") + x, (H,),
                         P[p + "attention.output.LayerNorm.weight"],
                         P[p + "attention.output.LayerNorm.bias"], eps)
        f = lin(F.gelu(lin(a, "intermediate.dense")), "output.dense")
        x = F.layer_norm(f + a, (H,), P[p + "output.LayerNorm.weight"],
                         P[p + "output.LayerNorm.bias"], eps)
    return x


class Head(nn.Module):
    """src/model.py:7-41: nn.LSTM + Linear (+ Identity)."""

    def __init__(self, inp, hid, layers, out):
        super().__init__()
        self.lstm = nn.LSTM(inp, hid, layers, batch_first=True, bidirectional=True)
        self.scaling_layer = nn.Sequential(nn.Linear(2 * hid, out), nn.Identity())

    def forward(self, features):
        return self.scaling_layer(self.lstm(features)[0])


def nce_loss(q, k, queue, T):
    """contrastive_loss.py:56-93 (the reference's masking and .repeat(2, 1))."""
    n = len(q)
    labels = torch.cat([torch.arange(n) for _ in range(2)], dim=0)
    labels = (labels.unsqueeze(0) == labels.unsqueeze(1)).float()
    feats = torch.cat([q, k], dim=0)
    sim = feats @ feats.T
    eye = torch.eye(labels.shape[0], dtype=torch.bool)
    labels = labels[~eye].view(labels.shape[0], -1)
    sim = sim[~eye].view(sim.shape[0], -1)
    pos = sim[labels.bool()].view(labels.shape[0], -1)
    neg = sim[~labels.bool()].view(sim.shape[0], -1)
    logits = [pos, neg]
    if queue is not None:
        logits.append(torch.einsum("nc,ck->nk", [q, queue.clone().detach()]).repeat(2, 1))
    logits = torch.cat(logits, dim=1) / T
    tgt = torch.zeros(logits.shape[0], dtype=torch.long)
    return F.cross_entropy(logits, tgt, reduction="sum") / 2


def train_step_baseline(bert_w, n_layers, heads, head_state, head_dims, queue, ids, mask,
                        steps=2, T=0.05, lr=2.5e-4, mom=0.9):
    """Times `steps` reference training steps of len(ids)//2 pairs (after one
    warm-up micro-batch of 8 pairs); returns (pairs/s, seconds per step)."""
    P = {k: torch.as_tensor(v, dtype=torch.float32) for k, v in bert_w.items()}
    hq = Head(*head_dims)
    hq.load_state_dict({k: torch.as_tensor(v) for k, v in head_state.items()})
    hk = Head(*head_dims)
    hk.load_state_dict(hq.state_dict())
    for p in hk.parameters():
        p.requires_grad_(False)
    opt = torch.optim.Adam(hq.parameters(), lr=lr, betas=(0.9, 0.999))
    queue = torch.as_tensor(queue, dtype=torch.float32).clone()
    ptr = 0
    ids, mask = torch.as_tensor(ids), torch.as_tensor(mask)
    n = ids.shape[0] // 2

    def step(ids, mask, nb):
        nonlocal queue, ptr
        with torch.no_grad():
            feats = bert_forward(P, ids, mask, n_layers, heads)
        eq = F.normalize(hq(feats[:nb]).mean(dim=1))
        with torch.no_grad():
            ek = F.normalize(hk(feats[nb:]).mean(dim=1))
        loss = nce_loss(eq, ek, queue, T) / nb
        loss.backward()
        torch.nn.utils.clip_grad_norm_(list(hq.parameters()), 1.0)
        opt.step()
        with torch.no_grad():
            for pk, pq in zip(hk.parameters(), hq.parameters()):
                pk.data = pk.data * mom + pq.data * (1.0 - mom)
            if queue.shape[1] % nb == 0:
                queue[:, ptr:ptr + nb] = ek.T
                ptr = (ptr + nb) % queue.shape[1]
        opt.zero_grad()

    w = 4  # warm-up: 4 pairs
    step(torch.cat([ids[:w], ids[n:n + w]]), torch.cat([mask[:w], mask[n:n + w]]), w)
    t0 = time.perf_counter()
    for _ in range(steps):
        step(ids, mask, n)
    dt = time.perf_counter() - t0
    return n * steps / dt, dt / steps


def scan_baseline(q, d, k, budget_s=10.0, chunk=65536):
    """q [Q, D], d [N, D] fp32 CPU tensors: exact top-k of q @ d.T over 64k-doc
    chunks with a running merge; repeats until budget_s; returns (queries/s, reps)."""
    def once():
        best_s = torch.full((q.shape[0], k), float("-inf"))
        best_i = torch.zeros((q.shape[0], k), dtype=torch.long)
        for c0 in range(0, d.shape[0], chunk):
            s = q @ d[c0:c0 + chunk].T
            ts, ti = torch.topk(s, min(k, s.shape[1]), dim=1)
            cs = torch.cat([best_s, ts], 1)
            ci = torch.cat([best_i, ti + c0], 1)
            best_s, o = torch.topk(cs, k, dim=1)
            best_i = torch.gather(ci, 1, o)
        return best_s, best_i

    once()
    reps, t0 = 0, time.perf_counter()
    while True:
        once()
        reps += 1
        if time.perf_counter() - t0 >= budget_s:
            break
    return q.shape[0] * reps / (time.perf_counter() - t0), reps
