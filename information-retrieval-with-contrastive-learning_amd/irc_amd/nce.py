"""In-batch NT-Xent / InfoNCE with the MoCo queue on the irc HIP kernels.

Reference: ``NCELoss._compute_info_loss`` (src/contrastor/contrastive_loss.py:56-93):
F = [q; k], S = F F^T with the diagonal dropped, positive column (i+N) mod 2N,
optional queue logits q.queue REUSED for the k-rows (.repeat(2, 1)), logits / T,
CrossEntropy(sum) with target 0, divided by 2.  With the momentum encoder (the
reference default) k is a no-grad key and the gradient flows into q only; with
``use_momentum: False`` the reference's k = seq2vec(positive) comes from
encoder_q WITH autograd (contrastive_module.py:82-83), so k receives
dk = G[N:] F + G[:, N:]^T F as well (S = F F^T; the queue logits use q only).

Fused path (the default for D in 32..256, D % 32 == 0: the LSTM head's 128):
csrc/nce_fused.hip streams 32-column tiles of [F ; queue^T] against 32-row blocks
on the exact-fp32 MFMA with an online row LSE, so S and LQ never land in HBM; the
backward recomputes each tile and folds it straight into dF.
Under data parallelism (info_nce_dist) each rank computes only its local pairs'
rows: the forward all-gathers q / k and then the rows' lse, the backward returns
d(global loss)/d(local rows) directly.

Unfused path (other widths, e.g. the trainable BERT's D = 768, and
IRC_NCE_FUSED=0): S = F F^T and LQ = q queue as exact-fp32 MFMA GEMMs, one row
kernel for log-sum-exp + NLL, a deterministic sum.  Backward: one elementwise
kernel for the softmax gradients (scaled on device by the upstream gradient -- no
host sync), then dq = G[:N] F + G[:, :N]^T F + GQ queue^T as three accumulating
GEMMs (and dk as two more when k requires grad).
"""
from __future__ import annotations

import os

import torch

from . import _lib, ops
from ._torch import ptr, stream_ptr, workspace


def fused_ok(D: int) -> bool:
    return os.environ.get("IRC_NCE_FUSED", "1") != "0" and 32 <= D <= 256 and D % 32 == 0


def _fused_ws(N, D, K, p_lo, p_hi, dev):
    nb = int(_lib.fn("irc_nce_fused_workspace")(N, D, K, p_lo, p_hi))
    return workspace(nb, dev, "nce_fused")


def _fused_fwd(F, qu, N, T, p_lo, p_hi, lse, loss_row):
    D = F.shape[1]
    K = qu.shape[1] if qu is not None else 0
    ws = _fused_ws(N, D, K, p_lo, p_hi, F.device)
    _lib.call("irc_nce_fused_fwd", ptr(F), ptr(qu), N, D, K, float(T), p_lo, p_hi, ptr(ws),
              ws.numel(), ptr(lse), ptr(loss_row), stream_ptr(F.device))


def _fused_bwd(F, qu, lse, N, T, g, p_lo, p_hi):
    D = F.shape[1]
    K = qu.shape[1] if qu is not None else 0
    ws = _fused_ws(N, D, K, p_lo, p_hi, F.device)
    rows = 2 * N if (p_lo == 0 and p_hi == N) else 2 * (p_hi - p_lo)
    dF = torch.empty((rows, D), dtype=torch.float32, device=F.device)
    _lib.call("irc_nce_fused_bwd", ptr(F), ptr(qu), ptr(lse), N, D, K, float(T), ptr(g), p_lo,
              p_hi, ptr(ws), ws.numel(), ptr(dF), stream_ptr(F.device))
    return dF


class _InfoNCEFused(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, queue, T):
        q = q.float().contiguous()
        k = k.float().contiguous()
        qu = queue.detach().float().clone(memory_format=torch.contiguous_format) \
            if queue is not None and queue.shape[1] > 0 else None
        N = q.shape[0]
        F = torch.cat([q, k], dim=0).contiguous()
        lse = torch.empty((2 * N,), dtype=torch.float32, device=q.device)
        loss_row = torch.empty_like(lse)
        _fused_fwd(F, qu, N, T, 0, N, lse, loss_row)
        ctx.save_for_backward(F, lse)
        ctx.queue, ctx.T, ctx.N = qu, T, N
        return ops.dsum(loss_row, 0.5)

    @staticmethod
    def backward(ctx, gloss):
        F, lse = ctx.saved_tensors
        N = ctx.N
        g = gloss.reshape(1).float().contiguous()
        dF = _fused_bwd(F, ctx.queue, lse, N, ctx.T, g, 0, N)
        ctx.queue = None
        return dF[:N], (dF[N:] if ctx.needs_input_grad[1] else None), None, None


class _InfoNCEDist(torch.autograd.Function):
    """Local-rows InfoNCE of a data-parallel rank: the global-batch loss over the
    all-gathered q / k (the value is all-reduced, identical on every rank), with
    this rank computing only its own pairs' rows and returning d(global loss)/d(its
    rows) -- no rank repeats another's logits."""

    @staticmethod
    def forward(ctx, q, k, queue, T, group):
        import torch.distributed as dist

        world, rank = dist.get_world_size(group), dist.get_rank(group)
        q = q.float().contiguous()
        k = k.float().contiguous()
        n = q.shape[0]
        qs = [torch.empty_like(q) for _ in range(world)]
        ks = [torch.empty_like(k) for _ in range(world)]
        dist.all_gather(qs, q, group=group)
        dist.all_gather(ks, k, group=group)
        N = n * world
        F = torch.cat(qs + ks, dim=0).contiguous()
        qu = queue.detach().float().clone(memory_format=torch.contiguous_format) \
            if queue is not None and queue.shape[1] > 0 else None
        p_lo, p_hi = rank * n, (rank + 1) * n
        lse = torch.empty((2 * N,), dtype=torch.float32, device=q.device)
        loss_row = torch.empty_like(lse)
        _fused_fwd(F, qu, N, T, p_lo, p_hi, lse, loss_row)
        mine = torch.cat([lse[p_lo:p_hi], lse[N + p_lo:N + p_hi]]).contiguous()
        parts = [torch.empty_like(mine) for _ in range(world)]
        dist.all_gather(parts, mine, group=group)
        lse = torch.cat([p[:n] for p in parts] + [p[n:] for p in parts]).contiguous()
        loss = ops.dsum(torch.cat([loss_row[p_lo:p_hi], loss_row[N + p_lo:N + p_hi]]).contiguous(),
                        0.5)
        dist.all_reduce(loss, group=group)
        ctx.save_for_backward(F, lse)
        ctx.queue, ctx.T, ctx.N, ctx.p = qu, T, N, (p_lo, p_hi)
        return loss

    @staticmethod
    def backward(ctx, gloss):
        F, lse = ctx.saved_tensors
        g = gloss.reshape(1).float().contiguous()
        p_lo, p_hi = ctx.p
        dF = _fused_bwd(F, ctx.queue, lse, ctx.N, ctx.T, g, p_lo, p_hi)
        n = p_hi - p_lo
        ctx.queue = None
        return dF[:n], (dF[n:] if ctx.needs_input_grad[1] else None), None, None, None


def info_nce_dist(q, k, queue, T, group):
    """The global-batch InfoNCE of a data-parallel group, each rank computing its own
    pairs' rows (fused path; needs the per-rank batch and the global batch to be
    multiples of 32 and D in 32..256)."""
    return _InfoNCEDist.apply(q, k, None if queue is None else queue.detach(), float(T), group)


def dist_fused_ok(n_local: int, D: int) -> bool:
    return fused_ok(D) and n_local % 32 == 0


def _logits(q, k, queue):
    F = torch.cat([q, k], dim=0).contiguous()  # [2N, D] (device copy)
    S = ops.gemm(F, F)  # F @ F.T, fp32 MFMA
    if queue is not None and queue.shape[1] > 0:
        LQ = ops.gemm(q, queue, b_is_nk=False)  # [N, K]
    else:
        LQ = None
    return F, S, LQ


class _InfoNCE(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, queue, T):
        q = q.float().contiguous()
        k = k.float().contiguous()
        # snapshot, as the reference's queue.clone().detach() (contrastive_loss.py:80):
        # the enqueue after forward() overwrites the live buffer before backward runs
        qu = queue.detach().float().clone(memory_format=torch.contiguous_format) \
            if queue is not None else None
        N = q.shape[0]
        F, S, LQ = _logits(q, k, qu)
        Kq = LQ.shape[1] if LQ is not None else 0
        lse, loss_row = ops.nce_lse(S, LQ, N, Kq, T)
        loss = ops.dsum(loss_row, 0.5)
        ctx.save_for_backward(F, S, lse)
        ctx.LQ, ctx.queue, ctx.T, ctx.N, ctx.Kq = LQ, qu, T, N, Kq
        return loss

    @staticmethod
    def backward(ctx, gloss):
        F, S, lse = ctx.saved_tensors
        N, Kq = ctx.N, ctx.Kq
        g = gloss.reshape(1).float().contiguous()
        GS, GQ = ops.nce_grads(S, ctx.LQ, lse, N, Kq, ctx.T, gscale=g)
        dq = ops.gemm(GS[:N], F, b_is_nk=False)  # sum_j G_nj F_j
        ops.gemm(GS[:, :N], F, trans_a=True, b_is_nk=False, out=dq, accumulate=True)  # G_jn F_j
        if Kq > 0:
            ops.gemm(GQ, ctx.queue, out=dq, accumulate=True)  # GQ @ queue^T
        dk = None
        if ctx.needs_input_grad[1]:
            dk = ops.gemm(GS[N:], F, b_is_nk=False)
            ops.gemm(GS[:, N:], F, trans_a=True, b_is_nk=False, out=dk, accumulate=True)
        ctx.LQ = ctx.queue = None
        return dq, dk, None, None


def info_nce(q, k, queue, T):
    """0-d fp32 loss tensor with autograd into q (and into k when k requires grad:
    the reference's use_momentum False configuration)."""
    qd = None if queue is None else queue.detach()
    if fused_ok(q.shape[1]):
        return _InfoNCEFused.apply(q, k, qd, float(T))
    return _InfoNCE.apply(q, k, qd, float(T))
