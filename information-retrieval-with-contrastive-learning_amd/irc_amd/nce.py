"""In-batch NT-Xent / InfoNCE with the MoCo queue on the irc HIP kernels.

Reference: ``NCELoss._compute_info_loss`` (src/contrastor/contrastive_loss.py:56-93):
F = [q; k], S = F F^T with the diagonal dropped, positive column (i+N) mod 2N,
optional queue logits q.queue REUSED for the k-rows (.repeat(2, 1)), logits / T,
CrossEntropy(sum) with target 0, divided by 2.  With the momentum encoder (the
reference default) k is a no-grad key and the gradient flows into q only; with
``use_momentum: False`` the reference's k = seq2vec(positive) comes from
encoder_q WITH autograd (contrastive_module.py:82-83), so k receives
dk = G[N:] F + G[:, N:]^T F as well (S = F F^T; the queue logits use q only).

Forward: S = F F^T and LQ = q queue as exact-fp32 MFMA GEMMs, one row kernel
for log-sum-exp + NLL, a deterministic sum.  Backward: one elementwise kernel
for the softmax gradients (scaled on device by the upstream gradient -- no host
sync), then dq = G[:N] F + G[:, :N]^T F + GQ queue^T as three accumulating GEMMs (and
dk as two more when k requires grad).
"""
from __future__ import annotations

import torch

from . import ops


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
    return _InfoNCE.apply(q, k, None if queue is None else queue.detach(), float(T))
