"""Data-parallel plumbing for the training step: one process per
GPU, RCCL ("nccl") on MI355X, gloo on CPU for the tests.

Global in-batch negatives: each rank encodes its own B/P pairs, the embeddings
are all-gathered (q with autograd, k without), and every rank evaluates the SAME
single-GPU InfoNCE over the global batch of B pairs (contrastive_loss.py:56-93
with N = B).  Because the loss is identical on every rank, the gradient reaching
the gathered q is identical too, so the backward of the gather is just the
local slice -- no collective.  Each rank then back-propagates its slice through
its own head and the flat head gradients are summed with one all-reduce, which
yields exactly d(global loss)/d(theta).  The key encoder and the queue are
replicated: every rank enqueues the same gathered keys.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def world_of(group) -> int:
    if group is None or not dist.is_initialized():
        return 1
    return dist.get_world_size(group)


class _GatherRows(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, group):
        world = dist.get_world_size(group)
        rank = dist.get_rank(group)
        x = x.contiguous()
        parts = [torch.empty_like(x) for _ in range(world)]
        dist.all_gather(parts, x, group=group)
        ctx.rank, ctx.n = rank, x.shape[0]
        return torch.cat(parts, dim=0)

    @staticmethod
    def backward(ctx, g):
        return g[ctx.rank * ctx.n:(ctx.rank + 1) * ctx.n], None


def gather_rows(x: torch.Tensor, group) -> torch.Tensor:
    """Concatenate every rank's ``x`` (equal row counts) along dim 0, in rank
    order.  Differentiable: the gradient of the result flows back to this rank's
    rows (valid when every rank computes the same function of the result)."""
    if world_of(group) == 1:
        return x
    if x.requires_grad:
        return _GatherRows.apply(x, group)
    with torch.no_grad():
        return _GatherRows.forward(_Ctx(), x, group)


class _Ctx:  # stand-in ctx for the no-grad gather
    pass


def all_reduce_sum_(t: torch.Tensor, group) -> None:
    if world_of(group) > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
