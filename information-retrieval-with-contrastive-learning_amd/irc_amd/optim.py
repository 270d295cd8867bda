"""Fused optimizers over the flat fp32 parameter buffer of the encoder head.

Reference semantics (src/model.py:44-58, src/train.py:150-169): Adam(lr, betas)
(eps 1e-8, no weight decay) or SGD(lr, momentum, weight_decay) over
model.parameters(); parameters without a gradient (frozen BERT, the momentum
encoder) are skipped, so only encoder_q moves.  ``param_groups[0]["lr"]`` is live
(the reference's cosine adjust_learning_rate writes it, src/train.py:18-23).  clip_grad_norm_(max_norm) is fused into the step: the global norm and
the clip coefficient are computed on the device and applied inside the update
kernel (no host sync).  The optimizer follows the module across .to(device):
it reads head.flat / head.flat_grad at step time and keeps its moments on the
same device.
"""
from __future__ import annotations

import math

import torch

from . import ops


class _LiveLR:
    """``lr`` backed by ``param_groups[0]["lr"]``, as torch.optim exposes it."""

    @property
    def lr(self):
        return float(self.param_groups[0]["lr"])

    @lr.setter
    def lr(self, v):
        self.param_groups[0]["lr"] = float(v)


class FusedAdam(_LiveLR):
    def __init__(self, head, lr=2.5e-4, betas=(0.9, 0.999), eps=1e-8):
        self.head = head
        self.param_groups = [{"lr": float(lr)}]
        self.b1, self.b2 = (float(b) for b in betas)
        self.eps = float(eps)
        self.step_count = 0
        self.exp_avg = None
        self.exp_avg_sq = None
        self.last_norm = None  # device tensor [grad norm, clip coef] of the last step

    def _moments(self):
        flat = self.head.flat
        if self.exp_avg is None:
            self.exp_avg = torch.zeros(flat.shape, dtype=torch.float32, device=flat.device)
            self.exp_avg_sq = torch.zeros_like(self.exp_avg)
        elif self.exp_avg.device != flat.device:
            self.to(flat.device)
        return self.exp_avg, self.exp_avg_sq

    def to(self, device):
        if self.exp_avg is not None:
            self.exp_avg = self.exp_avg.to(device)
            self.exp_avg_sq = self.exp_avg_sq.to(device)
        return self

    def clip_and_step(self, max_norm: float | None = None, faults=()):
        """clip_grad_norm_(max_norm) (if given) + one Adam step; returns the device
        tensor [norm, coef, gate, -].  ``faults``: device fault words (the cluster
        recurrences' sticky timeout words); when one is set the update is skipped on
        the device (coef[2] = 1) -- parameters and moments stay as they were."""
        g = self.head.flat_grad
        m, v = self._moments()
        coef = ops.grad_norm_clip(g, max_norm if max_norm is not None else float("inf"))
        faults = [f for f in faults if f is not None]
        if faults:
            ops.fault_gate(coef, *faults)
            if max_norm is None:
                max_norm = float("inf")  # the kernel reads the gate from coef
        self.last_norm = coef
        self.step_count += 1
        t = self.step_count
        bc1 = 1 - self.b1 ** t
        bc2 = 1 - self.b2 ** t
        shadow = self.head.shadow_buffer() if hasattr(self.head, "shadow_buffer") else None
        if shadow is not None:
            # trainable encoder: the bf16 MFMA-operand shadow is rewritten in the same pass
            ops.adam_step_bf16(self.head.flat.detach(), g, m, v,
                               coef if max_norm is not None else None, self.b1, self.b2,
                               self.lr / bc1, math.sqrt(bc2), self.eps, shadow)
            self.head.after_update(True)
        else:
            ops.adam_step(self.head.flat.detach(), g, m, v,
                          coef if max_norm is not None else None, self.b1, self.b2,
                          self.lr / bc1, math.sqrt(bc2), self.eps)
            if hasattr(self.head, "after_update"):
                self.head.after_update(False)
        return coef

    def step(self):
        return self.clip_and_step(None)

    def zero_grad(self, set_to_none: bool = False):
        self.head.flat_grad.zero_()

    # torch.optim-style checkpoint dict (flat state under parameter index 0)
    def state_dict(self):
        m, v = self._moments()
        return {"state": {0: {"step": torch.tensor(float(self.step_count)), "exp_avg": m,
                              "exp_avg_sq": v}},
                "param_groups": [{"lr": self.lr, "betas": (self.b1, self.b2), "eps": self.eps,
                                  "weight_decay": 0, "amsgrad": False, "params": [0]}]}

    def load_state_dict(self, sd):  # noqa: C901
        """Accepts this class's dict, or a reference torch.optim.Adam dict whose
        parameter indices 0..n-1 are encoder_q's parameters in nn.LSTM order."""
        m, v = self._moments()
        st = sd.get("state", {})
        specs = self.head.specs
        if 0 in st and st[0]["exp_avg"].numel() == m.numel():
            self.step_count = int(float(st[0]["step"]))
            m.copy_(st[0]["exp_avg"])
            v.copy_(st[0]["exp_avg_sq"])
        elif st:
            for i, (name, shape) in enumerate(specs):
                if i in st:
                    self.head.view(name, m).copy_(st[i]["exp_avg"].reshape(shape))
                    self.head.view(name, v).copy_(st[i]["exp_avg_sq"].reshape(shape))
                    self.step_count = int(float(st[i]["step"]))
        pg = sd["param_groups"][0]
        self.lr = float(pg["lr"])
        self.b1, self.b2 = (float(b) for b in pg["betas"])
        self.eps = float(pg.get("eps", self.eps))



class FusedSGD(_LiveLR):
    """torch.optim.SGD(params, lr, momentum, weight_decay) (dampening 0, nesterov
    False; src/model.py:45-51) as one fused launch over the flat buffer, with
    clip_grad_norm_ and the fault gate fused like FusedAdam.  The momentum buffer is
    created by the first step (torch: ``buf = d.clone()``)."""

    def __init__(self, head, lr=3e-4, momentum=0.9, weight_decay=1e-4):
        self.head = head
        self.param_groups = [{"lr": float(lr)}]
        self.momentum = float(momentum)
        self.weight_decay = float(weight_decay)
        self.buf = None
        self.started = False  # the momentum buffer holds a first step
        self.last_norm = None

    def _buffer(self):
        flat = self.head.flat
        if self.buf is None:
            self.buf = torch.zeros(flat.shape, dtype=torch.float32, device=flat.device)
        elif self.buf.device != flat.device:
            self.to(flat.device)
        return self.buf

    def to(self, device):
        if self.buf is not None:
            self.buf = self.buf.to(device)
        return self

    def clip_and_step(self, max_norm: float | None = None, faults=()):
        g = self.head.flat_grad
        buf = self._buffer()
        coef = ops.grad_norm_clip(g, max_norm if max_norm is not None else float("inf"))
        faults = [f for f in faults if f is not None]
        if faults:
            ops.fault_gate(coef, *faults)
        self.last_norm = coef
        shadow = self.head.shadow_buffer() if hasattr(self.head, "shadow_buffer") else None
        # unclipped and ungated (FusedAdam's rule): the kernel reads no coefficient, so a
        # non-finite norm cannot reach the update through inf / inf
        use = coef if (max_norm is not None or faults) else None
        ops.sgd_step(self.head.flat.detach(), g, buf, use, self.lr, self.momentum,
                     self.weight_decay, not self.started, shadow)
        # a gated first step leaves the zero buffer unwritten: the next step's
        # mom * 0 + d is then exactly torch's first-step d, so no host check is needed
        self.started = True
        if hasattr(self.head, "after_update"):
            self.head.after_update(shadow is not None)
        return coef

    def step(self):
        return self.clip_and_step(None)

    def zero_grad(self, set_to_none: bool = False):
        self.head.flat_grad.zero_()

    def state_dict(self):
        st = {0: {"momentum_buffer": self._buffer()}} if self.started else {}
        return {"state": st,
                "param_groups": [{"lr": self.lr, "momentum": self.momentum, "dampening": 0,
                                  "weight_decay": self.weight_decay, "nesterov": False,
                                  "maximize": False, "params": [0]}]}

    def load_state_dict(self, sd):
        """This class's dict, or a reference torch.optim.SGD dict whose parameter
        indices 0..n-1 are encoder_q's parameters in nn.LSTM order."""
        buf = self._buffer()
        st = sd.get("state", {})
        if 0 in st and st[0].get("momentum_buffer") is not None and \
                st[0]["momentum_buffer"].numel() == buf.numel():
            buf.copy_(st[0]["momentum_buffer"])
            self.started = True
        elif st:
            for i, (name, shape) in enumerate(self.head.specs):
                if i in st and st[i].get("momentum_buffer") is not None:
                    self.head.view(name, buf).copy_(st[i]["momentum_buffer"].reshape(shape))
                    self.started = True
        pg = sd["param_groups"][0]
        self.lr = float(pg["lr"])
        self.momentum = float(pg.get("momentum", self.momentum))
        self.weight_decay = float(pg.get("weight_decay", self.weight_decay))
