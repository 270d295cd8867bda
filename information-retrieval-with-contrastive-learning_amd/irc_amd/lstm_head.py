"""BiLSTM + Linear encoder head and its seq2vec tail on the irc HIP kernels.

Reference: ``LSTM`` in src/model.py:7-41 (nn.LSTM(input, hidden, num_layers,
batch_first, bidirectional) -> Linear(2*hidden -> output) -> Identity) and
``seq2vec`` in src/contrastor/contrastive_module.py:102-112 (mean over ALL L
positions, PAD included, then F.normalize).

Parameters live in ONE flat fp32 buffer (16-float aligned slices) with
nn.LSTM-named views, so the optimizer, clipping and the momentum update are
single fused launches over the buffer, and ``state_dict()`` keeps the
reference's keys (``lstm.weight_ih_l0`` ... ``scaling_layer.0.bias``).
Gradients go to a parallel flat buffer (``flat_grad``); each named parameter's
``.grad`` is a view of it.

Forward (per layer): xp = x W_ih^T + (b_ih + b_hh) for both directions in one
GEMM -> recurrence kernel -> next layer.  In bf16 mode at H = 256 the recurrence
runs on MFMA (csrc/lstm_mfma.hip; W_ih packed so each unit's four gates are
adjacent), otherwise on the VALU kernels (csrc/lstm.hip).  Head: mean over positions of the top
layer, then the Linear (mean and Linear commute exactly in real arithmetic),
then L2 normalisation.  Backward: l2norm bwd -> Linear grads -> broadcast /L ->
per layer BPTT kernel -> weight-gradient GEMMs over all (b, t).
"""
from __future__ import annotations

import math
import os

import torch
import torch.nn as nn

from . import ops
from ._torch import side_stream
from .precision import compute_dtype

ALIGN = 16  # floats (64 B) per slice start: GEMM operands need 16-byte alignment


def lstm_param_specs(input_size, hidden, num_layers, bidirectional, output_size):
    """(name, shape) in nn.LSTM + Linear named_parameters() order."""
    specs = []
    dirs = ["", "_reverse"] if bidirectional else [""]
    for l in range(num_layers):
        in_l = input_size if l == 0 else hidden * len(dirs)
        for d in dirs:
            specs += [(f"lstm.weight_ih_l{l}{d}", (4 * hidden, in_l)),
                      (f"lstm.weight_hh_l{l}{d}", (4 * hidden, hidden)),
                      (f"lstm.bias_ih_l{l}{d}", (4 * hidden,)),
                      (f"lstm.bias_hh_l{l}{d}", (4 * hidden,))]
    specs += [("scaling_layer.0.weight", (output_size, hidden * len(dirs))),
              ("scaling_layer.0.bias", (output_size,))]
    return specs


def _layout(specs):
    """Flat offsets: per layer [W_ih fwd | W_ih rev] and [W_hh fwd | W_hh rev] are
    adjacent so both directions are one GEMM operand / one kernel argument."""
    order = []
    names = [n for n, _ in specs]
    shapes = dict(specs)
    layers = sorted({int(n.split("_l")[1].split("_")[0].rstrip("_reverse")) for n in names
                     if n.startswith("lstm.")})
    for l in layers:
        for kind in ("weight_ih", "weight_hh", "bias_ih", "bias_hh"):
            for d in ("", "_reverse"):
                n = f"lstm.{kind}_l{l}{d}"
                if n in shapes:
                    order.append(n)
    order += ["scaling_layer.0.weight", "scaling_layer.0.bias"]
    offs, o = {}, 0
    for n in order:
        numel = math.prod(shapes[n])
        if not (n.startswith("lstm.") and n.endswith("_reverse")):
            o = (o + ALIGN - 1) // ALIGN * ALIGN
        offs[n] = o
        o += numel
    total = (o + ALIGN - 1) // ALIGN * ALIGN
    return offs, total



def _cu_count(dev) -> int:
    return torch.cuda.get_device_properties(dev).multi_processor_count


# Rows of the input projection past its last whole wave (256 x 256 output tiles on all CUs)
# run beside it on a side stream instead of as a nearly empty last wave of the same launch
# (B L = 256 x 65 = 16640 rows: 2 waves of 520 tiles + 8; IRC_HEAD_SPLIT=0: off)
_HEAD_SPLIT = os.environ.get("IRC_HEAD_SPLIT", "1") != "0"

# Split-K cap (256 x 256-tile blocks) of the MFMA-path BPTT's GEMMs: the weight gradients on
# their side stream and dX (irc_gemm_ex max_blocks; 0 = one full wave).  They run beside the
# encoder forward, whose GEMMs set the step: half a wave of blocks is slower alone but leaves
# it CUs (profiles/r05_zc_split_cap_ab.txt; a cap of 64 measured slower)
SPLIT_MAX_BLOCKS = int(os.environ.get("IRC_HEAD_SPLIT_BLOCKS", "128"))


def _gemm_rows_split(x, w, b):
    """xp = x . w^T + b (fp32 out) -- as one GEMM, or, when M sits just above a whole
    number of waves, as the whole-wave rows here plus the rest on a side stream."""
    M, N = x.shape[0], w.shape[0]
    ct = (N + 255) // 256
    ncu = _cu_count(x.device) if (_HEAD_SPLIT and x.is_cuda) else 0
    rpw = 256 * (ncu // ct) if ct and ncu % ct == 0 else 0  # rows per wave of tiles
    full = M // rpw * rpw if rpw else 0
    if full == 0 or M == full or M - full > rpw // 4:
        return ops.gemm(x, w, bias=b, epilogue=ops.EPI_BIAS, out_dtype=torch.float32)
    out = torch.empty((M, N), dtype=torch.float32, device=x.device)
    cur = torch.cuda.current_stream(x.device)
    side = side_stream(x.device, "head_tail")
    side.wait_stream(cur)
    with torch.cuda.stream(side):
        ops.gemm(x[full:], w, bias=b, epilogue=ops.EPI_BIAS, out=out[full:])
    for t in (x, w, b, out):
        t.record_stream(side)
    ops.gemm(x[:full], w, bias=b, epilogue=ops.EPI_BIAS, out=out[:full])
    cur.wait_stream(side)
    return out

class LSTMHead(nn.Module):
    """Drop-in for the reference ``LSTM`` module (same config keys and names)."""

    def __init__(self, config, init: bool = True, **kwargs):
        super().__init__()
        c = config["model"]["LSTM"]
        self.input_size = int(c["input_size"])
        self.hidden = int(c["hidden_size"])
        self.num_layers = int(c["num_layers"])
        self.bidirectional = bool(c["bidirectional"])
        self.output_size = int(c["output_size"])
        act = c.get("activation", "Identity")
        if act not in ops.ACTIVATIONS:
            raise ValueError(f"activation {act!r}: supported nn activations are "
                             f"{sorted(ops.ACTIVATIONS)}")
        self.activation = act
        self.act_kind = ops.ACTIVATIONS[act]
        self.ndir = 2 if self.bidirectional else 1
        self.specs = lstm_param_specs(self.input_size, self.hidden, self.num_layers,
                                      self.bidirectional, self.output_size)
        self.offsets, self.numel_flat = _layout(self.specs)
        self.flat = nn.Parameter(torch.zeros(self.numel_flat), requires_grad=True)
        self.register_buffer("flat_grad", torch.zeros(self.numel_flat), persistent=False)
        # sticky device word: OR of every cluster recurrence's timeout word since the
        # last check_fault() (the calls also NaN-poison their outputs on a timeout)
        self.register_buffer("coop_fault", torch.zeros(1, dtype=torch.int32), persistent=False)
        if init:
            self.reset_parameters()

    # ---- parameter plumbing ----
    def view(self, name, buf=None):
        buf = self.flat if buf is None else buf
        shape = dict(self.specs)[name]
        o = self.offsets[name]
        return buf.detach()[o:o + math.prod(shape)].view(shape)

    def named_flat_params(self):
        return [(n, self.view(n)) for n, _ in self.specs]

    def _save_to_state_dict(self, destination, prefix, keep_vars):
        # reference key layout: one entry per nn.LSTM / Linear parameter
        for n, _ in self.specs:
            destination[prefix + n] = self.view(n).clone()

    def _load_from_state_dict(self, state_dict, prefix, local_metadata, strict, missing_keys,
                              unexpected_keys, error_msgs):
        with torch.no_grad():
            for n, shape in self.specs:
                k = prefix + n
                if k in state_dict:
                    self.view(n).copy_(state_dict[k].reshape(shape))
                elif strict:
                    missing_keys.append(k)
        for k in state_dict:  # the head has no child modules: every prefixed key is ours
            if k.startswith(prefix) and k[len(prefix):] not in self.offsets and strict:
                unexpected_keys.append(k)

    @torch.no_grad()
    def reset_parameters(self):
        """nn.LSTM default init then the reference's init_weights (model.py:29-36):
        xavier_uniform_ (weight_ih*, Linear weight), orthogonal_ (weight_hh*),
        zero biases -- consuming torch's CPU RNG in the same order."""
        cpu = {n: torch.empty(s) for n, s in self.specs}
        stdv = 1.0 / math.sqrt(self.hidden)
        for n, _ in self.specs:  # nn.LSTM.reset_parameters
            if n.startswith("lstm."):
                cpu[n].uniform_(-stdv, stdv)
        w, b = cpu["scaling_layer.0.weight"], cpu["scaling_layer.0.bias"]  # nn.Linear init
        nn.init.kaiming_uniform_(w, a=math.sqrt(5))
        bound = 1 / math.sqrt(w.shape[1])
        nn.init.uniform_(b, -bound, bound)
        for n, _ in self.specs:  # LSTM.init_weights
            if "weight_ih" in n or "scaling_layer.0.weight" in n:
                nn.init.xavier_uniform_(cpu[n])
            elif "weight_hh" in n:
                nn.init.orthogonal_(cpu[n])
            elif "bias" in n:
                nn.init.constant_(cpu[n], 0)
        for n, _ in self.specs:
            self.view(n).copy_(cpu[n])

    # ---- compute ----
    def _layer_weights(self, l, dt):
        """(W_ih both dirs [ndir*4H, In], W_hh [ndir, 4H, H], bias [ndir*4H]) in dt."""
        H, nd = self.hidden, self.ndir
        wih0 = self.offsets[f"lstm.weight_ih_l{l}"]
        in_l = self.input_size if l == 0 else H * nd
        flat = self.flat.detach()
        wih = flat[wih0:wih0 + nd * 4 * H * in_l].view(nd * 4 * H, in_l)
        whh0 = self.offsets[f"lstm.weight_hh_l{l}"]
        whh = flat[whh0:whh0 + nd * 4 * H * H].view(nd, 4 * H, H)
        bih0 = self.offsets[f"lstm.bias_ih_l{l}"]
        bhh0 = self.offsets[f"lstm.bias_hh_l{l}"]
        bias = ops.axpby(flat[bih0:bih0 + nd * 4 * H], flat[bhh0:bhh0 + nd * 4 * H])
        if dt == torch.bfloat16:
            wih = ops.cast_bf16(wih)
            whh = ops.cast_bf16(whh)
        return wih, whh, bias

    def _layer_fp32(self, l):
        """fp32 views (W_ih [ndir*4H, In], b_ih, b_hh [ndir*4H], W_hh [ndir*4H, H])."""
        H, nd = self.hidden, self.ndir
        in_l = self.input_size if l == 0 else H * nd
        flat = self.flat.detach()
        o = self.offsets
        wih = flat[o[f"lstm.weight_ih_l{l}"]:][:nd * 4 * H * in_l].view(nd * 4 * H, in_l)
        whh = flat[o[f"lstm.weight_hh_l{l}"]:][:nd * 4 * H * H].view(nd * 4 * H, H)
        bih = flat[o[f"lstm.bias_ih_l{l}"]:][:nd * 4 * H]
        bhh = flat[o[f"lstm.bias_hh_l{l}"]:][:nd * 4 * H]
        return wih, bih, bhh, whh

    def _recurrence(self, dt):
        """'coop' (multi-CU MFMA, bf16 at H=256), 'mfma' (single-CU MFMA) or 'valu'
        (any width, and the fp32 parity mode).  IRC_LSTM_RECURRENCE overrides."""
        if dt != torch.bfloat16:
            return "valu"
        want = os.environ.get("IRC_LSTM_RECURRENCE", "coop")
        if want == "coop" and ops.lstm_coop_supported(self.hidden):
            return "coop"
        if want in ("coop", "mfma") and ops.lstm_mfma_supported(self.hidden):
            return "mfma"
        return "valu"

    def _use_mfma(self, dt):
        return self._recurrence(dt) != "valu"

    def _layer_fwd(self, l, x, B, L, dt, save):
        """One BiLSTM layer: (hout, saved-for-BPTT or None)."""
        H, nd = self.hidden, self.ndir
        kind = self._recurrence(dt)
        if kind in ("coop", "mfma"):
            # MFMA recurrence: packed W_ih columns so xp is read as per-unit float4s
            wih, bih, bhh, whh = self._layer_fp32(l)
            wp, bp, w, wT = ops.lstm_pack(wih, bih, bhh, whh, H, nd, whh_packs=kind != "coop")
            xp = _gemm_rows_split(x, wp, bp)
            if kind == "coop":
                wf, wb = ops.lstm_coop_pack(whh, H, nd)
                hout, gsave, csave, hprev, sync = ops.lstm_fwd_coop(xp, wf, B, L, H, nd,
                                                                    save=save)
                ops.lstm_coop_fault(sync, B, nd, self.coop_fault)
                wT = wb
            else:
                hout, gsave, csave, hprev = ops.lstm_fwd_mfma(xp, w, B, L, H, nd, save=save)
            # dx GEMM operand, transposed to [In, ndir*4H] so dx = dg . W_ih is an
            # A[M][K] . B[N][K] GEMM (the big-tile path)
            wih_c = ops.cast_bf16_t(wih) if (save and l > 0) else None
            return hout, ((kind, x, wih_c, wT, gsave, csave, hprev) if save else None)
        wih, whh, bias = self._layer_weights(l, dt)
        xp = ops.gemm(x, wih, bias=bias, epilogue=ops.EPI_BIAS, out_dtype=torch.float32)
        hout, gsave, csave, hprev = ops.lstm_fwd(xp, whh, B, L, H, nd, dt, save=save)
        return hout, (("valu", x, wih, whh, gsave, csave, hprev) if save else None)

    def forward_compute(self, features: torch.Tensor, save: bool):
        """features [B, L, In] -> (emb [B, D] fp32 unit-norm, saved state or None)."""
        B, L, In = features.shape
        if In != self.input_size:
            raise ValueError(f"feature dim {In} != input_size {self.input_size}")
        dt = compute_dtype()
        H, nd = self.hidden, self.ndir
        x = features.reshape(B * L, In)
        if x.dtype != dt:
            x = x.to(dt)  # dtype conversion of the frozen features (copy)
        x = x.contiguous()
        layers = []
        for l in range(self.num_layers):
            x, st = self._layer_fwd(l, x, B, L, dt, save)
            layers.append(st)
        wl = self.view("scaling_layer.0.weight")
        bl = self.view("scaling_layer.0.bias")
        if self.act_kind == 0:
            # Identity: the mean over L commutes with the Linear, so the small GEMM
            # runs on the [B, 2H] means instead of all B*L rows
            mh = ops.mean_rows(x, B, L, nd * H)  # [B, 2H] fp32
            m = ops.gemm(mh, wl, bias=bl, epilogue=ops.EPI_BIAS)
        else:  # y = act(x W^T + b) on every row, then the mean
            xf = (x if x.dtype == torch.float32 else x.float()).contiguous()
            u = ops.gemm(xf, wl, bias=bl, epilogue=ops.EPI_BIAS)  # [B*L, D] fp32
            m = ops.mean_rows(ops.activation(self.act_kind, u), B, L, u.shape[1])
            mh = (xf, u)
        emb, nrm = ops.l2norm_fwd(m)
        saved = (B, L, layers, mh, emb, nrm) if save else None
        return emb, saved

    def backward_compute(self, saved, demb: torch.Tensor):
        """Accumulate d(loss)/d(params) into self.flat_grad."""
        B, L, layers, mh, emb, nrm = saved
        H, nd = self.hidden, self.ndir
        g = self.flat_grad
        dm = ops.l2norm_bwd(demb.contiguous(), emb, nrm)
        if self.act_kind == 0:
            ops.gemm(dm, mh, trans_a=True, b_is_nk=False, accumulate=True,
                     out=self.view("scaling_layer.0.weight", g))
            ops.colsum(dm, out=self.view("scaling_layer.0.bias", g), accumulate=True)
            dmh = ops.gemm(dm, self.view("scaling_layer.0.weight"), b_is_nk=False)  # [B, 2H]
            dy = ops.bcast_rows(dmh, B, L, 1.0 / L)  # [B*L, 2H] fp32
        else:
            xf, u = mh
            du = ops.activation_bwd(self.act_kind, u, ops.bcast_rows(dm, B, L, 1.0 / L))
            ops.gemm(du, xf, trans_a=True, b_is_nk=False, accumulate=True,
                     out=self.view("scaling_layer.0.weight", g))
            ops.colsum(du, out=self.view("scaling_layer.0.bias", g), accumulate=True)
            dy = ops.gemm(du, self.view("scaling_layer.0.weight"), b_is_nk=False)  # [B*L, 2H]
        for l in range(self.num_layers - 1, -1, -1):
            kind, x, wih, whh, gsave, csave, hprev = layers[l]
            if kind in ("coop", "mfma"):
                dy = self._layer_bwd_mfma(l, dy, x, wih, whh, gsave, csave, hprev, B, L, kind)
                if l == 0:
                    torch.cuda.current_stream(x.device).wait_stream(self._wgrad_pending)
                continue
            dg = ops.lstm_bwd(dy, whh, gsave, csave, B, L, H, nd)  # [nd, B*L, 4H] fp32
            dgc = ops.cast_bf16(dg) if x.dtype == torch.bfloat16 else dg
            in_l = x.shape[1]
            dx = None
            for d in range(nd):
                sfx = f"l{l}" + ("_reverse" if d == 1 else "")
                ops.gemm(dgc[d], x, trans_a=True, b_is_nk=False, accumulate=True,
                         out=self.view(f"lstm.weight_ih_{sfx}", g), out_dtype=torch.float32)
                ops.gemm(dgc[d], hprev[d], trans_a=True, b_is_nk=False, accumulate=True,
                         out=self.view(f"lstm.weight_hh_{sfx}", g), out_dtype=torch.float32)
                ops.colsum(dg[d], out=self.view(f"lstm.bias_ih_{sfx}", g), accumulate=True)
                ops.colsum(dg[d], out=self.view(f"lstm.bias_hh_{sfx}", g), accumulate=True)
                if l > 0:
                    w_d = wih[d * 4 * H:(d + 1) * 4 * H]  # [4H, In] = [K][N]
                    dx = ops.gemm(dgc[d], w_d, b_is_nk=False, out=dx, accumulate=dx is not None,
                                  out_dtype=torch.float32)
            dy = dx

    def _layer_bwd_mfma(self, l, dy, x, wih_c, whhT, gsave, csave, hprev, B, L, kind="mfma"):
        """BPTT of one layer on the MFMA path; returns dL/dx (None for layer 0).

        dgates [B*L, ndir*4H] bf16 -> both directions' dW_ih / dW_hh as one batched
        GEMM each (K = B*L, deterministic split-K), the bias grads as one column
        sum over both directions, and dx as one GEMM with K = ndir*4H."""
        H, nd = self.hidden, self.ndir
        g = self.flat_grad
        o = self.offsets
        if kind == "coop":
            dg, sync = ops.lstm_bwd_coop(dy, whhT, gsave, csave, B, L, H, nd)
            ops.lstm_coop_fault(sync, B, nd, self.coop_fault)
        else:
            dg = ops.lstm_bwd_mfma(dy, whhT, gsave, csave, B, L, H, nd)
        In = x.shape[1]
        BL = B * L
        ih, hh = o[f"lstm.weight_ih_l{l}"], o[f"lstm.weight_hh_l{l}"]
        bi, bh = o[f"lstm.bias_ih_l{l}"], o[f"lstm.bias_hh_l{l}"]
        if nd == 2:  # both directions' slices are adjacent in the flat buffer
            assert o[f"lstm.weight_ih_l{l}_reverse"] == ih + 4 * H * In
            assert o[f"lstm.weight_hh_l{l}_reverse"] == hh + 4 * H * H
            assert o[f"lstm.bias_ih_l{l}_reverse"] == bi + 4 * H
            assert o[f"lstm.bias_hh_l{l}_reverse"] == bh + 4 * H
        # dx is the critical path (next layer's recurrence); the weight/bias
        # gradients go to a side stream and overlap that recurrence, which only
        # occupies B/32 * ndir CUs.  Joined in backward_compute.
        mb = SPLIT_MAX_BLOCKS
        dx = ops.gemm(dg, wih_c, out_dtype=torch.float32, max_blocks=mb) if l > 0 else None
        cur = torch.cuda.current_stream(dg.device)
        side = side_stream(dg.device, "lstm_wgrad")
        side.wait_stream(cur)
        # Half a wave of split-K blocks (SPLIT_MAX_BLOCKS): each dW GEMM is slower alone
        # (l0 112 vs 78 us) but leaves CUs to the encoder forward beside it.
        with torch.cuda.stream(side):
            ops.gemm_strided(dg, x, g[ih:], M=4 * H, N=In, K=BL, batch=nd, lda=nd * 4 * H,
                             sA=4 * H, ldb=x.stride(0), sB=0, ldc=In, sC=4 * H * In,
                             trans_a=True, b_is_nk=False, accumulate=True, max_blocks=mb)
            ops.gemm_strided(dg, hprev, g[hh:], M=4 * H, N=H, K=BL, batch=nd, lda=nd * 4 * H,
                             sA=4 * H, ldb=H, sB=BL * H, ldc=H, sC=4 * H * H, trans_a=True,
                             b_is_nk=False, accumulate=True, max_blocks=mb)
            db = ops.colsum(dg)  # d(b_ih) = d(b_hh): one column sum, added to both
            ops.axpby(g[bi:bi + nd * 4 * H], db, out=g[bi:bi + nd * 4 * H])
            ops.axpby(g[bh:bh + nd * 4 * H], db, out=g[bh:bh + nd * 4 * H])
        for t in (dg, x, hprev):  # allocated on cur, read on side
            t.record_stream(side)
        self._wgrad_pending = side
        return dx

    def check_fault(self):
        """Raise if any cluster recurrence timed out since the last check (host
        sync: called at the train loop's existing sync points)."""
        if self.coop_fault.device.type != "cuda":
            return
        if int(self.coop_fault.item()) != 0:
            self.coop_fault.zero_()
            raise ops.IRCError(
                "LSTM cluster recurrence (irc_lstm_fwd_coop / irc_lstm_bwd_coop) timed out: "
                "its workgroups were not co-resident; the affected outputs were NaN-poisoned")

    def forward(self, features, **kwargs):
        """Per-position head output [B, L, D] (reference LSTM.forward semantics);
        the training path uses the fused ``seq2vec`` instead."""
        B, L, In = features.shape
        dt = compute_dtype()
        x = features.reshape(B * L, In).to(dt).contiguous()
        for l in range(self.num_layers):
            x, _ = self._layer_fwd(l, x, B, L, dt, save=False)
        wl = self.view("scaling_layer.0.weight")
        bl = self.view("scaling_layer.0.bias")
        xf = x if x.dtype == torch.float32 else x.float()
        y = ops.gemm(xf.contiguous(), wl, bias=bl, epilogue=ops.EPI_BIAS)
        if self.act_kind != 0:
            y = ops.activation(self.act_kind, y)
        return y.view(B, L, -1)


class _Seq2VecFn(torch.autograd.Function):
    """emb = seq2vec(features) with grads accumulated into head.flat_grad."""

    @staticmethod
    def forward(ctx, features, flat, head):
        emb, saved = head.forward_compute(features, save=True)
        ctx.head = head
        ctx.saved = saved
        return emb

    @staticmethod
    def backward(ctx, demb):
        ctx.head.backward_compute(ctx.saved, demb)
        ctx.saved = None
        return None, None, None


def seq2vec(head: LSTMHead, features: torch.Tensor, grad: bool) -> torch.Tensor:
    if grad and torch.is_grad_enabled():
        return _Seq2VecFn.apply(features, head.flat, head)
    with torch.no_grad():
        emb, _ = head.forward_compute(features, save=False)
    return emb
