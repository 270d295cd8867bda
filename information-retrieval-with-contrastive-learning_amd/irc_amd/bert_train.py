"""Trainable BERT bi-encoder (``--model BERT``): forward with saved activations and
a full backward on the irc HIP kernels.

The reference trains only the BiLSTM head over a frozen HF BertModel
(src/contrastor/contrastive_module.py:30-41, src/model.py:61-70).  The north star
adds the encoder forward/backward: this module is the same BERT forward as
``irc_amd.bert`` (HF BertModel semantics, eval mode, no dropout) made
trainable, with seq2vec = mean over ALL L positions (PAD included, as the
reference's ``seq2vec``, contrastive_module.py:102-112) + F.normalize, so the
embedding dim is the hidden size.

Parameters live in ONE flat fp32 buffer with HF-named views (``state_dict()``
keys are HF's ``embeddings.*`` / ``encoder.layer.N.*`` / ``pooler.*``), the
gradients in a parallel flat buffer, so clip + Adam + the momentum update are
single fused launches (irc_amd.optim / contrastive_module), exactly as for the
LSTM head.  In bf16 mode the MFMA operands come from a flat bf16 shadow that the
Adam / momentum kernels rewrite in the same pass, plus transposed bf16 copies of
the weight matrices for the dX GEMMs (so they take the big-tile A[M][K].B[N][K]
path); fp32 mode (parity) runs every GEMM on the exact-fp32 MFMA.

Per layer, forward (saved for backward in brackets):
  qkv = x Wqkv^T + b [qkv] -> ctx = attention(qkv) [ctx] -> s1 = ctx Wo^T + bo + x
  [s1] -> a = LN1(s1) [a] -> g = gelu(u), u = a W1^T + b1 [u, g] -> s2 = g W2^T + b2
  + a [s2] -> y = LN2(s2) (next layer's x [x]).
Backward mirrors it: LN bwd (recomputed statistics) -> dX GEMMs with fused
residual / GELU' epilogues -> attention bwd -> ... -> the embedding LN bwd and the
word / position / token-type scatter; the weight / bias gradients are deferred and
formed per kind for all layers at once (one batched GEMM + one batched column
sum each) from [layers, B*L, dim] buffers.
"""
from __future__ import annotations

import copy
import math

import torch
import torch.nn as nn

from . import ops
from ._torch import side_stream
from .bert import BERT_BASE, PRESETS, BertConfig, BertModel
from .precision import compute_dtype

ALIGN = 16  # floats per slice start (16-byte-aligned bf16 shadow slices)


def bert_param_specs(c: BertConfig):
    """(name, shape) in HF BertModel.named_parameters() order, except that each
    layer's query/key/value weights (and biases) are listed adjacently so the
    fused [3H, H] QKV operand is a view of the flat buffer."""
    H, I = c.hidden_size, c.intermediate_size
    s = [("embeddings.word_embeddings.weight", (c.vocab_size, H)),
         ("embeddings.position_embeddings.weight", (c.max_position_embeddings, H)),
         ("embeddings.token_type_embeddings.weight", (c.type_vocab_size, H)),
         ("embeddings.LayerNorm.weight", (H,)), ("embeddings.LayerNorm.bias", (H,))]
    for l in range(c.num_hidden_layers):
        p = f"encoder.layer.{l}."
        s += [(p + "attention.self.query.weight", (H, H)),
              (p + "attention.self.key.weight", (H, H)),
              (p + "attention.self.value.weight", (H, H)),
              (p + "attention.self.query.bias", (H,)),
              (p + "attention.self.key.bias", (H,)),
              (p + "attention.self.value.bias", (H,)),
              (p + "attention.output.dense.weight", (H, H)),
              (p + "attention.output.dense.bias", (H,)),
              (p + "attention.output.LayerNorm.weight", (H,)),
              (p + "attention.output.LayerNorm.bias", (H,)),
              (p + "intermediate.dense.weight", (I, H)), (p + "intermediate.dense.bias", (I,)),
              (p + "output.dense.weight", (H, I)), (p + "output.dense.bias", (H,)),
              (p + "output.LayerNorm.weight", (H,)), (p + "output.LayerNorm.bias", (H,))]
    s += [("pooler.dense.weight", (H, H)), ("pooler.dense.bias", (H,))]
    return s


class BertEncoder(nn.Module):
    """Trainable BERT + mean-pool bi-encoder (the ``--model BERT`` base encoder)."""

    def __init__(self, config: BertConfig | dict | None = None, name: str = "bert-base-uncased",
                 seed: int | None = 0, init_from: BertModel | None = None):
        super().__init__()
        if isinstance(config, dict):
            config = BertConfig.from_dict(config)
        self.config = config or PRESETS.get(name, BERT_BASE)
        c = self.config
        if c.hidden_size % c.num_attention_heads:
            raise ValueError("hidden_size % num_attention_heads != 0")
        if c.hidden_size % ALIGN:
            raise ValueError(f"hidden_size must be a multiple of {ALIGN}")
        self.specs = bert_param_specs(c)
        self.offsets, o = {}, 0
        for n, shp in self.specs:
            o = (o + ALIGN - 1) // ALIGN * ALIGN
            self.offsets[n] = o
            o += math.prod(shp)
        self.numel_flat = (o + ALIGN - 1) // ALIGN * ALIGN
        for l in range(c.num_hidden_layers):  # fused QKV operand = one view
            p = f"encoder.layer.{l}.attention.self."
            H = c.hidden_size
            assert self.offsets[p + "key.weight"] == self.offsets[p + "query.weight"] + H * H
            assert self.offsets[p + "value.weight"] == self.offsets[p + "key.weight"] + H * H
            assert self.offsets[p + "key.bias"] == self.offsets[p + "query.bias"] + H
            assert self.offsets[p + "value.bias"] == self.offsets[p + "key.bias"] + H
        self.flat = nn.Parameter(torch.zeros(self.numel_flat), requires_grad=True)
        self.register_buffer("flat_grad", torch.zeros(self.numel_flat), persistent=False)
        self._shadow = None      # bf16 mirror of flat (MFMA operands)
        self._shadow_t = None    # {name: bf16 transposed weight} (dX GEMM operands)
        self._shadow_ok = False
        self._shadow_t_ok = False
        # data-parallel gradient reduction overlapped with the backward (set per
        # micro-batch by TrainState.set_process_group's caller; None: no reduce)
        self._reduce_group = None
        self._reduce_works = []
        self.reduce_bucket_layers = 4
        # single process: the same buckets' weight gradients on the side stream during the
        # dX chain (whose N = 768 GEMMs fill three quarters of a wave at B L = 16384), under
        # a split-K cap of wgrad_max_blocks 256 x 256 blocks (0 = one wave).  --model BERT
        # step: 19.19-19.43 ms after the chain, 18.95-18.98 overlapped, 18.73-18.76 with the
        # cap of 128 (three interleaved runs, profiles/r06_d_wgrad_ab.log)
        self.overlap_wgrad = True
        self.wgrad_max_blocks = 128
        if init_from is not None:
            self.load_from_bert(init_from)
        else:
            self.load_from_bert(BertModel(c, seed=seed))

    # ---- parameter plumbing (same interface as LSTMHead: view / specs / flat) ----
    def view(self, name, buf=None):
        buf = self.flat if buf is None else buf
        shape = dict(self.specs)[name]
        o = self.offsets[name]
        return buf.detach()[o:o + math.prod(shape)].view(shape)

    def _span(self, first, n, buf=None):
        buf = self.flat if buf is None else buf
        o = self.offsets[first]
        return buf.detach()[o:o + n]

    def named_flat_params(self):
        return [(n, self.view(n)) for n, _ in self.specs]

    @torch.no_grad()
    def load_from_bert(self, bert: BertModel):
        sd = bert.state_dict()
        for n, shape in self.specs:
            self.view(n).copy_(sd[n].reshape(shape).to(self.flat.device, torch.float32))
        self.invalidate_shadow()

    def invalidate_shadow(self):
        self._shadow_ok = False
        self._shadow_t_ok = False

    def _save_to_state_dict(self, destination, prefix, keep_vars):
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
        for k in state_dict:
            if k.startswith(prefix) and k[len(prefix):] not in self.offsets and strict \
                    and not k.endswith("position_ids"):
                unexpected_keys.append(k)
        self.invalidate_shadow()

    def _apply(self, fn, *a, **k):
        r = super()._apply(fn, *a, **k)
        self._shadow = self._shadow_t = None
        self.invalidate_shadow()
        return r

    # ---- bf16 shadows ----
    def shadow(self):
        """bf16 mirror of the flat buffer (rebuilt when invalid; otherwise kept
        current by the Adam / momentum kernels, which write it in their pass)."""
        if self._shadow is None or self._shadow.device != self.flat.device:
            self._shadow = torch.empty(self.numel_flat, dtype=torch.bfloat16,
                                       device=self.flat.device)
            self._shadow_ok = False
        if not self._shadow_ok:
            ops.cast_bf16_into(self.flat.detach(), self._shadow)
            self._shadow_ok = True
        return self._shadow

    def shadow_buffer(self):
        """The bf16 shadow storage for an update kernel that rewrites all of it
        (None in fp32 mode, where no shadow is used)."""
        if compute_dtype() != torch.bfloat16:
            return None
        if self._shadow is None or self._shadow.device != self.flat.device:
            self._shadow = torch.empty(self.numel_flat, dtype=torch.bfloat16,
                                       device=self.flat.device)
        return self._shadow

    def _matrices(self):
        c = self.config
        H = c.hidden_size
        out = []
        for l in range(c.num_hidden_layers):
            p = f"encoder.layer.{l}."
            out += [(p + "attention.self.query.weight", (3 * H, H)),
                    (p + "attention.output.dense.weight", (H, H)),
                    (p + "intermediate.dense.weight", (c.intermediate_size, H)),
                    (p + "output.dense.weight", (H, c.intermediate_size))]
        return out

    _KINDS = ("attention.self.query.weight", "attention.output.dense.weight",
              "intermediate.dense.weight", "output.dense.weight")

    def shadow_t(self):
        """{weight name: bf16 W^T} for the dX GEMMs (rebuilt after each update): per weight
        kind one [layers, in, out] buffer, rebuilt by ONE batched transposing cast over the
        layers' identically laid-out flat slices (48 launches a step -> 4)."""
        c = self.config
        nl = c.num_hidden_layers
        shapes = dict(self._matrices())
        if self._shadow_t is None or next(iter(self._shadow_t.values())).device != \
                self.flat.device:
            self._shadow_t, self._shadow_t_kind = {}, {}
            for kind in self._KINDS:
                r, cc = shapes[f"encoder.layer.0.{kind}"]
                buf = torch.empty((nl, cc, r), dtype=torch.bfloat16, device=self.flat.device)
                self._shadow_t_kind[kind] = buf
                for l in range(nl):
                    self._shadow_t[f"encoder.layer.{l}.{kind}"] = buf[l]
            self._shadow_t_ok = False
        if not self._shadow_t_ok:
            flat = self.flat.detach()
            for kind in self._KINDS:
                r, cc = shapes[f"encoder.layer.0.{kind}"]
                o = self.offsets[f"encoder.layer.0.{kind}"]
                ops.cast_bf16_t_batched(flat[o:], self._shadow_t_kind[kind], r, cc, nl,
                                        self._layer_stride(kind))
            self._shadow_t_ok = True
        return self._shadow_t

    def after_update(self, shadow_written: bool):
        """Called by the optimizer / momentum update after the flat buffer moved."""
        self._shadow_ok = bool(shadow_written) and self._shadow is not None
        self._shadow_t_ok = False

    def _weights(self, dt, with_t=False):
        """Per-layer operand views in the compute dtype."""
        c = self.config
        H, I = c.hidden_size, c.intermediate_size
        src = self.shadow() if dt == torch.bfloat16 else self.flat.detach()
        f32 = self.flat.detach()
        sT = self.shadow_t() if (with_t and dt == torch.bfloat16) else None

        def v(buf, name, shape):
            o = self.offsets[name]
            return buf[o:o + math.prod(shape)].view(shape)

        w = {"word": v(src, "embeddings.word_embeddings.weight", (c.vocab_size, H)),
             "pos": v(src, "embeddings.position_embeddings.weight",
                      (c.max_position_embeddings, H)),
             "type0": v(src, "embeddings.token_type_embeddings.weight", (c.type_vocab_size, H))[0],
             "ln_g": self.view("embeddings.LayerNorm.weight"),
             "ln_b": self.view("embeddings.LayerNorm.bias"), "layers": []}
        for l in range(c.num_hidden_layers):
            p = f"encoder.layer.{l}."
            lw = {"wqkv": v(src, p + "attention.self.query.weight", (3 * H, H)),
                  "bqkv": v(f32, p + "attention.self.query.bias", (3 * H,)),
                  "wo": v(src, p + "attention.output.dense.weight", (H, H)),
                  "bo": self.view(p + "attention.output.dense.bias"),
                  "ln1_g": self.view(p + "attention.output.LayerNorm.weight"),
                  "ln1_b": self.view(p + "attention.output.LayerNorm.bias"),
                  "w1": v(src, p + "intermediate.dense.weight", (I, H)),
                  "b1": self.view(p + "intermediate.dense.bias"),
                  "w2": v(src, p + "output.dense.weight", (H, I)),
                  "b2": self.view(p + "output.dense.bias"),
                  "ln2_g": self.view(p + "output.LayerNorm.weight"),
                  "ln2_b": self.view(p + "output.LayerNorm.bias")}
            if with_t:
                if sT is not None:
                    lw["wqkvT"] = sT[p + "attention.self.query.weight"]
                    lw["woT"] = sT[p + "attention.output.dense.weight"]
                    lw["w1T"] = sT[p + "intermediate.dense.weight"]
                    lw["w2T"] = sT[p + "output.dense.weight"]
                else:  # fp32: the KN operand layout directly (no transposed copies)
                    lw["wqkvT"] = lw["woT"] = lw["w1T"] = lw["w2T"] = None
            w["layers"].append(lw)
        return w

    # ---- compute ----
    def flops_per_sequence(self, L: int) -> float:
        c = self.config
        H, I = c.hidden_size, c.intermediate_size
        return c.num_hidden_layers * (2 * L * (4 * H * H + 2 * H * I) + 4 * L * L * H)

    def _dx_gemm(self, dY, w, wT, **kw):
        """dX = dY . W (W = nn.Linear weight [out, in]); big-tile path via W^T in bf16."""
        if wT is not None:
            return ops.gemm(dY, wT, **kw)
        return ops.gemm(dY, w, b_is_nk=False, **kw)

    def forward_compute(self, input_ids: torch.Tensor, attention_mask: torch.Tensor, save: bool):
        """ids/mask [B, L] -> (emb [B, H] fp32 unit-norm, saved state or None).

        With save, the four weight-gradient operands (layer input x, ctx, a, gelu
        output g) are written into per-type [layers, B*L, dim] buffers so the
        backward can form every layer's dW of one kind as ONE batched GEMM."""
        c = self.config
        ids = input_ids.to(torch.int64).contiguous()
        mask = attention_mask.to(torch.int64).contiguous()
        B, L = ids.shape
        if L > c.max_position_embeddings:
            raise ValueError(f"sequence length {L} > max_position_embeddings")
        H, I, heads, eps = c.hidden_size, c.intermediate_size, c.num_attention_heads, \
            c.layer_norm_eps
        nl = c.num_hidden_layers
        dt = compute_dtype()
        w = self._weights(dt, with_t=save)
        dev = self.flat.device
        BL = B * L
        if save:
            xs = torch.empty((nl, BL, H), dtype=dt, device=dev)
            ctxs = torch.empty((nl, BL, H), dtype=dt, device=dev)
            as_ = torch.empty((nl, BL, H), dtype=dt, device=dev)
            gs = torch.empty((nl, BL, I), dtype=dt, device=dev)
        x = ops.embed_ln(ids, w["word"], w["pos"], w["type0"], w["ln_g"], w["ln_b"], eps,
                         out=xs[0] if save else None)
        layers = []
        for l, lw in enumerate(w["layers"]):
            qkv = ops.gemm(x, lw["wqkv"], bias=lw["bqkv"], epilogue=ops.EPI_BIAS)
            ctx = ops.attention(qkv, mask, B, L, H, heads, out=ctxs[l] if save else None)
            s1 = ops.gemm(ctx, lw["wo"], bias=lw["bo"], residual=x, epilogue=ops.EPI_BIAS_RESID)
            a = ops.layernorm(s1, lw["ln1_g"], lw["ln1_b"], eps, out=as_[l] if save else s1)
            if save:
                g, u = ops.gemm_gelu_save(a, lw["w1"], lw["b1"], out=gs[l])
            else:
                g, u = ops.gemm(a, lw["w1"], bias=lw["b1"], epilogue=ops.EPI_BIAS_GELU), None
            s2 = ops.gemm(g, lw["w2"], bias=lw["b2"], residual=a, epilogue=ops.EPI_BIAS_RESID)
            last = l == nl - 1
            if save:
                y = ops.layernorm(s2, lw["ln2_g"], lw["ln2_b"], eps,
                                  out=None if last else xs[l + 1])
                layers.append((qkv, s1, u, s2))
            else:
                y = ops.layernorm(s2, lw["ln2_g"], lw["ln2_b"], eps, out=s2)
            x = y
        m = ops.mean_rows(x, B, L, H)  # [B, H] fp32, PAD positions included
        emb, nrm = ops.l2norm_fwd(m)
        saved = (ids, mask, B, L, w, layers, (xs, ctxs, as_, gs), emb, nrm) if save else None
        return emb, saved

    def backward_compute(self, saved, demb: torch.Tensor):
        """Accumulate d(loss)/d(params) into self.flat_grad.

        The dX chain runs layer by layer; each layer's four output gradients (dqkv,
        ds1, du, ds2) land in per-type [layers, B*L, dim] buffers, and after the
        chain every layer's dW / db of one kind is ONE batched GEMM (K = B*L, both
        operands K-outer) / one batched column sum, strided over the layers'
        identically laid-out flat-buffer slices."""
        ids, mask, B, L, w, layers, acts, emb, nrm = saved
        xs, ctxs, as_, gs = acts
        c = self.config
        H, I, heads, eps = c.hidden_size, c.intermediate_size, c.num_attention_heads, \
            c.layer_norm_eps
        nl = c.num_hidden_layers
        g = self.flat_grad
        dev = g.device
        BL = B * L
        dt = xs.dtype
        dqkvs = torch.empty((nl, BL, 3 * H), dtype=dt, device=dev)
        ds1s = torch.empty((nl, BL, H), dtype=dt, device=dev)
        dus = torch.empty((nl, BL, I), dtype=dt, device=dev)
        ds2s = torch.empty((nl, BL, H), dtype=dt, device=dev)
        dm = ops.l2norm_bwd(demb.float().contiguous(), emb, nrm)  # [B, H] fp32
        dy, bcast = dm, L  # top layer: the mean-pool backward folded into LN2's
        # DP (and, with overlap_wgrad, one process): buckets of reduce_bucket_layers
        # layers, top bucket first; bucket_lo maps each bucket's lowest layer to its
        # (exclusive) top
        reduce_on = self._reduce_group is not None
        overlap = reduce_on or (self.overlap_wgrad and g.is_cuda)
        nb = max(1, int(self.reduce_bucket_layers))
        bucket_lo = {}
        if overlap:
            hi = nl
            while hi > 0:
                lo = max(0, hi - nb)
                bucket_lo[lo] = hi
                hi = lo
        for l in range(nl - 1, -1, -1):
            qkv, s1, u, s2 = layers[l]
            lw = w["layers"][l]
            p = f"encoder.layer.{l}."
            ds2 = ops.layernorm_bwd(dy, s2, lw["ln2_g"], self.view(p + "output.LayerNorm.weight", g),
                                    self.view(p + "output.LayerNorm.bias", g), eps,
                                    bcast_L=bcast, dy_scale=1.0 / L if bcast else 1.0,
                                    out=ds2s[l])
            bcast = 0
            du = self._dx_gemm(ds2, lw["w2"], lw.get("w2T"), epilogue=ops.EPI_DGELU, residual=u,
                               out=dus[l])
            da = self._dx_gemm(du, lw["w1"], lw.get("w1T"), epilogue=ops.EPI_RESID, residual=ds2)
            ds1 = ops.layernorm_bwd(da, s1, lw["ln1_g"],
                                    self.view(p + "attention.output.LayerNorm.weight", g),
                                    self.view(p + "attention.output.LayerNorm.bias", g), eps,
                                    out=ds1s[l])
            dctx = self._dx_gemm(ds1, lw["wo"], lw.get("woT"))
            dqkv = ops.attention_bwd(qkv, mask, ctxs[l], dctx, B, L, H, heads, out=dqkvs[l])
            dy = self._dx_gemm(dqkv, lw["wqkv"], lw.get("wqkvT"), epilogue=ops.EPI_RESID,
                               residual=ds1)
            if overlap and l in bucket_lo and l > 0:
                self._bucket_wgrad_reduce(l, bucket_lo[l], acts, (dqkvs, ds1s, dus, ds2s),
                                          reduce=reduce_on)
        # layer-batched weight / bias gradients (the layers not yet reduced)
        lo_end = bucket_lo[0] if overlap else nl
        self._wgrad_layers(0, lo_end, acts, (dqkvs, ds1s, dus, ds2s))
        # embeddings: LN backward on the rebuilt fp32 sum, then the table scatter
        e = ops.embed_sum(ids, w["word"], w["pos"], w["type0"])
        de = ops.layernorm_bwd(dy, e, w["ln_g"], self.view("embeddings.LayerNorm.weight", g),
                               self.view("embeddings.LayerNorm.bias", g), eps)
        ops.embed_bwd(de, ids, self.view("embeddings.word_embeddings.weight", g),
                      self.view("embeddings.position_embeddings.weight", g),
                      self.view("embeddings.token_type_embeddings.weight", g)[0],
                      c.pad_token_id)
        if reduce_on:  # last bucket: embeddings + the bottom layers, on this stream
            self._reduce_async(0, self._layer_start(lo_end))
        elif overlap and len(bucket_lo) > 1:  # the side stream's buckets, before any reader
            torch.cuda.current_stream(dev).wait_stream(side_stream(dev, "grad_reduce"))

    # ---- data-parallel gradient all-reduce, bucketed and overlapped -------------
    def set_grad_reduce(self, group):
        """All-reduce (sum) flat_grad over ``group`` DURING the next backward, in
        buckets of ``reduce_bucket_layers`` layers: once the dX chain has passed a
        bucket's lowest layer, that bucket's weight gradients (one batched GEMM per
        kind) and its RCCL all-reduce run on a side stream while the chain goes on
        (the BERT-size gradient bucketed and overlapped with backward).
        None: no reduction (a micro-batch that does not step)."""
        self._reduce_group = group

    def wait_grad_reduce(self):
        """Make the current stream wait for the bucketed all-reduces."""
        for work in self._reduce_works:
            work.wait()
        self._reduce_works = []

    def _layer_start(self, l):
        """Flat offset where layer l's parameters start (the end for l = nl)."""
        c = self.config
        if l >= c.num_hidden_layers:
            return self.numel_flat
        return self.offsets[f"encoder.layer.{l}.attention.self.query.weight"]

    def _reduce_async(self, start, stop):
        import torch.distributed as dist

        self._reduce_works.append(dist.all_reduce(self.flat_grad.detach()[start:stop],
                                                  op=dist.ReduceOp.SUM,
                                                  group=self._reduce_group, async_op=True))

    def _wgrad_layers(self, lo, hi, acts, grads, max_blocks=0):
        xs, ctxs, as_, gs = acts
        dqkvs, ds1s, dus, ds2s = grads
        if hi <= lo:
            return
        for dY, X, wname, bname in ((dqkvs, xs, "attention.self.query.weight",
                                     "attention.self.query.bias"),
                                    (ds1s, ctxs, "attention.output.dense.weight",
                                     "attention.output.dense.bias"),
                                    (dus, as_, "intermediate.dense.weight",
                                     "intermediate.dense.bias"),
                                    (ds2s, gs, "output.dense.weight", "output.dense.bias")):
            self._wgrad_batched(dY[lo:hi], X[lo:hi], wname, bname, first=lo,
                                max_blocks=max_blocks)

    def _bucket_wgrad_reduce(self, lo, hi, acts, grads, reduce=True):
        """Layers [lo, hi): weight gradients (+ with reduce, the all-reduce of their flat
        slice, plus everything above it for the top bucket) on the "grad_reduce" side
        stream."""
        cur = torch.cuda.current_stream(self.flat_grad.device)
        side = side_stream(self.flat_grad.device, "grad_reduce")
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            self._wgrad_layers(lo, hi, acts, grads, self.wgrad_max_blocks)
            if reduce:
                top = hi >= self.config.num_hidden_layers
                self._reduce_async(self._layer_start(lo),
                                   self.numel_flat if top else self._layer_start(hi))
        for t in list(acts) + list(grads):
            t.record_stream(side)
        # no join here: the dX chain goes on; wait_grad_reduce() joins through the
        # all-reduce works (each enqueued behind its bucket's GEMMs on `side`)

    def _layer_stride(self, name):
        c = self.config
        if c.num_hidden_layers < 2:
            return 0
        st = self.offsets[f"encoder.layer.1.{name}"] - self.offsets[f"encoder.layer.0.{name}"]
        for l in range(2, c.num_hidden_layers):  # identical per-layer layout
            assert self.offsets[f"encoder.layer.{l}.{name}"] - \
                self.offsets[f"encoder.layer.{l - 1}.{name}"] == st
        return st

    def _wgrad_batched(self, dY, X, wname, bname, first=0, max_blocks=0):
        """dW[l] += dY[l]^T X[l] and db[l] += colsum(dY[l]) for the layers
        first .. first + len(dY) - 1."""
        g = self.flat_grad.detach()
        nl, BL, out_n = dY.shape
        in_n = X.shape[2]
        ow = self.offsets[f"encoder.layer.{first}.{wname}"]
        ob = self.offsets[f"encoder.layer.{first}.{bname}"]
        sw, sb = self._layer_stride(wname), self._layer_stride(bname)
        ops.gemm_strided(dY, X, g[ow:], M=out_n, N=in_n, K=BL, batch=nl, lda=out_n,
                         sA=BL * out_n, ldb=in_n, sB=BL * in_n, ldc=in_n, sC=sw, trans_a=True,
                         b_is_nk=False, accumulate=True, max_blocks=max_blocks)
        ops.colsum_batched(dY, g[ob:], sb, accumulate=True)

    def encode(self, input_ids, attention_mask):
        """last_hidden_state-free embedding path (no grad): [B, H] unit-norm."""
        with torch.no_grad():
            emb, _ = self.forward_compute(input_ids, attention_mask, save=False)
        return emb


class _EncodeFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ids, mask, flat, enc):
        emb, saved = enc.forward_compute(ids, mask, save=True)
        ctx.enc = enc
        ctx.saved = saved
        return emb

    @staticmethod
    def backward(ctx, demb):
        ctx.enc.backward_compute(ctx.saved, demb)
        ctx.saved = None
        return None, None, None, None


def seq2vec_ids(enc: BertEncoder, input_ids, attention_mask, grad: bool) -> torch.Tensor:
    """normalize(mean_L(BERT(ids))) with grads accumulated into enc.flat_grad."""
    if grad and torch.is_grad_enabled():
        return _EncodeFn.apply(input_ids, attention_mask, enc.flat, enc)
    return enc.encode(input_ids, attention_mask)


def clone_encoder(enc: BertEncoder) -> BertEncoder:
    k = copy.deepcopy(enc)
    k.invalidate_shadow()
    return k
