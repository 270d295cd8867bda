"""Drop-in for src/contrastor/contrastive_module.py (RetrievalModelWrapper).

Same constructor, attributes (encoder_q, encoder_k, queue [dim, K] buffer,
queue_ptr, add_queue_to_loss, use_momentum, use_queue, bert_tokenizer,
bert_model, criterion, loss_config) and methods (bert_extract,
_momentum_update_key_encoder, _dequeue_and_enqueue, forward, ctx2vec, seq2vec)
as the reference (contrastive_module.py:6-112).  Device work runs on the irc
HIP kernels: BERT on irc_amd.bert, the BiLSTM head + seq2vec on
irc_amd.lstm_head, the loss on irc_amd.nce, momentum and enqueue as single
fused launches.  Like the reference, ``use_momentum``/``use_queue`` arguments
are ignored in favour of loss_config (contrastive_module.py:12-13).

Extension (superset): the BERT source/config/tokenizer come from the optional
``bert`` section of config.yaml; offline, a preset name builds the architecture
with seeded random weights instead of fetching 'bert-base-uncased'.

``--model BERT`` (the north star's trainable encoder, irc_amd.bert_train): the
base encoder IS the BERT, run on the jointly tokenised/padded batch (the same
tokenisation as bert_extract), so there is no separate frozen ``bert_model``
(None); emb = normalize(mean_L(BERT(ids))) with D = hidden size; encoder_k is its
momentum copy, and the loss / queue / enqueue tail is shared with the LSTM path.
"""
import copy
import os

import torch
import torch.nn as nn

from irc_amd import ops
from irc_amd._torch import side_stream
from irc_amd.dist import gather_rows
from irc_amd.nce import dist_fused_ok, info_nce_dist
from irc_amd.bert import BertModel
from irc_amd.bert_train import BertEncoder, seq2vec_ids
from irc_amd.lstm_head import LSTMHead, seq2vec as head_seq2vec
from irc_amd.tokenizer import load_tokenizer
from irc_amd.wordpiece import GpuWordPiece


class RetrievalModelWrapper(nn.Module):
    def __init__(self, base_encoder, criterion, loss_config, use_momentum=True, use_queue=True,
                 use_LSTM=True, bert_config=None):
        super().__init__()
        self.criterion = criterion
        self.loss_config = loss_config
        self.use_momentum = self.loss_config["use_momentum"]
        self.use_queue = self.loss_config["use_queue"]
        self.use_LSTM = use_LSTM

        self.encoder_q = copy.deepcopy(base_encoder)
        if self.use_momentum:
            self.encoder_k = copy.deepcopy(base_encoder)
            with torch.no_grad():
                self.encoder_k.flat.copy_(self.encoder_q.flat)
            self.encoder_k.flat.requires_grad_(False)
            if hasattr(self.encoder_k, "invalidate_shadow"):
                self.encoder_k.invalidate_shadow()

        if self.use_queue:
            self.register_buffer("queue", torch.randn(self.loss_config["dim"],
                                                      self.loss_config["queue_size"]))
            self.queue = nn.functional.normalize(self.queue, dim=0)  # host-side init
            self.register_buffer("queue_ptr", torch.zeros(1, dtype=torch.long))
            self.add_queue_to_loss = False

        bc = dict(bert_config or {})
        name = bc.get("name", "bert-base-uncased")
        if use_LSTM:
            self.bert_model = BertModel.from_pretrained(name, config=bc.get("config"),
                                                        seed=int(bc.get("seed", 0)))
            self.bert_model.eval()
            vocab_size = self.bert_model.config.vocab_size
        else:  # --model BERT: the trainable encoder is the BERT
            self.bert_model = None
            vocab_size = self.encoder_q.config.vocab_size
        self.bert_tokenizer = load_tokenizer(bc.get("vocab"), vocab_size)
        # data-parallel group for global in-batch negatives (None: single process)
        self.dist_group = None
        self._gpu_tokenizers = {}  # device -> GpuWordPiece (built on first use)

    @torch.no_grad()
    def bert_extract(self, d1, d2, device):
        ids, mask = self.tokenize(list(d1) + list(d2), device)
        out = self.bert_model.encode(ids, mask)
        return out[:len(d1)], out[len(d1):]

    @torch.no_grad()
    def bert_extract_ids(self, input_ids, attention_mask, n_anchor):
        """Same as bert_extract for already-tokenised (device) batches."""
        out = self.bert_model.encode(input_ids, attention_mask)
        return out[:n_anchor], out[n_anchor:]

    @torch.no_grad()
    def bert_extract_async(self, input_ids, attention_mask, n_anchor, inputs_ready=False):
        """bert_extract_ids issued on the "bert_prefetch" side stream.

        BERT is frozen (contrastive_module.py:34-36: no_grad, eval, never in the
        optimizer), so the features of micro-batch t+1 do not depend on the heads'
        update of micro-batch t: issuing them here, before the heads' step of
        micro-batch t is enqueued, lets the BERT GEMMs fill the CUs the
        latency-bound BiLSTM recurrences leave idle.

        inputs_ready=False (default): the inputs may have just been produced on the
        current stream, so the side stream first waits for everything queued there
        -- including the previous micro-batch's backward, which serialises BERT
        behind it (on MI355X the side stream then idled ~2.5 ms of a 10 ms C2 step).
        inputs_ready=True: the inputs are already complete (resident, or produced on
        the side stream as in bert_extract_texts_async): no wait.  Returns a handle
        for features_ready()."""
        dev = input_ids.device
        cur = torch.cuda.current_stream(dev)
        side = side_stream(dev, "bert_prefetch")
        if not inputs_ready:
            side.wait_stream(cur)
        with torch.cuda.stream(side):
            out = self.bert_model.encode(input_ids, attention_mask)
            done = torch.cuda.Event()
            done.record(side)
        if side != cur:
            input_ids.record_stream(side)
            attention_mask.record_stream(side)
        return out, int(n_anchor), done

    @torch.no_grad()
    def bert_extract_texts_async(self, anchors, positives, device):
        """Tokenise (GPU WordPiece + joint padding) AND encode on the "bert_prefetch"
        side stream: the features of the next micro-batch depend on nothing the
        current stream is doing.  Returns a handle for features_ready()."""
        dev = torch.device(device)
        side = side_stream(dev, "bert_prefetch")
        with torch.cuda.stream(side):
            ids, mask = self.tokenize(list(anchors) + list(positives), dev)
        return self.bert_extract_async(ids, mask, len(anchors), inputs_ready=True)

    @torch.no_grad()
    def bert_extract_corpus_async(self, corpus, sel, n_anchor):
        """The device-corpus input path (irc_amd.corpus): gather + jointly pad the
        selected sentences' resident token ids AND encode them, all on the
        "bert_prefetch" side stream -- the micro-batch crosses the host boundary as
        its sentence indices only.  Returns a handle for features_ready()."""
        dev = corpus.device
        side = side_stream(dev, "bert_prefetch")
        with torch.cuda.stream(side):
            ids, mask = corpus.batch(sel)
        return self.bert_extract_async(ids, mask, n_anchor, inputs_ready=True)

    @staticmethod
    def features_ready(handle):
        """(anchor, positive) features of a bert_extract_async handle, usable on the
        current stream (which is made to wait for them)."""
        out, n_anchor, done = handle
        cur = torch.cuda.current_stream(out.device)
        cur.wait_event(done)
        out.record_stream(cur)
        return out[:n_anchor], out[n_anchor:]

    @torch.no_grad()
    def _momentum_update_key_encoder(self, gate=None):
        """theta_k <- m theta_k + (1 - m) theta_q: one fused launch over the flat buffers
        (for the trainable BERT also rewriting encoder_k's bf16 operand shadow).
        ``gate`` (superset): the step's [norm, coef, gate] device tensor; the update
        is skipped on the device when gate[2] is set (a recurrence timed out)."""
        mom = float(self.loss_config["momentum"])
        shadow = self.encoder_k.shadow_buffer() if hasattr(self.encoder_k, "shadow_buffer") \
            else None
        if gate is not None:
            ops.momentum_update_gated(self.encoder_k.flat.detach(), self.encoder_q.flat.detach(),
                                      mom, gate, shadow)
            if hasattr(self.encoder_k, "after_update"):
                self.encoder_k.after_update(shadow is not None)
        elif shadow is not None:
            ops.momentum_update_bf16(self.encoder_k.flat.detach(), self.encoder_q.flat.detach(),
                                     mom, shadow)
            self.encoder_k.after_update(True)
        else:
            ops.momentum_update(self.encoder_k.flat.detach(), self.encoder_q.flat.detach(), mom)
            if hasattr(self.encoder_k, "after_update"):
                self.encoder_k.after_update(False)

    @torch.no_grad()
    def _dequeue_and_enqueue(self, keys):
        batch_size = keys.shape[0]
        if self.loss_config["queue_size"] % batch_size == 0:  # reference rule (:59)
            ops.enqueue(self.queue, keys.float().contiguous(), self.queue_ptr)

    def tokenize(self, texts, device):
        """bert_tokenizer(texts, padding=True, truncation=True) as device tensors.
        On a HIP device the WordPiece + joint padding run on the GPU
        (irc_amd.wordpiece; IRC_TOKENIZER=host keeps the host tokenizer)."""
        device = torch.device(device)
        if device.type == "cuda" and os.environ.get("IRC_TOKENIZER", "gpu") != "host":
            wp = self._gpu_tokenizers.get(device)
            if wp is None:
                wp = self._gpu_tokenizers[device] = GpuWordPiece(self.bert_tokenizer, device)
            return wp(texts)
        t = self.bert_tokenizer(list(texts), padding=True, truncation=True, return_tensors="pt")
        return t["input_ids"].to(device), t["attention_mask"].to(device)

    def forward(self, anchor_sample, positive_sample, device, cluster_result=None, indexes=None):
        if indexes is not None:
            indexes = indexes.view(-1)
        if not self.use_LSTM:  # --model BERT: joint tokenisation as bert_extract, then encode
            ids, mask = self.tokenize(list(anchor_sample) + list(positive_sample), device)
            return self.forward_ids(ids, mask, len(anchor_sample), cluster_result, indexes)
        anchor_sample, positive_sample = self.bert_extract(anchor_sample, positive_sample, device)
        return self.forward_features(anchor_sample, positive_sample, cluster_result, indexes)

    def forward_ids(self, input_ids, attention_mask, n_anchor, cluster_result=None, indexes=None):
        """--model BERT forward from a jointly padded token batch (anchors first)."""
        qi, qm = input_ids[:n_anchor], attention_mask[:n_anchor]
        ki, km = input_ids[n_anchor:], attention_mask[n_anchor:]
        if self.use_momentum and input_ids.is_cuda:
            cur = torch.cuda.current_stream(input_ids.device)
            side = side_stream(input_ids.device, "key_encoder")
            side.wait_stream(cur)
            with torch.cuda.stream(side):
                emb_k = seq2vec_ids(self.encoder_k, ki, km, grad=False)
            input_ids.record_stream(side)
            attention_mask.record_stream(side)
            emb_q = seq2vec_ids(self.encoder_q, qi, qm, grad=True)
            cur.wait_stream(side)
            emb_k.record_stream(cur)
        else:
            emb_q = seq2vec_ids(self.encoder_q, qi, qm, grad=True)
            enc = self.encoder_k if self.use_momentum else self.encoder_q
            emb_k = seq2vec_ids(enc, ki, km, grad=not self.use_momentum)
        return self._loss_tail(emb_q, emb_k, cluster_result, indexes)

    def forward_features(self, anchor_feat, positive_feat, cluster_result=None, indexes=None):
        """forward() from BERT features on: heads, loss, enqueue."""
        if self.use_momentum and positive_feat.is_cuda:
            # the no-grad key encoder is independent of the query encoder until the
            # loss: run it on a side stream so the two recurrences share the chip
            cur = torch.cuda.current_stream(positive_feat.device)
            side = side_stream(positive_feat.device, "key_encoder")
            side.wait_stream(cur)
            with torch.cuda.stream(side):
                emb_k = self.seq2vec(positive_feat, query=False)
            positive_feat.record_stream(side)
            emb_q = self.seq2vec(anchor_feat)
            cur.wait_stream(side)
            emb_k.record_stream(cur)
        else:
            emb_q = self.seq2vec(anchor_feat)
            emb_k = self.seq2vec(positive_feat, query=False) if self.use_momentum else \
                self.seq2vec(positive_feat)
        return self._loss_tail(emb_q, emb_k, cluster_result, indexes)

    def _loss_tail(self, emb_q, emb_k, cluster_result, indexes):
        """contrastive_module.py:85-92: (global negatives,) loss, enqueue."""
        group = getattr(self, "dist_group", None)
        if group is not None and cluster_result is None and emb_q.is_cuda and \
                dist_fused_ok(emb_q.shape[0], emb_q.shape[1]):
            # data parallel, fused InfoNCE: this rank computes only its own pairs'
            # loss rows over the gathered batch (irc_amd.nce.info_nce_dist)
            keys = emb_k if not self.use_momentum else emb_k.detach()
            queue = None if not self.use_queue or not self.add_queue_to_loss else self.queue
            loss = info_nce_dist(emb_q, keys, queue, self.criterion.T, group)
            if self.use_queue and self.training:
                self._dequeue_and_enqueue(gather_rows(emb_k.detach(), group))
            return loss
        if group is not None:  # global in-batch negatives (irc_amd.dist)
            emb_q = gather_rows(emb_q, group)
            # keys carry autograd only without the momentum encoder (then they come
            # from encoder_q, contrastive_module.py:82-83 of the reference)
            emb_k = gather_rows(emb_k if not self.use_momentum else emb_k.detach(), group)
        queue = None if not self.use_queue or not self.add_queue_to_loss else self.queue
        loss = self.criterion(emb_q, emb_k, queue, cluster_result, indexes)
        if self.use_queue and self.training:
            self._dequeue_and_enqueue(emb_k.detach())
        return loss

    def ctx2vec(self, context, device):
        ids, mask = self.tokenize(context, device)
        if not self.use_LSTM:
            return seq2vec_ids(self.encoder_q, ids, mask, grad=True)
        out = self.bert_model.encode(ids, mask)
        return self.seq2vec(out)

    def seq2vec(self, seq, query=True):
        assert seq.ndim == 3
        if query:
            return head_seq2vec(self.encoder_q, seq, grad=True)
        return head_seq2vec(self.encoder_k, seq, grad=False)


__all__ = ["RetrievalModelWrapper", "LSTMHead", "BertEncoder"]
