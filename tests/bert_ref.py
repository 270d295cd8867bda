"""Plain PyTorch fp32 reference of the BERT bi-encoder (test infrastructure only).

HF BertModel semantics as the reference reaches them (contrastive_module.py:36-41,
96-112; modeling_bert: embeddings (word + token_type 0) + position -> LN; per layer
softmax(QK^T/sqrt(dh) + (1-mask)*finfo.min) V -> dense + residual -> LN ->
GELU(erf) FFN + residual -> LN), then seq2vec's mean over ALL L positions and
F.normalize.  Used with torch autograd as the gradient reference for the trainable
encoder (irc_amd.bert_train); pinned to the reference's own HF output by
tests/test_oracle_golden.py::test_bert_ref_matches_golden.
"""
import math

import torch
import torch.nn.functional as F


def layer_names(l):
    p = f"encoder.layer.{l}."
    return {k: p + v for k, v in {
        "q": "attention.self.query", "k": "attention.self.key", "v": "attention.self.value",
        "o": "attention.output.dense", "ln1": "attention.output.LayerNorm",
        "i": "intermediate.dense", "out": "output.dense", "ln2": "output.LayerNorm"}.items()}


def bert_hidden(P, ids, mask, n_layers, heads, eps=1e-12):
    """last_hidden_state [B, L, H] from a {HF name: tensor} parameter dict."""
    B, L = ids.shape
    # nn.Embedding(padding_idx=0): the PAD row never receives a gradient
    x = F.embedding(ids, P["embeddings.word_embeddings.weight"], padding_idx=0)
    x = x + P["embeddings.token_type_embeddings.weight"][0]
    x = x + P["embeddings.position_embeddings.weight"][:L][None]
    H = x.shape[-1]
    x = F.layer_norm(x, (H,), P["embeddings.LayerNorm.weight"], P["embeddings.LayerNorm.bias"], eps)
    dh = H // heads
    bias = (1.0 - mask.float())[:, None, None, :] * torch.finfo(torch.float32).min
    for l in range(n_layers):
        n = layer_names(l)

        def lin(t, k):
            return t @ P[n[k] + ".weight"].T + P[n[k] + ".bias"]

        q, k, v = (lin(x, kk).view(B, L, heads, dh).transpose(1, 2) for kk in "qkv")
        s = q @ k.transpose(-1, -2) / math.sqrt(dh) + bias
        ctx = (torch.softmax(s, -1) @ v).transpose(1, 2).reshape(B, L, H)
        a = F.layer_norm(lin(ctx, "o") + x, (H,), P[n["ln1"] + ".weight"], P[n["ln1"] + ".bias"], eps)
        f = lin(F.gelu(lin(a, "i")), "out")
        x = F.layer_norm(f + a, (H,), P[n["ln2"] + ".weight"], P[n["ln2"] + ".bias"], eps)
    return x


def bert_seq2vec(P, ids, mask, n_layers, heads, eps=1e-12):
    """normalize(mean_L(last_hidden_state)) -- PAD positions included (seq2vec)."""
    return F.normalize(bert_hidden(P, ids, mask, n_layers, heads, eps).mean(dim=1))
