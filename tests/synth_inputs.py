"""Deterministic synthetic inputs shared by the golden generator
(tests/golden/make_goldens.py, run against the reference in the build container)
and the tests that replay them on the GPU box: the large C2-shape inputs are
regenerated from numpy's PCG64 streams instead of being committed."""
import zlib

import numpy as np


def unit_rows(seed, n, d):
    """n unit-norm float32 rows (normalised in float64, then cast)."""
    x = np.random.default_rng(seed).standard_normal((n, d))
    return (x / np.linalg.norm(x, axis=1, keepdims=True)).astype(np.float32)


def unit_cols(seed, d, k):
    """[d, k] float32 with unit-norm columns (the MoCo queue's layout)."""
    x = np.random.default_rng(seed).standard_normal((d, k))
    return (x / np.linalg.norm(x, axis=0, keepdims=True)).astype(np.float32)


NCE_C2_CASES = [(256, 128, 12544, 21), (256, 768, 12544, 22)]  # (N, D, K, seed)
# C3 / C4 global batches (B = 1024 over 4 GPUs, 2048 over 8) with the LSTM head's D
NCE_C34_CASES = [(1024, 128, 12544, 31), (2048, 128, 12544, 32)]


def nce_c2_inputs(n, d, k, seed):
    return unit_rows(seed, n, d), unit_rows(seed + 1000, n, d), unit_cols(seed + 2000, d, k)


BERT_BASE = dict(vocab_size=30522, hidden_size=768, num_hidden_layers=12, num_attention_heads=12,
                 intermediate_size=3072, max_position_embeddings=512)


BERT_LARGE = dict(vocab_size=30522, hidden_size=1024, num_hidden_layers=24,
                  num_attention_heads=16, intermediate_size=4096, max_position_embeddings=512)
BERT_LARGE_LENS = (64, 29)  # B = 2 sequences, one full length, one padded


def bert_param(name, shape):
    """One BERT parameter from its own PCG64 stream (seed = crc32 of the HF name):
    LayerNorm gammas 1 + 0.1 N(0,1), every bias / beta 0.02 N(0,1), every weight
    and embedding 0.02 N(0,1) -- biases and LN affines nonzero so they are pinned."""
    rng = np.random.default_rng(zlib.crc32(name.encode()))
    x = rng.standard_normal(shape, dtype=np.float32)
    if name.endswith("LayerNorm.weight"):
        return (1.0 + 0.1 * x).astype(np.float32)
    return (0.02 * x).astype(np.float32)


def bert_base_batch(seed=7, lens=(64, 40, 17, 5), vocab=30522):
    """[CLS] w.. [SEP] [PAD].. token ids / mask, B = len(lens), L = max(lens)."""
    g = np.random.default_rng(seed)
    B, L = len(lens), max(lens)
    ids = g.integers(5, vocab, (B, L)).astype(np.int64)
    mask = (np.arange(L)[None] < np.array(lens)[:, None]).astype(np.int64)
    ids[:, 0] = 2
    ids = np.where(mask == 1, ids, 0)
    ids[np.arange(B), np.array(lens) - 1] = 3
    return ids, mask
