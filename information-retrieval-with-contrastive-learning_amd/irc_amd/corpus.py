"""Device-resident tokenised training corpus.

The reference hands every micro-batch to the model as two tuples of sentence
STRINGS pickled by DataLoader workers (src/dataset.py:89-101, 159-182) and
tokenises them on the host per call (src/contrastor/contrastive_module.py:36-41).
Here the sentences of docs_sentence.pkl are WordPiece-tokenised once at startup
on the GPU (irc_wordpiece, token-exact with the host tokenizer) and packed in HBM
as CSR (irc_corpus_pack); a micro-batch is then the sampler's sentence indices
(a few KB to the device) and irc_pair_batch gathers and jointly pads the ids --
the same [CLS] .. [SEP] [PAD] rows and mask the tokenizer would have produced
for those sentences with padding=True, truncation=True.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib
from ._torch import ptr, require_hip, stream_ptr
from .wordpiece import GpuWordPiece


class DeviceCorpus:
    """docs: list of documents, each a list of sentence strings (the
    docs_sentence.pkl format).  Sentence s of document d has global index
    doc_start[d] + s."""

    def __init__(self, docs, hf_tokenizer, device, chunk: int = 65536):
        self.device = torch.device(device)
        self.doc_start = np.zeros(len(docs) + 1, np.int64)
        np.cumsum([len(d) for d in docs], out=self.doc_start[1:])
        sents = [s for d in docs for s in d]
        self.wp = GpuWordPiece(hf_tokenizer, self.device)
        self.flat, self.offsets, self.lens = self.wp.tokenize_corpus(sents, chunk)
        require_hip(self.flat, self.offsets)
        self.n_sentences = len(sents)

    def sentence_index(self, doc: int, sent: int) -> int:
        return int(self.doc_start[doc] + sent)

    def batch(self, sel):
        """(input_ids, attention_mask) int64 [len(sel), L] of the selected sentences,
        jointly padded: L = min(longest, max_tokens) + 2, known on the host (no
        device sync).  Issued on the current stream."""
        sel = np.ascontiguousarray(np.asarray(sel, dtype=np.int64))
        n = sel.shape[0]
        longest = int(self.lens[sel].max()) if n else 0
        L = max(min(longest, self.wp.max_tokens) + 2, 2)
        sel_d = torch.from_numpy(sel).pin_memory().to(self.device, non_blocking=True)
        ids = torch.empty((n, L), dtype=torch.int64, device=self.device)
        mask = torch.empty((n, L), dtype=torch.int64, device=self.device)
        _lib.call("irc_pair_batch", ptr(self.flat), ptr(self.offsets), ptr(sel_d), n, L,
                  self.wp.cls_id, self.wp.sep_id, self.wp.pad_id, ptr(ids), ptr(mask),
                  stream_ptr(self.device))
        return ids, mask
