"""Host-side WordPiece tokenizer plumbing (not on the kernel path).

The reference calls ``BertTokenizer.from_pretrained('bert-base-uncased')``
(src/contrastor/contrastive_module.py:32), a network fetch.  Offline, this
loads a local vocab.txt / tokenizer directory when given, otherwise it builds a
deterministic synthetic vocabulary ([PAD] [UNK] [CLS] [SEP] [MASK] w0 w1 ...)
so the pipeline runs end to end without network access.
"""
from __future__ import annotations

import os
import tempfile
import warnings

SPECIALS = ["[PAD]", "[UNK]", "[CLS]", "[SEP]", "[MASK]"]


def synthetic_vocab_file(vocab_size: int = 30522) -> str:
    path = os.path.join(tempfile.gettempdir(), f"irc_synthetic_vocab_{vocab_size}.txt")
    if not os.path.exists(path):
        toks = SPECIALS + [f"w{i}" for i in range(vocab_size - len(SPECIALS))]
        # per-process temporary name: ranks started together each write their own
        # copy and rename it into place atomically (the same content either way)
        tmp = f"{path}.{os.getpid()}.tmp"
        with open(tmp, "w") as f:
            f.write("\n".join(toks) + "\n")
        os.replace(tmp, path)
    return path


# bert-base-uncased's tokenizer_config: `truncation=True` (contrastive_module.py:38,97)
# cuts at model_max_length, so a bare vocab file gets the same 512 limit
MODEL_MAX_LENGTH = 512


def load_tokenizer(name_or_path: str | None, vocab_size: int = 30522):
    from transformers import BertTokenizer

    if name_or_path and os.path.isdir(name_or_path):
        return BertTokenizer.from_pretrained(name_or_path, local_files_only=True)
    if name_or_path and os.path.isfile(name_or_path):
        return BertTokenizer(name_or_path, model_max_length=MODEL_MAX_LENGTH)
    warnings.warn("no local BERT vocab given: using a synthetic offline vocabulary "
                  f"({vocab_size} tokens)", stacklevel=2)
    return BertTokenizer(synthetic_vocab_file(vocab_size), model_max_length=MODEL_MAX_LENGTH)
