"""GPU WordPiece tokenisation + joint padding.

Drop-in for the reference's per-micro-batch host call
``bert_tokenizer(texts, padding=True, truncation=True, return_tensors='pt')``
(src/contrastor/contrastive_module.py:36-41, 96-100): the host only joins the
sentences' UTF-8 bytes; normalisation, pre-tokenisation, WordPiece and padding
run in csrc/wordpiece.hip (irc_wordpiece / irc_wordpiece_pad).

The device tables are derived from the tokenizer object itself, so the result
is the tokenizer's, character for character:
  * cmap / cpool: the BertNormalizer's output for every code point (it acts per
    character: clean text, CJK spacing, NFD + accent strip, lowercase);
  * cls: whitespace / punctuation as the BertPreTokenizer splits them;
  * the vocab as an open-addressing FNV-1a table over code points, pieces
    stored without their "##" (continuation flag kept separately).
Building cmap / cls calls the tokenizer's Rust normaliser and pre-tokeniser once
per code point (~4 s); the result is cached in a per-user cache directory, keyed
by the tokenizers version and the normaliser / pre-tokeniser configuration, and
spot-checked against the tokenizer on load (rebuilt when a check fails).

Not reproduced: special-token strings typed literally in the input text
("[SEP]" inside a sentence), which the host tokenizer matches before
normalisation; they are tokenised as ordinary text here.
"""
from __future__ import annotations

import hashlib
import json
import os
import tempfile

import numpy as np
import torch

from . import _lib
from ._torch import ptr, stream_ptr

N_CP = 0x110000
FNV_P = 16777619
SEED_WORD = 2166136261
SEED_CONT = 0x9E3779B9
MAXW = 100
MAXP = 64


def _fnv(seed, cps):
    h = seed
    for c in cps:
        h = ((h ^ c) * FNV_P) & 0xFFFFFFFF
    return h


def _cache_dir():
    """Per-user cache directory (not the shared temp directory: a stale or planted
    file there would change every token id the GPU path produces)."""
    base = os.environ.get("XDG_CACHE_HOME") or os.path.join(os.path.expanduser("~"), ".cache")
    d = os.path.join(base, "irc_amd")
    try:
        os.makedirs(d, mode=0o700, exist_ok=True)
        return d
    except OSError:  # read-only home: a private directory of our own under tmp
        d = os.path.join(tempfile.gettempdir(), f"irc_amd-{os.getuid()}")
        os.makedirs(d, mode=0o700, exist_ok=True)
        return d


def _char_entry(norm, pre, c):
    """(cmap word, pool code points, cls) of code point c: the normaliser's output
    (1 char inline, several in the pool) and the pre-tokeniser's class."""
    ch = chr(c)
    out = norm.normalize_str(ch)
    word, pool = 0, []
    if len(out) == 1:
        word = (ord(out) << 8) | 1
    elif len(out) > 1:
        if len(out) > 15:
            raise ValueError(f"normaliser maps U+{c:04X} to {len(out)} characters")
        word = (len(out) << 2) | 2  # pool offset added by the caller
        pool = [ord(o) for o in out]
    pieces = pre.pre_tokenize_str("a" + ch + "a")
    cls = 0
    if len(pieces) == 2 and [p[0] for p in pieces] == ["a", "a"]:
        cls = 1
    elif len(pieces) == 3 and pieces[1][0] == ch:
        cls = 2
    return word, pool, cls


def _tables_valid(norm, pre, cmap, cpool, cls, n_check=512):
    """Shapes / dtypes of a cached table set, and a spot check of n_check code
    points (ASCII, Latin-1 and a seeded random sample) against the tokenizer."""
    if cmap.shape != (N_CP,) or cls.shape != (N_CP,) or cmap.dtype != np.uint32 or \
            cls.dtype != np.uint8 or cpool.dtype != np.uint32 or cpool.ndim != 1:
        return False
    rng = np.random.default_rng(0x1D)
    sample = list(range(0x20, 0x100)) + [int(c) for c in rng.integers(0x100, N_CP, n_check)]
    for c in sample:
        if 0xD800 <= c < 0xE000:
            continue
        word, pool, cl = _char_entry(norm, pre, c)
        if int(cls[c]) != cl:
            return False
        got = int(cmap[c])
        if pool:
            off, n = got >> 8, (got >> 2) & 15
            if (got & 3) != 2 or n != len(pool) or off + n > len(cpool) or \
                    [int(x) for x in cpool[off:off + n]] != pool:
                return False
        elif got != word:
            return False
    return True


def _char_tables(backend):
    """(cmap uint32 [N_CP], cpool uint32, cls uint8 [N_CP]) from the tokenizer."""
    import tokenizers

    norm, pre = backend.normalizer, backend.pre_tokenizer
    key = json.dumps([tokenizers.__version__, str(norm.__getstate__()),
                      str(pre.__getstate__())])
    tag = hashlib.sha1(key.encode()).hexdigest()[:16]
    path = os.path.join(_cache_dir(), f"wordpiece_chars_{tag}.npz")
    if os.path.exists(path):
        try:
            with np.load(path, allow_pickle=False) as z:  # our own cache file
                cmap, cpool, cls = z["cmap"], z["cpool"], z["cls"]
            if _tables_valid(norm, pre, cmap, cpool, cls):
                return cmap, cpool, cls
        except Exception:  # truncated / foreign file: rebuild below
            pass
    cmap = np.zeros(N_CP, np.uint32)
    cls = np.zeros(N_CP, np.uint8)
    pool = []
    for c in range(N_CP):
        if 0xD800 <= c < 0xE000:
            continue
        word, p, cls[c] = _char_entry(norm, pre, c)
        if p:
            word |= len(pool) << 8
            pool.extend(p)
        cmap[c] = word
    cpool = np.array(pool if pool else [0], np.uint32)
    tmp = path + f".{os.getpid()}.npz"
    np.savez(tmp, cmap=cmap, cpool=cpool, cls=cls)
    os.replace(tmp, path)
    return cmap, cpool, cls


def _vocab_tables(vocab: dict, prefix: str):
    """Open-addressing table (size 4V rounded up to a power of two) of the
    pieces' code points, continuation pieces keyed with their own seed."""
    V = max(vocab.values()) + 1
    pieces = [None] * V
    for tok, i in vocab.items():
        pieces[i] = tok
    voff = np.zeros(V + 1, np.int32)
    vcont = np.zeros(V, np.uint8)
    cps = []
    for i, tok in enumerate(pieces):
        tok = tok or ""
        cont = tok.startswith(prefix) and len(tok) > len(prefix)
        body = tok[len(prefix):] if cont else tok
        vcont[i] = cont
        cps.extend(ord(ch) for ch in body)
        voff[i + 1] = len(cps)
    size = 1
    while size < 4 * V:
        size <<= 1
    hid = np.full(size, -1, np.int32)
    hh = np.zeros(size, np.uint32)
    max_piece = 1
    for i in range(V):
        body = cps[voff[i]:voff[i + 1]]
        if not body:
            continue
        if len(body) > MAXP:
            continue  # longer than any word the GPU matches (MAXW caps words at 100)
        max_piece = max(max_piece, len(body))
        h = _fnv(SEED_CONT if vcont[i] else SEED_WORD, body)
        j = h & (size - 1)
        while hid[j] >= 0:
            j = (j + 1) & (size - 1)
        hid[j], hh[j] = i, h
    return hid, hh, voff, np.array(cps if cps else [0], np.uint32), vcont, max_piece


class GpuWordPiece:
    """``__call__(texts) -> (input_ids, attention_mask)`` int64 [n, L] on the
    device, equal to the host tokenizer's padding=True, truncation=True output
    (max_length = min(tokenizer.model_max_length, 512), the reference's
    bert-base-uncased limit)."""

    def __init__(self, hf_tokenizer, device, max_length: int | None = None):
        be = hf_tokenizer.backend_tokenizer
        model = be.model
        if type(model).__name__ != "WordPiece":
            raise ValueError("GpuWordPiece needs a WordPiece tokenizer")
        if int(model.max_input_chars_per_word) != MAXW:
            raise ValueError("max_input_chars_per_word != 100")
        self.device = torch.device(device)
        ml = max_length or min(int(hf_tokenizer.model_max_length), 512)
        self.max_tokens = ml - 2
        vocab = hf_tokenizer.get_vocab()
        self.unk = vocab[model.unk_token]
        self.cls_id = hf_tokenizer.cls_token_id
        self.sep_id = hf_tokenizer.sep_token_id
        self.pad_id = hf_tokenizer.pad_token_id
        cmap, cpool, cls = _char_tables(be)
        hid, hh, voff, vcps, vcont, self.max_piece = _vocab_tables(
            vocab, model.continuing_subword_prefix)
        up = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(self.device)  # noqa: E731
        self._t = {"cmap": up(cmap.view(np.int32)), "cpool": up(cpool.view(np.int32)),
                   "cls": up(cls), "hid": up(hid), "hh": up(hh.view(np.int32)),
                   "voff": up(voff), "vcps": up(vcps.view(np.int32)), "vcont": up(vcont)}
        self.hsize = hid.shape[0]
        # high priority: its few waves are dispatched ahead of the training step's
        # GEMM workgroups queued on the other streams (the host waits on it)
        self.stream = torch.cuda.Stream(self.device, priority=-1)
        self._max_len = torch.zeros(1, dtype=torch.int32, device=self.device)
        self._host_len = torch.zeros(1, dtype=torch.int32, pin_memory=True)

    def _raw(self, texts, st):
        """WordPiece ids without special tokens on stream st: (tok int32 [n, max_tokens],
        tok_len int32 [n], the inputs kept alive); the longest length lands in
        self._max_len (device)."""
        n = len(texts)
        enc = [t.encode("utf-8") for t in texts]
        offs = np.zeros(n + 1, np.int64)
        np.cumsum([len(e) for e in enc], out=offs[1:])
        blob = np.frombuffer(b"".join(enc) or b"\0", np.uint8)
        with torch.cuda.stream(st):
            b = torch.from_numpy(blob.copy()).pin_memory().to(self.device, non_blocking=True)
            o = torch.from_numpy(offs).pin_memory().to(self.device, non_blocking=True)
            tok = torch.empty((max(n, 1), max(self.max_tokens, 1)), dtype=torch.int32,
                              device=self.device)
            tlen = torch.empty((max(n, 1),), dtype=torch.int32, device=self.device)
            t = self._t
            _lib.call("irc_wordpiece", ptr(b), ptr(o), n, ptr(t["cmap"]), ptr(t["cpool"]),
                      ptr(t["cls"]), ptr(t["hid"]), ptr(t["hh"]), self.hsize, ptr(t["voff"]),
                      ptr(t["vcps"]), ptr(t["vcont"]), self.max_piece, self.unk,
                      self.max_tokens, ptr(tok), ptr(tlen), ptr(self._max_len), stream_ptr(st))
        return tok, tlen, (b, o)

    def __call__(self, texts):
        texts = list(texts)
        n = len(texts)
        cur = torch.cuda.current_stream(self.device)
        st = self.stream  # independent of the compute in flight on `cur`: no wait
        tok, tlen, keep = self._raw(texts, st)
        with torch.cuda.stream(st):
            self._host_len.copy_(self._max_len, non_blocking=True)
            st.synchronize()  # this stream only: the tokenizer's own work
            L = max(int(self._host_len[0]), 2)
            ids = torch.empty((n, L), dtype=torch.int64, device=self.device)
            mask = torch.empty((n, L), dtype=torch.int64, device=self.device)
            _lib.call("irc_wordpiece_pad", ptr(tok), ptr(tlen), n, self.max_tokens, L, self.cls_id,
                      self.sep_id, self.pad_id, ptr(ids), ptr(mask), stream_ptr(st))
        cur.wait_stream(st)
        for x in (ids, mask):
            x.record_stream(cur)
        for x in (tok, tlen) + keep:
            x.record_stream(st)
        return ids, mask

    def tokenize_corpus(self, texts, chunk: int = 65536):
        """The whole sentence list tokenised once: (flat int32 ids, offsets int64
        [n + 1] on the device, host int32 lengths [n]) -- the DeviceCorpus layout."""
        texts = list(texts)
        n = len(texts)
        st = self.stream
        toks, lens = [], []
        for c0 in range(0, n, chunk):
            tok, tlen, keep = self._raw(texts[c0:c0 + chunk], st)
            toks.append((tok, tlen, keep))
            lens.append(tlen[:min(chunk, n - c0)])
        with torch.cuda.stream(st):
            tl = torch.cat(lens) if lens else torch.zeros(0, dtype=torch.int32, device=self.device)
            host_len = tl.cpu().numpy().astype(np.int32)  # synchronises st
        offs = np.zeros(n + 1, np.int64)
        np.cumsum(host_len, out=offs[1:])
        d_off = torch.from_numpy(offs).to(self.device)
        flat = torch.empty((max(int(offs[-1]), 1),), dtype=torch.int32, device=self.device)
        with torch.cuda.stream(st):
            for ci, (tok, tlen, _) in enumerate(toks):
                c0 = ci * chunk
                m = min(chunk, n - c0)
                _lib.call("irc_corpus_pack", ptr(tok), ptr(tlen), m, self.max_tokens,
                          ptr(d_off[c0:]), ptr(flat), stream_ptr(st))
            st.synchronize()
        return flat, d_off, host_len
