"""GPU WordPiece + joint padding (irc_amd.wordpiece, csrc/wordpiece.hip) against
the host tokenizer the reference calls (BertTokenizer, padding=True,
truncation=True: src/contrastor/contrastive_module.py:36-41).

The CPU test replays the kernel's algorithm in Python over the device tables
(test double of the kernel) to pin the table derivation; the GPU tests compare
the kernel's ids / masks with the tokenizer's, token for token."""
import os
import sys

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))


@pytest.fixture(scope="module")
def hf_tok(tmp_path_factory):
    from transformers import BertTokenizer

    from e2e_train import make_vocab

    path = str(tmp_path_factory.mktemp("vocab") / "vocab.txt")
    make_vocab(path, 30000)
    with open(path, "a") as f:
        f.write("\n".join(["中", "文", "字", "##ing", "hello", "world", "istanbul", "nandu",
                           "café", "##é", "über", "ﬁ", "ß", "σ", "ο", "δ"]) + "\n")
    return BertTokenizer(path, model_max_length=512)


def _corpus(rng):
    from e2e_train import make_vocab  # noqa: F401  (syllable words below)

    cons, vows = "bcdfghjklmnprstvwz", "aeiou"
    syl = [c + v for c in cons for v in vows]
    special = ["Héllo, WORLD!", "ñandú", "中文字 and 中", "a​b", "c\xa0d", "e　f",
               "g\x01h", "İstanbul", "ﬁne", "x́y", "ΟΔΟΣ", "naïve café's über-cool",
               "tabs\tand\nnewlines\r", "", "   ", "!!!???", "emoji 😀 ok", "𝔘𝔫𝔦", "q" * 101,
               "Z" + "ba" * 60, "xyzzy qwfp", "[brackets] (parens) {braces}", "don't-stop",
               "😀" * 3, "�\x00end", "ṩ̇", "ㄱㅏ 한국어", "１２３ＡＢＣ", "e.g. U.S.A."]
    out = list(special)
    for _ in range(400):
        words = []
        for _ in range(rng.integers(1, 40)):
            w = "".join(rng.choice(syl, rng.integers(1, 5)))
            if rng.random() < 0.1:
                w = w.capitalize()
            if rng.random() < 0.1:
                w += rng.choice(list(",.;:!?"))
            words.append(w)
        out.append(" ".join(words))
    out.append(" ".join(["ba"] * 700))  # truncated at 512 tokens
    return out


def _emulate(wp_tables, texts, max_tokens):
    """The kernel's algorithm over the device tables, in Python (test double)."""
    cmap, cpool, cls, vocab_pieces, unk, max_piece = wp_tables
    rows = []
    for t in texts:
        out = []
        word = []

        def flush():
            if len(word) > 100:
                out.append(unk)
            elif word:
                ids, start = [], 0
                while start < len(word):
                    got = None
                    for l in range(min(len(word) - start, max_piece), 0, -1):
                        key = (start > 0, tuple(word[start:start + l]))
                        if key in vocab_pieces:
                            got = (vocab_pieces[key], start + l)
                            break
                    if got is None:
                        ids = [unk]
                        break
                    ids.append(got[0])
                    start = got[1]
                out.extend(ids)
            word.clear()

        for ch in t:
            m = int(cmap[ord(ch)])
            kind = m & 3
            outs = [m >> 8] if kind == 1 else \
                [int(x) for x in cpool[(m >> 8):(m >> 8) + ((m >> 2) & 15)]] if kind == 2 else []
            for cp in outs:
                c = cls[cp]
                if c == 1:
                    flush()
                elif c == 2:
                    flush()
                    word.append(cp)
                    flush()
                else:
                    word.append(cp)
        flush()
        rows.append(out[:max_tokens])
    return rows


def test_tables_reproduce_tokenizer_cpu(hf_tok):
    from irc_amd import wordpiece as W

    cmap, cpool, cls = W._char_tables(hf_tok.backend_tokenizer)
    vocab = hf_tok.get_vocab()
    pieces = {}
    for tok, i in vocab.items():
        cont = tok.startswith("##") and len(tok) > 2
        body = tok[2:] if cont else tok
        pieces[(cont, tuple(ord(c) for c in body))] = i
    hid, hh, voff, vcps, vcont, max_piece = W._vocab_tables(vocab, "##")
    texts = _corpus(np.random.default_rng(0))
    got = _emulate((cmap, cpool, cls, pieces, vocab["[UNK]"], max_piece), texts, 510)
    ref = hf_tok(texts, truncation=True)["input_ids"]
    for t, g, r in zip(texts, got, ref):
        assert [2] + g + [3] == r, repr(t)


def test_table_cache_rejects_tampered_file(hf_tok, tmp_path, monkeypatch):
    """the cached normaliser / pre-tokeniser tables live in a per-user
    cache directory and are spot-checked on load: a tampered or truncated file is
    rebuilt, never used."""
    from irc_amd import wordpiece as W

    monkeypatch.setenv("XDG_CACHE_HOME", str(tmp_path))
    backend = hf_tok.backend_tokenizer
    cmap, cpool, cls = W._char_tables(backend)  # builds into tmp_path/irc_amd
    files = list((tmp_path / "irc_amd").glob("wordpiece_chars_*.npz"))
    assert len(files) == 1
    bad = cmap.copy()
    bad[ord("a")] = (ord("b") << 8) | 1  # 'a' would normalise to 'b'
    np.savez(files[0], cmap=bad, cpool=cpool, cls=cls)
    assert not W._tables_valid(backend.normalizer, backend.pre_tokenizer, bad, cpool, cls)
    c2, p2, k2 = W._char_tables(backend)
    assert np.array_equal(c2, cmap) and np.array_equal(p2, cpool) and np.array_equal(k2, cls)
    files[0].write_bytes(b"truncated")
    c3, _, _ = W._char_tables(backend)
    assert np.array_equal(c3, cmap)


@pytest.mark.gpu
def test_gpu_wordpiece_matches_tokenizer(gpu, hf_tok):
    from irc_amd.wordpiece import GpuWordPiece

    texts = _corpus(np.random.default_rng(1))
    ids, mask = GpuWordPiece(hf_tok, gpu)(texts)
    ref = hf_tok(texts, padding=True, truncation=True, return_tensors="pt")
    assert torch.equal(ids.cpu(), ref["input_ids"])
    assert torch.equal(mask.cpu(), ref["attention_mask"])


@pytest.mark.gpu
def test_gpu_wordpiece_training_batch(gpu, hf_tok):
    """A C2 micro-batch (2 x 256 sentences), repeated calls, and the empty batch."""
    from irc_amd.wordpiece import GpuWordPiece

    rng = np.random.default_rng(2)
    cons, vows = "bcdfghjklmnprstvwz", "aeiou"
    syl = [c + v for c in cons for v in vows]
    wp = GpuWordPiece(hf_tok, gpu)
    for _ in range(3):
        texts = [" ".join("".join(rng.choice(syl, rng.integers(1, 4)))
                          for _ in range(rng.integers(8, 31))).capitalize() + "."
                 for _ in range(512)]
        ids, mask = wp(texts)
        ref = hf_tok(texts, padding=True, truncation=True, return_tensors="pt")
        assert torch.equal(ids.cpu(), ref["input_ids"])
        assert torch.equal(mask.cpu(), ref["attention_mask"])
    ids, mask = wp([])
    assert ids.shape[0] == 0


def _vocab_worker(n):
    from irc_amd.tokenizer import synthetic_vocab_file
    return synthetic_vocab_file(n)


def test_synthetic_vocab_file_concurrent_writers():
    """Ranks that start together all create the synthetic vocab file: each writes its
    own temporary copy and renames it into place, so none fails on a rename (the
    2-rank DP test once did) and the file holds the full vocabulary."""
    import multiprocessing as mp
    import tempfile

    n = 101
    path = os.path.join(tempfile.gettempdir(), f"irc_synthetic_vocab_{n}.txt")
    if os.path.exists(path):
        os.remove(path)
    ctx = mp.get_context("spawn")
    with ctx.Pool(4) as pool:
        paths = pool.map(_vocab_worker, [n] * 16)
    assert set(paths) == {path}
    with open(path) as f:
        assert len(f.read().split()) == n


@pytest.mark.gpu
def test_device_corpus_batches_match_tokenizer(gpu, hf_tok):
    """irc_amd.corpus.DeviceCorpus: the corpus tokenised once (in several chunks)
    and packed in HBM; any selection of its sentences, gathered and jointly padded
    by irc_pair_batch, is token-exact with the tokenizer's padding=True,
    truncation=True output for those sentences (incl. one over the 512 limit)."""
    from irc_amd.corpus import DeviceCorpus

    texts = _corpus(np.random.default_rng(3))
    long_one = " ".join(["supercalifragilistic"] * 400)  # > 510 pieces: truncated
    docs = [texts[i:i + 5] for i in range(0, len(texts), 5)] + [[long_one, "short one ."]]
    flat = [s for d in docs for s in d]
    corpus = DeviceCorpus(docs, hf_tok, gpu, chunk=16)  # several tokenisation chunks
    assert corpus.n_sentences == len(flat)
    rng = np.random.default_rng(4)
    for n in (1, 7, 64, len(flat)):
        sel = rng.choice(len(flat), n, replace=False)
        ids, mask = corpus.batch(sel)
        ref = hf_tok([flat[i] for i in sel], padding=True, truncation=True, return_tensors="pt")
        assert torch.equal(ids.cpu(), ref["input_ids"]), n
        assert torch.equal(mask.cpu(), ref["attention_mask"]), n
    sel = np.array([corpus.sentence_index(len(docs) - 1, 0)])
    ids, _ = corpus.batch(sel)
    assert ids.shape[1] == 512
