"""End-to-end training throughput through the drop-in entrypoint (main.py ->
src.train.train: DataLoader workers, host WordPiece tokenisation + joint
padding, frozen-BERT prefetch, heads, loss, optimizer) at the C2 shapes, next
to the host tokenizer's own rate -- the measurement SURVEY 8f rank 1 asks for
before moving tokenisation to the GPU.

    python tools/e2e_train.py [--steps 30] [--workers 6]

Synthetic corpus: 20k documents x 3-8 sentences of 8-26 words (--max-words); each word is
1-3 syllables from a vocabulary that holds the syllables as words and as
'##' continuation pieces, so WordPiece does real greedy longest-match splits
(the offline image has no bert-base-uncased vocab)."""
import argparse
import os
import pickle
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "information-retrieval-with-contrastive-learning_amd")
for p in (ROOT, PKG):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import yaml  # noqa: E402


def make_vocab(path, size=30522):
    cons, vows = "bcdfghjklmnprstvwz", "aeiou"
    syl = [c + v for c in cons for v in vows] + [c + v + e for c in cons for v in vows
                                                  for e in "nrst"]
    toks = ["[PAD]", "[UNK]", "[CLS]", "[SEP]", "[MASK]"] + list("abcdefghijklmnopqrstuvwxyz")
    toks += ["##" + ch for ch in "abcdefghijklmnopqrstuvwxyz"] + list(".,;:!?'\"()-")
    toks += syl + ["##" + s for s in syl]
    rng = np.random.default_rng(0)
    words = set()
    while len(toks) + len(words) < size:
        words.add("".join(rng.choice(syl, rng.integers(2, 4))))
    toks += sorted(words)
    with open(path, "w") as f:
        f.write("\n".join(toks[:size]) + "\n")
    return syl


def make_corpus(path, syl, n_docs=20000, max_words=20):
    rng = np.random.default_rng(1)
    docs = []
    for _ in range(n_docs):
        sents = []
        for _ in range(rng.integers(3, 9)):
            words = ["".join(rng.choice(syl, rng.integers(1, 4)))
                     for _ in range(rng.integers(8, max_words + 1))]
            sents.append(" ".join(words).capitalize() + ".")
        docs.append(sents)
    with open(path, "wb") as f:
        pickle.dump(docs, f)
    return docs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--workers", type=int, default=6)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--max-words", type=int, default=26,
                    help="words per sentence 8..max (26: a joint batch of 512 pads to L ~ 64, the C2 "
                         "bench sequence length; 20: L ~ 52; 30: L ~ 72)")
    args = ap.parse_args()
    tmp = tempfile.mkdtemp()
    vocab = os.path.join(tmp, "vocab.txt")
    syl = make_vocab(vocab)
    docs = make_corpus(os.path.join(tmp, "docs_sentence.pkl"), syl, max_words=args.max_words)

    from irc_amd.tokenizer import load_tokenizer

    tok = load_tokenizer(vocab)
    sents = [s for d in docs[:400] for s in d][:2 * args.batch]
    t = tok(sents, padding=True, truncation=True, return_tensors="pt")
    reps, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < 5.0:
        t = tok(sents, padding=True, truncation=True, return_tensors="pt")
        reps += 1
    tok_rate = reps * len(sents) / (time.perf_counter() - t0)
    print(f"host tokenizer: {tok_rate:.0f} sentences/s = {tok_rate / 2:.0f} pairs/s "
          f"(joint batch of {len(sents)}, padded L = {t['input_ids'].shape[1]}, "
          f"{t['attention_mask'].sum().item() / len(sents):.1f} tokens/sentence)", flush=True)

    with open(os.path.join(PKG, "config.yaml")) as f:
        cfg = yaml.safe_load(f)
    cfg["dataset"]["docs_sentence"] = os.path.join(tmp, "docs_sentence.pkl")
    cfg["bert"] = {"name": "bert-base-uncased", "vocab": vocab, "seed": 0}
    cfg["train"].update(batch_size=args.batch, acml_batch_size=args.batch,
                        total_steps=args.steps, log_step=10 ** 6, n_jobs=args.workers)
    cpath = os.path.join(tmp, "config.yaml")
    with open(cpath, "w") as f:
        yaml.safe_dump(cfg, f)

    from src import train as T

    stamps, events = [], []
    orig = T.TrainState.micro_batch

    def timed(self, *a, **k):
        out = orig(self, *a, **k)
        stamps.append(time.perf_counter())
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()  # the step's work on the training stream (it joins the others)
        events.append(ev)
        return out

    # The rate is taken between device events recorded after step w and after the
    # last step, so the host's end-of-run work (checkpoint save, writer close) is
    # not charged to the loop; host stalls between steps (DataLoader, sampling,
    # tokenisation) still show as gaps between the events.
    T.TrainState.micro_batch = timed
    # host-time breakdown of the loop (seconds spent inside each call)
    from src.contrastor import contrastive_module as CM

    spent = {"tokenize": [], "bert_issue": [], "step_issue": [], "loader_next": []}

    def wrap(obj, name, key):
        f = getattr(obj, name)

        def g(*a, **k):
            t0 = time.perf_counter()
            try:
                return f(*a, **k)
            finally:
                spent[key].append(time.perf_counter() - t0)
        setattr(obj, name, g)

    wrap(CM.RetrievalModelWrapper, "tokenize", "tokenize")
    lens = []
    f_issue = CM.RetrievalModelWrapper.bert_extract_async

    def issue(self, ids, mask, n, **kw):
        lens.append(ids.shape[1])
        return f_issue(self, ids, mask, n, **kw)
    CM.RetrievalModelWrapper.bert_extract_async = issue
    wrap(CM.RetrievalModelWrapper, "bert_extract_async", "bert_issue")
    wrap(T.TrainState, "micro_batch", "step_issue")
    # host time the loop spends waiting in next(it) on the DataLoader
    from torch.utils.data import dataloader as DL

    for cls in (DL._SingleProcessDataLoaderIter, DL._MultiProcessingDataLoaderIter):
        wrap(cls, "__next__", "loader_next")
    t_start = time.perf_counter()
    import main as entry

    entry.main(["--config", cpath, "--gpu", "0", "--logdir", os.path.join(tmp, "log"),
                "--ckptdir", os.path.join(tmp, "ckpt")])
    torch.cuda.synchronize()
    t_end = time.perf_counter()
    w = min(5, len(stamps) - 2)
    dt = events[w].elapsed_time(events[-1]) * 1e-3 / (len(stamps) - 1 - w)
    print(f"end-to-end main.py train: {args.batch / dt:.0f} pairs/s ({dt * 1e3:.2f} ms/step over "
          f"{len(stamps) - 1 - w} steps, {args.workers} DataLoader workers, B = {args.batch})")
    tot = t_end - t_start
    print("host time per call, median after warm-up (ms): " + ", ".join(
        f"{k} {np.median(v[w:]) * 1e3:.2f}" for k, v in spent.items()) +
        f"; whole run {tot * 1e3 / len(stamps):.2f} per step (incl. startup); padded L mean "
        f"{np.mean(lens):.1f} (bench.py's synthetic batch: L = 64)")
    vals, cnt = np.unique(np.asarray(lens), return_counts=True)
    print("padded L histogram: " + ", ".join(f"{v}: {c}" for v, c in zip(vals, cnt)))


if __name__ == "__main__":
    main()
