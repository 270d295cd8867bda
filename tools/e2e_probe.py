"""Where the end-to-end main.py step loses to bench.py's synthetic train leg: the same
model / optimizer / TrainState as src.train.train on tools/e2e_train.py's corpus, with
one ingredient of the real loop changed at a time.

    python tools/e2e_probe.py [--steps 40]

  loop      src.train's loop body: PairSampler -> DeviceCorpus batch + BERT on the
            prefetch stream -> heads step (queue off: step < queue_start_steps)
  loop+q    the same with the 12544-key queue in the loss (the bench's steady state)
  presel    the sampler's batches drawn beforehand (no host sampling in the loop)
  fixed     one corpus batch, resident, reused every step (no gather / pad launch)
  synth     bench.py's synthetic batch (uniform ids, L = 64), reused every step
Prints ms per step (wall clock over the timed steps, device synchronised) per variant,
twice, interleaved."""
import argparse
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "information-retrieval-with-contrastive-learning_amd")
for p in (ROOT, PKG, os.path.join(ROOT, "tools")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import yaml  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--by-len", action="store_true")
    ap.add_argument("--lens", default="", help="with --by-len: only these padded L")
    a = ap.parse_args()
    import e2e_train as E
    import bench

    tmp = tempfile.mkdtemp()
    vocab = os.path.join(tmp, "vocab.txt")
    syl = E.make_vocab(vocab)
    E.make_corpus(os.path.join(tmp, "docs_sentence.pkl"), syl, max_words=26)
    with open(os.path.join(PKG, "config.yaml")) as f:
        cfg = yaml.safe_load(f)
    cfg["dataset"]["docs_sentence"] = os.path.join(tmp, "docs_sentence.pkl")
    cfg["bert"] = {"name": "bert-base-uncased", "vocab": vocab, "seed": 0}
    cfg["train"].update(batch_size=256, acml_batch_size=256, total_steps=10 ** 6, n_jobs=0)
    import argparse as ap_

    from irc_amd.corpus import DeviceCorpus
    from src.dataset import PairSampler
    from src.model import build_model, get_optimizer
    from src.train import TrainState

    dev = torch.device("cuda:0")
    args = ap_.Namespace(config=cfg, loss="InfoNCE", model="LSTM", opt="adam", sample="uniform",
                         data="doc", seed=0)
    torch.manual_seed(0)
    model = build_model(args).to(dev).train()
    opt = get_optimizer(args, model)
    st = TrainState(args, model, opt)
    sampler = PairSampler(args)
    corpus = DeviceCorpus(sampler.dataset.data, model.bert_tokenizer, dev)
    sels = []
    for idx, sel in sampler:
        sels.append((idx, sel))
        if len(sels) >= 200:
            break
    fixed = list(corpus.batch(sels[0][1]))
    syn_ids, syn_mask = bench.synthetic_batch(512, 64, 1337)
    syn_ids, syn_mask = syn_ids.to(dev), syn_mask.to(dev)
    B = 256

    def run(kind, n):
        model.add_queue_to_loss = kind == "loop+q"
        it = iter(sampler) if kind in ("loop", "loop+q") else None
        k = [0]

        def nxt():
            if it is not None:
                b = next(it, None)
                if b is None:
                    return nxt_restart()
                return b
            k[0] += 1
            return sels[k[0] % len(sels)]

        def nxt_restart():
            nonlocal it
            it = iter(sampler)
            return next(it)

        def issue(b):
            if kind == "fixed":
                return model.bert_extract_async(fixed[0], fixed[1], B, inputs_ready=True)
            if kind == "synth":
                return model.bert_extract_async(syn_ids, syn_mask, B, inputs_ready=True)
            return model.bert_extract_corpus_async(corpus, b[1], B)

        pending = issue(nxt())
        times = []
        for s in range(n + 5):
            if s == 5:
                torch.cuda.synchronize()
                t0 = time.perf_counter()
            handle = pending
            pending = issue(nxt())
            st.micro_batch(B, lambda h=handle: model.forward_features(*model.features_ready(h)),
                           sync_loss=False)
        torch.cuda.synchronize()
        model.features_ready(pending)
        return (time.perf_counter() - t0) * 1e3 / n

    if a.by_len:
        # real corpus batches grouped by their padded L, against synthetic batches of
        # the same L (token ids uniform, lengths uniform in [10, L]): data vs length
        by_len = {}
        for idx, sel in sels:
            ids, mask = corpus.batch(sel)
            by_len.setdefault(ids.shape[1], (ids, mask))
        keep = {int(v) for v in a.lens.split(",") if v}
        for L in sorted(by_len):
            if keep and L not in keep:
                continue
            sids, smask = bench.synthetic_batch(512, L, 1337)
            for name, (i_, m_) in (("real", by_len[L]), ("synth", (sids.to(dev), smask.to(dev)))):
                fixed[0], fixed[1] = i_, m_
                ms = run("fixed", a.steps)
                print(f"L={L:3d} {name:5s} {ms:7.3f} ms/step  {256 / ms * 1e3:8.0f} pairs/s",
                      flush=True)
        return
    for rep in range(2):
        for kind in ("loop", "loop+q", "presel", "fixed", "synth"):
            ms = run(kind, a.steps)
            print(f"{kind:7s} {ms:7.3f} ms/step  {256 / ms * 1e3:8.0f} pairs/s", flush=True)


if __name__ == "__main__":
    main()
