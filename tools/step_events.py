"""Un-traced timeline of the overlapped C2 training step (bench.py's train leg): HIP
events on each stream at the phase boundaries -- the BERT forward of the next
micro-batch (prefetch stream), the key encoder's heads forward (its side stream),
the query encoder's heads forward and the rest of the step (loss, backward, update)
on the current stream.  A rocprofv3 trace adds host cost per launch and distorts the
overlap; a dozen events per step do not.

    python tools/step_events.py [--steps 30] [--L 64]

Prints, per phase, its mean start / end in ms relative to the previous step's end."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "information-retrieval-with-contrastive-learning_amd"))

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--L", type=int, default=64)
    a = ap.parse_args()
    from irc_amd._torch import side_stream
    from src.model import build_model, get_optimizer
    from src.train import TrainState

    dev = torch.device("cuda:0")
    ns = argparse.Namespace(config=bench.c2_config(), loss="InfoNCE", model="LSTM", opt="adam",
                            sample="uniform")
    torch.manual_seed(1337)
    model = build_model(ns).to(dev).train()
    model.add_queue_to_loss = True
    st = TrainState(ns, model, get_optimizer(ns, model))
    B = bench.TRAIN_B
    ids, mask = bench.synthetic_batch(2 * B, a.L, 1337)
    ids, mask = ids.to(dev), mask.to(dev)
    rec = []

    def ev(stream):
        e = torch.cuda.Event(enable_timing=True)
        e.record(stream)
        return e

    orig_s2v, orig_bert = model.seq2vec, model.bert_extract_async

    def seq2vec(feat, query=True):
        s = torch.cuda.current_stream(dev)
        e0 = ev(s)
        out = orig_s2v(feat, query=query)
        rec.append(("heads fwd q" if query else "heads fwd k", e0, ev(s)))
        return out

    def bert(*args, **kw):
        side = side_stream(dev, "bert_prefetch")
        e0 = ev(side)
        h = orig_bert(*args, **kw)
        rec.append(("BERT (next)", e0, ev(side)))
        return h

    model.seq2vec, model.bert_extract_async = seq2vec, bert
    pending = [model.bert_extract_async(ids, mask, B)]
    ends = []

    def step():
        handle = pending[0]
        pending[0] = model.bert_extract_async(ids, mask, B, inputs_ready=True)
        cur = torch.cuda.current_stream(dev)
        e0 = ev(cur)
        st.micro_batch(B, lambda: model.forward_features(*model.features_ready(handle)),
                       sync_loss=False)
        e1 = ev(cur)
        rec.append(("micro_batch (cur)", e0, e1))
        ends.append(e1)

    for _ in range(5):
        step()
    torch.cuda.synchronize()
    rec.clear()
    ends.clear()
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize()
    # per step i (1..): phases recorded during step i, relative to ends[i-1]
    per = {}
    n_per_step = len(rec) // a.steps
    for i in range(1, a.steps):
        base = ends[i - 1]
        for name, e0, e1 in rec[i * n_per_step:(i + 1) * n_per_step]:
            per.setdefault(name, []).append((base.elapsed_time(e0), base.elapsed_time(e1)))
    wall = sum(ends[i - 1].elapsed_time(ends[i]) for i in range(1, a.steps)) / (a.steps - 1)
    print(f"L={a.L} step {wall:.3f} ms (mean over {a.steps - 1}); phases relative to the "
          f"previous step's end:")
    for name, v in per.items():
        s = sum(x for x, _ in v) / len(v)
        e = sum(y for _, y in v) / len(v)
        print(f"  {name:20s} {s:7.3f} -> {e:7.3f} ms  ({e - s:6.3f})")


if __name__ == "__main__":
    main()
