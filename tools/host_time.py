"""Host-side issue time of the C2 training step vs its wall time: whether the
Python/ctypes launch path, not the GPU, sets the step rate.

    python tools/host_time.py [--steps 30]"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "information-retrieval-with-contrastive-learning_amd"))

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=30)
    a = ap.parse_args()
    from src.model import build_model, get_optimizer
    from src.train import TrainState

    dev = torch.device("cuda:0")
    cfg = bench.c2_config()
    ns = argparse.Namespace(config=cfg, loss="InfoNCE", model="LSTM", opt="adam", sample="uniform")
    torch.manual_seed(1337)
    model = build_model(ns).to(dev).train()
    model.add_queue_to_loss = True
    st = TrainState(ns, model, get_optimizer(ns, model))
    ids, mask = bench.synthetic_batch(2 * bench.TRAIN_B, bench.TRAIN_L, 1337)
    ids, mask = ids.to(dev), mask.to(dev)
    pending = [model.bert_extract_async(ids, mask, bench.TRAIN_B)]

    hs = torch.cuda.current_stream(dev)

    def step():
        handle = pending[0]
        pending[0] = model.bert_extract_async(ids, mask, bench.TRAIN_B, inputs_ready=True)
        with torch.cuda.stream(hs):
            st.micro_batch(bench.TRAIN_B,
                           lambda: model.forward_features(*model.features_ready(handle)),
                           sync_loss=False)

    def timed(fn, n):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(n):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t) / n * 1e3

    feats = model.bert_extract_ids(ids, mask, bench.TRAIN_B)
    torch.cuda.synchronize()
    b_ms = timed(lambda: model.bert_extract_ids(ids, mask, bench.TRAIN_B), 10)
    h_ms = timed(lambda: st.micro_batch(bench.TRAIN_B, lambda: model.forward_features(*feats),
                                        sync_loss=False), 10)
    print(f"BERT forward alone {b_ms:.2f} ms, heads step alone {h_ms:.2f} ms")
    # BERT side-stream spans: an event before each encode and its done event
    spans = []
    from irc_amd._torch import side_stream as _ss

    bside = _ss(dev, "bert_prefetch")

    def step_ev():
        handle = pending[0]
        e0 = torch.cuda.Event(enable_timing=True)
        e0.record(bside)
        pending[0] = model.bert_extract_async(ids, mask, bench.TRAIN_B, inputs_ready=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e1.record(bside)
        spans.append((e0, e1))
        with torch.cuda.stream(hs):
            st.micro_batch(bench.TRAIN_B,
                           lambda: model.forward_features(*model.features_ready(handle)),
                           sync_loss=False)

    for _ in range(5):
        step_ev()
    torch.cuda.synchronize()
    spans.clear()
    tw = time.perf_counter()
    for _ in range(a.steps):
        step_ev()
    torch.cuda.synchronize()
    wall_ev = (time.perf_counter() - tw) / a.steps * 1e3
    busy = [s0.elapsed_time(s1) for s0, s1 in spans]
    gaps = [spans[i][1].elapsed_time(spans[i + 1][0]) for i in range(len(spans) - 1)]
    print(f"with side-stream events: wall {wall_ev:.2f} ms/step; BERT encode span "
          f"{sum(busy) / len(busy):.2f} ms, gap between encodes {sum(gaps) / len(gaps):.3f} ms")
    for _ in range(5):
        step()
    torch.cuda.synchronize()
    host = []
    t0 = time.perf_counter()
    for _ in range(a.steps):
        h0 = time.perf_counter()
        step()
        host.append(time.perf_counter() - h0)
    t_issue = time.perf_counter() - t0
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    host.sort()
    print(f"steps {a.steps}: wall {wall / a.steps * 1e3:.2f} ms/step, host issue "
          f"{t_issue / a.steps * 1e3:.2f} ms/step (median step() {host[len(host) // 2] * 1e3:.2f} ms, "
          f"max {host[-1] * 1e3:.2f})")


if __name__ == "__main__":
    main()
