"""Kernel-trace helper for the C2 step's BERT / heads overlap: --mode bert runs only
the frozen-BERT forward (one stream), --mode overlap the overlapped training step
(BERT prefetch on its side stream beside the heads), --mode heads the heads step
alone on cached features.  Run each under rocprofv3 --kernel-trace --stats and
compare the BERT kernels' average durations.

    python tools/overlap_prof.py --mode overlap --steps 20
"""
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
    ap.add_argument("--mode", choices=["bert", "overlap", "heads"], default="overlap")
    ap.add_argument("--steps", type=int, default=20)
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
    if a.mode == "bert":
        fn = lambda: model.bert_extract_ids(ids, mask, bench.TRAIN_B)  # noqa: E731
    elif a.mode == "heads":
        feats = model.bert_extract_ids(ids, mask, bench.TRAIN_B)
        fn = lambda: st.micro_batch(bench.TRAIN_B, lambda: model.forward_features(*feats),  # noqa: E731
                                    sync_loss=False)
    else:
        pending = [model.bert_extract_async(ids, mask, bench.TRAIN_B)]

        def fn():
            handle = pending[0]
            pending[0] = model.bert_extract_async(ids, mask, bench.TRAIN_B, inputs_ready=True)
            st.micro_batch(bench.TRAIN_B, lambda: model.forward_features(*model.features_ready(handle)),
                           sync_loss=False)
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        fn()
    torch.cuda.synchronize()
    print(f"mode {a.mode}: {(time.perf_counter() - t0) / a.steps * 1e3:.3f} ms per step", flush=True)


if __name__ == "__main__":
    main()
