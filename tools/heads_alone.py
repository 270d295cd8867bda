"""The C2 heads step alone (3-layer BiLSTM query + key encoders, InfoNCE with the queue,
backward, clip + Adam + momentum + enqueue) on fixed BERT features, no BERT beside it:
wall ms per step, and, under rocprofv3 --kernel-trace, each heads kernel's time alone.

    python tools/heads_alone.py [--steps 20]"""
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
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    from src.model import build_model, get_optimizer
    from src.train import TrainState

    dev = torch.device("cuda:0")
    ns = argparse.Namespace(config=bench.c2_config(), loss="InfoNCE", model="LSTM", opt="adam",
                            sample="uniform")
    torch.manual_seed(1337)
    model = build_model(ns).to(dev).train()
    model.add_queue_to_loss = True
    st = TrainState(ns, model, get_optimizer(ns, model))
    ids, mask = bench.synthetic_batch(2 * bench.TRAIN_B, bench.TRAIN_L, 1337)
    feats = model.bert_extract_ids(ids.to(dev), mask.to(dev), bench.TRAIN_B)
    torch.cuda.synchronize()

    def step():
        st.micro_batch(bench.TRAIN_B, lambda: model.forward_features(*feats), sync_loss=False)

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize()
    print(f"heads step alone {(time.perf_counter() - t) / a.steps * 1e3:.3f} ms")


if __name__ == "__main__":
    main()
