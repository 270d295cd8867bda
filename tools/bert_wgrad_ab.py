"""--model BERT step (bench.py run_train_bert's loop) with the trainable encoder's weight
gradients overlapped with its dX chain (BertEncoder.overlap_wgrad, on a side stream in
layer buckets) against all of them after the chain, interleaved A/B; optionally a split-K
cap on the overlapped ones (--cap).

    python tools/bert_wgrad_ab.py [--steps 10] [--reps 3] [--cap 0 128]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "information-retrieval-with-contrastive-learning_amd")):
    sys.path.insert(0, p)

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--cap", type=int, nargs="*", default=[0])
    ap.add_argument("--bucket", type=int, nargs="*", default=[4],
                    help="layers per weight-gradient bucket (reduce_bucket_layers)")
    a = ap.parse_args()
    from src.model import build_model, get_optimizer
    from src.train import TrainState

    dev = torch.device("cuda:0")
    cfg = bench.c2_config()
    ns = argparse.Namespace(config=cfg, loss="InfoNCE", model="BERT", opt="adam", sample="uniform")
    torch.manual_seed(1337)
    model = build_model(ns).to(dev).train()
    model.add_queue_to_loss = True
    st = TrainState(ns, model, get_optimizer(ns, model))
    ids, mask = bench.synthetic_batch(2 * bench.TRAIN_B, bench.TRAIN_L, 1337)
    ids, mask = ids.to(dev), mask.to(dev)
    enc = model.encoder_q

    def run(overlap, cap, bucket=4):
        enc.overlap_wgrad, enc.wgrad_max_blocks, enc.reduce_bucket_layers = overlap, cap, bucket
        for _ in range(3):
            st.micro_batch(bench.TRAIN_B, lambda: model.forward_ids(ids, mask, bench.TRAIN_B),
                           sync_loss=False)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            st.micro_batch(bench.TRAIN_B, lambda: model.forward_ids(ids, mask, bench.TRAIN_B),
                           sync_loss=False)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / a.steps

    for r in range(a.reps):
        dt = run(False, 0)
        print(f"rep {r} overlap=off       {dt * 1e3:7.2f} ms/step {bench.TRAIN_B / dt:8.0f} pairs/s",
              flush=True)
        for bucket in a.bucket:
            for cap in a.cap:
                dt = run(True, cap, bucket)
                print(f"rep {r} overlap=on bucket={bucket} cap={cap:<4d}{dt * 1e3:7.2f} ms/step "
                      f"{bench.TRAIN_B / dt:8.0f} pairs/s", flush=True)


if __name__ == "__main__":
    main()
