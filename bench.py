"""Benchmark of the contrastive-training + dense-retrieval hot path on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--part all|train|scan]

For N>1 the driver launches one process per GPU (torch.distributed.run); each
rank reads RANK/LOCAL_RANK/WORLD_SIZE and RCCL (backend "nccl") carries the
collectives.  Rank 0 prints ONE JSON line.

Metric (BASELINE.json): "query-doc pairs/sec (train) + queries/sec @ top-k over
N docs".  `value` = training pairs/s (whole job); `retrieval` = queries/s.

* Training step (config C2): frozen BERT-base encoder (bf16 MFMA)
  over 2x256 synthetic sequences (L=64, token ids uniform in [5, 30522), seeded)
  -> 3-layer BiLSTM head 768->256x2->128 q fwd+bwd and momentum-encoder k fwd
  -> InfoNCE with the 12544-key queue -> clip + Adam + momentum update + enqueue.
  One step = 256 (anchor, positive) pairs.  N>1: data-parallel, each rank its
  own 256 pairs; q/k embeddings all-gathered over RCCL so the InfoNCE negatives
  span the global batch (256*N pairs), head gradients all-reduced before the
  step (scaling: weak).
* Retrieval (C2): each rank keeps a 100k-doc shard (D=768 bf16 unit-norm,
  seed 2024+rank) in HBM; one batch = 256 query embeddings all-gathered,
  scanned against every shard, reduced to the global top-100.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "information-retrieval-with-contrastive-learning_amd")
for _p in (ROOT, PKG):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X spec (MI355X_MICROARCH.md chip table)
FP8_PEAK_TFS = 5000.0  # dense fp8 MFMA (MI355X_MICROARCH.md chip table)
BF16_PEAK_TFS = 2500.0  # dense bf16 MFMA spec

METRIC = "query-doc pairs/sec (train) + queries/sec @ top-k over N docs, 1/2/4/8 GPU"
TRAIN_B, TRAIN_L, VOCAB = 256, 64, 30522
SCAN_N_PER_GPU, SCAN_Q, SCAN_D, SCAN_K = 100_000, 256, 768, 100
# C4 / C5 retrieval legs: 5M docs over 8 GPUs = 625k docs per GPU (weak scaling),
# 2048 queries per batch; C4 is BERT-large (D = 1024, bf16), C5 fp8 (D = 768, e4m3)
FP8_N_PER_GPU = 625_000
C4_Q, C4_D, C5_Q = 2048, 1024, 2048
# C3 retrieval leg: 1M docs over 4 GPUs = 250k x 768 bf16 per GPU (384 MB: larger
# than the 256 MiB Infinity Cache, so its Q sweep is HBM-honest), 1024 queries
C3_N_PER_GPU, C3_Q = 250_000, 1024
# Strong scaling (the north star's ">= 6x at 8 GPUs on a 5M-doc sharded
# corpus"): a FIXED corpus split N_total / world per rank, the same global query batch at
# every world size.  (name, docs in total, dtype, global queries, dim)
STRONG_LEGS = (("retrieval_strong_c3", 1_000_000, "bf16", C3_Q, SCAN_D),
               ("retrieval_strong_c4", 5_000_000, "bf16", C4_Q, C4_D),
               ("retrieval_strong_c5", 5_000_000, "fp8", C5_Q, SCAN_D))
STRONG_CHUNKS = 8  # the corpus is drawn in n_total / 8 chunks, each from its own seed, so
# the docs (and the top-k) are the same at 1, 2, 4 and 8 ranks
PP_MIN_Q = 192  # irc_scan_topk's filter runs on the ping-pong GEMM kernel from this Q
SCAN_DEPTH = 3  # query batches in flight in the retrieval legs (search_many; 2 -> 3: C2 +13%,
# profiles/r05_zd_scan_depth.txt; 4 on the one-call native loop: 3.41-3.59M against
# 3.97-3.99M queries/s at 3, interleaved on one box, profiles/r06_m/)


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor()


def _blas_threads():
    try:
        from threadpoolctl import threadpool_info

        return max((i.get("num_threads", 1) for i in threadpool_info()), default=1)
    except Exception:
        return int(os.environ.get("OMP_NUM_THREADS", "1"))


def _pmc_traffic(tag: str):
    """HBM bytes per launch from a committed rocprofv3 --pmc summary, if present
    (profiles/pmc_<tag>.json, written by tools/pmc_summary.py)."""
    p = os.path.join(ROOT, "profiles", f"pmc_{tag}.json")
    try:
        with open(p) as f:
            return float(json.load(f)["hbm_bytes_per_launch"])
    except Exception:
        return None


def _pmc_source(tag: str):
    p = os.path.join("profiles", f"pmc_{tag}.json")
    if not os.path.exists(os.path.join(ROOT, p)):
        return None
    return (f"{p}: HBM bytes per launch = (2*FETCH_SIZE + WRITE_SIZE)*1024 from separate "
            "rocprofv3 --pmc passes of the same bench part (tools/pmc_traffic.sh)")


def _prof(lib, name):
    tot, cnt, work = ctypes.c_double(0), ctypes.c_int64(0), ctypes.c_double(0)
    lib.irc_prof_query(name.encode(), ctypes.byref(tot), ctypes.byref(cnt), ctypes.byref(work))
    return tot.value / 1e3, cnt.value, work.value  # seconds, launches, work


def _alg_bytes(lib, traffic, name="gemm_bf16_bytes"):
    """Algorithmic HBM bytes per GEMM launch of the last profiled pass (operands
    read once, C written once, residual read once: gemm.hip gemm_alg_bytes; MX-fp8:
    codes + E8M0 scales, fp8_linear.hip irc_gemm_mx) and the PMC traffic's ratio to
    them (same dispatch set: the bench part's GEMM launches)."""
    _, n, b = _prof(lib, name)
    per = b / n if n else None
    return {"alg_bytes_per_launch": per,
            "traffic_over_alg": (traffic / per) if (traffic and per) else None}


def _max_over_ranks(x, dev, world):
    if world == 1:
        return x
    t = torch.tensor([x], device=dev, dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def synthetic_batch(n_seq, L, seed):
    """[CLS] w... [SEP] [PAD]...; lengths uniform in [10, L], one row full length."""
    g = torch.Generator().manual_seed(seed)
    ids = torch.randint(5, VOCAB, (n_seq, L), generator=g)
    lens = torch.randint(10, L + 1, (n_seq,), generator=g)
    lens[0] = L
    pos = torch.arange(L)[None]
    mask = (pos < lens[:, None]).long()
    ids[:, 0] = 2
    ids = torch.where(mask.bool(), ids, torch.zeros_like(ids))
    ids[torch.arange(n_seq), lens - 1] = 3
    return ids, mask


def c2_config():
    import yaml

    with open(os.path.join(PKG, "config.yaml")) as f:
        cfg = yaml.safe_load(f)
    cfg["train"].update(batch_size=TRAIN_B, acml_batch_size=TRAIN_B)
    return cfg


def c4_config():
    """Config C4's per-rank step: BERT-large frozen encoder (24 layers, H = 1024,
    A = 16, I = 4096), so the BiLSTM head's input is 1024 wide; 256 pairs per rank
    (global batch 2048 on 8 GPUs)."""
    cfg = c2_config()
    cfg["bert"] = dict(cfg.get("bert") or {}, name="bert-large-uncased")
    cfg["model"]["LSTM"]["input_size"] = 1024
    return cfg


def _live_events(lib, name, fn, n):
    """The library's HIP-event timing of `name` over n more calls of fn.  Kept out of
    the timed regions: an event pair around every GEMM launch cost 5-8% of the C2
    training step on MI355X (9.1-9.6 ms/step clean, 9.9 with events)."""
    torch.cuda.synchronize()
    lib.irc_prof_reset()
    lib.irc_prof_enable(1)
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    lib.irc_prof_enable(0)
    return _prof(lib, name)


def run_train(args, rank, world, dev, weights="bf16", cfg=None):
    """weights "fp8": config C5 -- the frozen encoder's nn.Linear layers on e4m3
    (irc_gemm_mx: MX-fp8, e4m3 codes with one E8M0 scale per 32 k, inputs quantised by
    their producing LayerNorm / attention / GELU epilogues); same step.
    cfg: c2_config() (default) or c4_config() (BERT-large encoder)."""
    from irc_amd import _lib
    from src.model import build_model, get_optimizer
    from src.train import TrainState

    lib = _lib.load()
    cfg = cfg or c2_config()
    ns = argparse.Namespace(config=cfg, loss="InfoNCE", model="LSTM", opt="adam",
                            sample="uniform")
    torch.manual_seed(1337)
    model = build_model(ns).to(dev).train()
    model.bert_model.set_weight_format(weights)
    gname, gpeak = ("gemm_fp8", FP8_PEAK_TFS) if weights == "fp8" else ("gemm_bf16", BF16_PEAK_TFS)
    model.add_queue_to_loss = True  # steady state (step >= queue_start_steps)
    opt = get_optimizer(ns, model)
    st = TrainState(ns, model, opt)
    if world > 1:
        st.set_process_group(dist.group.WORLD)
    ids, mask = synthetic_batch(2 * TRAIN_B, TRAIN_L, 1337 + rank)
    ids, mask = ids.to(dev), mask.to(dev)

    # Frozen-BERT features of the next micro-batch are issued on a side stream
    # before this micro-batch's heads step (model.bert_extract_async), as src/train.py
    # does: every step still runs one BERT forward and one heads fwd/bwd + update.
    # the first call waits for the inputs' upload; later ones need not wait for
    # anything (resident inputs), so BERT never queues behind a heads backward
    pending = [model.bert_extract_async(ids, mask, TRAIN_B)]

    def step():
        handle = pending[0]
        pending[0] = model.bert_extract_async(ids, mask, TRAIN_B, inputs_ready=True)
        st.micro_batch(TRAIN_B, lambda: model.forward_features(*model.features_ready(handle)),
                       sync_loss=False)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    dt = _max_over_ranks(dt, dev, world)
    live_s, live_n, live_flops = _live_events(lib, gname, step, args.steps)
    # Kernel efficiency: the same steps once more, serialised (BERT features and
    # every side-stream launch on the current stream, no prefetch), so concurrent
    # streams do not stretch the GEMM launches' event durations; the overlapped
    # (live) figure is reported beside it.
    model.features_ready(pending[0])
    torch.cuda.synchronize()
    from irc_amd._torch import serial_streams

    lib.irc_prof_reset()
    lib.irc_prof_enable(1)
    with serial_streams():  # one stream: every GEMM runs alone
        for _ in range(args.steps):
            st.micro_batch(TRAIN_B, lambda: model.forward_features(
                *model.bert_extract_ids(ids, mask, TRAIN_B)), sync_loss=False)
        torch.cuda.synchronize()
    lib.irc_prof_enable(0)
    g_s, g_n, g_flops = _prof(lib, gname)
    large = "large" in str((cfg or {}).get("bert", {}).get("name", ""))
    # PMC traffic of THIS leg's GEMMs (profiles/pmc_<tag>.json; null when absent)
    ptag = ("gemm_bf16_c4" if large else gname) if weights == "bf16" else "gemm_mx"
    g_bytes = _alg_bytes(lib, _pmc_traffic(ptag), gname + "_bytes")
    flops_pair = 2 * model.bert_model.flops_per_sequence(TRAIN_L) + _lstm_flops_per_pair(cfg)
    pairs = TRAIN_B * args.steps * world
    achieved = g_flops / g_s / 1e12 if g_s > 0 else None
    loss = float(st.loss_record[-1]) if st.loss_record else None
    step_tflops = pairs * flops_pair / dt / 1e12
    return model, {
        "pairs_per_s": pairs / dt,
        "ms_per_step": dt * 1e3 / args.steps,
        "loss_last": loss,
        "flops_per_pair": flops_pair,
        "step_tflops": step_tflops,
        "roofline": _step_roofline(step_tflops, gpeak, flops_pair, {
                     "bound": "mfma", "achieved": achieved, "peak": gpeak,
                     "unit": "TFLOP/s", "frac": achieved / gpeak if achieved else None,
                     "traffic": _pmc_traffic(ptag),
                     "traffic_source": _pmc_source(ptag),
                     "kernel": ("bf16 GEMM kernels (gemm_big_kernel / gemm_pp_kernel / "
                                "gemm_kernel, and qkv_attn_kernel: the QKV GEMM with the "
                                "attention in its epilogue, priced on the QKV GEMM's flops "
                                "alone; all GEMM launches of a single-stream pass of the "
                                "same steps)") if weights == "bf16" else
                               ("MX-fp8 GEMM (gemm_pp_kernel F8 = 2: e4m3 codes, E8M0 scales "
                                "per 32 k applied by v_mfma_scale_f32_16x16x128_f8f6f4) of the "
                                "frozen encoder's linear layers, single-stream pass; the heads' "
                                "bf16 GEMMs are not in this figure"),
                     "launches_per_step": g_n / args.steps,
                     "gemm_ms_per_step": g_s * 1e3 / args.steps,
                     "alg_flops_per_step": g_flops / args.steps,
                     **g_bytes,
                     "live_overlapped": {
                         "achieved": live_flops / live_s / 1e12 if live_s > 0 else None,
                         "note": "timed region itself: BERT GEMMs share the chip with the "
                                 "heads' recurrences on other streams, so event durations "
                                 "overlap and are summed"}}),
    }


def run_train_bert(args, rank, world, dev):
    """--model BERT (the north star's trainable encoder): BERT-base fwd+bwd on the
    256 anchors, momentum-encoder fwd on the 256 positives, InfoNCE (D=768) with the
    12544-key queue, clip + Adam (110M params, bf16 shadow refresh), momentum update."""
    from irc_amd import _lib
    from src.model import build_model, get_optimizer
    from src.train import TrainState

    lib = _lib.load()
    cfg = c2_config()
    ns = argparse.Namespace(config=cfg, loss="InfoNCE", model="BERT", opt="adam",
                            sample="uniform")
    torch.manual_seed(1337)
    model = build_model(ns).to(dev).train()
    model.add_queue_to_loss = True
    opt = get_optimizer(ns, model)
    st = TrainState(ns, model, opt)
    if world > 1:
        st.set_process_group(dist.group.WORLD)
    ids, mask = synthetic_batch(2 * TRAIN_B, TRAIN_L, 1337 + rank)
    ids, mask = ids.to(dev), mask.to(dev)

    def step():
        st.micro_batch(TRAIN_B, lambda: model.forward_ids(ids, mask, TRAIN_B), sync_loss=False)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    dt = _max_over_ranks(dt, dev, world)
    live_s, _, live_flops = _live_events(lib, "gemm_bf16", step, args.steps)
    # kernel efficiency on one stream (the timed steps overlap the momentum
    # encoder and the weight-gradient GEMMs on side streams)
    from irc_amd._torch import serial_streams

    lib.irc_prof_reset()
    lib.irc_prof_enable(1)
    with serial_streams():
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
    lib.irc_prof_enable(0)
    g_s, g_n, g_flops = _prof(lib, "gemm_bf16")
    g_bytes = _alg_bytes(lib, _pmc_traffic("gemm_bf16_bert"))
    enc = model.encoder_q
    D, K = enc.config.hidden_size, cfg["loss"]["InfoNCE"]["queue_size"]
    loss_flops = 3 * (2 * (2 * TRAIN_B) ** 2 * D + 2 * TRAIN_B * D * K) / TRAIN_B
    flops_pair = 4 * enc.flops_per_sequence(TRAIN_L) + loss_flops
    pairs = TRAIN_B * args.steps * world
    achieved = g_flops / g_s / 1e12 if g_s > 0 else None
    loss = float(st.loss_record[-1]) if st.loss_record else None
    step_tflops = pairs * flops_pair / dt / 1e12
    return {
        "pairs_per_s": pairs / dt,
        "ms_per_step": dt * 1e3 / args.steps,
        "loss_last": loss,
        "flops_per_pair": flops_pair,
        "step_tflops": step_tflops,
        "step_mfma_frac": step_tflops / BF16_PEAK_TFS,
        "roofline": _step_roofline(step_tflops, BF16_PEAK_TFS, flops_pair, {
                     "bound": "mfma", "achieved": achieved, "peak": BF16_PEAK_TFS,
                     "unit": "TFLOP/s", "frac": achieved / BF16_PEAK_TFS if achieved else None,
                     "traffic": _pmc_traffic("gemm_bf16_bert"),
                     "traffic_source": _pmc_source("gemm_bf16_bert"),
                     "kernel": "gemm kernels, bf16 operands (all GEMM launches of a "
                               "single-stream pass of the same steps: fwd, dX, dW)",
                     "launches_per_step": g_n / args.steps,
                     "gemm_ms_per_step": g_s * 1e3 / args.steps,
                     "alg_flops_per_step": g_flops / args.steps,
                     **g_bytes,
                     "live_overlapped": {
                         "achieved": live_flops / live_s / 1e12 if live_s > 0 else None}}),
    }


def _step_roofline(step_tflops, peak, flops_pair, gemm):
    """The training leg's roofline object: the north star's quantity, the whole
    encoder + InfoNCE step against the dense MFMA peak (pairs/s x
    algorithmic FLOPs per pair / peak), with the dominant kernel family -- the GEMM
    launches, priced on their own HIP-event durations -- as the ``gemm`` sub-field
    (``traffic``: that family's PMC HBM bytes per launch)."""
    return {"bound": "mfma", "achieved": step_tflops, "peak": peak, "unit": "TFLOP/s",
            "frac": step_tflops / peak, "traffic": gemm.get("traffic"),
            "definition": f"step-level: pairs/s x {flops_pair / 1e9:.2f} GFLOP per pair "
                          "(algorithmic, SURVEY.md 8d) / dense peak; the GEMM family alone "
                          "in 'gemm'",
            "gemm": gemm}


def _lstm_flops_per_pair(cfg):
    c = cfg["model"]["LSTM"]
    H, In, nl = c["hidden_size"], c["input_size"], c["num_layers"]
    per_tok = sum(2 * 4 * H * ((In if l == 0 else 2 * H) + H) * 2 for l in range(nl))
    return 4 * per_tok * TRAIN_L  # q fwd+bwd (3x) + k fwd (1x)


def cpu_baseline_train(model, steps):
    """The reference's step restated with the same torch CPU ops (nn.LSTM, matmul,
    cross_entropy, HF BERT math, torch.optim.Adam) at the C2 shapes and B = 256
    (oracle/torch_cpu_step.py), on the host's torch threads."""
    from oracle import torch_cpu_step

    cfgb = model.bert_model.config
    bert_w = {k: v.detach().float().cpu() for k, v in model.bert_model.state_dict().items()}
    head = model.encoder_q
    hs = {k: v.cpu() for k, v in head.state_dict().items()}
    dims = (head.input_size, head.hidden, head.num_layers, head.output_size)
    ids, mask = synthetic_batch(2 * TRAIN_B, TRAIN_L, 99)
    v, sec = torch_cpu_step.train_step_baseline(
        bert_w, cfgb.num_hidden_layers, cfgb.num_attention_heads, hs, dims,
        model.queue.detach().cpu(), ids, mask, steps=steps)
    return {"value": v, "unit": "pairs/s", "cores": torch.get_num_threads(), "kind": "port",
            "cpu_model": _cpu_model(), "s_per_step": sec,
            "sample": f"{steps} reference training steps of {TRAIN_B} pairs at the C2 shapes "
                      f"(BERT-base L={TRAIN_L} frozen, nn.LSTM 768->256x2 x3 + Linear 128, "
                      "queue 12544, clip + Adam + momentum + enqueue) in torch CPU ops, after "
                      "a 4-pair warm-up"}


def _filter_kernel_name(q, d, dtype):
    if q >= PP_MIN_Q:
        mf = ("v_mfma_scale_f32_16x16x128_f8f6f4" if dtype == "fp8"
              else "v_mfma_f32_16x16x32_bf16")
        return f"gemm_pp_kernel<EPI_SCAN> (scan filter, 256x256 tiles, {mf})"
    mf = "v_mfma_f32_32x32x16_fp8_fp8" if dtype == "fp8" else "v_mfma_f32_32x32x16_bf16"
    return f"scan_tile_kernel<{d}> (scan filter, stationary queries, {mf})"


def run_scan(args, rank, world, dev, n_per_gpu=SCAN_N_PER_GPU, dtype="bf16", nq=SCAN_Q,
             dim=SCAN_D, sweep=True):
    from irc_amd import _lib, retrieval

    lib = _lib.load()
    g = torch.Generator(device=dev).manual_seed(2024 + rank)
    shard = torch.randn(n_per_gpu, dim, generator=g, device=dev)
    shard = torch.nn.functional.normalize(shard).bfloat16()
    gq = torch.Generator().manual_seed(7)
    allq = torch.nn.functional.normalize(torch.randn(nq, dim, generator=gq)).bfloat16()
    myq = allq[rank * nq // world:(rank + 1) * nq // world].to(dev)
    index = retrieval.ShardedDenseIndex(shard, doc_offset=rank * n_per_gpu,
                                        group=dist.group.WORLD if world > 1 else None,
                                        dtype=dtype)
    del shard
    # a C2 batch is ~0.1 ms: time enough batches that one launch hiccup does not
    # move the rate (the retrieval legs are reported beside the training value).
    # Serving: DEPTH batches in flight (ShardedDenseIndex.search_many, one stream
    # each), so one batch's latency-bound selects overlap the next one's filter.
    reps = max(args.steps, 100 if nq <= 256 else 20)
    batches = [myq] * reps
    for _ in range(max(args.warmup, 3)):
        index.search(myq, SCAN_K, equal_counts=True)
    index.search_many(batches[:4], SCAN_K, depth=args.scan_depth, equal_counts=True)
    torch.cuda.synchronize()
    # serial calls first: the single-call latency (whole irc_scan_topk + collectives);
    # the filter kernel's HIP-event durations (roofline) come from these calls, where
    # nothing else runs beside it
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        index.search(myq, SCAN_K, equal_counts=True)
    torch.cuda.synchronize()
    dt_serial = _max_over_ranks(time.perf_counter() - t0, dev, world)
    k_s, k_n, k_bytes = _live_events(lib, "scan_filter",
                                     lambda: index.search(myq, SCAN_K, equal_counts=True), reps)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    index.search_many(batches, SCAN_K, depth=args.scan_depth, equal_counts=True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    dt = _max_over_ranks(dt, dev, world)
    sweep = scan_q_sweep(index, dev, dim) if (rank == 0 and sweep) else None
    kavg = k_s / max(k_n, 1)
    gbs = (k_bytes / max(k_n, 1)) / kavg / 1e9 if k_n else None
    tfs = 2 * nq * n_per_gpu * dim / kavg / 1e12 if k_n else None
    # bound: arithmetic intensity 2*Q*D flops per D*b doc bytes against the ridge
    # (bf16 2.5 PF / 8 TB/s = 312 flop/B; fp8 5 PF / 8 TB/s = 625)
    b = 1 if dtype == "fp8" else 2
    mfma_peak = FP8_PEAK_TFS if dtype == "fp8" else BF16_PEAK_TFS
    mfma_bound = 2.0 * nq / b > mfma_peak * 1e12 / (HBM_PEAK_GBS * 1e9)
    if mfma_bound:
        roof = {"bound": "mfma", "achieved": tfs, "peak": mfma_peak, "unit": "TFLOP/s",
                "frac": tfs / mfma_peak if tfs else None, "traffic": None, "hbm_GB_s": gbs}
    else:
        roof = {"bound": "hbm", "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": gbs / HBM_PEAK_GBS if gbs else None,
                "traffic": _pmc_traffic("scan_filter") if dtype == "bf16" else None,
                "traffic_source": _pmc_source("scan_filter") if dtype == "bf16" else None,
                "mfma_tflops": tfs}
    roof.update({"kernel": _filter_kernel_name(nq, dim, dtype), "kernel_avg_us": kavg * 1e6,
                 "alg_bytes_per_launch": k_bytes / max(k_n, 1)})
    alg_call = n_per_gpu * dim * b + nq * dim * 2 + nq * SCAN_K * 8  # bytes per local call
    if roof["bound"] == "hbm":  # the whole irc_scan_topk call priced beside the filter kernel
        call_gbs = alg_call / (dt_serial / reps) / 1e9
        roof.update({"call_achieved": call_gbs, "call_frac": call_gbs / HBM_PEAK_GBS,
                     "call_note": "serial whole-call (every launch of the search) on the call's "
                                  "algorithmic bytes; frac/achieved are the filter kernel's"})
    return {
        "value": nq * reps / dt, "unit": "queries/s", "batches_timed": reps,
        "ms_per_batch": dt * 1e3 / reps, "dtype": dtype, "batches_in_flight": args.scan_depth,
        "call_level": {
            "note": "whole search (sample pass, threshold select, filter, final select, "
                    "collectives) vs HBM peak on the call's algorithmic bytes",
            "serial_us_per_call": dt_serial * 1e6 / reps,
            "serial_hbm_frac": alg_call / (dt_serial / reps) / (HBM_PEAK_GBS * 1e9),
            "pipelined_us_per_batch": dt * 1e6 / reps,
            "pipelined_hbm_frac": alg_call / (dt / reps) / (HBM_PEAK_GBS * 1e9),
            "filter_hbm_frac": gbs / HBM_PEAK_GBS if gbs else None},
        "docs_per_gpu": n_per_gpu,
        "docs_total": n_per_gpu * world, "queries": nq, "dim": dim, "k": SCAN_K,
        "query_doc_pairs_per_s": nq * n_per_gpu * world * reps / dt,
        "roofline": roof,
        "q_sweep_local": sweep,
        "shard_bytes": n_per_gpu * dim * b,
        "cache_resident": n_per_gpu * dim * b < 256 * 2**20 * 0.9,
        "cache_note": ("the shard fits the 256 MiB Infinity Cache and is re-scanned batch after "
                       "batch: its 'HBM' fractions are cache-assisted"
                       if n_per_gpu * dim * b < 256 * 2**20 * 0.9 else
                       "the shard exceeds the 256 MiB Infinity Cache: HBM-bound figures"),
    }


def strong_shard(n_total, dim, rank, world, dev):
    """This rank's rows [lo, hi) of the fixed corpus (unit-norm Gaussian, bf16): drawn
    chunk by chunk (STRONG_CHUNKS seeds), so every world size sees the same documents."""
    from irc_amd.retrieval import shard_bounds

    lo, hi = shard_bounds(n_total, world, rank)
    chunk = -(-n_total // STRONG_CHUNKS)
    parts = []
    for c in range(lo // chunk, (hi - 1) // chunk + 1):
        c0, c1 = c * chunk, min(n_total, (c + 1) * chunk)
        g = torch.Generator(device=dev).manual_seed(4049 + c)
        x = torch.nn.functional.normalize(torch.randn(c1 - c0, dim, generator=g, device=dev))
        parts.append(x[max(lo, c0) - c0:min(hi, c1) - c0].bfloat16())
        del x
    return (parts[0] if len(parts) == 1 else torch.cat(parts)), lo


def _sync(dev):
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


def run_scan_strong(args, rank, world, dev, n_total, dtype, nq, dim, k=SCAN_K, make_index=None,
                    reps=None):
    """Strong scaling of the sharded scan: the fixed corpus of n_total
    docs split n_total / world per rank (ShardedDenseIndex), the same nq global queries
    per batch (each rank contributes nq / world and receives the global top-k of all
    nq).  Reports global queries/s (serial calls and `--scan-depth` batches in flight),
    the ranks and backend the collectives ran on, and the three steps of one search
    timed apart -- query all-gather, local scan, per-shard list all-gather + merge --
    each max over ranks.  make_index(rank, world, dev) -> index lets the CPU tests
    drive the same orchestration with a host-side double of the local scan."""
    if make_index is None:
        from irc_amd import retrieval

        def make_index(rank, world, dev):
            shard, lo = strong_shard(n_total, dim, rank, world, dev)
            group = dist.group.WORLD if world > 1 else None
            return retrieval.ShardedDenseIndex(shard, doc_offset=lo, group=group, dtype=dtype)
    index = make_index(rank, world, dev)
    gq = torch.Generator().manual_seed(7)
    allq = torch.nn.functional.normalize(torch.randn(nq, dim, generator=gq)).bfloat16()
    myq = allq[rank * nq // world:(rank + 1) * nq // world].to(dev)
    equal = nq % world == 0
    reps = reps or max(args.steps, 10)

    def timed(fn, n):
        if world > 1:
            dist.barrier()
        _sync(dev)
        t0 = time.perf_counter()
        for _ in range(n):
            fn()
        _sync(dev)
        return _max_over_ranks(time.perf_counter() - t0, dev, world) / n

    search = lambda: index.search(myq, k, equal_counts=equal)  # noqa: E731
    for _ in range(max(args.warmup, 2)):
        res = search()
    _sync(dev)
    t_call = timed(search, reps)
    if dev.type == "cuda":
        index.search_many([myq] * 4, k, depth=args.scan_depth, equal_counts=equal)
        t_pipe = timed(lambda: index.search_many([myq] * reps, k, depth=args.scan_depth,
                                                 equal_counts=equal), 1) / reps
    else:
        t_pipe = t_call
    sharded = index._sharded()
    gathered = index._gather_queries(myq, equal) if sharded else myq
    s, i = index._local_topk(gathered, k)
    phases = {"query_allgather_us": timed(lambda: index._gather_queries(myq, equal), reps) * 1e6
              if sharded else 0.0,
              "local_scan_us": timed(lambda: index._local_topk(gathered, k), reps) * 1e6,
              "list_allgather_merge_us": timed(lambda: index._exchange_merge(s, i, k), reps) * 1e6
              if sharded else 0.0}
    local = index.docs.shape[0]
    counts = torch.tensor([local], dtype=torch.int64, device=dev)
    lo_hi = [counts.clone() for _ in range(world)]
    if world > 1:
        dist.all_gather(lo_hi, counts)
    per_rank = [int(c.item()) for c in lo_hi]
    return {
        "value": nq / t_pipe, "unit": "queries/s", "scaling": "strong",
        "serial_queries_per_s": nq / t_call, "serial_us_per_call": t_call * 1e6,
        "pipelined_us_per_batch": t_pipe * 1e6, "batches_in_flight": args.scan_depth,
        "phases": phases,
        "ranks": world, "backend": dist.get_backend() if world > 1 else None,
        "docs_total": n_total, "docs_per_rank": per_rank, "queries": nq,
        "queries_per_rank": nq // world, "dim": dim, "k": k, "dtype": dtype,
        "query_doc_pairs_per_s": nq * n_total / t_pipe,
        "result_shape": list(res[1].shape),
        "workload": (f"fixed {n_total}-doc corpus (D={dim}, {dtype}) split {n_total} / {world} "
                     f"per rank, {nq} global queries per batch, top-{k}; global queries/s"),
    }


def scan_q_sweep(index, dev, dim=SCAN_D, qs=(1, 16, 64, 256), reps=20):
    """Local scan filter at several query-batch sizes (SURVEY.md 8d grades the HBM
    fraction at Q in {1, 16, 64, 256}): kernel HIP-event time and algorithmic bytes
    (N*D*b + Q*D*b) -> GB/s, plus the whole call's queries/s (query quantisation
    included for fp8)."""
    from irc_amd import _lib

    lib = _lib.load()
    out = []
    for q in qs:
        g = torch.Generator().manual_seed(11 + q)
        qq = torch.nn.functional.normalize(torch.randn(q, dim, generator=g)).bfloat16().to(dev)
        for _ in range(3):
            index._local_topk(qq, SCAN_K)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            index._local_topk(qq, SCAN_K)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        k_s, k_n, k_bytes = _live_events(lib, "scan_filter", lambda: index._local_topk(qq, SCAN_K),
                                         reps)
        kavg = k_s / max(k_n, 1)
        gbs = (k_bytes / max(k_n, 1)) / kavg / 1e9 if k_n else None
        b = 1 if index.dtype == "fp8" else 2
        alg = index.docs.shape[0] * dim * b + q * dim * 2 + q * SCAN_K * 8
        out.append({"Q": q, "filter_us": kavg * 1e6, "filter_GB_s": gbs,
                    "hbm_frac": gbs / HBM_PEAK_GBS if gbs else None,
                    "call_us": dt / reps * 1e6, "call_hbm_frac": alg / (dt / reps) / (
                        HBM_PEAK_GBS * 1e9),
                    "queries_per_s": q * reps / dt})
    return out


def run_sparse(args, dev, cpu_baseline):
    """Sparse hashed n-gram TF-IDF ranking (the reference's own
    predict path): a synthetic Zipf-distributed TF-IDF matrix [2^22 hashes x 200k
    docs, ~100 n-grams per doc], 64 claims of 16 hashed n-grams, top-100 --
    GPU (irc_csr_spmv_f64 + irc_csr_union + irc_topk_f64, scores bit-identical to
    scipy) vs the reference's CPU arithmetic (scipy spvec * doc_mat + argpartition)."""
    import scipy.sparse as sp

    from irc_amd import sparse

    rng = np.random.default_rng(11)
    H, N, per_doc, Qn, per_q, k = 1 << 22, 200_000, 100, 64, 16, 100
    zipf = lambda size: np.minimum(rng.zipf(1.3, size), H) - 1  # noqa: E731
    rows = zipf(N * per_doc)
    cols = np.repeat(np.arange(N), per_doc)
    m = sp.csr_matrix((np.log1p(rng.integers(1, 4, N * per_doc)).astype(np.float64), (rows, cols)),
                      shape=(H, N))
    m.sum_duplicates()
    index = sparse.SparseIndex(m, device=dev)
    q_rows = [np.unique(zipf(per_q)) for _ in range(Qn)]
    q_w = [rng.random(len(r)) + 0.1 for r in q_rows]
    for _ in range(2):
        index.topk_rows(q_rows, q_w, k)
    torch.cuda.synchronize()
    reps = max(args.steps, 3)
    t0 = time.perf_counter()
    for _ in range(reps):
        index.topk_rows(q_rows, q_w, k)
    torch.cuda.synchronize()
    gpu_qps = Qn * reps / (time.perf_counter() - t0)
    out = {"value": gpu_qps, "unit": "queries/s", "queries": Qn, "k": k, "docs": N,
           "hash_size": H, "nnz": int(m.nnz),
           "workload": "Zipf(1.3) hashed n-gram TF-IDF, 200k docs x ~100 n-grams, 64 claims "
                       "x 16 n-grams, top-100 (includes host packing and result copies)"}
    if cpu_baseline:
        t0, n = time.perf_counter(), 0
        while time.perf_counter() - t0 < 5.0 and n < Qn:
            spv = sp.csr_matrix((q_w[n], q_rows[n], np.array([0, len(q_rows[n])])), shape=(1, H))
            res = spv * m
            if len(res.data) > k:
                o = np.argpartition(-res.data, k)[:k]
                o[np.argsort(-res.data[o])]
            n += 1
        out["cpu_baseline"] = {"value": n / (time.perf_counter() - t0), "unit": "queries/s",
                               "cores": 1, "kind": "reference",
                               "sample": f"{n} claims through the reference's arithmetic "
                                         "(scipy csr product + argpartition/argsort, "
                                         "tfidf_doc_ranker.py:60-75), single thread"}
    return out


def cpu_baseline_scan(budget_s, n=SCAN_N_PER_GPU, nq=SCAN_Q, dim=SCAN_D, max_q=SCAN_Q,
                      leg="C2"):
    """The reference's CPU arithmetic for one retrieval leg's shard (fp32 q @ d.T and an
    exact top-k, src/evaluation.py:110-112 / tfidf_doc_ranker.py:60-75), on the host's
    torch threads.  Bounded sample: at most max_q of the leg's nq queries per pass over
    the whole shard, repeated for budget_s; queries/s is per query, so it compares with
    the GPU leg's rate directly.  fp8 legs are timed on the same shapes in fp32 (the
    reference has no fp8 path)."""
    from oracle import torch_cpu_step

    g = torch.Generator().manual_seed(2024)
    d = torch.nn.functional.normalize(torch.randn(n, dim, generator=g))
    gq = torch.Generator().manual_seed(7)
    qn = min(nq, max_q)
    q = torch.nn.functional.normalize(torch.randn(qn, dim, generator=gq))
    v, reps = torch_cpu_step.scan_baseline(q.bfloat16().float(), d.bfloat16().float(), SCAN_K,
                                           budget_s)
    del d
    return {"value": v, "unit": "queries/s", "cores": torch.get_num_threads(), "kind": "port",
            "cpu_model": _cpu_model(),
            "sample": f"{reps} x {qn} of the {leg} batch's {nq} queries over the full shard "
                      f"(N={n}, D={dim}, k={SCAN_K}): torch CPU fp32 matmul over 64k-doc chunks "
                      "+ topk merge"}


def _r(x, n=4):
    return None if x is None else float(f"{x:.{n}g}")


def _leg_summary(name, d):
    """The few numbers of one leg that a reader checks first (value, step time, roofline
    fraction, Q sweep); the full leg goes to the detail file."""
    if name.startswith("train"):
        r = d.get("roofline") or {}
        gm = r.get("gemm") or {}
        return {"pairs_per_s": _r(d.get("pairs_per_s"), 5), "ms_per_step": _r(d.get("ms_per_step")),
                "step_frac": _r(r.get("frac"), 3), "step_tflops": _r(d.get("step_tflops")),
                "gemm_frac": _r(gm.get("frac"), 3), "gemm_ms_per_step": _r(gm.get("gemm_ms_per_step")),
                "traffic_over_alg": _r(gm.get("traffic_over_alg"), 3)}
    if name.startswith("retrieval_strong"):
        ph = d.get("phases") or {}
        return {"queries_per_s": _r(d.get("value"), 5), "scaling": "strong",
                "docs_total": d.get("docs_total"), "docs_per_rank": d.get("docs_per_rank"),
                "ranks": d.get("ranks"), "Q": d.get("queries"), "dtype": d.get("dtype"),
                "call_us": _r(d.get("serial_us_per_call")),
                "phases_us": {k.replace("_us", ""): _r(v) for k, v in ph.items()}}
    if name == "sparse_tfidf":
        c = d.get("cpu_baseline") or {}
        return {"queries_per_s": _r(d.get("value"), 5), "cpu_queries_per_s": _r(c.get("value"))}
    r, c = d.get("roofline") or {}, d.get("call_level") or {}
    cb = d.get("cpu_baseline") or {}
    out = {"queries_per_s": _r(d.get("value"), 5), "Q": d.get("queries"),
           "cpu_queries_per_s": _r(cb.get("value")), "cpu_cores": cb.get("cores"),
           "docs_per_gpu": d.get("docs_per_gpu"), "bound": r.get("bound"),
           "filter_frac": _r(r.get("frac"), 3), "filter_us": _r(r.get("kernel_avg_us")),
           "call_us": _r(c.get("serial_us_per_call")), "call_hbm_frac": _r(c.get("serial_hbm_frac"), 3)}
    if d.get("q_sweep_local"):
        out["sweep_call_us"] = {str(x["Q"]): _r(x["call_us"]) for x in d["q_sweep_local"]}
        out["sweep_call_frac"] = {str(x["Q"]): _r(x["call_hbm_frac"], 3) for x in d["q_sweep_local"]}
    return out


# summary order: the training legs last (nearest the end of the output)
LEGS = ("sparse_tfidf", "retrieval_strong_c3", "retrieval_strong_c4", "retrieval_strong_c5",
        "retrieval_fp8", "retrieval_c4", "retrieval_c3", "retrieval", "train_bert", "train_c4",
        "train_fp8", "train")


def _compact(line):
    """The printed line keeps the contract keys and one short summary per leg, placed
    last so that a reader holding only the output's tail still sees every leg; the
    full per-leg objects (Q sweeps, traffic sources, notes) go to bench_detail.json
    (gpurun_out/ when present, else the working directory) and are named in the line."""
    legs = {k: line[k] for k in LEGS if k in line}
    if not legs:
        return line
    detail = os.path.join(ROOT, "gpurun_out") if os.path.isdir(os.path.join(ROOT, "gpurun_out")) \
        else os.getcwd()
    path = os.path.join(detail, "bench_detail.json")
    try:
        with open(path, "w") as f:
            json.dump(line, f)
    except OSError:
        path = None
    out = {k: v for k, v in line.items() if k not in LEGS}
    out["detail_file"] = path and os.path.relpath(path, ROOT)
    out["legs"] = {k: _leg_summary(k, legs[k]) for k in LEGS if k in legs}
    return out


def _free_port():
    import socket

    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def _launch_ranks(n):
    """`bench.py --gpus N` without a launcher: start N ranks under
    torch.distributed.run as CHILD processes (nothing here has touched the GPU)
    and exit with their status."""
    import subprocess

    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}",
           os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd, env=env)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--part", default="all",
                    choices=["all", "train", "train_fp8", "train_c4", "scan", "scan_c2",
                             "scan_c3", "bert", "strong"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=10.0)
    ap.add_argument("--cpu-steps", type=int, default=2)
    ap.add_argument("--scan-depth", type=int, default=SCAN_DEPTH,
                    help="query batches in flight in the retrieval legs")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(_launch_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}: one rank per GPU")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # IRC_DIST_BACKEND=gloo (as main.py): a rehearsal of the N-rank path where RCCL cannot
    # run it, e.g. N ranks sharing a 1-GPU box (ranks beyond the visible devices wrap
    # round them); the default is RCCL with one rank per GPU
    backend = os.environ.get("IRC_DIST_BACKEND", "nccl")
    ndev = torch.cuda.device_count()
    if backend == "gloo" and ndev and local >= ndev:
        local %= ndev
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    train = scan = None
    model = None
    if args.part in ("all", "train"):
        model, train = run_train(args, rank, world, dev)
    train8 = None
    if args.part in ("all", "train_fp8"):
        _, train8 = run_train(args, rank, world, dev, weights="fp8")
        torch.cuda.empty_cache()
    train_c4 = None
    if args.part in ("all", "train_c4"):
        _, train_c4 = run_train(args, rank, world, dev, cfg=c4_config())
        torch.cuda.empty_cache()
    bert = None
    if args.part in ("all", "bert"):
        bert = run_train_bert(args, rank, world, dev)
    scan_fp8 = scan_c4 = scan_c3 = None
    if args.part == "scan_c2":  # the C2 leg alone (PMC passes: tools/pmc_traffic.sh)
        scan = run_scan(args, rank, world, dev, sweep=False)
    if args.part in ("all", "scan", "scan_c3"):
        scan_c3 = run_scan(args, rank, world, dev, C3_N_PER_GPU, "bf16", C3_Q, SCAN_D)
        torch.cuda.empty_cache()
    if args.part in ("all", "scan"):
        scan = run_scan(args, rank, world, dev)
        torch.cuda.empty_cache()
        scan_c4 = run_scan(args, rank, world, dev, FP8_N_PER_GPU, "bf16", C4_Q, C4_D,
                           sweep=False)
        torch.cuda.empty_cache()
        scan_fp8 = run_scan(args, rank, world, dev, FP8_N_PER_GPU, "fp8", C5_Q, SCAN_D)
    strong = {}
    if args.part in ("all", "strong"):
        for name, n_total, sdt, snq, sdim in STRONG_LEGS:
            torch.cuda.empty_cache()
            strong[name] = run_scan_strong(args, rank, world, dev, n_total, sdt, snq, sdim)
        torch.cuda.empty_cache()
    cpu_t = cpu_s = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        if train is not None:
            cpu_t = cpu_baseline_train(model, args.cpu_steps)
        if scan is not None:
            cpu_s = cpu_baseline_scan(args.cpu_budget)
        # the other retrieval legs, each beside its own CPU figure (shorter budgets)
        for leg, n, nq, dim, name in ((scan_c3, C3_N_PER_GPU, C3_Q, SCAN_D, "C3"),
                                      (scan_c4, FP8_N_PER_GPU, C4_Q, C4_D, "C4"),
                                      (scan_fp8, FP8_N_PER_GPU, C5_Q, SCAN_D, "C5")):
            if leg is not None:
                leg["cpu_baseline"] = cpu_baseline_scan(args.cpu_budget / 2, n, nq, dim,
                                                        max_q=128, leg=name)
    if scan is not None:
        scan["cpu_baseline"] = cpu_s
    sparse_leg = None
    if args.part in ("all", "scan") and rank == 0 and world == 1:
        torch.cuda.empty_cache()
        sparse_leg = run_sparse(args, dev, not args.no_cpu_baseline)
    if rank == 0:
        if train is not None:
            head = {"value": train["pairs_per_s"], "unit": "pairs/s",
                    "ms_per_step": train["ms_per_step"], "roofline": train["roofline"],
                    "cpu_baseline": cpu_t}
        elif train_c4 is not None:
            head = {"value": train_c4["pairs_per_s"], "unit": "pairs/s",
                    "ms_per_step": train_c4["ms_per_step"], "roofline": train_c4["roofline"],
                    "cpu_baseline": None}
        elif train8 is not None:
            head = {"value": train8["pairs_per_s"], "unit": "pairs/s",
                    "ms_per_step": train8["ms_per_step"], "roofline": train8["roofline"],
                    "cpu_baseline": None}
        elif bert is not None:
            head = {"value": bert["pairs_per_s"], "unit": "pairs/s",
                    "ms_per_step": bert["ms_per_step"], "roofline": bert["roofline"],
                    "cpu_baseline": None}
        elif scan is None and scan_c3 is None:
            leg = strong["retrieval_strong_c4"]
            head = {"value": leg["value"], "unit": "queries/s",
                    "ms_per_step": leg["pipelined_us_per_batch"] / 1e3, "roofline": None,
                    "cpu_baseline": None}
        elif scan is None:
            head = {"value": scan_c3["value"], "unit": "queries/s",
                    "ms_per_step": scan_c3["ms_per_batch"], "roofline": scan_c3["roofline"],
                    "cpu_baseline": None}
        else:
            head = {"value": scan["value"], "unit": "queries/s",
                    "ms_per_step": scan["ms_per_batch"], "roofline": scan["roofline"],
                    "cpu_baseline": cpu_s}
        line = {
            "metric": METRIC, "value": head["value"], "unit": head["unit"], "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": head["ms_per_step"],
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "bf16",
            "data": "synthetic (seeded token ids / unit-norm Gaussian corpus; random-init "
                    "BERT-base weights, no checkpoint)",
            "config": {"workload": "C2: BERT-base bi-encoder (frozen, bf16) + 3-layer BiLSTM "
                                   "head, 256 pairs/step, L=64, in-batch + 12544-key queue "
                                   "negatives; retrieval 100k docs/GPU, 256 queries, top-100",
                       "pairs_per_step_per_gpu": TRAIN_B, "seq_len": TRAIN_L,
                       "global_batch": TRAIN_B * world,
                       "parallelism": f"dp{world} (train) / corpus-sharded x{world} (scan)"},
            "roofline": head["roofline"], "cpu_baseline": head["cpu_baseline"],
        }
        if world > 1:
            line["config"]["backend"] = dist.get_backend()  # "gloo": a rehearsal, not RCCL
        if train is not None:
            line["train"] = {k: train[k] for k in ("pairs_per_s", "ms_per_step", "step_tflops",
                                                   "flops_per_pair", "loss_last", "roofline")}
        if bert is not None:
            line["train_bert"] = bert
        if train_c4 is not None:
            line["train_c4"] = dict(train_c4, workload=(
                "C4 per-rank step: BERT-large frozen encoder (24L, H=1024, A=16, I=4096, bf16) "
                "+ 3-layer BiLSTM 1024->256x2->128, 256 pairs per rank (global batch 2048 on "
                "8 GPUs), L=64, queue 12544"))
        if train8 is not None:
            line["train_fp8"] = dict(train8, workload=(
                "C5: fp8 (e4m3) frozen-encoder weights, d=768: the C2 step with every BERT-base "
                "nn.Linear on irc_gemm_mx (MX-fp8: e4m3 codes, one E8M0 scale per 32 k; inputs "
                "quantised by their producing LayerNorm / attention / GELU epilogues)"))
        if scan is not None:
            line["retrieval"] = scan
        if scan_c3 is not None:
            scan_c3["workload"] = (f"C3 retrieval shard: {C3_N_PER_GPU} bf16 docs/GPU x D="
                                   f"{SCAN_D} (1M over 4 GPUs; 384 MB, beyond the 256 MiB "
                                   f"Infinity Cache), {C3_Q} queries, top-{SCAN_K}; q_sweep "
                                   "on this shard is the HBM-honest one")
            line["retrieval_c3"] = scan_c3
        if scan_c4 is not None:
            scan_c4["workload"] = (f"C4 retrieval shard: {FP8_N_PER_GPU} bf16 docs/GPU x D="
                                   f"{C4_D} (BERT-large, 5M over 8 GPUs), {C4_Q} queries, "
                                   f"top-{SCAN_K}")
            line["retrieval_c4"] = scan_c4
        if sparse_leg is not None:
            line["sparse_tfidf"] = sparse_leg
        line.update(strong)
        if scan_fp8 is not None:
            scan_fp8["workload"] = (f"C5 retrieval shard: {FP8_N_PER_GPU} e4m3 docs/GPU "
                                    f"(5M over 8 GPUs), {C5_Q} queries, top-{SCAN_K}")
            line["retrieval_fp8"] = scan_fp8
        print(json.dumps(_compact(line)), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
