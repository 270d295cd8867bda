"""Dense retrieval: corpus-wide cosine top-k over a (sharded) document corpus.

Semantics: scores = <e_q, e_n> of L2-normalised
``ctx2vec`` embeddings (src/evaluation.py:110-112, src/contrastor/
contrastive_module.py:96-100), per-query top-k by descending score as in
``TfidfDocRanker.closest_docs`` (preprocessing/drqa/retriever/
tfidf_doc_ranker.py:60-75); equal scores -> lower global doc index.

Multi-GPU: the corpus is split into contiguous shards, one per
rank, resident in HBM.  A search all-gathers the query embeddings over RCCL,
scans the local shard (global indices via the shard offset), all-gathers the
per-shard top-k lists and merges them with the same exact rule.
"""
from __future__ import annotations

import ctypes
import itertools

import torch

from . import _lib
from ._torch import contig, ptr, require_hip, stream_ptr, workspace


def scan_topk(queries: torch.Tensor, docs: torch.Tensor, k: int, doc_offset: int = 0,
              ws_tag: str = "scan"):
    """Exact top-k of queries @ docs.T (bf16 inputs, fp32 scores).

    queries [Q, D], docs [N, D] on the same HIP device.  Returns
    (scores fp32 [Q, k], idx int64 [Q, k]) sorted by (score desc, idx asc);
    slots past N are (-inf, -1).
    """
    require_hip(queries, docs)
    q = contig(queries, torch.bfloat16)
    d = contig(docs, torch.bfloat16)
    Q, D = q.shape
    N = d.shape[0]
    if d.shape[1] != D:
        raise ValueError(f"dim mismatch: queries D={D}, docs D={d.shape[1]}")
    out_s = torch.empty((Q, k), dtype=torch.float32, device=q.device)
    out_i = torch.empty((Q, k), dtype=torch.int64, device=q.device)
    nbytes = int(_lib.fn("irc_scan_topk_workspace")(Q, N, D, k))
    ws = workspace(nbytes, q.device, ws_tag)
    _lib.call("irc_scan_topk", ptr(q), ptr(d), Q, N, D, k, doc_offset, ptr(ws), ws.numel(),
              ptr(out_s), ptr(out_i), stream_ptr(q.device))
    return out_s, out_i


def scan_topk_many(batches, docs: torch.Tensor, k: int, doc_offset: int, streams,
                   ws_tag: str = "scan"):
    """scan_topk over query batches of one shape [Q, D], len(streams) of them in flight
    (batch b on streams[b % depth], each stream with its own workspace), in ONE native
    call (irc_scan_topk_many): the streams wait for the current stream first and the
    current stream waits for all of them after.  Returns [(scores, idx)] per batch, views
    of two [len(batches), Q, k] tensors; identical to scan_topk per batch."""
    qs = [contig(q, torch.bfloat16) for q in batches]
    d = contig(docs, torch.bfloat16)
    require_hip(d, *qs)
    Q, D = qs[0].shape
    N = d.shape[0]
    if d.shape[1] != D or any(q.shape != qs[0].shape for q in qs):
        raise ValueError("scan_topk_many: every batch [Q, D] with the docs' D")
    nb, depth = len(qs), len(streams)
    out_s = torch.empty((nb, Q, k), dtype=torch.float32, device=d.device)
    out_i = torch.empty((nb, Q, k), dtype=torch.int64, device=d.device)
    if nb == 0:
        return []
    nbytes = int(_lib.fn("irc_scan_topk_workspace")(Q, N, D, k))
    wss = [workspace(nbytes, d.device, f"{ws_tag}{j}") for j in range(depth)]
    qp = (ctypes.c_void_p * nb)(*[q.data_ptr() for q in qs])
    wp = (ctypes.c_void_p * depth)(*[w.data_ptr() for w in wss])
    sp = (ctypes.c_void_p * depth)(*[s.cuda_stream for s in streams])
    _lib.call("irc_scan_topk_many", qp, nb, ptr(d), Q, N, D, k, doc_offset, wp, nbytes, depth,
              ptr(out_s), ptr(out_i), sp, stream_ptr(d.device))
    return list(zip(out_s.unbind(0), out_i.unbind(0)))


def scan_scores(queries: torch.Tensor, docs: torch.Tensor) -> torch.Tensor:
    """Raw fp32 score matrix from the same MFMA path (tests / diagnostics)."""
    require_hip(queries, docs)
    q = contig(queries, torch.bfloat16)
    d = contig(docs, torch.bfloat16)
    out = torch.empty((q.shape[0], d.shape[0]), dtype=torch.float32, device=q.device)
    _lib.call("irc_scan_scores", ptr(q), ptr(d), q.shape[0], d.shape[0], q.shape[1], ptr(out),
              stream_ptr(q.device))
    return out


# fp8 corpus (BASELINE config C5): e4m3fn embeddings, stored as uint8 bytes.
# Unit-norm components times 16 sit in e4m3's normal range and far below its
# 448 maximum; a power of two keeps the descale exact.
FP8_SCALE = 16.0


def quantize_fp8(x: torch.Tensor, scale: float = FP8_SCALE) -> torch.Tensor:
    """e4m3fn(RNE(x * scale)) as a uint8 tensor of x's shape (irc_quantize_fp8)."""
    require_hip(x)
    if x.dtype not in (torch.bfloat16, torch.float32):
        x = x.float()
    xc = x.contiguous()
    out = torch.empty(xc.shape, dtype=torch.uint8, device=xc.device)
    _lib.call("irc_quantize_fp8", 0 if xc.dtype == torch.bfloat16 else 1, ptr(xc), xc.numel(),
              float(scale), ptr(out), stream_ptr(xc.device))
    return out


def _fp8_operands(queries, docs):
    require_hip(queries, docs)
    for t in (queries, docs):
        if t.dtype != torch.uint8:
            raise TypeError("fp8 scan operands are e4m3 bytes (torch.uint8, see quantize_fp8)")
    q, d = queries.contiguous(), docs.contiguous()
    if d.shape[1] != q.shape[1]:
        raise ValueError(f"dim mismatch: queries D={q.shape[1]}, docs D={d.shape[1]}")
    return q, d


def scan_topk_fp8(queries: torch.Tensor, docs: torch.Tensor, k: int, doc_offset: int = 0,
                  score_scale: float = 1.0, ws_tag: str = "scan"):
    """Exact top-k over e4m3 queries [Q, D] and docs [N, D] (uint8 bytes); the
    returned scores are the fp32 dot products of the quantised values times
    score_scale (a power of two)."""
    q, d = _fp8_operands(queries, docs)
    Q, D = q.shape
    N = d.shape[0]
    out_s = torch.empty((Q, k), dtype=torch.float32, device=q.device)
    out_i = torch.empty((Q, k), dtype=torch.int64, device=q.device)
    nbytes = int(_lib.fn("irc_scan_topk_fp8_workspace")(Q, N, D, k))
    ws = workspace(nbytes, q.device, ws_tag)
    _lib.call("irc_scan_topk_fp8", ptr(q), ptr(d), Q, N, D, k, doc_offset, float(score_scale),
              ptr(ws), ws.numel(), ptr(out_s), ptr(out_i), stream_ptr(q.device))
    return out_s, out_i


def scan_scores_fp8(queries: torch.Tensor, docs: torch.Tensor) -> torch.Tensor:
    """Raw fp32 dot products of e4m3 operands (the fp8 filter's arithmetic)."""
    q, d = _fp8_operands(queries, docs)
    out = torch.empty((q.shape[0], d.shape[0]), dtype=torch.float32, device=q.device)
    _lib.call("irc_scan_scores_fp8", ptr(q), ptr(d), q.shape[0], d.shape[0], q.shape[1],
              ptr(out), stream_ptr(q.device))
    return out


def set_single_pass_min_q(q: int) -> int:
    """Smallest query batch of the single-pass GEMM filter (irc_scan_set_ppl_min_q:
    Q in [q, 256]; q > 256 selects the sampled-threshold pipeline).  Both are exact.
    Returns the previous value."""
    return int(_lib.load().irc_scan_set_ppl_min_q(int(q)))


def rescan_stats(reset: bool = True):
    """(queries whose single-pass select rescanned, workers rescanned) since the
    last reset -- synchronises the device (tests / diagnostics)."""
    import ctypes

    out = (ctypes.c_uint64 * 2)()
    _lib.call("irc_scan_rescan_stats", ctypes.addressof(out), 1 if reset else 0)
    return int(out[0]), int(out[1])


def topk_merge(scores: torch.Tensor, idx: torch.Tensor, k: int):
    """Merge [P, Q, kin] per-shard lists into [Q, k] with the exact rule."""
    require_hip(scores, idx)
    s = contig(scores, torch.float32)
    i = contig(idx, torch.int64)
    P, Q, kin = s.shape
    out_s = torch.empty((Q, k), dtype=torch.float32, device=s.device)
    out_i = torch.empty((Q, k), dtype=torch.int64, device=s.device)
    _lib.call("irc_topk_merge", ptr(s), ptr(i), P, Q, kin, k, ptr(out_s), ptr(out_i),
              stream_ptr(s.device))
    return out_s, out_i


def shard_bounds(n_docs: int, world: int, rank: int):
    """Contiguous shard [start, stop) of rank `rank` (first n % world ranks get +1)."""
    base, rem = divmod(n_docs, world)
    start = rank * base + min(rank, rem)
    return start, start + base + (1 if rank < rem else 0)


class ShardedDenseIndex:
    """One rank's HBM-resident shard of the corpus embedding matrix.

    ``docs`` is this rank's shard [N_local, D] (bf16), ``doc_offset`` its first
    global index.  ``search`` is collective over ``group`` when one is given:
    every rank passes its local query slice (may be empty) and receives the
    global top-k for ALL gathered queries (queries ordered by rank).

    ``dtype="fp8"`` keeps the shard as e4m3 bytes (half the HBM bytes per scan,
    BASELINE config C5): queries are quantised with the same power-of-two
    ``fp8_scale`` per search and the scores returned are those of the
    quantised embeddings, descaled exactly.
    """

    def __init__(self, docs: torch.Tensor, doc_offset: int = 0, group=None, dtype: str = "bf16",
                 fp8_scale: float = FP8_SCALE):
        if dtype not in ("bf16", "fp8"):
            raise ValueError(f"dtype must be 'bf16' or 'fp8', not {dtype!r}")
        self.dtype = dtype
        self.fp8_scale = float(fp8_scale)
        if dtype == "fp8":
            self.docs = quantize_fp8(docs, self.fp8_scale)
        else:
            self.docs = docs.to(torch.bfloat16).contiguous()
        self.doc_offset = int(doc_offset)
        self.group = group

    # ------------------------------------------------------------ persistence
    # On-disk corpus index: one .npy per shard (bf16 as
    # uint16 bits, or e4m3 bytes), a JSON header, and the DrQA-style doc-id map
    # (doc_dict = (DOC2IDX, doc_ids), preprocessing/drqa/build_tfidf.py:126,198-205).
    def save(self, directory: str, rank: int = 0, doc_ids=None) -> None:
        import json
        import os

        import numpy as np

        os.makedirs(directory, exist_ok=True)
        raw = self.docs.view(torch.uint16) if self.dtype == "bf16" else self.docs
        np.save(os.path.join(directory, f"shard_{rank}.npy"), raw.cpu().numpy())
        meta = {"dtype": self.dtype, "fp8_scale": self.fp8_scale, "doc_offset": self.doc_offset,
                "rows": int(self.docs.shape[0]), "dim": int(self.docs.shape[1])}
        with open(os.path.join(directory, f"shard_{rank}.json"), "w") as f:
            json.dump(meta, f)
        if doc_ids is not None:
            with open(os.path.join(directory, "doc_ids.json"), "w") as f:
                json.dump(list(doc_ids), f)

    @classmethod
    def load(cls, directory: str, rank: int = 0, device=None, group=None):
        """(index, doc_dict or None): the shard saved by save() for this rank,
        resident on `device` (no re-quantisation: the stored bytes are used)."""
        import json
        import os

        import numpy as np

        with open(os.path.join(directory, f"shard_{rank}.json")) as f:
            meta = json.load(f)
        raw = torch.from_numpy(np.load(os.path.join(directory, f"shard_{rank}.npy")))
        raw = raw.to(device or "cuda")
        self = cls.__new__(cls)
        self.dtype = meta["dtype"]
        self.fp8_scale = float(meta["fp8_scale"])
        self.docs = raw.view(torch.bfloat16) if self.dtype == "bf16" else raw
        self.doc_offset = int(meta["doc_offset"])
        self.group = group
        doc_dict = None
        ids_path = os.path.join(directory, "doc_ids.json")
        if os.path.exists(ids_path):
            with open(ids_path) as f:
                ids = json.load(f)
            doc_dict = ({d: i for i, d in enumerate(ids)}, ids)
        return self, doc_dict

    # The two device steps are methods so the collective orchestration can be
    # exercised on CPU (gloo) with a test double in tests/test_dist_cpu.py.
    def _local_topk(self, queries, k, ws_tag="scan"):
        if self.dtype == "fp8":
            q8 = quantize_fp8(queries, self.fp8_scale)
            return scan_topk_fp8(q8, self.docs, k, self.doc_offset,
                                 1.0 / (self.fp8_scale * self.fp8_scale), ws_tag=ws_tag)
        return scan_topk(queries, self.docs, k, self.doc_offset, ws_tag=ws_tag)

    def _merge(self, scores, idx, k):
        return topk_merge(scores, idx, k)

    def search(self, queries: torch.Tensor, k: int, equal_counts: bool = False,
               ws_tag: str = "scan"):
        """Global top-k of the gathered queries.  ``equal_counts``: every rank
        passes the same number of queries, so the ragged-count exchange (a host
        sync) is skipped and the whole search stays stream-ordered."""
        if not self._sharded():
            return self._local_topk(queries, k, ws_tag)
        allq = self._gather_queries(queries, equal_counts)  # (1)
        s, i = self._local_topk(allq, k, ws_tag)  # (2)
        return self._exchange_merge(s, i, k)  # (3)

    # The three steps of a sharded search, separately callable (bench.py times each).
    def _sharded(self):
        import torch.distributed as dist

        return not (self.group is None or not dist.is_initialized() or
                    dist.get_world_size(self.group) == 1)

    def _gather_queries(self, queries, equal_counts=False):
        """(1) every rank's query slice, all-gathered in rank order (ragged: the counts
        are exchanged first, a host sync that ``equal_counts`` skips)."""
        import torch.distributed as dist

        world = dist.get_world_size(self.group)
        if equal_counts:
            counts = [queries.shape[0]] * world
        else:
            n_local = torch.tensor([queries.shape[0]], dtype=torch.int64, device=queries.device)
            cnt = [torch.zeros_like(n_local) for _ in range(world)]
            dist.all_gather(cnt, n_local, group=self.group)
            counts = [int(c.item()) for c in cnt]
        qmax = max(counts)
        if qmax == queries.shape[0]:
            qpad = queries.contiguous()
        else:
            qpad = torch.zeros((qmax, queries.shape[1]), dtype=queries.dtype,
                               device=queries.device)
            qpad[: queries.shape[0]] = queries
        gathered = [torch.empty_like(qpad) for _ in range(world)]
        dist.all_gather(gathered, qpad, group=self.group)
        return torch.cat([g[:c] for g, c in zip(gathered, counts)], dim=0)

    def _exchange_merge(self, s, i, k):
        """(3) every shard's exact top-k lists (global doc ids) all-gathered and merged
        by the (score desc, index asc) rule: every rank gets the global result."""
        import torch.distributed as dist

        world = dist.get_world_size(self.group)
        ss = [torch.empty_like(s) for _ in range(world)]
        ii = [torch.empty_like(i) for _ in range(world)]
        dist.all_gather(ss, s.contiguous(), group=self.group)
        dist.all_gather(ii, i.contiguous(), group=self.group)
        return self._merge(torch.stack(ss), torch.stack(ii), k)

    def search_many(self, batches, k: int, depth: int = 3, equal_counts: bool = False,
                    graphs: bool = False):
        """search() over a sequence of query batches with up to ``depth`` batches
        in flight on as many HIP streams (each with its own scan workspace): one
        batch's latency-bound selects overlap the next batch's HBM-bound filter.
        Single process, bf16, batches of one shape: the whole loop is one native call
        (irc_scan_topk_many: the host issues a C2 batch in 13-17 us against 39-43 us for
        search() per batch, so the loop stays GPU-bound -- 60.6 us a batch at depth 3 on
        a box where the Python loop also kept up, profiles/r06_i_scan_depth.log; the C2
        leg on boxes since: 3.97-4.09M queries/s, profiles/r06_m/, against 3.27M with the
        Python loop in profiles/r06_fin1_bench.log).  ``graphs`` (single process, every batch of one
        shape): each stream replays a HIP graph of the whole local search captured once
        -- measured slower than direct launches at C2 (77-80 us a batch at depth 3).
        Results are identical to calling search() per batch; returned in order, usable
        on the current stream."""
        import torch.distributed as dist

        batches = list(batches)
        dev = self.docs.device
        cur = torch.cuda.current_stream(dev)
        streams = _search_streams(dev, depth)
        single = self.group is None or not dist.is_initialized() or \
            dist.get_world_size(self.group) == 1
        if graphs and not single:
            raise ValueError("graphed search_many needs a single-process index")
        if single and not graphs and self.dtype == "bf16" and batches and \
                all(q.shape == batches[0].shape for q in batches):
            # the whole loop in one native call (irc_scan_topk_many): the per-batch Python
            # of search() paced a C2 batch's ~70 us of GPU work
            return scan_topk_many(batches, self.docs, k, self.doc_offset, streams)
        slots = self._graph_slots(batches[0], k, depth, streams) if (graphs and batches) else None
        out = []
        for n, q in enumerate(batches):
            st = streams[n % depth]
            st.wait_stream(cur)  # the batch's inputs were produced on `cur`
            with torch.cuda.stream(st):
                if slots is not None:
                    g, qin, so, io, _ws = slots[n % depth]
                    qin.copy_(q)
                    g.replay()
                    res = (so.clone(), io.clone())
                else:
                    res = self.search(q, k, equal_counts=equal_counts, ws_tag=f"scan{n % depth}")
            q.record_stream(st)
            out.append(res)
        for st in streams:
            cur.wait_stream(st)
        for s, i in out:
            s.record_stream(cur)
            i.record_stream(cur)
        return out

    def _graph_slots(self, q0, k, depth, streams):
        """Per stream: (graph, static query buffer, static scores, static ids, workspace)
        of the local search for q0's shape, captured once and cached on the index.

        Each slot OWNS its scan workspace: it is taken out of the shared grow-only
        cache right after capture (under a tag no other call uses), so no later
        call on any index can grow -- and free -- memory a captured graph points
        into.  The key includes the shard tensor, so replacing ``self.docs``
        captures anew instead of replaying against the old one."""
        from ._torch import take_workspace

        key = (tuple(q0.shape), q0.dtype, int(k), depth, self.docs.data_ptr(),
               tuple(self.docs.shape), self.dtype)
        cache = self.__dict__.setdefault("_graphs", {})
        if key in cache:
            return cache[key]
        slots = []
        for st in streams:
            qin = torch.empty_like(q0)
            qin.copy_(q0)
            tag = f"gscan:{next(_GRAPH_SERIAL)}"
            with torch.cuda.stream(st):
                self._local_topk(qin, k, tag)  # warm-up: workspace sized outside the graph
            st.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=st):
                so, io = self._local_topk(qin, k, tag)
            ws = take_workspace(self.docs.device, tag)  # owned by this slot from now on
            slots.append((g, qin, so, io, ws))
        cache[key] = slots
        return slots


_GRAPH_SERIAL = itertools.count()  # unique workspace tags of captured searches
_SEARCH_STREAMS = {}


def _search_streams(dev, depth):
    key = (dev.index if dev.index is not None else torch.cuda.current_device(), depth)
    st = _SEARCH_STREAMS.get(key)
    if st is None:
        st = _SEARCH_STREAMS[key] = [torch.cuda.Stream(dev) for _ in range(depth)]
    return st
