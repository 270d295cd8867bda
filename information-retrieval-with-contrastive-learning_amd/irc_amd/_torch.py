"""Thin torch plumbing for the C ABI: device checks, raw pointers, the current
HIP stream, and the workspace allocator.  PyTorch is plumbing only here: memory,
streams, autograd bookkeeping and torch.distributed -- never the compute."""
from __future__ import annotations


import torch

from ._lib import IRCError


def require_hip(*tensors: torch.Tensor) -> None:
    for t in tensors:
        if t is None:
            continue
        if not t.is_cuda:
            raise IRCError(
                "irc_amd kernels run on a HIP device (MI355X / gfx950) only; got a tensor on "
                f"{t.device}. There is no CPU fallback in the product path.")


def ptr(t: torch.Tensor | None):
    return None if t is None else t.data_ptr()


def stream_ptr(device: torch.device | None = None):
    return torch.cuda.current_stream(device).cuda_stream


_side: dict = {}


# Every side stream has the default priority.  The frozen encoder's feature prefetch at high
# priority gained the C2 step 0.6-1.1% in round 4 (profiles/r04_q_priority_ab.txt) and later
# cost it 0.5-1%; once such a stream exists in the process the pipelined retrieval
# (search_many) runs slower too -- C2 3.58M -> 2.1M queries/s (profiles/r05_zh_priority_ab.txt,
# r04_t_priority_retrieval.txt); the heads' streams at high priority measured 3% slower.


_serial = [0]


class serial_streams:
    """Context: side_stream() hands out the current stream, so every launch runs
    in issue order with nothing beside it (kernel-efficiency measurements)."""

    def __enter__(self):
        _serial[0] += 1
        return self

    def __exit__(self, *exc):
        _serial[0] -= 1
        return False


def side_stream(device: torch.device, tag: str = "side") -> torch.cuda.Stream:
    """A persistent secondary HIP stream per (device, tag) for overlapping
    independent launches (e.g. the key encoder, weight-gradient GEMMs)."""
    if _serial[0]:
        return torch.cuda.current_stream(device)
    key = (torch.device(device).index, tag)
    s = _side.get(key)
    if s is None:
        s = _side[key] = torch.cuda.Stream(device=device)
    return s


def contig(t: torch.Tensor, dtype: torch.dtype) -> torch.Tensor:
    if t.dtype != dtype:
        t = t.to(dtype)
    return t.contiguous()


_ws_cache: dict = {}


def workspace(nbytes: int, device: torch.device, tag: str = "default") -> torch.Tensor:
    """Grow-only per-(device, tag) scratch buffer from the caching allocator.

    Stream-ordered reuse is safe because every IRC call on a tag is issued on the
    same (current) stream; callers on other streams must pass their own tag."""
    key = (device.index if device.index is not None else torch.cuda.current_device(), tag)
    buf = _ws_cache.get(key)
    if buf is None or buf.numel() < nbytes:
        buf = torch.empty(max(nbytes, 256), dtype=torch.uint8, device=device)
        _ws_cache[key] = buf
    return buf


def take_workspace(device: torch.device, tag: str):
    """Remove (device, tag)'s buffer from the shared cache and return it: the caller
    (a captured HIP graph's slot) keeps it alive and nothing else can grow it."""
    key = (device.index if device.index is not None else torch.cuda.current_device(), tag)
    return _ws_cache.pop(key, None)
