"""Typed wrappers over the libirc_hip.so entry points (include/irc.h).

Each wrapper validates devices/dtypes, allocates outputs from the PyTorch
caching allocator and launches on the current HIP stream.  None of them has a
fallback: a CPU tensor or a missing library raises.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib
from ._lib import IRCError  # noqa: F401  (re-exported for callers of ops)
from ._torch import ptr, require_hip, stream_ptr

BF16, F32 = torch.bfloat16, torch.float32
_DT = {BF16: 0, F32: 1}

EPI_NONE, EPI_BIAS, EPI_BIAS_GELU, EPI_BIAS_RESID, EPI_RESID = 0, 1, 2, 3, 4


def _code(t: torch.Tensor) -> int:
    try:
        return _DT[t.dtype]
    except KeyError:
        raise TypeError(f"irc kernels take bf16 or fp32, got {t.dtype}") from None


def gemm_set_big_ring(on) -> int:
    """K loop of the big-tile bf16 GEMM (irc_gemm_set_big_ring): True = 4-slot ring of
    32-deep K-tiles, False = two 64-deep slots (the default; the ring measured no
    faster on MI355X).  Bit-identical results.
    Returns the previous setting."""
    return int(_lib.load().irc_gemm_set_big_ring(1 if on else 0))



class LnStats:
    """Per-row statistics of a pre-LayerNorm activation: partial (sum, sum of squares)
    pairs over column tiles, [rows, nt, 2] fp32, written by irc_gemm_ln."""

    def __init__(self, t: torch.Tensor, nt: int, h: int):
        self.t, self.nt, self.h = t, nt, h


def gemm_ln(a, b, bias, *, epilogue, stats=None, gamma=None, beta=None, eps=1e-12,
            colsum=None, residual=None, want_stats=False, out=None):
    """irc_gemm_ln (include/irc.h): the BERT encoder's LayerNorm-fold GEMMs, bf16.
    epilogue EPI_BIAS / EPI_BIAS_GELU: out = LN(a) . W^T + bias' with b = W diag(gamma)
    (the fold: stats of a, colsum of b); EPI_BIAS_RESID: out = a . b^T + bias + LN(residual)
    (stats, gamma, beta of the residual) or + residual.  Returns out, or (out, LnStats)."""
    require_hip(a, b, bias, residual, out, gamma, beta, colsum,
                stats.t if stats is not None else None)
    for t in (a, b, residual, out):
        if t is not None and (t.dtype != BF16 or t.dim() != 2 or t.stride(-1) != 1):
            raise TypeError("gemm_ln: a, b, residual and out must be 2-D bf16, unit column stride")
    for t in (bias, gamma, beta, colsum):
        if t is not None and (t.dtype != F32 or not t.is_contiguous()):
            raise TypeError("gemm_ln: bias, gamma, beta and colsum must be contiguous fp32")
    M, K = a.shape
    N = b.shape[0]
    if b.shape[1] != K:
        raise ValueError(f"gemm_ln inner dims differ: {K} vs {b.shape[1]}")
    # the kernels read bias / colsum per output column and gamma / beta per statistics
    # column with 16-byte loads: a short vector would be a device fault
    for t, n, name in ((bias, N, "bias"), (colsum, N, "colsum"),
                       (gamma, stats.h if stats is not None else None, "gamma"),
                       (beta, stats.h if stats is not None else None, "beta")):
        if t is not None and n is not None and t.numel() != n:
            raise ValueError(f"gemm_ln: {name} has {t.numel()} elements, needs {n}")
    # the statistics describe a (the fold, epilogues 1 / 2) or the residual (epilogue 3)
    if stats is not None and (stats.t.shape[0] != M or stats.h != (N if residual is not None else K)):
        raise ValueError("gemm_ln: the statistics describe another activation")
    if out is None:
        out = torch.empty((M, N), dtype=BF16, device=a.device)
    st_out = None
    if want_stats:
        st_out = torch.empty((M, (N + 127) // 128, 2), dtype=F32, device=a.device)
    nt = ctypes.c_int(0)
    _lib.call("irc_gemm_ln", int(epilogue), M, N, K, ptr(a), a.stride(0), ptr(b), b.stride(0),
              ptr(bias), ptr(residual), residual.stride(0) if residual is not None else 0,
              ptr(out), out.stride(0), ptr(stats.t) if stats is not None else None,
              stats.nt if stats is not None else 0, ptr(gamma), ptr(beta), float(eps),
              stats.h if stats is not None else 0, ptr(colsum), ptr(st_out),
              ctypes.addressof(nt) if want_stats else None, stream_ptr(a.device))
    if want_stats:
        n = int(nt.value)
        return out, LnStats(st_out.view(-1)[:M * n * 2].view(M, n, 2), n, N)
    return out


def gemm_set_big_mf16(on) -> int:
    """MFMA shape of the big-tile bf16 GEMM's 2-slot loop (irc_gemm_set_big_mf16):
    True = 16x16x32 (the default), False = 32x32x16.  Returns the previous setting."""
    return int(_lib.load().irc_gemm_set_big_mf16(1 if on else 0))


def gemm_set_persistent(mode) -> int:
    """Persistent tile loop of the 256x256 bf16 GEMM (irc_gemm_set_persistent): 0 off
    (the default), 1 / True dynamic tiles with the next tile's first K-tile prestaged
    during the epilogue, 2 static waves + prestage, 3 static.  Returns the previous
    mode.  Results are bit-identical in every mode."""
    return int(_lib.load().irc_gemm_set_persistent(int(mode)))


def gemm(a, b, *, trans_a=False, b_is_nk=True, bias=None, epilogue=EPI_NONE, residual=None,
         alpha=1.0, out=None, out_dtype=None, accumulate=False, max_blocks=0):
    """out[M, N] = alpha * op(a) @ op(b) (+ bias) (-> gelu) (+ residual).

    a: [M, K] (or [K, M] with trans_a); b: [N, K] when b_is_nk (nn.Linear weight
    layout, i.e. a @ b.T) else [K, N].  Inputs bf16 or fp32 (same dtype);
    fp32 inputs run the exact fp32 MFMA.  2-D only (see gemm_strided).  max_blocks
    caps a split-K launch (irc_gemm_ex; 0 = one wave); a negative value caps the grid of an
    unsplit launch at -max_blocks workgroups instead (a static persistent tile loop).
    """
    require_hip(a, b, bias, residual, out)
    if a.dtype != b.dtype:
        raise TypeError(f"gemm operands must share a dtype ({a.dtype} vs {b.dtype})")
    if a.stride(-1) != 1 or b.stride(-1) != 1:
        raise ValueError("gemm operands must be contiguous in their last dim")
    M, K = (a.shape[1], a.shape[0]) if trans_a else (a.shape[0], a.shape[1])
    N, Kb = (b.shape[0], b.shape[1]) if b_is_nk else (b.shape[1], b.shape[0])
    if K != Kb:
        raise ValueError(f"gemm inner dims differ: {K} vs {Kb}")
    if out is None:
        od = out_dtype or a.dtype
        out = torch.empty((M, N), dtype=od, device=a.device)
        if accumulate:
            out.zero_()
    if bias is not None and bias.dtype != F32:
        raise TypeError("bias must be fp32")
    if residual is not None and residual.dtype != out.dtype:
        raise TypeError("residual dtype must match the output")
    ws, nws = _splitk_ws(a, out, epilogue, M, N, K, 1, max_blocks)
    _lib.call("irc_gemm_ex", _code(a), _code(out), 1 if trans_a else 0, 0 if b_is_nk else 1,
              int(epilogue), M, N, K, float(alpha), ptr(a), a.stride(0), 0, ptr(b), b.stride(0),
              0, ptr(bias), 0, ptr(residual), residual.stride(0) if residual is not None else 0, 0,
              ptr(out), out.stride(0), 0, 1 if accumulate else 0, 1, ptr(ws), nws,
              int(max_blocks), stream_ptr(a.device))
    return out


def _splitk_ws(a, out, epilogue, M, N, K, batch, max_blocks=0):
    """Device workspace for the GEMM's deterministic split-K (None when unused)."""
    nws = _lib.load().irc_gemm_workspace_ex(_code(a), _code(out), int(epilogue), M, N, K, batch,
                                            int(max_blocks))
    if nws <= 0:
        return None, 0
    return torch.empty((nws,), dtype=torch.uint8, device=a.device), nws


def gemm_strided(a, b, out, *, M, N, K, batch, lda, sA, ldb, sB, ldc, sC, trans_a=False,
                 b_is_nk=True, alpha=1.0, accumulate=False, max_blocks=0):
    """Batched C_i (=|+=) alpha * op(A_i) @ op(B_i) over raw strides (elements):
    A_i = a + i*sA, etc.  Same operand layouts as ``gemm``; no epilogue.  max_blocks caps
    a split-K launch (irc_gemm_ex; 0 = one wave)."""
    require_hip(a, b, out)
    if a.dtype != b.dtype:
        raise TypeError("gemm operands must share a dtype")
    ws, nws = _splitk_ws(a, out, EPI_NONE, M, N, K, batch, max_blocks)
    _lib.call("irc_gemm_ex", _code(a), _code(out), 1 if trans_a else 0, 0 if b_is_nk else 1,
              EPI_NONE, M, N, K, float(alpha), ptr(a), lda, sA, ptr(b), ldb, sB, None, 0, None,
              0, 0, ptr(out), ldc, sC, 1 if accumulate else 0, batch, ptr(ws), nws,
              int(max_blocks), stream_ptr(a.device))
    return out


def embed_ln(ids, word, pos, type0, gamma, beta, eps=1e-12, out=None):
    require_hip(ids, word, pos, type0, gamma, beta, out)
    B, L = ids.shape
    H = word.shape[1]
    y = torch.empty((B * L, H), dtype=word.dtype, device=word.device) if out is None else out
    _lib.call("irc_embed_ln", _code(word), ptr(ids), ptr(word), ptr(pos), ptr(type0), ptr(gamma),
              ptr(beta), ptr(y), B * L, L, H, float(eps), stream_ptr(word.device))
    return y


def layernorm(x, gamma, beta, eps=1e-12, out=None):
    require_hip(x, gamma, beta)
    out = torch.empty_like(x) if out is None else out
    H = x.shape[-1]
    _lib.call("irc_layernorm", _code(x), ptr(x), ptr(out), ptr(gamma), ptr(beta),
              x.numel() // H, H, float(eps), stream_ptr(x.device))
    return out


def attention(qkv, mask, B, L, H, heads, out=None):
    require_hip(qkv, mask, out)
    ctx = torch.empty((B * L, H), dtype=qkv.dtype, device=qkv.device) if out is None else out
    _lib.call("irc_attention", _code(qkv), ptr(qkv), ptr(mask), ptr(ctx), B, L, H, heads,
              stream_ptr(qkv.device))
    return ctx


def qkv_perm_index(H: int, device=None) -> torch.Tensor:
    """Row order of Wqkv [3H][H] (query | key | value) for qkv_attention: block n of 384
    rows = Q, K, V rows of heads 2n and 2n + 1 (head dim 64)."""
    n = torch.arange(H // 128).view(-1, 1, 1) * 128
    part = torch.arange(3).view(1, -1, 1) * H
    return (n + part + torch.arange(128).view(1, 1, -1)).reshape(-1).to(device)


# The L the frozen encoder sends to the fused kernel: a sequence takes a 64-row (L <= 64)
# or 128-row (L <= 128) slot of the QKV GEMM, or 256 // L sequences share a packed tile, so
# the slot's or tile's unused rows are extra QKV work, against the separate attention
# launch and the QKV activation's HBM round trip the fusion saves.  Measured at B = 512
# (a C2 / C4 micro-batch), us per layer fused vs two-launch (profiles/r06_k/): L = 30-36:
# 77-92 vs 85-97; 40: 113 vs 98; 44-64: 116-125 vs 120-146; 65-76: 222-225 vs 180-220;
# 80: 224-225 vs 225-226; 85: 225 vs 237; 88-128: 240-263 vs 253-413.
QKV_ATTN_FUSED_L = ((29, 36), (44, 64), (80, 128))


def qkv_attention_supported(L: int, H: int, heads: int, ranges=((1, 128),)) -> bool:
    return any(lo <= L <= hi for lo, hi in ranges) and heads * 64 == H and H % 128 == 0


def qkv_attention(x, wqkv_perm, bias_perm, mask, B, L, H, heads, out=None):
    """irc_qkv_attention: ctx [B*L, H] bf16 = attention(x . Wqkv^T + b) in one launch
    (the QKV activation stays on chip).  wqkv_perm / bias_perm: rows in qkv_perm_index
    order.  One 64-row (L <= 64) or 128-row (L <= 128) slot per sequence.  Same result
    as gemm(EPI_BIAS) + attention on the big-tile shapes."""
    require_hip(x, wqkv_perm, bias_perm, mask, out)
    if x.dtype != BF16 or wqkv_perm.dtype != BF16 or bias_perm.dtype != F32:
        raise TypeError("qkv_attention: bf16 x / weights, fp32 bias")
    if not qkv_attention_supported(L, H, heads):
        raise ValueError("qkv_attention: needs L <= 128, head dim 64, H % 128 == 0")
    if x.shape != (B * L, H) or x.stride(-1) != 1 or tuple(wqkv_perm.shape) != (3 * H, H):
        raise ValueError("qkv_attention: x [B*L, H], Wqkv [3H, H]")
    if mask is not None and (mask.dtype != torch.int64 or not mask.is_contiguous()
                             or mask.numel() != B * L):
        raise ValueError("qkv_attention: mask must be a contiguous int64 [B, L] tensor")
    ctx = torch.empty((B * L, H), dtype=BF16, device=x.device) if out is None else out
    _lib.call("irc_qkv_attention", B * L, H, heads, L, ptr(x), x.stride(0), ptr(wqkv_perm),
              ptr(bias_perm), ptr(mask), ptr(ctx), ctx.stride(0), stream_ptr(x.device))
    return ctx


def lstm_fwd(xp, whh, B, L, H, ndir, h_dtype, save=True):
    """xp [B*L, ndir*4H] fp32 -> hout [B*L, ndir*H] (+ saved state for BPTT)."""
    require_hip(xp, whh)
    dev = xp.device
    hout = torch.empty((B * L, ndir * H), dtype=h_dtype, device=dev)
    gsave = torch.empty((ndir, B * L, 4 * H), dtype=F32, device=dev) if save else None
    csave = torch.empty((ndir, B * L, H), dtype=F32, device=dev) if save else None
    hprev = torch.empty((ndir, B * L, H), dtype=h_dtype, device=dev) if save else None
    if whh.dtype != h_dtype:
        raise TypeError("W_hh dtype must match the hidden-state dtype")
    _lib.call("irc_lstm_fwd", _code(whh), ptr(xp), ptr(whh), ptr(hout), ptr(gsave), ptr(csave),
              ptr(hprev), B, L, H, ndir, stream_ptr(dev))
    return hout, gsave, csave, hprev


def lstm_bwd(dy, whh, gsave, csave, B, L, H, ndir):
    require_hip(dy, whh, gsave, csave)
    dg = torch.empty((ndir, B * L, 4 * H), dtype=F32, device=dy.device)
    _lib.call("irc_lstm_bwd", _code(whh), ptr(dy), ptr(whh), ptr(gsave), ptr(csave), ptr(dg), B,
              L, H, ndir, stream_ptr(dy.device))
    return dg


def lstm_mfma_supported(H):
    return bool(_lib.load().irc_lstm_mfma_supported(H))


def lstm_pack(wih, bih, bhh, whh, H, ndir, whh_packs=True):
    """fp32 weights of one layer -> (wih_packed bf16, bias_packed fp32, whh bf16, whhT bf16);
    whh_packs=False skips the single-CU recurrence's W_hh packs (None, None): the cluster
    recurrence packs W_hh itself (lstm_coop_pack)."""
    require_hip(wih, bih, bhh, whh)
    dev = wih.device
    In = wih.shape[1]
    wp = torch.empty((ndir * 4 * H, In), dtype=BF16, device=dev)
    bp = torch.empty((ndir * 4 * H,), dtype=F32, device=dev)
    w = torch.empty((ndir, 4 * H, H), dtype=BF16, device=dev) if whh_packs else None
    wT = torch.empty((ndir, H, 4 * H), dtype=BF16, device=dev) if whh_packs else None
    _lib.call("irc_lstm_pack", ptr(wih), ptr(bih), ptr(bhh), ptr(whh), In, H, ndir, ptr(wp),
              ptr(bp), ptr(w), ptr(wT), stream_ptr(dev))
    return wp, bp, w, wT


def lstm_fwd_mfma(xp_packed, whh_bf16, B, L, H, ndir, save=True):
    require_hip(xp_packed, whh_bf16)
    dev = xp_packed.device
    lib = _lib.load()
    hout = torch.empty((B * L, ndir * H), dtype=BF16, device=dev)
    gsave = csave = hprev = None
    if save:
        gsave = torch.empty((lib.irc_lstm_mfma_save_floats(B, L, H, ndir, 0),), dtype=F32,
                            device=dev)
        csave = torch.empty((lib.irc_lstm_mfma_save_floats(B, L, H, ndir, 1),), dtype=F32,
                            device=dev)
        hprev = torch.empty((ndir, B * L, H), dtype=BF16, device=dev)
    _lib.call("irc_lstm_fwd_mfma", ptr(xp_packed), ptr(whh_bf16), ptr(hout), ptr(gsave),
              ptr(csave), ptr(hprev), B, L, H, ndir, stream_ptr(dev))
    return hout, gsave, csave, hprev


def lstm_bwd_mfma(dy, whhT_bf16, gsave, csave, B, L, H, ndir):
    require_hip(dy, whhT_bf16, gsave, csave)
    dg = torch.empty((B * L, ndir * 4 * H), dtype=BF16, device=dy.device)
    _lib.call("irc_lstm_bwd_mfma", ptr(dy), ptr(whhT_bf16), ptr(gsave), ptr(csave), ptr(dg), B, L,
              H, ndir, stream_ptr(dy.device))
    return dg


def lstm_coop_supported(H):
    return bool(_lib.load().irc_lstm_coop_supported(H))


def lstm_coop_pack(whh, H, ndir):
    """W_hh fp32 [ndir*4H, H] -> (wf, wb) resident-slice layouts (bf16)."""
    require_hip(whh)
    wf = torch.empty((ndir * 4 * H * H,), dtype=BF16, device=whh.device)
    wb = torch.empty_like(wf)
    _lib.call("irc_lstm_coop_pack", ptr(whh), H, ndir, ptr(wf), ptr(wb), stream_ptr(whh.device))
    return wf, wb


def _coop_bytes(B, L, H, ndir, which):
    return int(_lib.load().irc_lstm_coop_sizes(B, L, H, ndir, which))


def lstm_fwd_coop(xp_packed, wf, B, L, H, ndir, save=True):
    """Multi-CU forward recurrence -> (hout, gsave, csave, hprev, sync)."""
    require_hip(xp_packed, wf)
    dev = xp_packed.device
    hout = torch.empty((B * L, ndir * H), dtype=BF16, device=dev)
    gsave = csave = hprev = None
    if save:
        gsave = torch.empty((_coop_bytes(B, L, H, ndir, 0),), dtype=F32, device=dev)
        csave = torch.empty((_coop_bytes(B, L, H, ndir, 1),), dtype=F32, device=dev)
        # h_{t-1} for dW_hh, written by the recurrence itself alongside hout
        hprev = torch.empty((ndir, B * L, H), dtype=BF16, device=dev)
    xch = torch.empty((_coop_bytes(B, L, H, ndir, 2),), dtype=torch.uint8, device=dev)
    sync = torch.empty((_coop_bytes(B, L, H, ndir, 4) // 4,), dtype=torch.int32, device=dev)
    _lib.call("irc_lstm_fwd_coop", ptr(xp_packed), ptr(wf), ptr(hout), ptr(gsave), ptr(csave),
              ptr(hprev), ptr(xch), ptr(sync), B, L, H, ndir, stream_ptr(dev))
    return hout, gsave, csave, hprev, sync


def lstm_bwd_coop(dy, wb, gsave, csave, B, L, H, ndir):
    """Multi-CU BPTT -> (dgates bf16 [B*L, ndir*4H], sync)."""
    require_hip(dy, wb, gsave, csave)
    dev = dy.device
    dg = torch.empty((B * L, ndir * 4 * H), dtype=BF16, device=dev)
    xch = torch.empty((_coop_bytes(B, L, H, ndir, 3),), dtype=torch.uint8, device=dev)
    sync = torch.empty((_coop_bytes(B, L, H, ndir, 4) // 4,), dtype=torch.int32, device=dev)
    _lib.call("irc_lstm_bwd_coop", ptr(dy), ptr(wb), ptr(gsave), ptr(csave), ptr(dg), ptr(xch),
              ptr(sync), B, L, H, ndir, stream_ptr(dev))
    return dg, sync


def lstm_coop_fault(sync, B, ndir, fault):
    """fault (int32 device word) |= the coop call's timeout word -- stream-ordered,
    no host sync (the call has already NaN-poisoned its output on a timeout)."""
    require_hip(sync, fault)
    _lib.call("irc_lstm_coop_fault", ptr(sync), B, ndir, ptr(fault), stream_ptr(sync.device))


def lstm_coop_timed_out(sync, B, ndir):
    """Host check (synchronising) of a coop call's timeout word."""
    n = ndir * ((B + 31) // 32) * 16  # after the P * NW = 16 flag words per (dir, group)
    return int(sync[n].item()) != 0


def mean_rows(x, B, L, C, ldx=None):
    require_hip(x)
    out = torch.empty((B, C), dtype=F32, device=x.device)
    _lib.call("irc_mean_rows", _code(x), ptr(x), ptr(out), B, L, C, ldx or C,
              stream_ptr(x.device))
    return out


def bcast_rows(g, B, L, scale):
    require_hip(g)
    C = g.shape[1]
    y = torch.empty((B * L, C), dtype=F32, device=g.device)
    _lib.call("irc_bcast_rows", ptr(g), ptr(y), B, L, C, float(scale), stream_ptr(g.device))
    return y


def l2norm_fwd(x, eps=1e-12):
    require_hip(x)
    y = torch.empty_like(x)
    nrm = torch.empty((x.shape[0],), dtype=F32, device=x.device)
    _lib.call("irc_l2norm_fwd", ptr(x), ptr(y), ptr(nrm), x.shape[0], x.shape[1], float(eps),
              stream_ptr(x.device))
    return y, nrm


def l2norm_bwd(dy, y, nrm, eps=1e-12):
    require_hip(dy, y, nrm)
    dx = torch.empty_like(dy)
    _lib.call("irc_l2norm_bwd", ptr(dy), ptr(y), ptr(nrm), ptr(dx), dy.shape[0], dy.shape[1],
              float(eps), stream_ptr(dy.device))
    return dx


def nce_lse(S, LQ, N, K, T):
    require_hip(S, LQ)
    lse = torch.empty((2 * N,), dtype=F32, device=S.device)
    loss_row = torch.empty((2 * N,), dtype=F32, device=S.device)
    _lib.call("irc_nce_lse", ptr(S), ptr(LQ), N, K, float(T), ptr(lse), ptr(loss_row),
              stream_ptr(S.device))
    return lse, loss_row


def nce_grads(S, LQ, lse, N, K, T, gscale=None):
    """Softmax gradients of the InfoNCE rows, times the device scalar gscale."""
    require_hip(S, LQ, lse, gscale)
    GS = torch.empty_like(S)
    GQ = torch.empty((N, K), dtype=F32, device=S.device) if K > 0 else None
    _lib.call("irc_nce_grads", ptr(S), ptr(LQ), ptr(lse), N, K, float(T), ptr(gscale), ptr(GS),
              ptr(GQ), stream_ptr(S.device))
    return GS, GQ


def axpby(x, y, a=1.0, b=1.0, out=None):
    require_hip(x, y, out)
    out = torch.empty_like(x) if out is None else out
    _lib.call("irc_axpby", ptr(out), ptr(x), ptr(y), float(a), float(b), x.numel(),
              stream_ptr(x.device))
    return out


def dsum(x, scale=1.0):
    """Deterministic fp32 sum (fixed order) -> 0-d tensor."""
    require_hip(x)
    partial = torch.empty((1024,), dtype=F32, device=x.device)
    out = torch.empty((2,), dtype=F32, device=x.device)
    _lib.call("irc_sum", ptr(x), x.numel(), float(scale), ptr(partial), ptr(out),
              stream_ptr(x.device))
    return out[0]


def grad_norm_clip(g, max_norm):
    """[||g||, min(1, max_norm / (||g|| + 1e-6))] as a device tensor (no sync)."""
    require_hip(g)
    partial = torch.empty((1024,), dtype=F32, device=g.device)
    out = torch.empty((4,), dtype=F32, device=g.device)  # [norm, coef, step gate, pad]
    _lib.call("irc_grad_norm_clip", ptr(g), g.numel(), float(max_norm), ptr(partial), ptr(out),
              stream_ptr(g.device))
    return out


def adam_step(p, g, m, v, coef, b1, b2, step_size, bc2_sqrt, eps):
    require_hip(p, g, m, v, coef)
    _lib.call("irc_adam_step", ptr(p), ptr(g), ptr(m), ptr(v), p.numel(), ptr(coef), float(b1),
              float(b2), float(step_size), float(bc2_sqrt), float(eps), stream_ptr(p.device))


def sgd_step(p, g, buf, coef, lr, momentum, weight_decay, first, shadow=None):
    """torch.optim.SGD step (dampening 0, nesterov False) over a flat buffer, the clip
    coefficient / gate read from coef (None: unclipped); shadow: bf16 copy of p."""
    require_hip(p, g, buf)
    _lib.call("irc_sgd_step", ptr(p), ptr(g), ptr(buf), p.numel(),
              ptr(coef) if coef is not None else None, float(lr), float(momentum),
              float(weight_decay), int(bool(first)), ptr(shadow) if shadow is not None else None,
              stream_ptr(p.device))


# nn activation name -> irc kind code (include/irc.h IRC_ACT_*), torch default arguments
ACTIVATIONS = {name: i for i, name in enumerate(
    ["Identity", "ReLU", "ReLU6", "LeakyReLU", "ELU", "CELU", "SELU", "GELU", "SiLU", "Mish",
     "Sigmoid", "Tanh", "Softplus", "Softsign", "Hardtanh", "Hardsigmoid", "Hardswish",
     "Tanhshrink"])}


def activation(kind: int, u, out=None):
    """y = act(u) elementwise, fp32."""
    require_hip(u)
    if u.dtype != F32 or not u.is_contiguous():
        raise TypeError("activation: contiguous fp32 input")
    y = torch.empty_like(u) if out is None else out
    _lib.call("irc_activation", int(kind), ptr(u), ptr(y), u.numel(), stream_ptr(u.device))
    return y


def activation_bwd(kind: int, u, g):
    """g *= act'(u) in place (fp32)."""
    require_hip(u, g)
    if u.dtype != F32 or g.dtype != F32 or g.numel() != u.numel():
        raise TypeError("activation_bwd: fp32 u / g of equal size")
    _lib.call("irc_activation_bwd", int(kind), ptr(u), ptr(g), u.numel(), stream_ptr(u.device))
    return g


def fault_gate(coef, *faults):
    """coef[2] = 1 if any of the (<= 2) uint32 fault words is set: the gated updates
    of this step are skipped on the device."""
    require_hip(coef)
    f = [t for t in faults if t is not None]
    if len(f) > 2:
        raise ValueError("fault_gate takes at most two fault words")
    f += [None] * (2 - len(f))
    _lib.call("irc_fault_gate", ptr(f[0]), ptr(f[1]), ptr(coef), stream_ptr(coef.device))


def momentum_update_gated(pk, pq, mom, gate, shadow=None):
    require_hip(pk, pq, gate)
    _lib.call("irc_momentum_update_gated", ptr(pk), ptr(pq), pk.numel(), float(mom), ptr(gate),
              ptr(shadow), stream_ptr(pk.device))


def momentum_update(pk, pq, mom):
    require_hip(pk, pq)
    _lib.call("irc_momentum_update", ptr(pk), ptr(pq), pk.numel(), float(mom),
              stream_ptr(pk.device))


def enqueue(queue, keys, qptr):
    require_hip(queue, keys, qptr)
    D, K = queue.shape
    _lib.call("irc_enqueue", ptr(queue), ptr(keys), ptr(qptr), D, K, keys.shape[0],
              stream_ptr(queue.device))


def cast_bf16(x):
    require_hip(x)
    y = torch.empty(x.shape, dtype=BF16, device=x.device)
    _lib.call("irc_cast_bf16", ptr(x), ptr(y), x.numel(), stream_ptr(x.device))
    return y


def cast_bf16_t(x):
    """x fp32 [R, C] -> bf16 [C, R] (transposed copy)."""
    require_hip(x)
    R, C = x.shape
    y = torch.empty((C, R), dtype=BF16, device=x.device)
    _lib.call("irc_cast_bf16_t", ptr(x), ptr(y), R, C, stream_ptr(x.device))
    return y


def colsum(x, out=None, accumulate=False):
    require_hip(x)
    R, C = x.shape
    if out is None:
        out = torch.empty((C,), dtype=F32, device=x.device)
    partial = torch.empty((max(1, (R + 63) // 64) * C,), dtype=F32, device=x.device)
    _lib.call("irc_colsum", _code(x), ptr(x), ptr(out), R, C, x.stride(0), 1 if accumulate else 0,
              ptr(partial), stream_ptr(x.device))
    return out


# ---------------------------------------------------------------- encoder backward
EPI_DGELU, EPI_BIAS_GELU_SAVE = 5, 6


def gemm_gelu_save(a, b, bias, out=None, pre=None):
    """(gelu(a @ b.T + bias), a @ b.T + bias): FFN1 forward that also keeps the
    pre-activation for the GELU backward (epilogue 6 writes both)."""
    require_hip(a, b, bias)
    M, N = a.shape[0], b.shape[0]
    out = torch.empty((M, N), dtype=a.dtype, device=a.device) if out is None else out
    pre = torch.empty_like(out) if pre is None else pre
    return gemm(a, b, bias=bias, epilogue=EPI_BIAS_GELU_SAVE, residual=pre, out=out), pre


def layernorm_bwd(dy, x, gamma, dgamma, dbeta, eps=1e-12, bcast_L=0, dy_scale=1.0,
                  accumulate=True, out_dtype=None, out=None):
    """dL/dx of y = LN(x) * gamma + beta (statistics recomputed from x); dgamma /
    dbeta (+)= their deterministic column sums.  With bcast_L > 0, dy is [rows /
    bcast_L, H] and row r of the gradient is dy[r // bcast_L] * dy_scale."""
    require_hip(dy, x, gamma, dgamma, dbeta)
    H = x.shape[-1]
    rows = x.numel() // H
    dx = torch.empty((rows, H), dtype=out_dtype or x.dtype, device=x.device) if out is None \
        else out
    if dx.dtype != x.dtype:
        raise TypeError("layernorm_bwd: dx dtype must match x")
    nws = int(_lib.load().irc_layernorm_bwd_workspace(rows, H))
    ws = torch.empty((nws,), dtype=F32, device=x.device)
    _lib.call("irc_layernorm_bwd", _code(x), _code(dy), ptr(dy), ptr(x), ptr(gamma), ptr(dx),
              ptr(dgamma), ptr(dbeta), ptr(ws), nws, rows, H, float(eps), int(bcast_L),
              float(dy_scale), 1 if accumulate else 0, stream_ptr(x.device))
    return dx


def attention_bwd(qkv, mask, ctx, dctx, B, L, H, heads, out=None):
    """dqkv [B*L, 3H] of the fused-QKV masked self-attention (P recomputed)."""
    require_hip(qkv, mask, ctx, dctx, out)
    dqkv = torch.empty_like(qkv) if out is None else out
    _lib.call("irc_attention_bwd", _code(qkv), ptr(qkv), ptr(mask), ptr(ctx), ptr(dctx),
              ptr(dqkv), B, L, H, heads, stream_ptr(qkv.device))
    return dqkv


def embed_sum(ids, word, pos, type0):
    """fp32 [B*L, H] = word[ids] + type0 + pos[l]: the embedding-LN input, rebuilt
    for its backward (the forward fuses it into irc_embed_ln)."""
    require_hip(ids, word, pos, type0)
    B, L = ids.shape
    H = word.shape[1]
    y = torch.empty((B * L, H), dtype=F32, device=word.device)
    _lib.call("irc_embed_sum", _code(word), ptr(ids), ptr(word), ptr(pos), ptr(type0), ptr(y),
              B * L, L, H, stream_ptr(word.device))
    return y


def embed_bwd(dx, ids, dword, dpos, dtype0, pad_id):
    require_hip(dx, ids, dword, dpos, dtype0)
    B, L = ids.shape
    H = dx.shape[-1]
    ws = torch.empty((L * H,), dtype=F32, device=dx.device)
    _lib.call("irc_embed_bwd", _code(dx), ptr(dx), ptr(ids), ptr(dword), ptr(dpos), ptr(dtype0),
              ptr(ws), L * H, B, L, H, int(pad_id), stream_ptr(dx.device))


def adam_step_bf16(p, g, m, v, coef, b1, b2, step_size, bc2_sqrt, eps, shadow):
    require_hip(p, g, m, v, coef, shadow)
    _lib.call("irc_adam_step_bf16", ptr(p), ptr(g), ptr(m), ptr(v), p.numel(), ptr(coef),
              float(b1), float(b2), float(step_size), float(bc2_sqrt), float(eps), ptr(shadow),
              stream_ptr(p.device))


def momentum_update_bf16(pk, pq, mom, shadow):
    require_hip(pk, pq, shadow)
    _lib.call("irc_momentum_update_bf16", ptr(pk), ptr(pq), pk.numel(), float(mom), ptr(shadow),
              stream_ptr(pk.device))


def cast_bf16_t_into(x, y):
    """y bf16 [C, R] (a view is fine if contiguous) <- transpose of x fp32 [R, C]."""
    require_hip(x, y)
    R, C = x.shape
    _lib.call("irc_cast_bf16_t", ptr(x), ptr(y), R, C, stream_ptr(x.device))
    return y


def cast_bf16_t_batched(x_first, y, R, C, batch, sx):
    """y bf16 [batch, C, R] <- the transposes of `batch` fp32 [R, C] matrices that start at
    x_first's storage and lie sx floats apart (irc_cast_bf16_t_batched)."""
    require_hip(x_first, y)
    _lib.call("irc_cast_bf16_t_batched", ptr(x_first), ptr(y), R, C, batch, sx, C * R,
              stream_ptr(y.device))
    return y


def cast_bf16_into(x, y):
    require_hip(x, y)
    _lib.call("irc_cast_bf16", ptr(x), ptr(y), x.numel(), stream_ptr(x.device))
    return y


def colsum_batched(x, out, out_stride, accumulate=True):
    """x [batch, R, C] (bf16 / fp32, contiguous rows) -> out[b * out_stride + c] (+)=
    column sums of x[b] (deterministic)."""
    require_hip(x, out)
    nb, R, C = x.shape
    nws = int(_lib.load().irc_colsum_batched_workspace(nb, R, C))
    ws = torch.empty((max(nws, 1),), dtype=F32, device=x.device)
    _lib.call("irc_colsum_batched", _code(x), ptr(x), nb, R, C, x.stride(1), x.stride(0), ptr(out),
              int(out_stride), 1 if accumulate else 0, ptr(ws), nws, stream_ptr(x.device))


# ---- fp8 (e4m3) linear layers of the frozen encoder (csrc/fp8_linear.hip, config C5)
def quantize_rows_fp8(x):
    """x bf16 / fp32 [M, K] -> (e4m3 bytes uint8 [M, K], per-row fp32 scales [M]):
    q = e4m3(RNE(x * 448 / amax_row)), scale = amax_row / 448."""
    require_hip(x)
    if x.dtype not in (BF16, F32):
        raise TypeError(f"quantize_rows_fp8: bf16 or fp32 input, got {x.dtype}")
    if x.stride(-1) != 1:
        x = x.contiguous()
    M, K = x.shape
    q = torch.empty((M, K), dtype=torch.uint8, device=x.device)
    s = torch.empty((M,), dtype=F32, device=x.device)
    _lib.call("irc_quantize_rows_fp8", 0 if x.dtype == BF16 else 1, ptr(x), x.stride(0), M, K,
              ptr(q), K, ptr(s), stream_ptr(x.device))
    return q, s


def gemm_fp8(aq, sa, bq, sb, bias=None, epilogue=EPI_NONE, residual=None):
    """bf16 [M, N] = (aq . bq^T) * sa[:, None] * sb[None, :] (+ bias) (-> GELU)
    (+ residual): aq [M, K], bq [N, K] e4m3 bytes with their row scales."""
    require_hip(aq, sa, bq, sb, bias, residual)
    M, K = aq.shape
    N = bq.shape[0]
    if bq.shape[1] != K:
        raise ValueError(f"gemm_fp8 inner dims differ: {K} vs {bq.shape[1]}")
    out = torch.empty((M, N), dtype=BF16, device=aq.device)
    _lib.call("irc_gemm_fp8", ptr(aq), aq.stride(0), ptr(sa), ptr(bq), bq.stride(0), ptr(sb), M, N,
              K, ptr(bias), ptr(residual), residual.stride(0) if residual is not None else 0,
              ptr(out), out.stride(0), int(epilogue), stream_ptr(aq.device))
    return out


# ---- MX-fp8 (e4m3 + E8M0 per-32 block scales; csrc/mx.h, config C5) ----
class MX:
    """An MX-fp8 matrix: codes uint8 [rows, K] and block scales uint8 in the MX
    layout (K / 128 records of mpad * 4 bytes, mpad = rows rounded up to 256)."""

    __slots__ = ("codes", "scales", "mpad")

    def __init__(self, codes, scales, mpad):
        self.codes, self.scales, self.mpad = codes, scales, int(mpad)

    @property
    def shape(self):
        return self.codes.shape


def mx_pad(rows: int) -> int:
    return (int(rows) + 255) // 256 * 256


def mx_empty(rows, K, device):
    """Codes + scales of an MX operand.  Scale slots of the padding rows (rows..mpad) are
    zeroed (finite); with no padding every slot is written by the producer, so the zero
    fill (a separate launch per activation) is skipped."""
    mp = mx_pad(rows)
    n = (K // 128) * mp * 4
    scales = (torch.empty if mp == rows else torch.zeros)(n, dtype=torch.uint8, device=device)
    return MX(torch.empty((rows, K), dtype=torch.uint8, device=device), scales, mp)


def quantize_mx(x):
    """x bf16 / fp32 [M, K] (K % 128 == 0) -> MX: per 32 consecutive values of a row
    the smallest power-of-two scale s with max|x| / s <= 448, codes e4m3(RNE(x / s))."""
    require_hip(x)
    if x.dtype not in (BF16, F32):
        raise TypeError(f"quantize_mx: bf16 or fp32 input, got {x.dtype}")
    if x.stride(-1) != 1:
        x = x.contiguous()
    M, K = x.shape
    out = mx_empty(M, K, x.device)
    _lib.call("irc_quantize_mx_fp8", 0 if x.dtype == BF16 else 1, ptr(x), x.stride(0), M, K,
              ptr(out.codes), K, ptr(out.scales), out.mpad, stream_ptr(x.device))
    return out


def gemm_mx(a: MX, b: MX, bias=None, epilogue=EPI_NONE, residual=None, out_mx=False):
    """a [M, K] . b [N, K]^T of two MX-fp8 operands (block scales applied in the MFMA)
    (+ bias) (-> GELU) (+ residual bf16): bf16 [M, N], or MX when out_mx (epilogues
    EPI_BIAS / EPI_BIAS_GELU; the FFN1 output that FFN2 reads)."""
    require_hip(a.codes, b.codes, bias, residual)
    M, K = a.codes.shape
    N = b.codes.shape[0]
    if b.codes.shape[1] != K:
        raise ValueError(f"gemm_mx inner dims differ: {K} vs {b.codes.shape[1]}")
    if out_mx:
        out = mx_empty(M, N, a.codes.device)
        c, ldc, cx = out.codes, N, out.scales
    else:
        out = torch.empty((M, N), dtype=BF16, device=a.codes.device)
        c, ldc, cx = out, N, None
    _lib.call("irc_gemm_mx", ptr(a.codes), a.codes.stride(0), ptr(a.scales), a.mpad,
              ptr(b.codes), b.codes.stride(0), ptr(b.scales), b.mpad, M, N, K, ptr(bias),
              ptr(residual), residual.stride(0) if residual is not None else 0, ptr(c), ldc,
              ptr(cx), int(epilogue), stream_ptr(a.codes.device))
    return out


def layernorm_mx(x, gamma, beta, eps=1e-12, out=None):
    """(bf16 LN(x), its MX-fp8 copy) in one pass (x bf16 [rows, H])."""
    require_hip(x, gamma, beta)
    out = torch.empty_like(x) if out is None else out
    H = x.shape[-1]
    rows = x.numel() // H
    mx = mx_empty(rows, H, x.device)
    _lib.call("irc_layernorm_mx", ptr(x), ptr(out), ptr(gamma), ptr(beta), rows, H, float(eps),
              ptr(mx.codes), ptr(mx.scales), mx.mpad, stream_ptr(x.device))
    return out, mx


def attention_mx(qkv, mask, B, L, H, heads):
    """The attention context as MX-fp8 only (the fp8 out-projection's A operand)."""
    require_hip(qkv, mask)
    mx = mx_empty(B * L, H, qkv.device)
    _lib.call("irc_attention_mx", ptr(qkv), ptr(mask), ptr(mx.codes), ptr(mx.scales), mx.mpad,
              B, L, H, heads, stream_ptr(qkv.device))
    return mx
