"""ctypes binding of libirc_hip.so (the C ABI declared in include/irc.h).

The product path has NO fallback: if the library is missing or the device is not
a HIP GPU, every op raises.  Build the library with ``__graft_entry__.build()``
(or ``make -C information-retrieval-with-contrastive-learning_amd/csrc``).
"""
from __future__ import annotations

import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "libirc_hip.so")
# IRC_LIB_PATH: load a differently built copy (A/B experiments of kernel variants)
LIB_PATH = os.environ.get("IRC_LIB_PATH") or LIB_PATH

_c = ctypes
P = _c.c_void_p
I64 = _c.c_int64
I32 = _c.c_int
F32 = _c.c_float

# name -> (restype, argtypes).  Keep in sync with include/irc.h
# (tests/test_abi.py checks every declared symbol is exported and bound here).
SIGNATURES = {
    "irc_last_error": (_c.c_char_p, []),
    "irc_abi_version": (I32, []),
    "irc_scan_topk_workspace": (I64, [I64, I64, I64, I64]),
    "irc_scan_topk": (I32, [P, P, I64, I64, I64, I64, I64, P, I64, P, P, P]),
    "irc_scan_topk_many": (I32, [P, I64, P, I64, I64, I64, I64, I64, P, I64, I64, P, P, P, P]),
    "irc_corpus_pack": (I32, [P, P, I64, I64, P, P, P]),
    "irc_pair_sample": (I32, [P, P, P, P, I64, P, P]),
    "irc_pair_batch": (I32, [P, P, P, I64, I64, I64, I64, I64, P, P, P]),
    "irc_nce_fused_workspace": (I64, [I64, I64, I64, I64, I64]),
    "irc_nce_fused_fwd": (I32, [P, P, I64, I64, I64, F32, I64, I64, P, I64, P, P, P]),
    "irc_nce_fused_bwd": (I32, [P, P, P, I64, I64, I64, F32, P, I64, I64, P, I64, P, P]),
    "irc_scan_rescan_stats": (I32, [P, I32]),
    "irc_topk_merge": (I32, [P, P, I64, I64, I64, I64, P, P, P]),
    "irc_scan_scores": (I32, [P, P, I64, I64, I64, P, P]),
    "irc_scan_topk_fp8_workspace": (I64, [I64, I64, I64, I64]),
    "irc_scan_topk_fp8": (I32, [P, P, I64, I64, I64, I64, I64, F32, P, I64, P, P, P]),
    "irc_scan_scores_fp8": (I32, [P, P, I64, I64, I64, P, P]),
    "irc_quantize_fp8": (I32, [I32, P, I64, F32, P, P]),
    "irc_csr_union_chunks": (I64, [I64]),
    "irc_csr_union_count": (I32, [P, P, I64, P, P, I64, I64, P, P, P]),
    "irc_csr_union_emit": (I32, [P, I64, I64, P, P, P, P]),
    "irc_csr_spmv_f64": (I32, [P, P, P, I64, P, P, P, I64, P, P]),
    "irc_topk_f64": (I32, [P, I64, P, P, I64, I64, P, P, P, P]),
    "irc_proto_ce": (I32, [P, P, I64, I64, P, P, P, P]),
    "irc_argmax_bias": (I32, [P, P, I64, I64, P, P, P]),
    "irc_centroid_accumulate": (I32, [P, P, I64, I64, P, P, P]),
    "irc_centroid_finalize": (I32, [P, P, I64, I64, P, P, P]),
    "irc_gemm": (I32, [I32, I32, I32, I32, I32, I64, I64, I64, F32, P, I64, I64, P, I64, I64,
                       P, I64, P, I64, I64, P, I64, I64, I32, I64, P, I64, P]),
    "irc_gemm_workspace": (I64, [I32, I32, I32, I64, I64, I64, I64]),
    "irc_gemm_ex": (I32, [I32, I32, I32, I32, I32, I64, I64, I64, F32, P, I64, I64, P, I64, I64,
                          P, I64, P, I64, I64, P, I64, I64, I32, I64, P, I64, I64, P]),
    "irc_gemm_workspace_ex": (I64, [I32, I32, I32, I64, I64, I64, I64, I64]),
    "irc_gemm_set_persistent": (I32, [I32]),
    "irc_gemm_set_big_ring": (I32, [I32]),
    "irc_gemm_ln": (I32, [I32, I64, I64, I64, P, I64, P, I64, P, P, I64, P, I64, P, I32, P, P, F32,
                          I64, P, P, P, P]),
    "irc_gemm_set_big_mf16": (I32, [I32]),
    "irc_scan_set_ppl_min_q": (I32, [I32]),
    "irc_embed_ln": (I32, [I32, P, P, P, P, P, P, P, I64, I64, I64, F32, P]),
    "irc_layernorm": (I32, [I32, P, P, P, P, I64, I64, F32, P]),
    "irc_attention": (I32, [I32, P, P, P, I64, I64, I64, I64, P]),
    "irc_qkv_attention": (I32, [I64, I64, I64, I64, P, I64, P, P, P, P, I64, P]),
    "irc_layernorm_bwd_workspace": (I64, [I64, I64]),
    "irc_layernorm_bwd": (I32, [I32, I32, P, P, P, P, P, P, P, I64, I64, I64, F32, I64, F32, I32,
                                P]),
    "irc_attention_bwd": (I32, [I32, P, P, P, P, P, I64, I64, I64, I64, P]),
    "irc_embed_sum": (I32, [I32, P, P, P, P, P, I64, I64, I64, P]),
    "irc_embed_bwd": (I32, [I32, P, P, P, P, P, P, I64, I64, I64, I64, I64, P]),
    "irc_lstm_fwd": (I32, [I32, P, P, P, P, P, P, I64, I64, I64, I64, P]),
    "irc_lstm_bwd": (I32, [I32, P, P, P, P, P, I64, I64, I64, I64, P]),
    "irc_lstm_mfma_supported": (I32, [I64]),
    "irc_lstm_mfma_save_floats": (I64, [I64, I64, I64, I64, I32]),
    "irc_lstm_pack": (I32, [P, P, P, P, I64, I64, I64, P, P, P, P, P]),
    "irc_lstm_fwd_mfma": (I32, [P, P, P, P, P, P, I64, I64, I64, I64, P]),
    "irc_lstm_bwd_mfma": (I32, [P, P, P, P, P, I64, I64, I64, I64, P]),
    "irc_lstm_hprev": (I32, [P, P, I64, I64, I64, I64, P]),
    "irc_lstm_coop_supported": (I32, [I64]),
    "irc_lstm_coop_sizes": (I64, [I64, I64, I64, I64, I32]),
    "irc_lstm_coop_pack": (I32, [P, I64, I64, P, P, P]),
    "irc_lstm_fwd_coop": (I32, [P, P, P, P, P, P, P, P, I64, I64, I64, I64, P]),
    "irc_lstm_bwd_coop": (I32, [P, P, P, P, P, P, P, I64, I64, I64, I64, P]),
    "irc_lstm_coop_fault": (I32, [P, I64, I64, P, P]),
    "irc_mean_rows": (I32, [I32, P, P, I64, I64, I64, I64, P]),
    "irc_bcast_rows": (I32, [P, P, I64, I64, I64, F32, P]),
    "irc_l2norm_fwd": (I32, [P, P, P, I64, I64, F32, P]),
    "irc_l2norm_bwd": (I32, [P, P, P, P, I64, I64, F32, P]),
    "irc_nce_lse": (I32, [P, P, I64, I64, F32, P, P, P]),
    "irc_nce_grads": (I32, [P, P, P, I64, I64, F32, P, P, P, P]),
    "irc_axpby": (I32, [P, P, P, F32, F32, I64, P]),
    "irc_sum": (I32, [P, I64, F32, P, P, P]),
    "irc_grad_norm_clip": (I32, [P, I64, F32, P, P, P]),
    "irc_sgd_step": (I32, [P, P, P, I64, P, F32, F32, F32, I32, P, P]),
    "irc_activation": (I32, [I32, P, P, I64, P]),
    "irc_activation_bwd": (I32, [I32, P, P, I64, P]),
    "irc_adam_step": (I32, [P, P, P, P, I64, P, F32, F32, F32, F32, F32, P]),
    "irc_fault_gate": (I32, [P, P, P, P]),
    "irc_momentum_update_gated": (I32, [P, P, I64, F32, P, P, P]),
    "irc_momentum_update": (I32, [P, P, I64, F32, P]),
    "irc_adam_step_bf16": (I32, [P, P, P, P, I64, P, F32, F32, F32, F32, F32, P, P]),
    "irc_momentum_update_bf16": (I32, [P, P, I64, F32, P, P]),
    "irc_enqueue": (I32, [P, P, P, I64, I64, I64, P]),
    "irc_cast_bf16": (I32, [P, P, I64, P]),
    "irc_cast_bf16_t": (I32, [P, P, I64, I64, P]),
    "irc_cast_bf16_t_batched": (I32, [P, P, I64, I64, I64, I64, I64, P]),
    "irc_colsum": (I32, [I32, P, P, I64, I64, I64, I32, P, P]),
    "irc_colsum_batched_workspace": (I64, [I64, I64, I64]),
    "irc_colsum_batched": (I32, [I32, P, I64, I64, I64, I64, I64, P, I64, I32, P, I64, P]),
    "irc_quantize_rows_fp8": (I32, [I32, P, I64, I64, I64, P, I64, P, P]),
    "irc_gemm_fp8": (I32, [P, I64, P, P, I64, P, I64, I64, I64, P, P, I64, P, I64, I32, P]),
    "irc_quantize_mx_fp8": (I32, [I32, P, I64, I64, I64, P, I64, P, I64, P]),
    "irc_gemm_mx": (I32, [P, I64, P, I64, P, I64, P, I64, I64, I64, I64, P, P, I64, P, I64, P,
                          I32, P]),
    "irc_layernorm_mx": (I32, [P, P, P, P, I64, I64, F32, P, P, I64, P]),
    "irc_attention_mx": (I32, [P, P, P, P, I64, I64, I64, I64, I64, P]),
    "irc_wordpiece": (I32, [P, P, I64, P, P, P, P, P, I64, P, P, P, I64, I64, I64, P, P, P, P]),
    "irc_wordpiece_pad": (I32, [P, P, I64, I64, I64, I64, I64, I64, P, P, P]),
    "irc_prof_enable": (I32, [I32]),
    "irc_prof_query": (I32, [_c.c_char_p, _c.POINTER(_c.c_double), _c.POINTER(I64),
                             _c.POINTER(_c.c_double)]),
    "irc_prof_reset": (I32, []),
}

_lock = threading.Lock()
_lib = None


class IRCError(RuntimeError):
    pass


def load():
    """Load (once) and return the library; raises IRCError if it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise IRCError(
                f"libirc_hip.so not found at {LIB_PATH}: build it first "
                "(python -c 'import __graft_entry__ as g; g.build()'). "
                "There is no CPU fallback.")
        lib = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
        return lib


def call(name: str, *args):
    """Call an IRC entry point; raise on a non-zero status with the library's
    thread-local message ("out of memory" is kept in the text so the
    reference's OOM handler, src/train.py:190-195, still matches)."""
    lib = load()
    rc = getattr(lib, name)(*args)
    if rc != 0:
        msg = lib.irc_last_error().decode(errors="replace")
        if rc == 2:  # hipErrorOutOfMemory
            msg = "HIP out of memory: " + msg
        raise IRCError(f"{name} failed (rc={rc}): {msg}")
    return rc


def fn(name: str):
    return getattr(load(), name)
