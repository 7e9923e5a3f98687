"""ctypes binding of libclassmate_hip.so (the C ABI in include/classmate_hip.h).

cffi is not installed on this image, so the binding is ctypes.  torch is
imported first when available: torch-ROCm ships its own ``libamdhip64.so.7``
and loading it before our library makes both share ONE HIP runtime (same
SONAME), so device pointers from torch tensors are valid in our kernels.

There is deliberately no fallback: if the shared library is missing the
import fails with instructions to build it.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

try:  # share torch's HIP runtime when torch is present
    import torch  # noqa: F401
except Exception:  # pragma: no cover - torch is optional for the C-ABI itself
    torch = None

LIB_NAME = "libclassmate_hip.so"
LIB_PATH = Path(os.environ.get("CLASSMATE_HIP_LIB", Path(__file__).with_name(LIB_NAME)))

CM_OK, CM_EINVAL, CM_ENOMEM, CM_EDEVICE, CM_EZERODIV, CM_EUNSUPPORTED = 0, -1, -2, -3, -4, -5
CM_FOP_EQ, CM_FOP_NE, CM_FOP_BITS, CM_FOP_TRUE, CM_FOP_FALSE, CM_FOP_AND, CM_FOP_OR, CM_FOP_NOT = range(1, 9)
CM_FILTER_MAX_OPS, CM_FILTER_MAX_SOURCES = 64, 16
CM_DTYPE_F32, CM_DTYPE_BF16, CM_DTYPE_F16, CM_DTYPE_I32, CM_DTYPE_I64 = 0, 1, 2, 3, 4

if not LIB_PATH.exists():
    raise ImportError(
        f"{LIB_PATH} not found: build the HIP extension first "
        f"(python -c 'import __graft_entry__ as g; g.build()' or make -C classmate-rag_amd)")

lib = C.CDLL(str(LIB_PATH), mode=C.RTLD_GLOBAL)

c_int, c_i32, c_i64, c_u8, c_u32 = C.c_int, C.c_int32, C.c_int64, C.c_uint8, C.c_uint32
c_f32, c_f64, c_vp, c_char_p = C.c_float, C.c_double, C.c_void_p, C.c_char_p
P = C.POINTER


def _fn(name, restype, *argtypes):
    f = getattr(lib, name)
    f.restype = restype
    f.argtypes = list(argtypes)
    return f


# name -> (restype, argtypes); keep in sync with include/classmate_hip.h
SIGNATURES = {
    "cm_last_error": (c_char_p,),
    "cm_version": (c_int,),
    "cm_device_count": (c_int, P(c_int)),
    "cm_stream_create_cu_masked": (c_int, c_int, P(C.c_uint32), c_int, P(c_vp)),
    "cm_stream_destroy": (c_int, c_vp),
    "cm_max_topk": (c_int,),
    "cm_dense_create": (c_int, c_int, c_i32, c_i64, P(c_vp)),
    "cm_dense_destroy": (None, c_vp),
    "cm_dense_reserve": (c_int, c_vp, c_i64),
    "cm_dense_mem_stats": (c_int, c_vp, c_vp, c_vp, c_vp),
    "cm_dense_set_growth": (c_int, c_vp, c_i32),
    "cm_dense_upsert": (c_int, c_vp, c_vp, c_vp, c_i64),
    "cm_dense_upsert_dev": (c_int, c_vp, c_vp, c_i64, c_i64, c_vp),
    "cm_dense_delete": (c_int, c_vp, c_vp, c_i64),
    "cm_dense_reset": (c_int, c_vp),
    "cm_dense_live_count": (c_i64, c_vp),
    "cm_dense_size": (c_i64, c_vp),
    "cm_dense_dim": (c_i32, c_vp),
    "cm_dense_search": (c_int, c_vp, c_vp, c_i32, c_i32, c_vp, c_vp, c_vp, c_vp),
    "cm_dense_search_workspace": (c_i64, c_vp, c_i32, c_i32),
    "cm_dense_search_kind": (c_i32, c_vp, c_i32, c_i32),
    "cm_dense_set_path": (c_int, c_vp, c_i32),
    "cm_dense_workspace_fallbacks": (c_i32, c_vp, c_i32, c_i32, c_vp),
    "cm_dense_last_fallbacks": (c_i32, c_vp),
    "cm_dense_workspace_wide_reranks": (c_i32, c_vp, c_i32, c_i32, c_vp),
    "cm_dense_last_wide_reranks": (c_i32, c_vp),
    "cm_dense_timing": (c_int, c_vp, c_i32),
    "cm_dense_set_seed_event": (c_int, c_vp, c_vp),
    "cm_dense_timing_drain": (c_i32, c_vp, c_vp, c_i32),
    "cm_bm25_timing": (c_int, c_vp, c_i32),
    "cm_bm25_timing_drain": (c_i32, c_vp, c_vp, c_i32),
    "cm_dense_search_dev": (c_int, c_vp, c_vp, c_i32, c_i32, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp),
    "cm_shard_merge_topk_dev": (c_int, c_vp, c_i32, c_i32, c_i32, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp),
    "cm_dense_search_dev_deferred": (c_int, c_vp, c_vp, c_i32, c_i32, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp),
    "cm_dense_exact_fallback_dev": (c_int, c_vp, c_vp, c_i32, c_i32, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp),
    "cm_dense_export": (c_int, c_vp, c_i64, c_i64, c_vp, c_vp),
    "cm_dense_gather_dev": (c_int, c_vp, c_vp, c_i64, c_vp, c_vp),
    "cm_dense_live_bits_dev": (c_vp, c_vp),
    "cm_bm25_create": (c_int, c_int, P(c_vp)),
    "cm_bm25_destroy": (None, c_vp),
    "cm_bm25_build": (c_int, c_vp, c_vp, c_vp, c_i64, c_i32, c_vp),
    "cm_bm25_build_dev": (c_int, c_vp, c_vp, c_vp, c_i64, c_i64, c_i32, c_vp),
    "cm_bm25_num_docs": (c_i64, c_vp),
    "cm_bm25_num_postings": (c_i64, c_vp),
    "cm_bm25_stats": (c_int, c_vp, P(c_i64), P(c_i64), P(c_f64), P(c_f64)),
    "cm_bm25_export": (c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp),
    "cm_bm25_set_head_policy": (c_int, c_vp, c_f64, c_i64),
    "cm_bm25_num_head_terms": (c_i32, c_vp),
    "cm_bm25_set_path": (c_int, c_vp, c_i32),
    "cm_bm25_workspace_rescored": (c_i32, c_vp, c_i32, c_i32, c_i32, c_vp),
    "cm_bm25_last_rescored": (c_i32, c_vp),
    "cm_bm25_term_stats": (c_int, c_vp, c_vp, c_vp),
    "cm_bm25_set_stats": (c_int, c_vp, c_vp, c_i32, c_i64, c_i64, c_f64),
    "cm_bm25_search": (c_int, c_vp, c_vp, c_vp, c_i32, c_i32, c_vp, c_vp, c_vp, c_vp),
    "cm_bm25_workspace_items": (c_i64, c_vp, c_i32, c_i32, c_i32, c_vp, c_vp, c_i64),
    "cm_bm25_workspace_subblocks": (c_i64, c_vp, c_i32, c_i32, c_i32, c_vp, c_vp, c_i64),
    "cm_bm25_timing_drain_block": (c_i32, c_vp, c_vp, c_i32),
    "cm_bm25_search_idf": (c_int, c_vp, c_vp, c_vp, c_i32, c_i32, c_vp, c_vp, c_f64, c_i64, c_vp, c_vp, c_vp),
    "cm_bm25_search_workspace": (c_i64, c_vp, c_i32, c_i32, c_i32),
    "cm_bm25_search_dev": (c_int, c_vp, c_vp, c_vp, c_i32, c_i32, c_i32, c_vp, c_vp, c_vp, c_i64, c_vp),
    "cm_bm25_search_dev_gated": (c_int, c_vp, c_vp, c_vp, c_i32, c_i32, c_i32, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp),
    "cm_bm25_prepare_filtered": (c_int, c_vp, c_i64),
    "cm_bm25_filter_stats_dev": (c_int, c_vp, c_vp, c_vp, c_i32, c_vp, c_vp, c_vp),
    "cm_bm25_filter_term_stats_dev": (c_int, c_vp, c_vp, c_vp, c_vp, c_vp),
    "cm_bm25_filter_eps": (c_int, c_vp, c_vp, P(c_f64)),
    "cm_bm25_search_stats_dev": (c_int, c_vp, c_vp, c_vp, c_i32, c_i32, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                                 c_vp, c_vp, c_i64, c_vp),
    "cm_bm25_search_filtered_dev": (c_int, c_vp, c_vp, c_vp, c_i32, c_i32, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp,
                                    c_vp, c_i64, c_vp),
    "cm_mmr": (c_int, c_vp, c_vp, c_vp, c_i32, c_i32, c_i32, c_i32, c_f64, c_vp),
    "cm_mmr_dev": (c_int, c_vp, c_vp, c_vp, c_i32, c_i32, c_i32, c_i32, c_f64, c_vp, c_vp),
    "cm_rrf_fuse": (c_int, c_vp, c_vp, c_i32, c_vp, c_i32, c_vp, c_vp, P(c_i32)),
    "cm_rrf_merge": (c_int, c_vp, c_vp, c_vp, c_i32, c_vp, c_vp, c_vp, c_i32, c_i32, c_f64, c_f64, c_i32, c_i32,
                     c_vp, c_vp, c_vp, c_vp, c_vp, c_vp),
    "cm_rrf_pool_prep_dev": (c_int, c_vp, c_vp, c_i32, c_vp, c_i32, c_vp, c_i32, c_i32, c_vp, c_vp, c_vp, c_vp,
                             c_vp),
    "cm_rrf_merge_dev": (c_int, c_vp, c_vp, c_vp, c_i32, c_vp, c_vp, c_vp, c_i32, c_i32, c_f64, c_f64, c_i32, c_i32,
                         c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp),
    "cm_filter_eval": (c_int, c_vp, c_i32, c_vp, c_i32, c_vp, c_i32, c_i64, c_vp, c_vp, c_vp),
    "cm_meanpool_l2norm": (c_int, c_vp, c_i32, c_vp, c_i32, c_i32, c_i32, c_i32, c_i32, c_vp, c_vp),
    "cm_short_attention": (c_int, c_vp, c_i32, c_i32, c_i32, c_i32, c_f32, c_i32, c_vp, c_vp),
    "cm_add_layernorm": (c_int, c_vp, c_vp, c_i64, c_vp, c_vp, c_i64, c_i32, c_f32, c_i32, c_vp, c_vp),
    "cm_f16x3_plane_rows": (c_i64, c_i64),
    "cm_f16x3_split_rows": (c_int, c_vp, c_i64, c_i32, c_f32, c_vp, c_vp),
    "cm_f16x3_split_weights": (c_int, c_vp, c_i32, c_i32, c_f32, c_vp, c_vp),
    "cm_linear_f16x3": (c_int, c_vp, c_i64, c_i32, c_vp, c_vp, c_f32, c_i32, c_i32, c_vp, c_f32, c_vp, c_vp),
    "cm_add_layernorm_split": (c_int, c_vp, c_vp, c_i64, c_vp, c_vp, c_i64, c_i32, c_f32, c_vp, c_f32, c_vp, c_vp),
    "cm_short_attention_split": (c_int, c_vp, c_i32, c_i32, c_i32, c_i32, c_f32, c_f32, c_vp, c_vp),
    "cm_short_attention_split_masked": (c_int, c_vp, c_i32, c_i32, c_i32, c_i32, c_f32, c_f32, c_vp, c_vp, c_vp),
    "cm_long_attention_split": (c_int, c_vp, c_i32, c_i32, c_i32, c_i32, c_f32, c_f32, c_vp, c_vp, c_vp),
    "cm_planes_attention": (c_int, c_vp, c_i32, c_i32, c_i32, c_i32, c_f32, c_f32, c_f32, c_vp, c_vp, c_vp),
}
CM_EPI_BIAS, CM_EPI_BIAS_GELU, CM_EPI_PLANES_GELU, CM_EPI_PLANES_QKV = 0, 1, 2, 3

fn = {name: _fn(name, sig[0], *sig[1:]) for name, sig in SIGNATURES.items()}


def last_error() -> str:
    msg = fn["cm_last_error"]()
    return msg.decode("utf-8", "replace") if msg else ""


def check(rc: int, what: str = "") -> None:
    """Map C-ABI return codes to the reference's Python exception types."""
    if rc == CM_OK:
        return
    msg = last_error() or f"error {rc}"
    if what:
        msg = f"{what}: {msg}"
    if rc == CM_EINVAL:
        raise ValueError(msg)
    if rc == CM_EZERODIV:
        raise ZeroDivisionError(msg)
    if rc == CM_ENOMEM:
        raise MemoryError(msg)
    raise RuntimeError(msg)


def ptr(a) -> int | None:
    """Address of a numpy array (C-contiguous) or torch tensor, None for None."""
    if a is None:
        return None
    if hasattr(a, "data_ptr"):
        return a.data_ptr()
    return a.ctypes.data


def device_count() -> int:
    n = C.c_int(0)
    rc = fn["cm_device_count"](C.byref(n))
    return n.value if rc == CM_OK else 0


def max_topk() -> int:
    return int(fn["cm_max_topk"]())
