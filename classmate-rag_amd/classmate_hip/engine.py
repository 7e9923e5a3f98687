"""Device-resident retrieval engines over the C ABI (include/classmate_hip.h).

``DenseIndex`` (cosine k-NN, K1), ``BM25Index`` (postings + BM25, K2/K3/K7)
and the fusion / pooling ops (K4 MMR, K5 RRF, K6 mean-pool).  Two call styles:

* host arrays (numpy) — used by the drop-in classes in ``classmate_hip.retrieval``;
* device tensors (torch) on torch's current HIP stream — used by the batched
  pipeline and ``bench.py`` (inputs resident in HBM, graph-capturable).

Rows are the integer positions the stores assign; string ids / documents /
metadata stay on the host (classmate_hip.retrieval).
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Optional, Sequence

import numpy as np

from . import _lib as L

try:
    import torch
except Exception:  # pragma: no cover
    torch = None


def default_device() -> int:
    env = os.environ.get("CM_DEVICE")
    if env:
        return int(env)
    if torch is not None and torch.cuda.is_available():
        return torch.cuda.current_device()
    return 0


def _stream(device: int):
    if torch is None:
        return None
    return C.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def _c(a, dtype):
    return np.ascontiguousarray(a, dtype=dtype)


def cu_masked_stream(device: int, cus):
    """A torch.cuda.ExternalStream whose kernels run only on the CU indices in ``cus``
    (``cm_stream_create_cu_masked``); the HIP stream lives as long as the returned object."""
    n_cu = torch.cuda.get_device_properties(device).multi_processor_count
    words = np.zeros((n_cu + 31) // 32, np.uint32)
    for c in cus:
        if not 0 <= c < n_cu:
            raise ValueError(f"CU index {c} outside 0..{n_cu - 1}")
        words[c // 32] |= np.uint32(1 << (c % 32))
    ptr = C.c_void_p()
    L.check(L.fn["cm_stream_create_cu_masked"](device, words.ctypes.data_as(C.POINTER(C.c_uint32)), words.size,
                                                C.byref(ptr)), "cm_stream_create_cu_masked")
    st = torch.cuda.ExternalStream(ptr.value, device=torch.device("cuda", device))
    st._cm_keep = (words, _StreamOwner(ptr.value))
    return st


class _StreamOwner:
    def __init__(self, ptr):
        self.ptr = ptr

    def __del__(self):
        try:
            L.fn["cm_stream_destroy"](C.c_void_p(self.ptr))
        except Exception:
            pass


class DenseIndex:
    """HBM-resident fp32 corpus + exact cosine top-k (replaces Chroma's HNSW)."""

    def __init__(self, dim: int, device: Optional[int] = None, capacity: int = 0):
        self.device = default_device() if device is None else int(device)
        h = C.c_void_p()
        L.check(L.fn["cm_dense_create"](self.device, int(dim), int(capacity), C.byref(h)), "cm_dense_create")
        self._h = h
        self.dim = int(dim)
        self._ws = None

    # -- lifecycle -------------------------------------------------------
    def close(self):
        if getattr(self, "_h", None):
            L.fn["cm_dense_destroy"](self._h)
            self._h = None

    def __del__(self):  # pragma: no cover - interpreter shutdown order
        try:
            self.close()
        except Exception:
            pass

    # -- mutation --------------------------------------------------------
    def reserve(self, capacity: int):
        L.check(L.fn["cm_dense_reserve"](self._h, int(capacity)), "cm_dense_reserve")

    def set_growth(self, mode: int):
        """0 auto (device-to-device copy when old + new fit in free HBM, else host-staged), 1 always
        host-staged above 1 GiB (peak = the final allocation) -- cm_dense_set_growth."""
        L.check(L.fn["cm_dense_set_growth"](self._h, int(mode)), "cm_dense_set_growth")

    def mem_stats(self) -> dict:
        """Device bytes of the row arrays now / at most at once, and the growths staged through
        host memory (cm_dense_mem_stats)."""
        cur, peak, staged = C.c_int64(), C.c_int64(), C.c_int64()
        L.check(L.fn["cm_dense_mem_stats"](self._h, C.byref(cur), C.byref(peak), C.byref(staged)),
                "cm_dense_mem_stats")
        return {"bytes": cur.value, "peak_bytes": peak.value, "staged_growths": staged.value}

    def upsert(self, vecs: np.ndarray, rows: np.ndarray):
        v = _c(vecs, np.float32)
        r = _c(rows, np.int64)
        if v.ndim != 2 or v.shape[1] != self.dim or v.shape[0] != r.shape[0]:
            raise ValueError(f"expected ({r.shape[0]}, {self.dim}) embeddings, got {v.shape}")
        L.check(L.fn["cm_dense_upsert"](self._h, L.ptr(v), L.ptr(r), int(r.shape[0])), "cm_dense_upsert")

    def upsert_dev(self, vecs, row0: int):
        """vecs: contiguous float32 device tensor (n, dim) -> rows [row0, row0+n)."""
        assert vecs.is_cuda and vecs.dtype == torch.float32 and vecs.is_contiguous() and vecs.shape[1] == self.dim
        L.check(L.fn["cm_dense_upsert_dev"](self._h, L.ptr(vecs), int(row0), int(vecs.shape[0]),
                                            _stream(self.device)), "cm_dense_upsert_dev")

    def delete(self, rows):
        r = _c(rows, np.int64)
        L.check(L.fn["cm_dense_delete"](self._h, L.ptr(r), int(r.shape[0])), "cm_dense_delete")

    def reset(self):
        L.check(L.fn["cm_dense_reset"](self._h), "cm_dense_reset")

    # -- queries ---------------------------------------------------------
    @property
    def size(self) -> int:
        return int(L.fn["cm_dense_size"](self._h))

    def live_count(self) -> int:
        n = int(L.fn["cm_dense_live_count"](self._h))
        if n < 0:
            raise RuntimeError(L.last_error())
        return n

    def search(self, q: np.ndarray, k: int, allow_bits: Optional[np.ndarray] = None, return_vectors: bool = False):
        """q: (nq, dim) -> dist (nq,k) f32, rows (nq,k) i64 (-1 pad)[, vecs (nq,k,dim)]."""
        qq = _c(np.atleast_2d(q), np.float32)
        if qq.shape[1] != self.dim:
            raise ValueError(f"query dim {qq.shape[1]} != index dim {self.dim}")
        nq = qq.shape[0]
        dist = np.empty((nq, k), np.float32)
        rows = np.empty((nq, k), np.int64)
        vecs = np.empty((nq, k, self.dim), np.float32) if return_vectors else None
        ab = None
        if allow_bits is not None:  # host words, or a device tensor from filter_bits
            ab = allow_bits if hasattr(allow_bits, "data_ptr") else _c(allow_bits, np.uint32)
            need = (self.size + 31) // 32
            if ab.shape[0] < need:
                raise ValueError(f"allow bitmap has {ab.shape[0]} words, need {need}")
        L.check(L.fn["cm_dense_search"](self._h, L.ptr(qq), nq, int(k), L.ptr(ab), L.ptr(dist), L.ptr(rows),
                                        L.ptr(vecs)), "cm_dense_search")
        return (dist, rows, vecs) if return_vectors else (dist, rows)

    def export(self, row0: int = 0, n: Optional[int] = None, with_live: bool = False):
        """Host copy of rows [row0, row0+n) (and their live mask)."""
        n = self.size - row0 if n is None else int(n)
        out = np.empty((max(n, 0), self.dim), np.float32)
        live = np.zeros(max((n + 31) // 32, 1), np.uint32) if with_live else None
        L.check(L.fn["cm_dense_export"](self._h, int(row0), n, L.ptr(out), L.ptr(live)), "cm_dense_export")
        if not with_live:
            return out
        mask = np.unpackbits(live.view(np.uint8), bitorder="little")[:n].astype(bool)
        return out, mask

    # scan kernels (cm_dense_search_kind / cm_dense_set_path)
    PATH_AUTO, PATH_F32, PATH_COARSE, PATH_STREAM, PATH_Q8, PATH_Q8S = 0, 1, 3, 4, 5, 6

    def set_path(self, kind: int):
        """Force the scan kernel (0 auto, 1 fp32 K1, 3 K1c coarse + re-rank, 4 K1s <= 32-query f16
        streams, 5 K1q int8 resident passes, 6 K1q-s <= 32-query int8 streams -- the coarse kinds with
        the certified re-rank; 2 = the retired K1b, automatic)."""
        L.check(L.fn["cm_dense_set_path"](self._h, int(kind)), "cm_dense_set_path")

    def search_kind(self, nq: int, k: int) -> int:
        return int(L.fn["cm_dense_search_kind"](self._h, int(nq), int(k)))

    def last_fallbacks(self) -> int:
        """K1c/K1s queries re-run by the exact fp32 pass in the last host search()."""
        return int(L.fn["cm_dense_last_fallbacks"](self._h))

    def last_wide_reranks(self) -> int:
        """K1q/K1q-s queries whose band overflowed the re-rank's LDS and that the wide re-rank
        finished from the complete candidate buffers (no exact scan) in the last host search()."""
        return int(L.fn["cm_dense_last_wide_reranks"](self._h))

    def timing(self, enable: bool = True):
        """Record HIP events around every search's scan kernel (see timing_drain)."""
        L.check(L.fn["cm_dense_timing"](self._h, int(bool(enable))), "cm_dense_timing")

    def set_seed_event(self, event=None):
        """Record ``event`` (a torch.cuda.Event, kept alive here; None clears) on the search stream right
        after K1q's seed pass of every later batched search (cm_dense_set_seed_event)."""
        self._seed_event = event
        L.check(L.fn["cm_dense_set_seed_event"](self._h, event.cuda_event if event is not None else None),
                "cm_dense_set_seed_event")

    def timing_drain(self, cap: int = 4096) -> list:
        """Synchronise on the recorded events -> per-launch scan-kernel times (ms)."""
        buf = np.zeros(cap, np.float32)
        n = int(L.fn["cm_dense_timing_drain"](self._h, L.ptr(buf), int(cap)))
        if n < 0:
            raise RuntimeError(L.last_error())
        return buf[:min(n, cap)].tolist()

    def workspace_fallbacks(self, nq: int, k: int, workspace) -> int:
        """K1c/K1s queries re-run by the exact fp32 pass in the last search_dev() that used `workspace`."""
        return int(L.fn["cm_dense_workspace_fallbacks"](self._h, int(nq), int(k), L.ptr(workspace)))

    def workspace_wide_reranks(self, nq: int, k: int, workspace) -> int:
        """last_wide_reranks for the device search that last used ``workspace`` (synchronous read)."""
        return int(L.fn["cm_dense_workspace_wide_reranks"](self._h, int(nq), int(k), L.ptr(workspace)))

    def workspace_bytes(self, nq: int, k: int) -> int:
        n = int(L.fn["cm_dense_search_workspace"](self._h, int(nq), int(k)))
        if n < 0:
            raise ValueError("bad (nq, k) for dense search")
        return n

    def search_dev(self, q, k: int, allow=None, out=None, workspace=None, defer_exact: bool = False):
        """q: (nq, dim) float32 device tensor. Returns (dist f32 (nq,k), rows i64 (nq,k)) device tensors.
        defer_exact: leave the certificate's exact pass (queries whose certified band overflowed) to a
        later ``exact_fallback_dev`` call with the same arguments on the same stream -- enqueued after
        other streams' work has joined, so its large-LDS grid does not wait behind their kernels."""
        nq = q.shape[0]
        dev = q.device
        wsb = self.workspace_bytes(nq, k)
        if workspace is None:
            if self._ws is None or self._ws.numel() < wsb:
                self._ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
            workspace = self._ws
        if out is None:
            out = (torch.empty((nq, k), dtype=torch.float32, device=dev),
                   torch.empty((nq, k), dtype=torch.int64, device=dev))
        name = "cm_dense_search_dev_deferred" if defer_exact else "cm_dense_search_dev"
        L.check(L.fn[name](self._h, L.ptr(q), nq, int(k), L.ptr(allow), L.ptr(out[0]), L.ptr(out[1]),
                           L.ptr(workspace), int(workspace.numel()), _stream(self.device)), name)
        return out

    def exact_fallback_dev(self, q, k: int, out, workspace=None, allow=None):
        """Second part of ``search_dev(..., defer_exact=True)``: the exact fp32 pass for the queries
        whose certificate failed, merged into ``out`` (device-gated: nothing runs when none failed)."""
        if workspace is None:
            workspace = self._ws
        L.check(L.fn["cm_dense_exact_fallback_dev"](self._h, L.ptr(q), q.shape[0], int(k), L.ptr(allow),
                                                    L.ptr(out[0]), L.ptr(out[1]), L.ptr(workspace),
                                                    int(workspace.numel()), _stream(self.device)),
                "cm_dense_exact_fallback_dev")
        return out

    def gather_dev(self, rows, out=None):
        n = rows.numel()
        if out is None:
            out = torch.empty((n, self.dim), dtype=torch.float32, device=rows.device)
        L.check(L.fn["cm_dense_gather_dev"](self._h, L.ptr(rows), n, L.ptr(out), _stream(self.device)),
                "cm_dense_gather_dev")
        return out


class BM25Index:
    """HBM-resident postings + BM25 Okapi with rank_bm25 0.2.x semantics."""

    def __init__(self, device: Optional[int] = None):
        self.device = default_device() if device is None else int(device)
        h = C.c_void_p()
        L.check(L.fn["cm_bm25_create"](self.device, C.byref(h)), "cm_bm25_create")
        self._h = h
        self.vocab = 0
        self._ws = None

    def close(self):
        if getattr(self, "_h", None):
            L.fn["cm_bm25_destroy"](self._h)
            self._h = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    def build(self, term_ids: np.ndarray, doc_off: np.ndarray, vocab: int, live: Optional[np.ndarray] = None):
        t = _c(term_ids, np.int32)
        o = _c(doc_off, np.int64)
        lv = None if live is None else _c(live, np.uint8)
        L.check(L.fn["cm_bm25_build"](self._h, L.ptr(t), L.ptr(o), int(o.shape[0] - 1), int(vocab), L.ptr(lv)),
                "cm_bm25_build")
        self.vocab = int(vocab)

    def build_dev(self, term_ids, doc_off, vocab: int):
        assert term_ids.dtype == torch.int32 and doc_off.dtype == torch.int64
        L.check(L.fn["cm_bm25_build_dev"](self._h, L.ptr(term_ids), L.ptr(doc_off), int(doc_off.numel() - 1),
                                          int(term_ids.numel()), int(vocab), _stream(self.device)),
                "cm_bm25_build_dev")
        self.vocab = int(vocab)

    @property
    def num_docs(self) -> int:
        return int(L.fn["cm_bm25_num_docs"](self._h))

    @property
    def num_postings(self) -> int:
        return int(L.fn["cm_bm25_num_postings"](self._h))

    def stats(self):
        n, s = C.c_int64(), C.c_int64()
        a, e = C.c_double(), C.c_double()
        L.check(L.fn["cm_bm25_stats"](self._h, C.byref(n), C.byref(s), C.byref(a), C.byref(e)), "cm_bm25_stats")
        return dict(n_live=n.value, sum_len=s.value, avgdl=a.value, eps=e.value)

    def export(self):
        """Host copy of the CSR index: dict(term_off, post_doc, post_tf, post_pos, dl)."""
        v, p, n = self.vocab, self.num_postings, self.num_docs
        out = dict(term_off=np.empty(v + 1, np.int64), post_doc=np.empty(max(p, 1), np.int32),
                   post_tf=np.empty(max(p, 1), np.uint16), post_pos=np.empty(max(p, 1), np.uint32),
                   dl=np.empty(max(n, 1), np.int32))
        L.check(L.fn["cm_bm25_export"](self._h, *[L.ptr(out[k]) for k in ("term_off", "post_doc", "post_tf",
                                                                          "post_pos", "dl")]), "cm_bm25_export")
        for k in ("post_doc", "post_tf", "post_pos"):
            out[k] = out[k][:p]
        out["dl"] = out["dl"][:n]
        return out

    def set_head_policy(self, min_df_frac: float = 1.0 / 128, max_bytes: int = 8 << 30):
        """Dense tf tiles for high-df terms (same results; max_bytes=0 disables)."""
        L.check(L.fn["cm_bm25_set_head_policy"](self._h, float(min_df_frac), int(max_bytes)), "cm_bm25_set_head_policy")

    # search strategy (cm_bm25_set_path): identical results either way
    PATH_AUTO, PATH_FULL, PATH_PRUNED = 0, 1, 2

    def set_path(self, kind: int):
        """0 auto (pruned), 1 full K2 scan of every (query, range), 2 tail pass + bounded re-score."""
        L.check(L.fn["cm_bm25_set_path"](self._h, int(kind)), "cm_bm25_set_path")

    def last_rescored(self) -> int:
        """(query, range) pairs K2 re-scored by the last host search() (-1 on the full path)."""
        return int(L.fn["cm_bm25_last_rescored"](self._h))

    def workspace_rescored(self, nq: int, total_terms: int, k: int, workspace) -> int:
        """Same for the last search_dev() that used `workspace`."""
        return int(L.fn["cm_bm25_workspace_rescored"](self._h, int(nq), int(total_terms), int(k),
                                                      L.ptr(workspace)))

    def timing(self, enable: bool = True):
        """Record HIP events around every search's scoring launches (see timing_drain)."""
        L.check(L.fn["cm_bm25_timing"](self._h, int(bool(enable))), "cm_bm25_timing")

    def timing_drain(self, cap: int = 4096) -> list:
        buf = np.zeros(cap, np.float32)
        n = int(L.fn["cm_bm25_timing_drain"](self._h, L.ptr(buf), int(cap)))
        if n < 0:
            raise RuntimeError(L.last_error())
        return buf[:min(n, cap)].tolist()

    def timing_drain_block(self, cap: int = 4096) -> list:
        """Per-launch times (ms) of K2b (bm25_block_kernel) since timing(True)."""
        buf = np.zeros(cap, np.float32)
        n = int(L.fn["cm_bm25_timing_drain_block"](self._h, L.ptr(buf), int(cap)))
        if n < 0:
            raise RuntimeError(L.last_error())
        return buf[:min(n, cap)].tolist()

    def workspace_items(self, nq: int, total_terms: int, k: int, workspace, cap: int = 1 << 22) -> np.ndarray:
        """K2b's planned items (q << 40 | range << 16 | 64-doc block mask) of the last pruned search
        that used ``workspace`` (synchronous read)."""
        buf = np.zeros(cap, np.uint64)
        n = int(L.fn["cm_bm25_workspace_items"](self._h, int(nq), int(total_terms), int(k), L.ptr(workspace),
                                                 L.ptr(buf), int(cap)))
        if n < 0:
            raise RuntimeError(L.last_error() or "no planned items (full path?)")
        return buf[:min(n, cap)]

    def workspace_subblocks(self, nq: int, total_terms: int, k: int, workspace, cap: int = 1 << 22) -> np.ndarray:
        """The planned items' 16-doc sub-block masks (bit 4 b + x), item for item with workspace_items."""
        buf = np.zeros(cap, np.uint64)
        n = int(L.fn["cm_bm25_workspace_subblocks"](self._h, int(nq), int(total_terms), int(k), L.ptr(workspace),
                                                     L.ptr(buf), int(cap)))
        if n < 0:
            raise RuntimeError(L.last_error() or "no planned items (full path?)")
        return buf[:min(n, cap)]

    @property
    def num_head_terms(self) -> int:
        return int(L.fn["cm_bm25_num_head_terms"](self._h))

    def term_stats(self):
        """Local (df[V] int32, first_key[V] uint64 = row << 32 | first position, ~0 if absent)."""
        df = np.zeros(max(self.vocab, 1), np.int32)
        fk = np.zeros(max(self.vocab, 1), np.uint64)
        L.check(L.fn["cm_bm25_term_stats"](self._h, L.ptr(df), L.ptr(fk)), "cm_bm25_term_stats")
        return df[: self.vocab], fk[: self.vocab]

    def set_stats(self, idf: np.ndarray, n_live: int, sum_len: int, eps: float):
        """Install corpus-wide statistics (sharded index: every rank scores with the global idf/avgdl)."""
        v = _c(idf, np.float64)
        L.check(L.fn["cm_bm25_set_stats"](self._h, L.ptr(v), int(v.shape[0]), int(n_live), int(sum_len), float(eps)),
                "cm_bm25_set_stats")

    def search(self, queries: Sequence[Sequence[int]], k: int, allow_bits: Optional[np.ndarray] = None):
        """queries: per query a list of term ids (-1 unknown). -> scores f64 (nq,k), rows i64, n i32."""
        nq = len(queries)
        off = np.zeros(nq + 1, np.int32)
        for i, q in enumerate(queries):
            off[i + 1] = off[i] + len(q)
        flat = np.concatenate([np.asarray(q, np.int32) for q in queries]) if off[-1] else np.zeros(1, np.int32)
        flat = _c(flat, np.int32)
        scores = np.empty((nq, k), np.float64)
        rows = np.empty((nq, k), np.int64)
        nvalid = np.empty(nq, np.int32)
        ab = None  # host words, or a device tensor from filter_bits
        if allow_bits is not None:
            ab = allow_bits if hasattr(allow_bits, "data_ptr") else _c(allow_bits, np.uint32)
            if ab.shape[0] < (self.num_docs + 31) // 32:
                raise ValueError(f"allow bitmap has {ab.shape[0]} words, need {(self.num_docs + 31) // 32}")
        L.check(L.fn["cm_bm25_search"](self._h, L.ptr(flat), L.ptr(off), nq, int(k), L.ptr(ab), L.ptr(scores),
                                       L.ptr(rows), L.ptr(nvalid)), "cm_bm25_search")
        return scores, rows, nvalid

    def workspace_bytes(self, nq: int, total_terms: int, k: int) -> int:
        n = int(L.fn["cm_bm25_search_workspace"](self._h, int(nq), int(total_terms), int(k)))
        if n < 0:
            raise ValueError("bad BM25 workspace request")
        return n

    def search_dev(self, q_terms, q_off, k: int, out=None, workspace=None, gate=None):
        """Unfiltered device search: q_terms int32 (T,), q_off int32 (nq+1,) device tensors.  ``gate``
        (a recorded torch.cuda.Event): the scoring kernels wait for it, the query preparation does not
        (cm_bm25_search_dev_gated)."""
        nq = q_off.numel() - 1
        total = q_terms.numel()
        wsb = self.workspace_bytes(nq, total, k)
        if workspace is None:
            if self._ws is None or self._ws.numel() < wsb:
                self._ws = torch.empty(wsb, dtype=torch.uint8, device=q_terms.device)
            workspace = self._ws
        if out is None:
            out = (torch.empty((nq, k), dtype=torch.float64, device=q_terms.device),
                   torch.empty((nq, k), dtype=torch.int64, device=q_terms.device))
        L.check(L.fn["cm_bm25_search_dev_gated"](self._h, L.ptr(q_terms), L.ptr(q_off), nq, total, int(k),
                                                 L.ptr(out[0]), L.ptr(out[1]), L.ptr(workspace), int(workspace.numel()),
                                                 _stream(self.device), gate.cuda_event if gate is not None else None),
                "cm_bm25_search_dev_gated")
        return out


    # ---- filtered device search (quirk Q2 on the device; SURVEY §8e for shards) -----------------
    FILT_EPS_MISSING, FILT_ZERO_DIV, FILT_TABLE = 1, 2, 4

    def prepare_filtered(self, max_docs: int = 0):
        """Upload the log table the device idf needs (once per index, before any graph capture;
        max_docs = the global corpus size when this index is a shard)."""
        L.check(L.fn["cm_bm25_prepare_filtered"](self._h, int(max_docs)), "cm_bm25_prepare_filtered")

    def filter_stats_dev(self, allow, q_terms, stats=None, df=None):
        """Candidate statistics of a device allow bitmap: stats int64 (2,) = {Nc, sum of lengths},
        df int64 (T,) per query term (device tensors, torch's stream, async)."""
        dev = q_terms.device
        if stats is None:
            stats = torch.empty(2, dtype=torch.int64, device=dev)
        if df is None:
            df = torch.empty(max(q_terms.numel(), 1), dtype=torch.int64, device=dev)
        L.check(L.fn["cm_bm25_filter_stats_dev"](self._h, L.ptr(allow), L.ptr(q_terms), int(q_terms.numel()),
                                                 L.ptr(stats), L.ptr(df), _stream(self.device)),
                "cm_bm25_filter_stats_dev")
        return stats, df

    def filter_term_stats_dev(self, allow):
        """Per-term candidate df (int64 (V,)) and first-occurrence keys (int64 view of the uint64
        row << 32 | position keys, -1 = none) of a device allow bitmap."""
        dev = torch.device("cuda", self.device)
        df = torch.empty(max(self.vocab, 1), dtype=torch.int64, device=dev)
        fk = torch.empty(max(self.vocab, 1), dtype=torch.int64, device=dev)
        L.check(L.fn["cm_bm25_filter_term_stats_dev"](self._h, L.ptr(allow), L.ptr(df), L.ptr(fk),
                                                      _stream(self.device)), "cm_bm25_filter_term_stats_dev")
        return df[: self.vocab], fk[: self.vocab]

    def filter_eps(self, allow) -> float:
        """rank_bm25's epsilon floor over the candidates of one filter (host or device words)."""
        ab = allow if hasattr(allow, "data_ptr") else _c(allow, np.uint32)
        e = C.c_double(0.0)
        L.check(L.fn["cm_bm25_filter_eps"](self._h, L.ptr(ab), C.byref(e)), "cm_bm25_filter_eps")
        return e.value

    def search_stats_dev(self, q_terms, q_off, k: int, allow, stats, df, eps=None, out=None, status=None,
                         workspace=None):
        """Device search of the allowed documents with the given candidate statistics (device
        tensors; eps: device float64 (1,) or None).  Returns (scores, rows, status int32 (1,))."""
        nq = q_off.numel() - 1
        total = q_terms.numel()
        dev = q_terms.device
        wsb = self.workspace_bytes(nq, total, k)
        if workspace is None:
            if self._ws is None or self._ws.numel() < wsb:
                self._ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
            workspace = self._ws
        if out is None:
            out = (torch.empty((nq, k), dtype=torch.float64, device=dev),
                   torch.empty((nq, k), dtype=torch.int64, device=dev))
        if status is None:
            status = torch.empty(1, dtype=torch.int32, device=dev)
        L.check(L.fn["cm_bm25_search_stats_dev"](self._h, L.ptr(q_terms), L.ptr(q_off), nq, total, int(k),
                                                 L.ptr(allow), L.ptr(stats), L.ptr(df), L.ptr(eps), L.ptr(out[0]),
                                                 L.ptr(out[1]), L.ptr(status), L.ptr(workspace),
                                                 int(workspace.numel()), _stream(self.device)),
                "cm_bm25_search_stats_dev")
        return out[0], out[1], status

    def search_filtered_dev(self, q_terms, q_off, k: int, allow, eps=None, out=None, status=None, workspace=None):
        """One-index filtered device search (statistics over the allowed candidates on the device,
        graph-capturable).  Returns (scores, rows, status); see FILT_* for the status bits."""
        nq = q_off.numel() - 1
        total = q_terms.numel()
        dev = q_terms.device
        wsb = self.workspace_bytes(nq, total, k)
        if workspace is None:
            if self._ws is None or self._ws.numel() < wsb:
                self._ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
            workspace = self._ws
        if out is None:
            out = (torch.empty((nq, k), dtype=torch.float64, device=dev),
                   torch.empty((nq, k), dtype=torch.int64, device=dev))
        if status is None:
            status = torch.empty(1, dtype=torch.int32, device=dev)
        L.check(L.fn["cm_bm25_search_filtered_dev"](self._h, L.ptr(q_terms), L.ptr(q_off), nq, total, int(k),
                                                    L.ptr(allow), L.ptr(eps), L.ptr(out[0]), L.ptr(out[1]),
                                                    L.ptr(status), L.ptr(workspace), int(workspace.numel()),
                                                    _stream(self.device)), "cm_bm25_search_filtered_dev")
        return out[0], out[1], status

    def search_filtered(self, q_terms, q_off, k: int, allow):
        """search_filtered_dev with the eps recovery step: when an idf is negative the filter's
        epsilon is computed (cm_bm25_filter_eps) and the batch searched again.  Synchronises."""
        s, r, st = self.search_filtered_dev(q_terms, q_off, k, allow)
        code = int(st.item())
        if code & self.FILT_EPS_MISSING:
            eps = torch.tensor([self.filter_eps(allow)], dtype=torch.float64, device=q_terms.device)
            s, r, st = self.search_filtered_dev(q_terms, q_off, k, allow, eps=eps)
            code = int(st.item())
        if code & self.FILT_ZERO_DIV:
            raise ZeroDivisionError("float division by zero (candidate documents have no tokens)")
        if code:
            raise RuntimeError(f"filtered BM25 search status {code}")
        return s, r


# ---------------------------------------------------------------------------
# Fusion and pooling ops
# ---------------------------------------------------------------------------
def mmr_order_batch(q: np.ndarray, cands: np.ndarray, k: int, lambd: float = 0.5,
                    n_valid: Optional[np.ndarray] = None) -> np.ndarray:
    """_mmr_order for nq queries on device. q (nq,d), cands (nq,P,d) -> (nq,k) int32 (-1 pad)."""
    qq = _c(np.atleast_2d(q), np.float32)
    cc = _c(cands, np.float32)
    nq, pool, dim = cc.shape
    out = np.empty((nq, k), np.int32)
    nv = None if n_valid is None else _c(n_valid, np.int32)
    L.check(L.fn["cm_mmr"](L.ptr(qq), L.ptr(cc), L.ptr(nv), nq, pool, dim, int(k), float(lambd), L.ptr(out)),
            "cm_mmr")
    return out


def mmr_dev(q, cands, k: int, lambd: float = 0.5, n_valid=None, out=None):
    nq, pool, dim = cands.shape
    if out is None:
        out = torch.empty((nq, k), dtype=torch.int32, device=q.device)
    L.check(L.fn["cm_mmr_dev"](L.ptr(q), L.ptr(cands), L.ptr(n_valid), nq, pool, dim, int(k), float(lambd),
                               L.ptr(out), _stream(q.device.index)), "cm_mmr_dev")
    return out


def rrf_fuse_keys(lists: Sequence[Sequence[int]], weights: Optional[Sequence[float]], rrf_k: int):
    """rrf_fuse over int keys on device -> (keys in first-appearance order, scores)."""
    nl = len(lists)
    off = np.zeros(nl + 1, np.int32)
    for i, l in enumerate(lists):
        off[i + 1] = off[i] + len(l)
    total = int(off[-1])
    keys = np.asarray([x for l in lists for x in l] or [0], np.int64)
    w = None if weights is None else _c([float(x) for x in weights], np.float64)
    out_k = np.empty(max(total, 1), np.int64)
    out_s = np.empty(max(total, 1), np.float64)
    n = C.c_int32(0)
    L.check(L.fn["cm_rrf_fuse"](L.ptr(keys), L.ptr(off), nl, L.ptr(w), int(rrf_k), L.ptr(out_k), L.ptr(out_s),
                                C.byref(n)), "cm_rrf_fuse")
    return out_k[:n.value], out_s[:n.value]


def rrf_merge(vkeys, vdist, vn, bkeys, bscore, bn, *, w_vec: float, w_bm25: float, rrf_k: int, top_k: int):
    """Batched HybridRetriever merge on device (host arrays in/out)."""
    vkeys = _c(vkeys, np.int64)
    nq = vkeys.shape[0]
    kv = vkeys.shape[1]
    bkeys = _c(bkeys, np.int64).reshape(nq, -1)
    kb = bkeys.shape[1]
    vdist = _c(vdist, np.float32).reshape(nq, kv)
    bscore = _c(bscore, np.float64).reshape(nq, kb)
    vn = _c(vn, np.int32)
    bn = _c(bn, np.int32)
    ok = np.empty((nq, top_k), np.int64)
    of = np.empty((nq, top_k), np.float64)
    ov = np.empty((nq, top_k), np.float32)
    ob = np.empty((nq, top_k), np.float64)
    ofl = np.empty((nq, top_k), np.int32)
    on = np.empty(nq, np.int32)
    L.check(L.fn["cm_rrf_merge"](L.ptr(vkeys), L.ptr(vdist), L.ptr(vn), kv, L.ptr(bkeys), L.ptr(bscore), L.ptr(bn), kb,
                                 nq, float(w_vec), float(w_bm25), int(rrf_k), int(top_k), L.ptr(ok), L.ptr(of),
                                 L.ptr(ov), L.ptr(ob), L.ptr(ofl), L.ptr(on)), "cm_rrf_merge")
    return ok, of, ov, ob, ofl, on


def rrf_pool_prep_dev(pool_keys, pool_dist, order, bkeys, out=None):
    """vkeys/vdist (MMR-ordered pool entries), vn, bn for rrf_merge_dev in one device pass
    (cm_rrf_pool_prep_dev).  pool_keys int64 (nq, pool), pool_dist float32 (nq, pool), order int32
    (nq, kv), bkeys int64 (nq, kb); all contiguous on one device."""
    nq, pool = pool_keys.shape
    kv, kb = order.shape[1], bkeys.shape[1]
    dev = pool_keys.device
    for t, dt in ((pool_keys, torch.int64), (pool_dist, torch.float32), (order, torch.int32), (bkeys, torch.int64)):
        if t.dtype != dt or not t.is_contiguous() or t.device != dev or t.shape[0] != nq:
            raise ValueError("rrf_pool_prep_dev: bad input tensor")
    if out is None:
        out = (torch.empty((nq, kv), dtype=torch.int64, device=dev), torch.empty((nq, kv), dtype=torch.float32, device=dev),
               torch.empty((nq,), dtype=torch.int32, device=dev), torch.empty((nq,), dtype=torch.int32, device=dev))
    L.check(L.fn["cm_rrf_pool_prep_dev"](L.ptr(pool_keys), L.ptr(pool_dist), pool, L.ptr(order), kv, L.ptr(bkeys), kb,
                                         nq, *[L.ptr(t) for t in out], _stream(dev.index)), "cm_rrf_pool_prep_dev")
    return out


def rrf_merge_dev(vkeys, vdist, vn, bkeys, bscore, bn, *, w_vec, w_bm25, rrf_k, top_k, out=None):
    nq, kv = vkeys.shape
    kb = bkeys.shape[1]
    dev = vkeys.device
    if out is None:
        out = (torch.empty((nq, top_k), dtype=torch.int64, device=dev),
               torch.empty((nq, top_k), dtype=torch.float64, device=dev),
               torch.empty((nq, top_k), dtype=torch.float32, device=dev),
               torch.empty((nq, top_k), dtype=torch.float64, device=dev),
               torch.empty((nq, top_k), dtype=torch.int32, device=dev),
               torch.empty((nq,), dtype=torch.int32, device=dev))
    L.check(L.fn["cm_rrf_merge_dev"](L.ptr(vkeys), L.ptr(vdist), L.ptr(vn), kv, L.ptr(bkeys), L.ptr(bscore),
                                     L.ptr(bn), kb, nq, float(w_vec), float(w_bm25), int(rrf_k), int(top_k),
                                     *[L.ptr(t) for t in out], _stream(dev.index)), "cm_rrf_merge_dev")
    return out


def meanpool_l2norm(hidden, mask, normalize: bool = True, out=None):
    """hidden (B,S,D) f32/bf16/f16 device, mask (B,S) int32/int64 -> (B,D) f32 (K6)."""
    B, S, D = hidden.shape
    hd = {torch.float32: L.CM_DTYPE_F32, torch.bfloat16: L.CM_DTYPE_BF16, torch.float16: L.CM_DTYPE_F16}[hidden.dtype]
    md = {torch.int32: L.CM_DTYPE_I32, torch.int64: L.CM_DTYPE_I64}[mask.dtype]
    hidden = hidden.contiguous()
    mask = mask.contiguous()
    if out is None:
        out = torch.empty((B, D), dtype=torch.float32, device=hidden.device)
    L.check(L.fn["cm_meanpool_l2norm"](L.ptr(hidden), hd, L.ptr(mask), md, B, S, D, int(bool(normalize)),
                                       L.ptr(out), _stream(hidden.device.index)), "cm_meanpool_l2norm")
    return out



def add_layernorm(x, r, weight, bias, eps: float, out=None):
    """LayerNorm(x + r) over the last dim in one pass (cm_add_layernorm; the XLM-R block epilogue).

    x: (..., D) f32/bf16 device; r: same shape as x, or (R, D) broadcast over rows (row i uses
    r[i % R]), or None; weight/bias: (D,) of x's dtype.  The sum is rounded to x's dtype before the
    statistics, as ``F.layer_norm(x + r, ...)`` does."""
    D = x.shape[-1]
    dt = {torch.float32: L.CM_DTYPE_F32, torch.bfloat16: L.CM_DTYPE_BF16}[x.dtype]
    x = x.contiguous()
    rows = x.numel() // D
    if r is not None:
        r = r.contiguous()
        if r.dtype != x.dtype or r.shape[-1] != D or rows % (r.numel() // D):
            raise ValueError("residual must match x's dtype and feature dim and tile its rows")
    for t in (weight, bias):
        if t.dtype != x.dtype or t.numel() != D or not t.is_contiguous():
            raise ValueError("weight/bias must be contiguous (D,) of x's dtype")
    if out is None:
        out = torch.empty_like(x)
    L.check(L.fn["cm_add_layernorm"](L.ptr(x), L.ptr(r) if r is not None else None,
                                     (r.numel() // D) if r is not None else 0, L.ptr(weight), L.ptr(bias), rows, D,
                                     float(eps), dt, L.ptr(out), _stream(x.device.index)), "cm_add_layernorm")
    return out


def short_attention(qkv, heads: int, scale: float, out=None):
    """Unmasked self-attention straight from a fused QKV projection (cm_short_attention).

    qkv: (B, S, 3*heads*64) f32/bf16 device, S <= 64 -> (B, S, heads*64): per head
    softmax(q k^T * scale) v, fp32 softmax."""
    B, S, F3 = qkv.shape
    if F3 != 3 * heads * 64 or not 0 < S <= 64:
        raise ValueError("qkv must be (B, S<=64, 3*heads*64)")
    dt = {torch.float32: L.CM_DTYPE_F32, torch.bfloat16: L.CM_DTYPE_BF16}[qkv.dtype]
    qkv = qkv.contiguous()
    if out is None:
        out = torch.empty((B, S, heads * 64), dtype=qkv.dtype, device=qkv.device)
    L.check(L.fn["cm_short_attention"](L.ptr(qkv), B, S, heads, 64, float(scale), dt, L.ptr(out),
                                       _stream(qkv.device.index)), "cm_short_attention")
    return out


# ---------------------------------------------------------------------------
# K10: fp32-accurate linear layers on the f16 matrix cores (split precision)
def _pow2_at_most(x: float) -> float:
    """Largest power of two <= x (x > 0)."""
    import math
    m, e = math.frexp(x)          # x = m * 2**e, 0.5 <= m < 1
    return math.ldexp(1.0, e - 1)


class F16x3Weight:
    """An nn.Linear weight (N, K) fp32 prepared for ``linear_f16x3``: the split blocks (f16 hi
    and lo halves) of W * scale in the fragment-major order the kernel streams
    (cm_f16x3_split_weights), scale a power of two putting max|W| in [2^14, 2^15).  Keeps the fp32
    bias (or None)."""

    def __init__(self, weight, bias=None):
        if weight.dtype != torch.float32 or weight.dim() != 2 or not weight.is_cuda:
            raise ValueError("weight must be a 2-D fp32 device tensor")
        N, K = weight.shape
        if N % 64 or K % 32:
            raise ValueError("need N % 64 == 0 and K % 32 == 0")
        w = weight.detach().contiguous()
        amax = float(w.abs().max())
        self.scale = (2.0 ** 14) / _pow2_at_most(amax) if amax > 0 else 1.0
        self.N, self.K = N, K
        self.planes = torch.empty((N, K, 2), dtype=torch.float16, device=w.device)   # split blocks
        self.bias = bias.detach().float().contiguous() if bias is not None else None
        if self.bias is not None and self.bias.numel() != N:
            raise ValueError("bias must have N elements")
        L.check(L.fn["cm_f16x3_split_weights"](L.ptr(w), N, K, float(self.scale), L.ptr(self.planes),
                                               _stream(w.device.index)), "cm_f16x3_split_weights")


class Planes:
    """An M x K fp32 matrix as K10 split planes: one f16 buffer of cm_f16x3_plane_rows(M) x K x 2
    halves (2 KiB split blocks [hi 1 KiB][lo 1 KiB], fragment-major; include/classmate_hip.h),
    holding the values times ``scale``."""

    __slots__ = ("data", "M", "K", "scale")

    def __init__(self, M: int, K: int, scale: float, device):
        rows = int(L.fn["cm_f16x3_plane_rows"](int(M)))
        self.data = torch.empty((max(rows, 1), K, 2), dtype=torch.float16, device=device)
        self.M, self.K, self.scale = M, K, float(scale)

    def halves(self):
        """(hi, lo) f16 views of rows 0 .. M-1 in row-major (M, K) order (for tests)."""
        kb = self.K // 32
        blk = self.data.view(-1, kb, 2, 4, 16, 8)          # [row block][kb][plane][g][c][e]
        v = blk.permute(2, 0, 4, 1, 3, 5).reshape(2, -1, self.K)   # [plane][row][k]
        return v[0, :self.M], v[1, :self.M]


def split_rows(x, scale: float = 1.0) -> Planes:
    """fp32 (..., K) device rows -> Planes of x * scale (cm_f16x3_split_rows)."""
    if x.dtype != torch.float32 or x.shape[-1] % 32:
        raise ValueError("x must be fp32 with a last dim that is a multiple of 32")
    x = x.contiguous()
    K = x.shape[-1]
    p = Planes(x.numel() // K, K, scale, x.device)
    L.check(L.fn["cm_f16x3_split_rows"](L.ptr(x), p.M, K, p.scale, L.ptr(p.data), _stream(x.device.index)),
            "cm_f16x3_split_rows")
    return p


def linear_f16x3(x, w: "F16x3Weight", a_scale: float = 1.0, gelu: bool = False, out=None, planes_out: float = 0.0,
                 qkv: bool = False):
    """y = x W^T + b (then exact-erf GELU if ``gelu``) at fp32 accuracy on the f16 MFMAs (K10).

    x: ``Planes`` (its own scale), or (..., K) fp32 device rows (split here with ``a_scale``, a
    power of two with |x| * a_scale <= 2^15).  Returns (M, N) fp32 -- or, with
    ``planes_out`` = s > 0 (requires gelu), the Planes of GELU(y) * s for the next projection; or,
    with ``qkv`` and ``planes_out`` = s (no gelu), the fused QKV projection as planes of y * s for
    ``planes_attention`` (Q, K thirds standard, V third transposed; CM_EPI_PLANES_QKV)."""
    if not isinstance(x, Planes):
        if x.dtype != torch.float32 or x.shape[-1] != w.K:
            raise ValueError(f"x must be (..., {w.K}) fp32")
        lead = x.shape[:-1]
        x = split_rows(x, a_scale)
    else:
        lead = (x.M,)
    if x.K != w.K:
        raise ValueError(f"planes have K={x.K}, the weight K={w.K}")
    dev = x.data.device
    common = (L.ptr(x.data), x.M, w.K, L.ptr(w.planes), L.ptr(w.bias) if w.bias is not None else None,
              float(1.0 / (x.scale * w.scale)), w.N)
    if planes_out:
        if gelu == qkv:
            raise ValueError("planes_out is the fused FFN-up epilogue (gelu=True) or the QKV planes (qkv=True)")
        p = Planes(x.M, w.N, planes_out, dev)
        L.check(L.fn["cm_linear_f16x3"](*common, L.CM_EPI_PLANES_QKV if qkv else L.CM_EPI_PLANES_GELU, None, p.scale,
                                        L.ptr(p.data), _stream(dev.index)), "cm_linear_f16x3")
        return p
    if qkv:
        raise ValueError("qkv=True writes planes: give planes_out")
    if out is None:
        out = torch.empty((*lead, w.N), dtype=torch.float32, device=dev)
    L.check(L.fn["cm_linear_f16x3"](*common, L.CM_EPI_BIAS_GELU if gelu else L.CM_EPI_BIAS, L.ptr(out), 0.0, None,
                                    _stream(dev.index)), "cm_linear_f16x3")
    return out


def add_layernorm_split(x, r, weight, bias, eps: float, a_scale: float, out=None):
    """add_layernorm (fp32) that also returns its output * a_scale as K10 Planes
    (cm_add_layernorm_split).  Returns (out, planes)."""
    D = x.shape[-1]
    if x.dtype != torch.float32:
        raise ValueError("add_layernorm_split is fp32")
    x = x.contiguous()
    rows = x.numel() // D
    if r is not None:
        r = r.contiguous()
        if r.dtype != x.dtype or r.shape[-1] != D or rows % (r.numel() // D):
            raise ValueError("residual must match x's dtype and feature dim and tile its rows")
    if out is None:
        out = torch.empty_like(x)
    p = Planes(rows, D, a_scale, x.device)
    L.check(L.fn["cm_add_layernorm_split"](L.ptr(x), L.ptr(r) if r is not None else None,
                                           (r.numel() // D) if r is not None else 0, L.ptr(weight), L.ptr(bias), rows,
                                           D, float(eps), L.ptr(out), p.scale, L.ptr(p.data),
                                           _stream(x.device.index)), "cm_add_layernorm_split")
    return out, p


def short_attention_split(qkv, heads: int, scale: float, a_scale: float, key_mask=None) -> Planes:
    """cm_short_attention (fp32) writing the context * a_scale as K10 Planes (B*S x heads*64).
    key_mask (B, S) int32 on the device, nonzero = attend (padded batches, S <= 32): padded keys
    leave the softmax (cm_short_attention_split_masked)."""
    B, S, F3 = qkv.shape
    if F3 != 3 * heads * 64 or not 0 < S <= 64 or qkv.dtype != torch.float32:
        raise ValueError("qkv must be fp32 (B, S<=64, 3*heads*64)")
    qkv = qkv.contiguous()
    p = Planes(B * S, heads * 64, a_scale, qkv.device)
    if key_mask is None:
        L.check(L.fn["cm_short_attention_split"](L.ptr(qkv), B, S, heads, 64, float(scale), p.scale, L.ptr(p.data),
                                                 _stream(qkv.device.index)), "cm_short_attention_split")
        return p
    if tuple(key_mask.shape) != (B, S) or key_mask.dtype != torch.int32 or key_mask.device != qkv.device or S > 32:
        raise ValueError("key_mask must be int32 (B, S) on the qkv device, S <= 32")
    key_mask = key_mask.contiguous()
    L.check(L.fn["cm_short_attention_split_masked"](L.ptr(qkv), B, S, heads, 64, float(scale), p.scale,
                                                    L.ptr(key_mask), L.ptr(p.data), _stream(qkv.device.index)),
            "cm_short_attention_split_masked")
    return p

def long_attention_split(qkv, heads: int, scale: float, a_scale: float, key_mask=None) -> Planes:
    """Attention of any sequence length at fp32 accuracy (K9L, cm_long_attention_split) writing the
    context * a_scale as K10 Planes (B*S x heads*64).  qkv: fp32 (B, S, 3*heads*64); key_mask:
    optional int32 (B, S) on the device, nonzero = attend (padded keys leave the softmax)."""
    B, S, F3 = qkv.shape
    if F3 != 3 * heads * 64 or not 0 < S <= 4096 or qkv.dtype != torch.float32:
        raise ValueError("qkv must be fp32 (B, 0 < S <= 4096, 3*heads*64)")
    qkv = qkv.contiguous()
    if key_mask is not None:
        if tuple(key_mask.shape) != (B, S) or key_mask.dtype != torch.int32 or key_mask.device != qkv.device:
            raise ValueError("key_mask must be int32 (B, S) on the qkv device")
        key_mask = key_mask.contiguous()
    p = Planes(B * S, heads * 64, a_scale, qkv.device)
    L.check(L.fn["cm_long_attention_split"](L.ptr(qkv), B, S, heads, 64, float(scale), p.scale,
                                            L.ptr(key_mask) if key_mask is not None else None, L.ptr(p.data),
                                            _stream(qkv.device.index)), "cm_long_attention_split")
    return p


def planes_attention(qkv: "Planes", B: int, S: int, heads: int, scale: float, a_scale: float,
                     key_mask=None) -> Planes:
    """K9P (cm_planes_attention): K9L's attention from the QKV projection's planes
    (``linear_f16x3(..., qkv=True, planes_out=s)``), writing the context * a_scale as K10 Planes
    (B*S x heads*64).  S % 64 == 0, S <= 512; key_mask: optional int32 (B, S), nonzero = attend."""
    if not isinstance(qkv, Planes) or qkv.K != 3 * heads * 64 or qkv.M != B * S:
        raise ValueError("qkv must be the (B*S) x 3*heads*64 QKV planes")
    if S <= 0 or S % 64 or S > 512:
        raise ValueError("planes attention: need S % 64 == 0 and 0 < S <= 512")
    dev = qkv.data.device
    if key_mask is not None:
        if tuple(key_mask.shape) != (B, S) or key_mask.dtype != torch.int32 or key_mask.device != dev:
            raise ValueError("key_mask must be int32 (B, S) on the qkv device")
        key_mask = key_mask.contiguous()
    p = Planes(B * S, heads * 64, a_scale, dev)
    L.check(L.fn["cm_planes_attention"](L.ptr(qkv.data), B, S, heads, 64, float(scale), qkv.scale, p.scale,
                                        L.ptr(key_mask) if key_mask is not None else None, L.ptr(p.data),
                                        _stream(dev.index)), "cm_planes_attention")
    return p


def qkv_planes_v(p: "Planes"):
    """(hi, lo) f16 row-major (M, N/3) views of the V third of CM_EPI_PLANES_QKV planes (tests)."""
    N = p.K
    nkbv = N // 96
    blk = p.data.view(-1, N // 32, 2, 4, 16, 8)        # [row block][kb][plane][g][c][e]
    rows = blk.shape[0] // 2 * 2
    v = blk[:rows, 2 * nkbv:].reshape(rows // 2, 2 * nkbv, 2, 4, 16, 8)   # [32-row unit][dblk][plane][g][c][e]
    # e 0-3: rows 4 g + e, e 4-7: rows 16 + 4 g + e - 4 of the unit; c = column within the 16-block
    v = v.view(rows // 2, 2 * nkbv, 2, 4, 16, 2, 4).permute(2, 0, 5, 3, 6, 1, 4)   # [plane][u][half][g][r][dblk][c]
    v = v.reshape(2, rows * 16, N // 3)
    return v[0, :p.M], v[1, :p.M]


# ---------------------------------------------------------------------------
# Where-filters on the device: retrieval.filters compiles, cm_filter_eval runs.
def filter_bits(prog, device: Optional[int] = None):
    """Run a compiled ``FilterProgram`` in HBM -> (allow words as a device int32 tensor, set bits).

    The MetaIndex's code columns and live bits are copied to the device once per metadata
    version and reused by every later filter; host-evaluated leaves are uploaded per call.
    """
    from .retrieval.filters import pack_bits
    device = default_device() if device is None else int(device)
    meta, n = prog.meta, prog.n
    dev = torch.device("cuda", device)
    cache = meta._dev_cache
    if cache is None or (cache["version"], cache["n"], cache["device"]) != (meta.version, n, device):
        cache = meta._dev_cache = {"version": meta.version, "n": n, "device": device, "cols": {}, "live": None}
    cols = []
    for slot, ck in enumerate(prog.cols):
        t = cache["cols"].get(ck)
        if t is None:
            t = cache["cols"][ck] = torch.from_numpy(np.ascontiguousarray(prog.column(slot))).to(dev)
        cols.append(t)
    bits = []
    for b in prog.bits:
        if isinstance(b, str):  # "live"
            if cache["live"] is None:
                cache["live"] = torch.from_numpy(pack_bits(meta.live[:n]).view(np.int32)).to(dev)
            bits.append(cache["live"])
        else:
            bits.append(torch.from_numpy(pack_bits(b).view(np.int32)).to(dev))
    nw = max((n + 31) // 32, 1)
    out = torch.zeros(nw, dtype=torch.int32, device=dev) if n == 0 else torch.empty(nw, dtype=torch.int32, device=dev)
    cnt = torch.empty(1, dtype=torch.int64, device=dev)
    ops = np.ascontiguousarray(np.asarray(prog.ops, np.int32).reshape(-1))
    col_p = (C.c_void_p * max(len(cols), 1))(*[t.data_ptr() for t in cols])
    bit_p = (C.c_void_p * max(len(bits), 1))(*[t.data_ptr() for t in bits])
    L.check(L.fn["cm_filter_eval"](L.ptr(ops), len(prog.ops), col_p, len(cols), bit_p, len(bits), int(n),
                                   out.data_ptr(), cnt.data_ptr(), _stream(device)), "cm_filter_eval")
    return out, int(cnt.item())  # .item() orders the handle-stream searches after the kernel


def where_bits(meta, where, semantics: str, device: Optional[int] = None):
    """Allow bitmap + candidate count of ``where`` under "bm25" (rag/retrieval/bm25.py:79-107) or
    "chroma" semantics: the compiled program on the device; a program over the kernel's limits
    (e.g. a 40-value $in) is evaluated by the MetaIndex in numpy and uploaded as host words."""
    from .retrieval.filters import pack_bits
    prog = meta.bm25_program(where) if semantics == "bm25" else meta.chroma_program(where)
    if prog.fits_device:
        return filter_bits(prog, device)
    mask = meta.bm25_mask(where) if semantics == "bm25" else meta.chroma_mask(where)
    return pack_bits(mask), int(mask.sum())
