"""ctypes wrapper of oracle/liboracle.so — CPU ORACLE, TEST INFRASTRUCTURE ONLY.

Used by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, as
the checker / CPU baseline; never by the product path.
"""
from __future__ import annotations

import ctypes as C
from pathlib import Path

import numpy as np

import os

# CM_ORACLE_LIB: an alternative build of the same source (tools/asan_check.sh: ASan/UBSan)
_LIB = Path(os.environ.get("CM_ORACLE_LIB") or Path(__file__).with_name("liboracle.so"))
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not _LIB.exists():
            raise ImportError(f"{_LIB} missing: run `make -C oracle`")
        _lib = C.CDLL(str(_LIB))
        vp, i32, i64, f64 = C.c_void_p, C.c_int32, C.c_int64, C.c_double
        _lib.orc_bm25_idf.argtypes = [i32, vp, vp, i64, vp, vp]
        _lib.orc_bm25_csr_topk.argtypes = [i32, vp, vp, vp, i64, vp, vp, vp, f64, i32, vp, vp, i32, vp, vp]
        _lib.orc_count_postings.argtypes = [vp, vp, i64, i32]
        _lib.orc_count_postings.restype = i64
        _lib.orc_build_csr.argtypes = [vp, vp, i64, i32, vp, vp, vp, vp, vp, vp]
        _lib.orc_dense_topk_f64.argtypes = [i64, i32, vp, i32, vp, i32, vp, vp]
        _lib.orc_num_threads.restype = C.c_int
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data


def num_threads() -> int:
    return int(lib().orc_num_threads())


def build_csr(term_ids: np.ndarray, doc_off: np.ndarray, vocab: int):
    t = np.ascontiguousarray(term_ids, np.int32)
    o = np.ascontiguousarray(doc_off, np.int64)
    nd = o.shape[0] - 1
    npost = lib().orc_count_postings(_p(t), _p(o), nd, vocab)
    term_off = np.empty(vocab + 1, np.int64)
    post_doc = np.empty(max(npost, 1), np.int32)
    post_tf = np.empty(max(npost, 1), np.uint16)
    dl = np.empty(max(nd, 1), np.int32)
    df = np.empty(max(vocab, 1), np.int64)
    fk = np.empty(max(vocab, 1), np.uint64)
    lib().orc_build_csr(_p(t), _p(o), nd, vocab, _p(term_off), _p(post_doc), _p(post_tf), _p(dl), _p(df), _p(fk))
    return dict(term_off=term_off, post_doc=post_doc[:npost], post_tf=post_tf[:npost], dl=dl[:nd],
                df=df[:vocab], first_key=fk[:vocab], vocab=vocab, ndocs=nd)


def bm25_idf(df: np.ndarray, first_key: np.ndarray, n_docs: int):
    v = df.shape[0]
    idf = np.empty(max(v, 1), np.float64)
    eps = C.c_double(0.0)
    rc = lib().orc_bm25_idf(v, _p(np.ascontiguousarray(df, np.int64)),
                            _p(np.ascontiguousarray(first_key, np.uint64)), int(n_docs), _p(idf), C.byref(eps))
    if rc == -4:
        raise ZeroDivisionError("float division by zero")
    return idf[:v], eps.value


def bm25_topk(csr: dict, idf: np.ndarray, avgdl: float, queries, k: int, allow=None):
    nq = len(queries)
    off = np.zeros(nq + 1, np.int32)
    for i, q in enumerate(queries):
        off[i + 1] = off[i] + len(q)
    flat = np.ascontiguousarray(np.concatenate([np.asarray(q, np.int32) for q in queries]) if off[-1]
                                else np.zeros(1, np.int32))
    sc = np.empty((nq, k), np.float64)
    rw = np.empty((nq, k), np.int64)
    al = None if allow is None else np.ascontiguousarray(allow, np.uint8)
    lib().orc_bm25_csr_topk(csr["vocab"], _p(csr["term_off"]), _p(csr["post_doc"]), _p(csr["post_tf"]),
                            csr["ndocs"], _p(csr["dl"]), _p(al), _p(np.ascontiguousarray(idf, np.float64)),
                            float(avgdl), nq, _p(flat), _p(off), int(k), _p(sc), _p(rw))
    return sc, rw


def dense_topk_f64(emb: np.ndarray, q: np.ndarray, k: int):
    c = np.ascontiguousarray(emb, np.float32)
    qq = np.ascontiguousarray(np.atleast_2d(q), np.float32)
    d = np.empty((qq.shape[0], k), np.float64)
    r = np.empty((qq.shape[0], k), np.int64)
    lib().orc_dense_topk_f64(c.shape[0], c.shape[1], _p(c), qq.shape[0], _p(qq), int(k), _p(d), _p(r))
    return d, r
