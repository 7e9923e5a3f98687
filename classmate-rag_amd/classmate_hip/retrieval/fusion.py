"""Hybrid retrieval with RRF + MMR, drop-in for rag/retrieval/fusion.py.

``rrf_fuse`` (fusion.py:17-36), ``_mmr_order`` (:39-61) and
``HybridRetriever.retrieve`` (:64-167) keep their signatures and return
values; the arithmetic runs in HIP kernels (K4 MMR, K5 RRF merge) instead of
Python/numpy.  ``HybridRetriever.retrieve_batch`` is the batched form: one
embedder call, one dense search, one MMR launch, one BM25 launch and one RRF
launch for the whole batch (per-query semantics unchanged).  Hybrid MMR
queries -- single or batched, filtered or not -- stay on the device end to end
(``device_batch``; CM_RETRIEVE_DEVICE=0 takes the host path).
"""
from __future__ import annotations

import contextlib
import os
from dataclasses import dataclass
from typing import Any, Dict, List, Mapping, Optional, Sequence

import numpy as np

from .. import engine
from . import device_batch
from .filters import build_where_filter


def rrf_fuse(*, rank_lists: Sequence[Sequence[str]], weights: Optional[Sequence[float]] = None,
             rrf_k: int = 60) -> Dict[str, float]:
    """score[id] += w_l / (rrf_k + rank + 1), computed on the GPU; dict in first-appearance order."""
    if not rank_lists:
        return {}
    n = len(rank_lists)
    if weights is not None and len(weights) != n:
        raise ValueError("weights length must match rank_lists length")
    intern: Dict[Any, int] = {}
    names: List[Any] = []
    lists = []
    for l in rank_lists:
        ks = []
        for x in l:
            k = intern.get(x)
            if k is None:
                k = intern[x] = len(names)
                names.append(x)
            ks.append(k)
        lists.append(ks)
    keys, scores = engine.rrf_fuse_keys(lists, None if weights is None else [float(w) for w in weights], rrf_k)
    return {names[int(k)]: float(s) for k, s in zip(keys, scores)}


def _mmr_order(q: np.ndarray, cands: np.ndarray, ids: List[str], k: int, lambd: float = 0.5) -> List[int]:
    """Greedy MMR over a candidate pool on the GPU (same tie rules as the reference)."""
    if len(ids) == 0:
        return []
    cands = np.asarray(cands, dtype=np.float32)
    order = engine.mmr_order_batch(np.asarray(q, np.float32).reshape(1, -1), cands[None], int(k), float(lambd),
                                   n_valid=np.array([len(ids)], np.int32))
    return [int(x) for x in order[0] if x >= 0]


@contextlib.contextmanager
def _stores_locked(retr):
    """The vector store's collection lock, then the BM25 store's (always in this order, so two
    retrievers sharing a store cannot deadlock), held across one retrieve: concurrent callers --
    each ask_question thread building its own stores on one directory -- are serialised on the
    handles they share (SURVEY §8(b) Threading; rag/pipeline/rag.py:531-534).  It also keeps a
    deferred dense search and its exact fallback (device_batch: search_dev(defer_exact=True) ...
    exact_fallback_dev, the shared index workspace and the kind chosen at search time) inside one
    critical section, so no other request's search or upsert lands between them.  Stores
    without a ``lock()`` (the reference's own classes) are not locked."""
    with contextlib.ExitStack() as stack:
        for s in (retr.vector_store, retr.bm25_store):
            lk = getattr(s, "lock", None)
            if callable(lk):
                stack.enter_context(lk())
        yield


def _vd_term(item) -> float:
    vd = item.get("distance")
    return float(vd) if isinstance(vd, (int, float)) else 0.0


@dataclass
class HybridRetriever:
    vector_store: Any
    bm25_store: Any
    embedder: Any

    k_vector: int = 8
    k_bm25: int = 8
    rrf_k: int = 60
    weight_vector: float = 1.0
    weight_bm25: float = 1.0

    use_mmr: bool = True
    mmr_lambda: float = 0.5
    mmr_max_pool: int = 24

    # ---- single query: the reference's control flow, device arithmetic ----------
    def _vector_search(self, *, query: str, where: Optional[Mapping[str, object]], k: int):
        q_vec = self.embedder.encode_queries([query])[0]
        pool_size = max(k, self.mmr_max_pool) if self.use_mmr else k
        res = self.vector_store.query(query_embeddings=q_vec, where=where, top_k=pool_size, include_documents=True,
                                      include_embeddings=self.use_mmr)
        if not self.use_mmr:
            return res[:k]
        ids, embs = [], []
        for r in res:
            if "embedding" in r and isinstance(r["embedding"], np.ndarray):
                ids.append(r["id"])
                embs.append(r["embedding"])
        if not ids:
            return res[:k]
        order = _mmr_order(q=q_vec, cands=np.stack(embs, axis=0), ids=ids, k=k, lambd=self.mmr_lambda)
        id_to_item = {r["id"]: r for r in res}
        return [id_to_item[ids[i]] for i in order if ids[i] in id_to_item]

    def _bm25_search(self, *, query: str, where: Optional[Mapping[str, object]], k: int):
        return self.bm25_store.search(query=query, where=where, top_k=k)

    def _merge(self, vec_res, bm25_res, top_k: int, hybrid: bool) -> List[Dict[str, object]]:
        """by_id assembly + RRF + (fused, -distance) stable sort (fusion.py:132-167), K5 on device."""
        return self._merge_batch([vec_res], [bm25_res], top_k, hybrid)[0]

    def _merge_batch(self, vec_batch, bm_batch, top_k: int, hybrid: bool) -> List[List[Dict[str, object]]]:
        nq = len(vec_batch)
        kv = max(1, max((len(v) for v in vec_batch), default=0))
        kb = max(1, max((len(b) for b in bm_batch), default=0)) if hybrid else 1
        vkeys = np.full((nq, kv), -1, np.int64)
        vdist = np.zeros((nq, kv), np.float32)
        bkeys = np.full((nq, kb), -1, np.int64)
        bscore = np.zeros((nq, kb), np.float64)
        vn = np.zeros(nq, np.int32)
        bn = np.zeros(nq, np.int32)
        interns = []
        for i in range(nq):
            intern: Dict[Any, int] = {}
            for j, r in enumerate(vec_batch[i]):
                vkeys[i, j] = intern.setdefault(r["id"], len(intern))
                vdist[i, j] = _vd_term(r)
            vn[i] = len(vec_batch[i])
            if hybrid:
                for j, r in enumerate(bm_batch[i]):
                    bkeys[i, j] = intern.setdefault(r["id"], len(intern))
                    bscore[i, j] = float(r.get("score") or 0.0)
                bn[i] = len(bm_batch[i])
            interns.append(intern)
        wv, wb = (self.weight_vector, self.weight_bm25) if hybrid else (1.0, 0.0)
        # fused_list[:top_k] (fusion.py:167) with Python slice semantics: the device merge ranks
        # every item (kv + kb of them) and a negative / zero top_k is applied to that full order
        k_dev = top_k if top_k > 0 else kv + kb
        ok, of, _, _, ofl, on = engine.rrf_merge(vkeys, vdist, vn, bkeys, bscore, bn, w_vec=wv, w_bm25=wb,
                                                 rrf_k=self.rrf_k, top_k=k_dev)
        out = []
        for i in range(nq):
            by_id: Dict[Any, Dict[str, object]] = {}
            for r in vec_batch[i]:
                it = by_id.setdefault(r["id"], {"id": r["id"], "document": None, "metadata": {},
                                                "scores": {"vector_distance": None, "bm25_score": None, "fused": 0.0}})
                it["document"] = it["document"] or r.get("document")
                it["metadata"] = it["metadata"] or r.get("metadata") or {}
                it["scores"]["vector_distance"] = r.get("distance")
            for r in (bm_batch[i] if hybrid else []):
                it = by_id.setdefault(r["id"], {"id": r["id"], "document": None, "metadata": {},
                                                "scores": {"vector_distance": None, "bm25_score": None, "fused": 0.0}})
                if not it["document"] and r.get("document"):
                    it["document"] = r.get("document")
                if not it["metadata"] and r.get("metadata"):
                    it["metadata"] = r.get("metadata") or {}
                it["scores"]["bm25_score"] = r.get("score")
            names = {v: k for k, v in interns[i].items()}
            res = []
            m = int(on[i])
            m = len(range(m)[:top_k])                    # Python slice of the full order
            for j in range(m):
                it = by_id[names[int(ok[i, j])]]
                it["scores"]["fused"] = float(of[i, j])
                res.append(it)
            out.append(res)
        return out

    def retrieve(self, *, question: str, filters: Optional[Mapping[str, object]] = None, top_k: int = 8,
                 hybrid: bool = True) -> List[Dict[str, object]]:
        with _stores_locked(self):
            return self._retrieve(question, filters, top_k, hybrid)

    def _retrieve(self, question, filters, top_k, hybrid):
        raw_filters = filters or {}
        if os.environ.get("CM_RETRIEVE_DEVICE", "1") != "0" and device_batch.applicable(self, raw_filters, hybrid):
            # the device chain of retrieve_batch for a batch of one (equal dicts: tests/test_gpu_dropin.py)
            out = device_batch.retrieve_batch(self, [question], top_k, raw_filters)
            if out is not None:
                return out[0]
        chroma_where = build_where_filter(raw_filters) if raw_filters else None
        bm_where = raw_filters or None
        bm25_res: List[Mapping[str, object]] = []
        if hybrid:
            vec_res = self._vector_search(query=question, where=chroma_where, k=self.k_vector)
            bm25_res = self._bm25_search(query=question, where=bm_where, k=self.k_bm25)
        else:
            vec_res = self._vector_search(query=question, where=chroma_where, k=max(top_k, self.k_vector))
        return self._merge(vec_res, bm25_res, top_k, hybrid)

    # ---- batched: one device launch per stage for the whole batch -----------------
    def retrieve_batch(self, *, questions: Sequence[str], filters: Optional[Mapping[str, object]] = None,
                       top_k: int = 8, hybrid: bool = True) -> List[List[Dict[str, object]]]:
        with _stores_locked(self):
            return self._retrieve_batch(questions, filters, top_k, hybrid)

    def _retrieve_batch(self, questions, filters, top_k, hybrid):
        questions = list(questions)
        if not questions:
            return []
        raw_filters = filters or {}
        if os.environ.get("CM_RETRIEVE_DEVICE", "1") != "0" and device_batch.applicable(self, raw_filters, hybrid):
            out = device_batch.retrieve_batch(self, questions, top_k, raw_filters)   # whole batch on the device
            if out is not None:
                return out
        chroma_where = build_where_filter(raw_filters) if raw_filters else None
        bm_where = raw_filters or None
        k = self.k_vector if hybrid else max(top_k, self.k_vector)
        q_vecs = self.embedder.encode_queries(questions)
        pool = max(k, self.mmr_max_pool) if self.use_mmr else k
        if hasattr(self.vector_store, "query_batch"):
            res_all = self.vector_store.query_batch(query_embeddings=q_vecs, where=chroma_where, top_k=pool,
                                                    include_documents=True, include_embeddings=self.use_mmr)
        else:
            res_all = [self.vector_store.query(query_embeddings=q, where=chroma_where, top_k=pool,
                                               include_documents=True, include_embeddings=self.use_mmr)
                       for q in q_vecs]
        vec_batch = []
        if self.use_mmr:
            P = max(1, max(len(r) for r in res_all))
            dim = q_vecs.shape[1]
            cands = np.zeros((len(questions), P, dim), np.float32)
            nv = np.zeros(len(questions), np.int32)
            ids_all = []
            for i, res in enumerate(res_all):
                ids = [r["id"] for r in res if isinstance(r.get("embedding"), np.ndarray)]
                for j, r in enumerate([r for r in res if isinstance(r.get("embedding"), np.ndarray)]):
                    cands[i, j] = r["embedding"]
                nv[i] = len(ids)
                ids_all.append(ids)
            order = engine.mmr_order_batch(q_vecs, cands, k, self.mmr_lambda, n_valid=nv)
            for i, res in enumerate(res_all):
                if nv[i] == 0:
                    vec_batch.append(res[:k])
                    continue
                by = {r["id"]: r for r in res}
                vec_batch.append([by[ids_all[i][j]] for j in order[i] if j >= 0 and ids_all[i][j] in by])
        else:
            vec_batch = [r[:k] for r in res_all]
        if hybrid:
            if hasattr(self.bm25_store, "search_batch"):
                bm_batch = self.bm25_store.search_batch(queries=questions, where=bm_where, top_k=self.k_bm25)
            else:
                bm_batch = [self.bm25_store.search(query=q, where=bm_where, top_k=self.k_bm25) for q in questions]
        else:
            bm_batch = [[] for _ in questions]
        return self._merge_batch(vec_batch, bm_batch, top_k, hybrid)
