"""``HybridRetriever.retrieve`` / ``retrieve_batch`` with the whole batch resident on the device.

The drop-in path (fusion.py) follows the reference's control flow per stage: the vector store
returns result dicts with their embeddings, MMR runs over host copies of the pools, the BM25 store
returns result dicts, and the merge matches items by id on the host (rag/retrieval/fusion.py:
108-167).  For a hybrid query with MMR -- the configuration the reference's callers use
(rag/pipeline/rag.py:531-554: ``ask_question`` sends ONE question with ``filters.to_dict()``) --
every one of those steps has a device form: where-filters as allow bitmaps (cm_filter_eval: Chroma
semantics for the dense side, ``_matches_filter`` semantics with quirk Q4 for BM25), cosine pool
search (K1c/K1s), pool gather + MMR (K4), BM25 top-k (K2a/K2b/K2 + K3; with a filter, K2f's
statistics over the allowed candidates, quirk Q2), pool preparation + RRF merge (K5).  This module
chains them without a host round trip and builds result dicts only for the final top_k items of
each query.  Single questions are a batch of one (their E5 encode replays a small-batch graph).

Id matching: the merge compares integer keys.  A document's key is its vector-store row; a BM25
document that the vector store does not hold gets ``n_vector_rows + bm25_row``.  The BM25-row ->
key map is a device array rebuilt when either store changes (their ``_version`` counters).

The result dicts equal the host path's (tests/test_gpu_dropin.py checks both on the same
stores): same ids, documents, metadata objects, distances (fp32 -> float), BM25 scores and fused
scores, in the same order.
"""
from __future__ import annotations

from typing import Any, Dict, List, Mapping, Optional, Sequence

import os

import numpy as np

from .. import _lib as L
from .. import engine


class _KeyMap:
    """BM25 rows <-> merge keys for one (vector store version, BM25 store version)."""

    def __init__(self, vs, bm, device: int):
        import torch
        ids_bm = bm._id_list
        nvr = len(vs._ids)
        if len(ids_bm) == nvr and ids_bm == vs._ids:          # the common case: one corpus, same order
            bm2key = np.arange(nvr, dtype=np.int64)
            vs2bm = np.arange(nvr, dtype=np.int64)
        else:
            rowmap = vs._row
            bm2key = np.fromiter((rowmap.get(i, -1) for i in ids_bm), dtype=np.int64, count=len(ids_bm))
            only = bm2key < 0
            bm2key[only] = nvr + np.nonzero(only)[0]
            vs2bm = np.full(nvr, -1, np.int64)
            both = ~only
            vs2bm[bm2key[both]] = np.nonzero(both)[0]
        self.nvr = nvr
        self.vs2bm = vs2bm
        self.bm2key_dev = torch.from_numpy(bm2key).to(torch.device("cuda", device))


def applicable(retr, filters, hybrid: bool) -> bool:
    """The device path covers hybrid retrieval with MMR over this package's stores, filtered or not
    (anything else takes the host path).  With a filter, ``retrieve_batch`` may still decline
    (None) when fewer vectors than the MMR pool pass it: the host path's k clamp covers that."""
    from .bm25 import BM25Store
    from .vector_store import GpuVectorStore
    vs, bm = retr.vector_store, retr.bm25_store
    if not hybrid or not retr.use_mmr:
        return False
    if not isinstance(vs, GpuVectorStore) or not isinstance(bm, BM25Store):
        return False
    vs._ensure_loaded()
    if vs._index is None or not bm._entries:
        return False
    pool = max(retr.k_vector, retr.mmr_max_pool)
    limit = L.max_topk()
    if not (0 < retr.k_vector <= pool <= limit and 0 < retr.k_bm25 <= limit):
        return False
    # the host path clamps k to the candidates; the device path needs full lists
    # live rows = the store's id -> row map (a device popcount + sync per call before)
    return len(vs._row) >= pool and len(bm._id_list) >= retr.k_bm25


def _query_vectors(embedder, questions: Sequence[str], dev):
    import torch
    enc = getattr(embedder, "encode_queries_dev", None)
    if enc is not None:
        q = enc(questions)
        if q is not None and q.device == dev and q.dtype == torch.float32:
            return q.contiguous()
    q = np.ascontiguousarray(np.asarray(embedder.encode_queries(list(questions)), np.float32))
    return torch.from_numpy(q).to(dev)


_ALLOW_CACHE_MAX = 64
# Process-level device caches, keyed by the stores' never-reused uids and version counters rather
# than held by one HybridRetriever: the reference builds a new retriever (and new stores) for every
# ask_question call (rag/pipeline/rag.py:531-545), so caches on the retriever object would be rebuilt
# per question -- the key map alone is O(corpus).
_ALLOW_CACHE: dict = {}
_KEYMAPS: dict = {}
_KEYMAPS_MAX = 4
_SIDE_STREAMS: dict = {}


def _canon(v):
    """Hashable, type-exact form of a where clause (True, 1 and "1" stay distinct; None when a
    value has no stable form)."""
    if isinstance(v, Mapping):
        return ("d", tuple(sorted(((str(type(k).__name__), k), _canon(x)) for k, x in v.items())))
    if isinstance(v, (list, tuple)):
        return (type(v).__name__, tuple(_canon(x) for x in v))
    if v is None or isinstance(v, (bool, int, float, str)):
        return (type(v).__name__, v)
    raise TypeError(type(v).__name__)


def _filter_key(meta, where, semantics: str):
    """Cache key of a filter over one metadata object and version: the object's uid (never reused,
    unlike id()), its version and the typed canonical clause (None when ``where`` has no stable
    form)."""
    try:
        return (meta.uid, meta.version, semantics, _canon(where))
    except (TypeError, ValueError):
        return None


def _allow(meta, where, semantics: str, device: int, n_words: int, cache: dict):
    """Device allow words + candidate count of ``where`` (engine.where_bits), cached per (metadata
    version, filter): a caller repeating one filter -- ask_question's to_dict() -- pays the filter
    program once per store change."""
    import torch
    key = _filter_key(meta, where, semantics)
    hit = cache.get(key) if key is not None else None
    if hit is not None and hit[0].numel() >= n_words:
        return hit
    from .. import engine as E
    words, n = E.where_bits(meta, where, semantics, device)
    if not hasattr(words, "data_ptr"):
        words = torch.from_numpy(np.ascontiguousarray(words).view(np.int32)).to(torch.device("cuda", device))
    if words.numel() < n_words:             # rows past the metadata (never written): not allowed
        words = torch.cat([words, torch.zeros(n_words - words.numel(), dtype=words.dtype, device=words.device)])
    if key is not None:
        if len(cache) >= _ALLOW_CACHE_MAX:
            cache.clear()
        cache[key] = (words, n)
    return words, n


def _bm25_filtered(bm, q_terms, q_off, k: int, allow, where, cache: dict):
    """Filtered BM25 top-k on the device (K2f: rank_bm25's statistics over the allowed candidates,
    quirk Q2).  rank_bm25's epsilon floor (0.25 x the mean idf over the candidates' vocabulary,
    needed when some query term's idf is negative) depends on the candidate set only, not on the
    query, so it is computed once per (BM25 version, filter) -- a pass over every posting -- and
    handed to later searches with the same filter."""
    import torch
    index = bm._index
    if getattr(index, "sharded", False):        # multidev: the candidates' statistics over every shard
        return index.search_filtered(q_terms, q_off, k, allow)
    index.prepare_filtered()                    # the device log table (once per index)
    fk = _filter_key(bm._meta, where, "bm25")
    ekey = None if fk is None else ("eps", bm._uid, bm._version) + fk
    eps_t = cache.get(ekey) if ekey is not None else None
    s, r, st = index.search_filtered_dev(q_terms, q_off, k, allow, eps=eps_t)
    code = int(st.item())
    if code & index.FILT_EPS_MISSING:
        eps_t = torch.tensor([index.filter_eps(allow)], dtype=torch.float64, device=q_terms.device)
        if ekey is not None:
            cache[ekey] = eps_t
        s, r, st = index.search_filtered_dev(q_terms, q_off, k, allow, eps=eps_t)
        code = int(st.item())
    if code & index.FILT_ZERO_DIV:
        raise ZeroDivisionError("float division by zero (candidate documents have no tokens)")
    if code:
        raise RuntimeError(f"filtered BM25 search status {code}")
    return s, r


def retrieve_batch(retr, questions: Sequence[str], top_k: int,
                   filters: Optional[Dict[str, Any]] = None) -> Optional[List[List[Dict[str, Any]]]]:
    """retr.retrieve_batch(questions, filters, top_k, hybrid=True) on the device (see module
    docstring); the caller checked ``applicable``.  Returns None when a filter leaves fewer vectors
    than the MMR pool (the host path then clamps k as the reference does)."""
    import torch
    from .filters import build_where_filter
    vs, bm = retr.vector_store, retr.bm25_store
    index = vs._index
    dev = torch.device("cuda", index.device)
    nq = len(questions)
    kv, kb = retr.k_vector, retr.k_bm25
    pool = max(kv, retr.mmr_max_pool)
    bm._ensure_index()
    allow_v = allow_b = None
    cache = _ALLOW_CACHE
    if filters:
        chroma_where = build_where_filter(filters)
        if chroma_where:
            allow_v, n_ok = _allow(vs._meta, chroma_where, "chroma", index.device, (index.size + 31) // 32, cache)
            if n_ok < pool:
                return None
        bm._ensure_meta()
        allow_b, n_cand = _allow(bm._meta, filters, "bm25", index.device, (len(bm._id_list) + 31) // 32, cache)
        kb = min(kb, n_cand)
    key = (vs._uid, vs._version, bm._uid, bm._version)   # the stores themselves (never-reused uids)
    km = _KEYMAPS.get(key)
    if km is None:
        km = _KeyMap(vs, bm, index.device)
        if len(_KEYMAPS) >= _KEYMAPS_MAX:
            _KEYMAPS.clear()
        _KEYMAPS[key] = km
    # BM25 runs on a side stream that waits only for the allow bitmaps / key map above, so it
    # overlaps the encode and the dense search (a filtered search's status read then waits for the
    # BM25 kernels alone, not for the dense scan queued ahead of it)
    main = torch.cuda.current_stream(dev)
    if os.environ.get("CLASSMATE_BM25_SAME_STREAM") == "1":     # A/B: the serial schedule
        side = main
    else:
        side = _SIDE_STREAMS.get(dev)
        if side is None:
            side = _SIDE_STREAMS[dev] = torch.cuda.Stream(device=dev)
    ready = torch.cuda.Event()
    ready.record(main)
    # E5 encode first (its launches return at once), so the host tokenizes the BM25 queries while
    # the device encodes; then dense pool + MMR
    q = _query_vectors(retr.embedder, questions, dev)
    # the certificate's exact pass (device-gated; normally nothing runs) waits for the BM25 join
    # below: its large-LDS grid would otherwise queue behind the BM25 kernels on the CUs
    d, r = index.search_dev(q, pool, allow=allow_v, defer_exact=True)
    blank = np.array([not q_.strip() for q_ in questions], bool)
    qids = [[] if blank[i] else bm._query_ids(q_) for i, q_ in enumerate(questions)]
    off = np.zeros(nq + 1, np.int32)
    off[1:] = np.cumsum([len(x) for x in qids])
    flat = np.asarray([t for x in qids for t in x] or [0], np.int32)
    with torch.cuda.stream(side):
        side.wait_event(ready)
        # pinned, stream-ordered copies: a pageable copy would wait here for the encode and search
        q_terms = torch.from_numpy(flat).pin_memory().to(dev, non_blocking=True)
        q_off = torch.from_numpy(off).pin_memory().to(dev, non_blocking=True)
        # BM25 top-k (whitespace-only queries: no BM25 list, bm25.py:178); with a filter, rank_bm25's
        # statistics over the allowed candidates (K2f; no candidate: empty lists, bm25.py:187)
        if allow_b is None:
            bs, br = bm._index.search_dev(q_terms, q_off, kb)
        elif kb > 0:
            bs, br = _bm25_filtered(bm, q_terms, q_off, kb, allow_b, filters, cache)
        else:
            bs = torch.zeros((nq, 1), dtype=torch.float64, device=dev)
            br = torch.full((nq, 1), -1, dtype=torch.int64, device=dev)
        bkeys = torch.where(br >= 0, km.bm2key_dev[br.clamp(min=0)], torch.full_like(br, -1))
        if blank.any():
            blank_dev = torch.from_numpy(blank).pin_memory().to(dev, non_blocking=True)
            bkeys = torch.where(blank_dev[:, None], torch.full_like(bkeys, -1), bkeys)   # no boolean-index sync
    main.wait_stream(side)
    index.exact_fallback_dev(q, pool, (d, r), allow=allow_v)
    vecs = index.gather_dev(r.reshape(-1)).view(nq, pool, index.dim)
    order = engine.mmr_dev(q, vecs, kv, float(retr.mmr_lambda))
    # side-stream tensors read on main: tell the caching allocator, so an exception
    # between here and the host copies below cannot recycle their blocks under main's kernels
    for t in (bs, br, bkeys, q_terms, q_off):
        t.record_stream(main)
    vk, vd, vn, bn = engine.rrf_pool_prep_dev(r.contiguous(), d.contiguous(), order, bkeys.contiguous())
    k_dev = top_k if top_k > 0 else kv + kb
    ok, of, ov, ob, ofl, on = engine.rrf_merge_dev(vk, vd, vn, bkeys.contiguous(), bs.contiguous(), bn,
                                                   w_vec=retr.weight_vector, w_bm25=retr.weight_bm25,
                                                   rrf_k=retr.rrf_k, top_k=k_dev)
    # one device-to-host copy of all six outputs (byte views concatenated; six .cpu() calls were six
    # synchronising copies), then Python lists once (per-element numpy indexing + float() costs ~40 %
    # of the dict loop)
    outs = (ok, of, ov, ob, ofl, on)
    blob = torch.cat([t.contiguous().view(-1).view(torch.uint8) for t in outs]).cpu().numpy()
    parts, o = [], 0
    for t in outs:
        nb = t.numel() * t.element_size()
        arr = blob[o:o + nb].view(np.dtype(str(t.dtype).replace("torch.", ""))).reshape(tuple(t.shape))
        parts.append(arr.tolist())
        o += nb
    ok, of, ov, ob, ofl, on = parts
    flush = getattr(retr.embedder, "flush_pending", None)     # CachingEmbedder: the misses' .npy files
    if flush is not None:
        flush()
    # result dicts of the final top_k items only (fusion.py:132-167 field rules)
    out: List[List[Dict[str, Any]]] = []
    nvr, vs2bm = km.nvr, km.vs2bm
    vids, vdocs, vmetas = vs._ids, vs._docs, vs._meta.metas
    bids, entries = bm._id_list, bm._entries
    dget = dict.__getitem__            # the catalog's stored value without its Python __getitem__ frame;
                                       # a pending (int: not yet parsed) record goes through entries[...]
    for i in range(nq):
        m = len(range(on[i])[:top_k])                    # Python slice of the full order
        res = []
        oki, fli, ofi, ovi, obi = ok[i], ofl[i], of[i], ov[i], ob[i]
        for j in range(m):
            kk, fl = oki[j], fli[j]
            if fl & 1:                                   # a vector item (the vector store's fields first)
                _id = vids[kk]
                doc, meta = vdocs[kk], vmetas[kk] or {}
                if fl & 2 and (not doc or not meta):
                    key = bids[int(vs2bm[kk])]
                    e = dget(entries, key)
                    if type(e) is int:
                        e = entries[key]
                    if not doc and e.text:
                        doc = e.text
                    if not meta and e.metadata:
                        meta = e.metadata
            else:                                        # BM25-only: the BM25 entry's fields (fusion.py:146-151)
                key = bids[int(vs2bm[kk])] if kk < nvr else bids[kk - nvr]
                e = dget(entries, key)
                if type(e) is int:
                    e = entries[key]
                _id, doc, meta = e.id, e.text or None, e.metadata or {}
            res.append({"id": _id, "document": doc, "metadata": meta,
                        "scores": {"vector_distance": ovi[j] if fl & 1 else None,
                                   "bm25_score": obi[j] if fl & 2 else None,
                                   "fused": ofi[j]}})
        out.append(res)
    return out
