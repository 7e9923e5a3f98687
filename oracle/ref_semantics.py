"""CPU ORACLE — TEST INFRASTRUCTURE ONLY.

A plain-Python/numpy restatement of the CLASSMATE-RAG hybrid-retrieval path
(rag/retrieval/{bm25,fusion,vector_chroma}.py).  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
it, and only as the checker / CPU baseline — never as a product path.

Pinning: every function below is checked in ``tests/test_oracle_golden.py``
against ``tests/golden/*.json``, which ``tests/golden/gen_goldens.py`` produced
by importing the reference's own ``BM25Store``, ``rrf_fuse``, ``_mmr_order``,
``HybridRetriever`` and ``build_where_filter`` (with import stubs for the
absent third-party packages).  The third-party arithmetic itself is restated:

* ``BM25Okapi`` — rank_bm25 0.2.2 (requirements.txt:4 pins ``>=0.2.2,<0.3``),
  not installed here: restated from its published source; the reference's
  call sites are ``rag/retrieval/bm25.py:145,191,197``.  Parity with the real
  package is UNPINNED (no reference test or fixture holds its output).
* Chroma/hnswlib cosine k-NN is approximate (HNSW); the oracle is exact fp64
  brute force, ``distance = 1 - cos`` (``vector_chroma.py:156`` sets
  ``hnsw:space=cosine``).  Parity with HNSW output is UNPINNED.
"""
from __future__ import annotations

import math
import re
from typing import Any, Dict, List, Mapping, Optional, Sequence

import numpy as np

# --------------------------------------------------------------------------
# Tokenizer — rag/retrieval/bm25.py:34-70
# --------------------------------------------------------------------------
TOKEN_RE = re.compile(r"[A-Za-zÀ-ÖØ-öø-ÿ]+")

STOP_EN = set("""a an the and or but if then else for to of in on at by with from as is are was
were be been being it its this that these those i you he she we they them his her their my your
our me us not no yes do does did doing can could should would may might will shall about into
over under again further there here when where why how what which who whom""".split())

STOP_IT = set("""un uno una le la il lo gli i l e o ma se allora altrimenti per di a da in su con
come è era sono siamo siete fui fu furono essere stato questo questa questi queste quello quella
quelli quelle ciò cio io tu lui lei noi voi loro mio mia tuo tua suo sua nostro vostro non no si
sia fare fa fatto posso può puo puoi possono dovrebbe potrebbe sarà sara sarebbe saremmo sarete
siano che perché perche quando dove cosa quale chi""".split())


def tokenize(text: str, lang_hint: Optional[str] = None) -> List[str]:
    """bm25.py:54-70: regex words, lowercase, drop stopwords (IT if hint startswith 'it'), len>1."""
    lang = (lang_hint or "").lower()
    sw = STOP_IT if lang.startswith("it") else STOP_EN
    toks = [m.group(0).lower() for m in TOKEN_RE.finditer(text or "")]
    return [t for t in toks if t not in sw and len(t) > 1]


# --------------------------------------------------------------------------
# rank_bm25 0.2.2 BM25Okapi (third-party, restated)
# --------------------------------------------------------------------------
class BM25Okapi:
    """rank_bm25.BM25Okapi(corpus, k1=1.5, b=0.75, epsilon=0.25)."""

    def __init__(self, corpus, k1=1.5, b=0.75, epsilon=0.25):
        self.k1, self.b, self.epsilon = k1, b, epsilon
        self.corpus_size = 0
        self.doc_len: List[int] = []
        self.doc_freqs: List[Dict[str, int]] = []
        self.idf: Dict[str, float] = {}
        nd: Dict[str, int] = {}
        num_doc = 0
        for document in corpus:
            self.doc_len.append(len(document))
            num_doc += len(document)
            freqs: Dict[str, int] = {}
            for word in document:
                freqs[word] = freqs.get(word, 0) + 1
            self.doc_freqs.append(freqs)
            for word in freqs:
                nd[word] = nd.get(word, 0) + 1
            self.corpus_size += 1
        self.avgdl = num_doc / self.corpus_size
        idf_sum = 0.0
        negative = []
        for word, freq in nd.items():
            idf = math.log(self.corpus_size - freq + 0.5) - math.log(freq + 0.5)
            self.idf[word] = idf
            idf_sum += idf
            if idf < 0:
                negative.append(word)
        self.average_idf = idf_sum / len(self.idf)        # ZeroDivisionError on empty vocab (Q7)
        eps = self.epsilon * self.average_idf
        for word in negative:
            self.idf[word] = eps

    def get_scores(self, query: Sequence[str]) -> np.ndarray:
        score = np.zeros(self.corpus_size)
        doc_len = np.array(self.doc_len)
        for q in query:
            q_freq = np.array([(doc.get(q) or 0) for doc in self.doc_freqs])
            score += (self.idf.get(q) or 0) * (q_freq * (self.k1 + 1) /
                                               (q_freq + self.k1 * (1 - self.b + self.b * doc_len / self.avgdl)))
        return score


# --------------------------------------------------------------------------
# Filters
# --------------------------------------------------------------------------
SIMPLE_FIELDS = ["course", "unit", "language", "doc_type", "author", "semester"]


def bm25_matches_filter(meta: Mapping[str, Any], where: Optional[Mapping[str, Any]]) -> bool:
    """bm25.py:79-107 (keeps quirk Q4: a present-but-None key must equal meta.get)."""
    if not where:
        return True
    if "$and" in where:
        return all(bm25_matches_filter(meta, c) for c in where["$and"])
    if "tags" in where and isinstance(where["tags"], dict) and "$contains" in where["tags"]:
        t = where["tags"]["$contains"]
        if not t:
            return True
        want = {t} if isinstance(t, str) else set(t)
        return want.issubset(set(meta.get("tags") or []))
    for f in SIMPLE_FIELDS:
        if f in where and meta.get(f) != where[f]:
            return False
    return True


def _slug_tag(t: str) -> str:
    s = re.sub(r"[^a-z0-9]+", "_", (t or "").lower().strip())
    return s.strip("_")


def _parse_tags(obj) -> List[str]:
    if not obj:
        return []
    vals = [str(x) for x in obj] if isinstance(obj, (list, tuple)) else str(obj).split(",")
    return [v.strip() for v in vals if v.strip()]


def build_where_filter(meta_like: Mapping[str, Any]):
    """vector_chroma.py:45-78."""
    if not meta_like:
        return None
    clauses = []
    for f in SIMPLE_FIELDS:
        v = meta_like.get(f)
        if v is None:
            continue
        if isinstance(v, str):
            v = v.strip()
            if not v or (f == "doc_type" and v.lower() == "other"):
                continue
        clauses.append({f: v})
    for t in _parse_tags(meta_like.get("tags")):
        s = _slug_tag(t)
        if s:
            clauses.append({f"tag_{s}": True})
    if not clauses:
        return None
    return clauses[0] if len(clauses) == 1 else {"$and": clauses}


def chroma_matches(meta: Mapping[str, Any], where: Optional[Mapping[str, Any]]) -> bool:
    """Chroma where semantics for the operators build_where_filter emits (+$or/$eq/$ne/$in)."""
    if not where:
        return True
    for key, cond in where.items():
        if key == "$and":
            if not all(chroma_matches(meta, c) for c in cond):
                return False
            continue
        if key == "$or":
            if not any(chroma_matches(meta, c) for c in cond):
                return False
            continue
        if key not in meta:
            return False
        v = meta[key]
        if isinstance(cond, dict):
            (op, arg), = cond.items()
            same = type(v) is type(arg) and v == arg
            if op == "$eq" and not same:
                return False
            if op == "$ne" and same:
                return False
            if op == "$in" and not any(type(v) is type(a) and v == a for a in arg):
                return False
            if op == "$nin" and any(type(v) is type(a) and v == a for a in arg):
                return False
        elif not (type(v) is type(cond) and v == cond):
            return False
    return True


# --------------------------------------------------------------------------
# BM25Store.search — bm25.py:147-212
# --------------------------------------------------------------------------
class BM25Oracle:
    """Insertion-ordered entries {id: (text, tokens, metadata)} with reference search()."""

    def __init__(self):
        self.entries: Dict[str, tuple] = {}

    def upsert_many(self, ids, texts, metadatas, lang_detect=lambda t: "en"):
        if not (len(ids) == len(texts) == len(metadatas)):
            raise ValueError("ids, texts, metadatas must have the same length")
        for i, doc_id in enumerate(ids):
            text = texts[i] or ""
            meta = dict(metadatas[i] or {})
            lang = meta.get("language")
            if not lang or lang == "auto":
                lang = lang_detect(text)
                meta["language"] = lang
            self.entries[doc_id] = (text, tokenize(text, lang), meta)
        if self.entries:
            BM25Okapi([e[1] for e in self.entries.values()])   # reference rebuild may raise (Q7)

    def delete_many(self, ids):
        for i in ids:
            self.entries.pop(i, None)

    def search(self, query: str, where=None, top_k: int = 8, lang_detect=lambda t: "en"):
        if not query.strip() or not self.entries:
            return []
        cands = [i for i in self.entries if bm25_matches_filter(self.entries[i][2], where)]
        if not cands:
            return []
        bm = BM25Okapi([self.entries[i][1] for i in cands] or [[""]])
        scores = bm.get_scores(tokenize(query, lang_detect(query)))
        ranked = sorted(zip(cands, scores), key=lambda x: x[1], reverse=True)[:top_k]
        return [{"id": i, "document": self.entries[i][0], "metadata": self.entries[i][2],
                 "score": float(s)} for i, s in ranked]


# --------------------------------------------------------------------------
# Exact dense cosine (stand-in for Chroma HNSW)
# --------------------------------------------------------------------------
def dense_topk_exact(emb: np.ndarray, q: np.ndarray, k: int, allow: Optional[np.ndarray] = None):
    """fp64 cosine distance 1 - q.c/(|q||c|); ascending, ties -> lower row. Returns (rows, dist64)."""
    c = emb.astype(np.float64)
    qq = np.atleast_2d(q).astype(np.float64)
    cn = np.linalg.norm(c, axis=1)
    cn[cn == 0] = np.inf
    qn = np.linalg.norm(qq, axis=1, keepdims=True)
    qn[qn == 0] = np.inf
    d = 1.0 - (qq @ c.T) / qn / cn[None, :]
    if allow is not None:
        d[:, ~allow] = np.inf
    rows, dists = [], []
    for i in range(d.shape[0]):
        ordr = np.lexsort((np.arange(d.shape[1]), d[i]))
        ordr = ordr[np.isfinite(d[i][ordr])][:k]
        rows.append(ordr)
        dists.append(d[i][ordr])
    return rows, dists


class ExactVectorStore:
    """Duck-typed ChromaVectorStore.query (vector_chroma.py:204-253) over exact fp64 cosine."""

    def __init__(self, ids, documents, metadatas, embeddings):
        self.ids = list(ids)
        self.docs = list(documents)
        self.metas = list(metadatas)
        self.emb = np.asarray(embeddings, dtype=np.float32)

    def query(self, *, query_embeddings, where=None, top_k=8, include_documents=True,
              include_embeddings=False):
        q = np.asarray(query_embeddings, dtype=np.float32)
        q = q[None, :] if q.ndim == 1 else q
        allow = np.array([chroma_matches(m, where) for m in self.metas]) if where else None
        rows, dists = dense_topk_exact(self.emb, q[:1], top_k, allow)
        out = []
        for r, dd in zip(rows[0], dists[0]):
            item = {"id": self.ids[r], "document": self.docs[r] if include_documents else None,
                    "metadata": self.metas[r], "distance": float(np.float32(dd))}
            if include_embeddings:
                item["embedding"] = self.emb[r].copy()
            out.append(item)
        return out


# --------------------------------------------------------------------------
# Fusion — fusion.py:17-167
# --------------------------------------------------------------------------
def rrf_fuse(*, rank_lists, weights=None, rrf_k: int = 60) -> Dict[str, float]:
    if not rank_lists:
        return {}
    n = len(rank_lists)
    if weights is None:
        weights = [1.0] * n
    elif len(weights) != n:
        raise ValueError("weights length must match rank_lists length")
    scores: Dict[str, float] = {}
    for li, ids in enumerate(rank_lists):
        w = float(weights[li])
        for r, _id in enumerate(ids):
            scores[_id] = scores.get(_id, 0.0) + w * (1.0 / (rrf_k + (r + 1)))
    return scores


def mmr_order(q: np.ndarray, cands: np.ndarray, ids: List[str], k: int, lambd: float = 0.5) -> List[int]:
    """fusion.py:39-61 (numpy>=2 NEP-50 float32 scalar arithmetic)."""
    if len(ids) == 0:
        return []
    q = q.reshape(1, -1).astype("float32")
    sims_q = (cands @ q.T).ravel()
    sims_cc = cands @ cands.T
    selected = [int(np.argmax(sims_q))]
    remaining = set(range(len(ids)))
    remaining.discard(selected[0])
    while remaining and len(selected) < min(k, len(ids)):
        best_idx, best = None, -1e9
        for i in sorted(remaining):
            div = np.max(sims_cc[i, selected])
            s = lambd * sims_q[i] - (1.0 - lambd) * div
            if s > best:
                best, best_idx = s, i
        selected.append(int(best_idx))
        remaining.discard(int(best_idx))
    return selected


def retrieve(vector_store, bm25_store, embedder, *, question, filters=None, top_k=8, hybrid=True,
             k_vector=8, k_bm25=8, rrf_k=60, weight_vector=1.0, weight_bm25=1.0,
             use_mmr=True, mmr_lambda=0.5, mmr_max_pool=24):
    """HybridRetriever.retrieve (fusion.py:80-167)."""
    raw = filters or {}
    cw = build_where_filter(raw) if raw else None
    bw = raw or None

    def vsearch(k):
        qv = embedder.encode_queries([question])[0]
        pool = max(k, mmr_max_pool) if use_mmr else k
        res = vector_store.query(query_embeddings=qv, where=cw, top_k=pool, include_documents=True,
                                 include_embeddings=use_mmr)
        if not use_mmr:
            return res[:k]
        ids = [r["id"] for r in res if isinstance(r.get("embedding"), np.ndarray)]
        embs = [r["embedding"] for r in res if isinstance(r.get("embedding"), np.ndarray)]
        if not ids:
            return res[:k]
        order = mmr_order(qv, np.stack(embs), ids, k, mmr_lambda)
        by = {r["id"]: r for r in res}
        return [by[ids[i]] for i in order if ids[i] in by]

    vec, bm = [], []
    if hybrid:
        vec = vsearch(k_vector)
        bm = bm25_store.search(query=question, where=bw, top_k=k_bm25)
    else:
        vec = vsearch(max(top_k, k_vector))
    fused = rrf_fuse(rank_lists=[[r["id"] for r in vec], [r["id"] for r in bm]] if hybrid
                     else [[r["id"] for r in vec]],
                     weights=[weight_vector, weight_bm25] if hybrid else [1.0], rrf_k=rrf_k)
    by_id: Dict[str, Dict[str, Any]] = {}
    for r in vec:
        it = by_id.setdefault(r["id"], {"id": r["id"], "document": None, "metadata": {},
                                        "scores": {"vector_distance": None, "bm25_score": None, "fused": 0.0}})
        it["document"] = it["document"] or r.get("document")
        it["metadata"] = it["metadata"] or r.get("metadata") or {}
        it["scores"]["vector_distance"] = r.get("distance")
    for r in bm:
        it = by_id.setdefault(r["id"], {"id": r["id"], "document": None, "metadata": {},
                                        "scores": {"vector_distance": None, "bm25_score": None, "fused": 0.0}})
        if not it["document"] and r.get("document"):
            it["document"] = r.get("document")
        if not it["metadata"] and r.get("metadata"):
            it["metadata"] = r.get("metadata") or {}
        it["scores"]["bm25_score"] = r.get("score")
    for _id, s in fused.items():
        if _id in by_id:
            by_id[_id]["scores"]["fused"] = float(s)

    def key(it):
        s = it["scores"]
        vd = s.get("vector_distance")
        return (s.get("fused") or 0.0, -(vd if isinstance(vd, (int, float)) else 0.0))

    return sorted(by_id.values(), key=key, reverse=True)[:top_k]
