"""BM25 lexical store, drop-in for ``rag.retrieval.bm25.BM25Store``.

Same dataclass fields, methods, JSONL persistence format and return dicts as
rag/retrieval/bm25.py:114-256.  Tokenization stays on the host (same regex,
stopwords and language handling); the index lives in HBM as CSR postings
(``engine.BM25Index``) and ``search`` is the HIP kernels K2/K3 with
rank_bm25 0.2.x semantics — statistics over the filtered candidates (Q2),
duplicate query tokens counted twice (Q3), zero-score padding in insertion
order (Q1), ZeroDivisionError on an all-empty vocabulary (Q7).

The reference rebuilds BM25Okapi on every mutation and again per search; here
mutations mark the device index dirty and the next search rebuilds it once.
"""
from __future__ import annotations

import json
from dataclasses import dataclass, field
from pathlib import Path
from typing import Any, Dict, List, Mapping, Optional, Sequence

import numpy as np

from .. import engine
from .filters import MetaIndex, pack_bits
from .tokenize import _tokenize, detect_lang_tag


@dataclass
class _Entry:
    id: str
    text: str
    tokens: List[str]
    metadata: Dict[str, Any]
    term_ids: Optional[np.ndarray] = None


@dataclass
class BM25Store:
    index_dir: Optional[Path] = Path("./indexes/bm25")
    index_file: str = "bm25_index.jsonl"
    device: Optional[int] = None

    _entries: Dict[str, _Entry] = field(default_factory=dict)
    _id_list: List[str] = field(default_factory=list)
    _vocab: Dict[str, int] = field(default_factory=dict, repr=False)
    _index: Optional[engine.BM25Index] = field(default=None, repr=False)
    _meta: MetaIndex = field(default_factory=MetaIndex, repr=False)
    _dirty: bool = field(default=True, repr=False)

    # ---------- core ops ----------
    def _term_ids(self, tokens: Sequence[str]) -> np.ndarray:
        v = self._vocab
        return np.fromiter((v.setdefault(t, len(v)) for t in tokens), dtype=np.int32, count=len(tokens))

    def _rebuild(self) -> None:
        """bm25.py:140-145: the reference rebuilds BM25Okapi here; it raises ZeroDivisionError when
        entries exist but every token list is empty.  We check that and defer the device build."""
        self._id_list = list(self._entries.keys())
        if self._entries and all(len(e.tokens) == 0 for e in self._entries.values()):
            raise ZeroDivisionError("float division by zero")
        self._dirty = True

    def _ensure_index(self) -> None:
        if not self._dirty and self._index is not None:
            return
        entries = [self._entries[i] for i in self._id_list]
        for e in entries:
            if e.term_ids is None:
                e.term_ids = self._term_ids(e.tokens)
        off = np.zeros(len(entries) + 1, np.int64)
        if entries:
            off[1:] = np.cumsum([e.term_ids.shape[0] for e in entries])
        flat = np.concatenate([e.term_ids for e in entries]) if off[-1] else np.zeros(0, np.int32)
        if self._index is None:
            self._index = engine.BM25Index(device=self.device)
        self._index.build(flat, off, max(len(self._vocab), 1))
        self._meta = MetaIndex()
        for r, e in enumerate(entries):
            self._meta.set(r, e.metadata)
        self._dirty = False

    def upsert_many(self, *, ids: Sequence[str], texts: Sequence[str], metadatas: Sequence[Mapping[str, Any]]) -> None:
        """bm25.py:147-166: language from metadata (or detected), tokenize, replace in place."""
        if not (len(ids) == len(texts) == len(metadatas)):
            raise ValueError("ids, texts, metadatas must have the same length")
        for i, doc_id in enumerate(ids):
            text = texts[i] or ""
            meta = dict(metadatas[i] or {})
            lang = meta.get("language")
            if not lang or lang == "auto":
                lang = detect_lang_tag(text)
                meta["language"] = lang
            toks = _tokenize(text, lang_hint=lang)
            self._entries[doc_id] = _Entry(id=doc_id, text=text, tokens=toks, metadata=meta)
        self._rebuild()

    def delete_many(self, ids: Sequence[str]) -> None:
        for doc_id in ids:
            self._entries.pop(doc_id, None)
        self._rebuild()

    # ---------- query ----------
    def _query_ids(self, query: str) -> List[int]:
        q_lang = detect_lang_tag(query)
        return [self._vocab.get(t, -1) for t in _tokenize(query, lang_hint=q_lang)]

    def search(self, *, query: str, where: Optional[Mapping[str, Any]] = None, top_k: int = 8) -> List[Dict[str, Any]]:
        """bm25.py:175-212 on the GPU."""
        return self.search_batch(queries=[query], where=where, top_k=top_k)[0]

    def search_batch(self, *, queries: Sequence[str], where: Optional[Mapping[str, Any]] = None,
                     top_k: int = 8) -> List[List[Dict[str, Any]]]:
        """Many queries sharing one filter: one device launch (build-side addition)."""
        out: List[List[Dict[str, Any]]] = [[] for _ in queries]
        live = [i for i, q in enumerate(queries) if q.strip()]
        if not live or not self._entries:
            return out
        self._ensure_index()
        mask = self._meta.bm25_mask(where)
        n_cand = int(mask.sum())
        if n_cand == 0:
            return out
        k = top_k if top_k >= 0 else n_cand + top_k      # python slice semantics of [:top_k]
        k = min(k, n_cand)
        if k <= 0:
            return out
        if k > engine.L.max_topk():
            raise ValueError(f"top_k={top_k} exceeds the GPU top-k limit {engine.L.max_topk()}")
        allow = pack_bits(mask) if where else None
        qids = [self._query_ids(queries[i]) for i in live]
        scores, rows, nvalid = self._index.search(qids, k, allow)
        for j, i in enumerate(live):
            res = []
            for s, r in zip(scores[j][: nvalid[j]], rows[j][: nvalid[j]]):
                e = self._entries[self._id_list[int(r)]]
                res.append({"id": e.id, "document": e.text, "metadata": e.metadata, "score": float(s)})
            out[i] = res
        return out

    def row_of(self, row: int) -> str:
        return self._id_list[row]

    # ---------- persistence (bm25.py:216-248) ----------
    @property
    def index_path(self) -> Path:
        return Path(self.index_dir) / self.index_file

    def save(self) -> None:
        if self.index_dir is None:
            return
        Path(self.index_dir).mkdir(parents=True, exist_ok=True)
        with self.index_path.open("w", encoding="utf-8") as f:
            for e in self._entries.values():
                rec = {"id": e.id, "text": e.text, "tokens": e.tokens, "metadata": e.metadata}
                f.write(json.dumps(rec, ensure_ascii=False) + "\n")

    def load(self) -> None:
        self._entries.clear()
        if self.index_dir is None or not self.index_path.exists():
            self._rebuild()
            return
        with self.index_path.open("r", encoding="utf-8") as f:
            for line in f:
                if not line.strip():
                    continue
                rec = json.loads(line)
                self._entries[rec["id"]] = _Entry(id=rec["id"], text=rec.get("text", ""),
                                                  tokens=list(rec.get("tokens", [])),
                                                  metadata=dict(rec.get("metadata", {})))
        self._rebuild()

    @classmethod
    def load_or_create(cls, index_dir: str | Path = "./indexes/bm25") -> "BM25Store":
        store = cls(index_dir=Path(index_dir))
        store.load()
        return store
