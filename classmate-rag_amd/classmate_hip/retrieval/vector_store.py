"""HBM-resident cosine vector store, drop-in for ``ChromaVectorStore``.

Same constructor, methods and return shapes as rag/retrieval/vector_chroma.py:81-278
(``upsert`` / ``query`` / ``count`` / ``reset_collection`` / ``from_config``);
the Chroma client + HNSW server is replaced by ``engine.DenseIndex`` (exact
brute-force cosine on the GPU, kernel K1).  Extra, build-side: ``query_batch``
(many query rows at once — the reference returns row 0 only, quirk Q6),
persistence under ``persist_dir/collection_name`` (replacing the
Chroma persistent dir):

* ``vectors.f32`` -- row-aligned fp32 rows (row r at byte r * dim * 4), written in
  place through a memory map; the load streams it to HBM in 64k-row slabs;
* ``rows.log.jsonl`` -- an append-only log of ``{"row", "id", "document",
  "metadata"}`` records (``"id": null`` = tombstone), replayed on load, last
  record per row wins;
* ``meta.json`` -- ``{"format", "dim", "rows"}``, rewritten after every append.

With ``autosave`` (the reference persists every ``upsert``/``delete``) a call
writes only its own rows and log records: O(batch), not O(collection).
``save()`` writes everything from the device copy and compacts the log.

String ids, documents and metadata stay on the host; rows are assigned in
insertion order and re-upserting an id overwrites its row in place.
"""
from __future__ import annotations

import json
import os
import shutil
import threading
from collections import OrderedDict
from dataclasses import dataclass
from pathlib import Path
from typing import Any, Dict, List, Mapping, Optional, Sequence

import numpy as np

from .. import engine
from .filters import MetaIndex, next_uid


_FORMAT = 2


class _State:
    """The collection itself: device index, row <-> id tables, documents, metadata.  One per
    (collection directory, device) in a process, shared by every GpuVectorStore constructed on it
    -- as every ChromaVectorStore on one persist directory or server shares the Chroma collection
    (rag/retrieval/vector_chroma.py:102-163) -- so the reference's construct-per-call pattern
    (rag/pipeline/rag.py:531, ``ChromaVectorStore.from_config()`` on every ask) attaches to the
    resident index instead of re-reading the directory."""

    def __init__(self):
        self.index: Optional[engine.DenseIndex] = None
        self.ids: List[Optional[str]] = []
        self.row: Dict[str, int] = {}
        self.docs: List[Optional[str]] = []
        self.meta = MetaIndex()
        self.loaded = False
        self.version = 0            # bumped by every mutation (device key maps)
        self.uid = next_uid()       # identity in device caches (never reused)
        self.sig = None             # on-disk signature this state matches
        self.unsaved = False        # changed without a write (autosave=False): not attachable


def _disk_sig(d: Optional[Path]):
    """(size, mtime_ns) of the files a load reads: any writer -- this process or another --
    changes it."""
    if d is None:
        return None
    out = []
    for name in ("meta.json", "rows.log.jsonl", "vectors.f32"):
        try:
            st = os.stat(d / name)
            out.append((st.st_size, st.st_mtime_ns))
        except OSError:
            out.append(None)
    return tuple(out)


_REGISTRY: "OrderedDict[tuple, _State]" = OrderedDict()   # most recently attached last
_REGISTRY_MAX = 8
_REG_LOCK = threading.Lock()


def release_all() -> None:
    """Forget every registered collection (their device memory is freed once no store holds it)."""
    with _REG_LOCK:
        _REGISTRY.clear()


def _proxy(name: str):
    return property(lambda self: getattr(self._st, name), lambda self, v: setattr(self._st, name, v))


@dataclass
class GpuVectorStore:
    persist_dir: Optional[Path] = Path("./indexes/chroma")
    collection_name: str = "classmate_rag"
    distance: str = "cosine"
    device: Optional[int] = None
    autosave: bool = True

    # the collection's state (shared per directory, see _State)
    _index = _proxy("index")
    _ids = _proxy("ids")
    _row = _proxy("row")
    _docs = _proxy("docs")
    _meta = _proxy("meta")
    _loaded = _proxy("loaded")
    _version = _proxy("version")
    _uid = _proxy("uid")

    def __post_init__(self):
        if self.distance != "cosine":
            raise ValueError(f"only the 'cosine' space is implemented (got {self.distance!r})")
        if self.persist_dir is not None:
            self.persist_dir = Path(self.persist_dir)
        self._st = self._attach()

    def _attach(self) -> _State:
        """This process's state of the collection when the directory still matches it (no writer
        since, no unsaved change), else a fresh state (loaded on first use) that replaces it."""
        d = self._dir
        if d is None:
            return _State()
        dev = engine.default_device() if self.device is None else int(self.device)
        key = (str(d.resolve()), dev)
        sig = _disk_sig(d)
        with _REG_LOCK:
            st = _REGISTRY.get(key)
            if st is None or st.unsaved or st.sig != sig:
                st = _State()
                st.sig = sig
                _REGISTRY[key] = st
            _REGISTRY.move_to_end(key)
            while len(_REGISTRY) > _REGISTRY_MAX:
                _REGISTRY.popitem(last=False)
            return st

    def _changed(self, written: bool):
        """After a mutation: with a write the state matches the directory again, without one it
        no longer does (later constructions then read the directory, as the reference's would)."""
        if written and self._dir is not None:
            self._st.sig = _disk_sig(self._dir)
            self._st.unsaved = False
        elif self._dir is not None:
            self._st.unsaved = True

    # ---- persistence ----------------------------------------------------
    @property
    def _dir(self) -> Optional[Path]:
        return None if self.persist_dir is None else self.persist_dir / self.collection_name

    def _ensure_loaded(self):
        if self._loaded:
            return
        self._loaded = True
        d = self._dir
        if d is not None and (d / "meta.json").exists():
            self._load_from(d)

    def _load_from(self, d: Path):
        meta = json.loads((d / "meta.json").read_text(encoding="utf-8"))
        if meta.get("format") != _FORMAT:
            raise ValueError(f"{d}: unsupported vector store format {meta.get('format')!r}")
        dim, n = int(meta["dim"]), int(meta["rows"])
        recs: Dict[int, Mapping[str, Any]] = {}
        with (d / "rows.log.jsonl").open("r", encoding="utf-8") as f:
            for line in f:
                if line.strip():
                    rec = json.loads(line)
                    if rec["row"] < n:   # records past meta.rows belong to an interrupted append
                        recs[rec["row"]] = rec
        vecs = np.memmap(d / "vectors.f32", dtype=np.float32, mode="r", shape=(n, dim)) if n else None
        self._index = engine.DenseIndex(dim, device=self.device, capacity=max(n, 1))
        self._version += 1
        live = []
        for r in range(n):
            rec = recs.get(r)
            _id = rec.get("id") if rec else None
            self._ids.append(_id)
            self._docs.append(rec.get("document") if _id is not None else None)
            if _id is not None:
                self._row[_id] = r
                self._meta.set(r, rec.get("metadata"))
                live.append(r)
        if live:
            idx = np.asarray(live, np.int64)
            for s in range(0, idx.shape[0], 1 << 16):
                part = idx[s: s + (1 << 16)]
                self._index.upsert(np.asarray(vecs[part], np.float32), part)
        del vecs

    def _record(self, r: int) -> str:
        _id = self._ids[r]
        rec = {"row": r, "id": _id, "document": self._docs[r] if _id is not None else None,
               "metadata": (self._meta.metas[r] if r < len(self._meta.metas) else None) if _id is not None else None}
        return json.dumps(rec, ensure_ascii=False) + "\n"

    def _write_meta(self, d: Path):
        tmp = d / "meta.tmp.json"
        tmp.write_text(json.dumps({"format": _FORMAT, "dim": self._index.dim, "rows": len(self._ids)}),
                       encoding="utf-8")
        os.replace(tmp, d / "meta.json")

    def _append(self, rows: np.ndarray, emb: Optional[np.ndarray]):
        """Autosave of one upsert (emb given) or delete: its rows' vectors and log records only."""
        d = self._dir
        if d is None or self._index is None:
            return
        if not (d / "meta.json").exists():   # first write of this collection: the full layout
            self.save()
            return
        if emb is not None:
            n, dim = len(self._ids), self._index.dim
            with open(d / "vectors.f32", "r+b") as f:
                if f.seek(0, 2) < n * dim * 4:
                    f.truncate(n * dim * 4)
            mm = np.memmap(d / "vectors.f32", dtype=np.float32, mode="r+", shape=(n, dim))
            mm[rows] = emb
            mm.flush()
            del mm
        with (d / "rows.log.jsonl").open("a", encoding="utf-8") as f:
            f.write("".join(self._record(int(r)) for r in rows))
        self._write_meta(d)

    def save(self):
        """Full write from the device copy + a compacted log (one record per row)."""
        d = self._dir
        if d is None or self._index is None:
            return
        d.mkdir(parents=True, exist_ok=True)
        if (d / "meta.json").exists():
            os.remove(d / "meta.json")    # invalid until the rewrite below completes
        vecs = np.ascontiguousarray(self._index.export(), np.float32)
        n, dim = len(self._ids), self._index.dim
        with open(d / "vectors.tmp.f32", "wb") as f:
            f.write(vecs[:n].tobytes())
            # the device copy ends at the last row ever written after a reload (trailing rows that
            # are tombstones were never re-uploaded): pad so the file always holds meta.rows rows
            if vecs.shape[0] < n:
                f.truncate(n * dim * 4)
        os.replace(d / "vectors.tmp.f32", d / "vectors.f32")
        with (d / "rows.tmp.jsonl").open("w", encoding="utf-8") as f:
            for r in range(len(self._ids)):
                f.write(self._record(r))
        os.replace(d / "rows.tmp.jsonl", d / "rows.log.jsonl")
        self._write_meta(d)
        self._changed(True)

    # ---- upsert (vector_chroma.py:168-200) ---------------------------------
    def upsert(self, *, ids: Sequence[str], documents: Sequence[str], metadatas: Sequence[Mapping[str, Any]],
               embeddings: np.ndarray, batch_size: int = 512) -> None:
        if len(ids) != len(documents) or len(ids) != len(metadatas) or len(ids) != len(embeddings):
            raise ValueError("Lengths of ids, documents, metadatas, and embeddings must match.")
        self._ensure_loaded()
        if len(ids) == 0:
            return
        if len(set(ids)) != len(ids):
            raise ValueError("Expected IDs to be unique within one upsert call")
        emb = np.ascontiguousarray(np.asarray(embeddings, dtype=np.float32))
        if emb.ndim != 2:
            raise ValueError("embeddings must be a 2-D array (n, dim)")
        if self._index is None:
            self._index = engine.DenseIndex(emb.shape[1], device=self.device, capacity=len(ids))
        elif emb.shape[1] != self._index.dim:
            raise ValueError(f"Embedding dimension {emb.shape[1]} does not match collection dimensionality "
                             f"{self._index.dim}")
        rows = np.empty(len(ids), np.int64)
        self._version += 1
        for i, _id in enumerate(ids):
            r = self._row.get(_id)
            if r is None:
                r = len(self._ids)
                self._ids.append(_id)
                self._docs.append(None)
                self._row[_id] = r
            rows[i] = r
            self._docs[r] = documents[i]
            self._meta.set(r, metadatas[i])
        self._index.upsert(emb, rows)
        if self.autosave:
            self._append(rows, emb)
        self._changed(self.autosave)

    def delete(self, ids: Sequence[str]) -> None:
        """col.delete(ids=...) (vector_chroma.py:181-187); unknown ids are ignored."""
        self._ensure_loaded()
        rows = [self._row.pop(i) for i in ids if i in self._row]
        if not rows:
            return
        self._version += 1
        for r in rows:
            self._ids[r] = None
            self._docs[r] = None
            self._meta.remove(r)
        self._index.delete(np.asarray(rows, np.int64))
        if self.autosave:
            self._append(np.asarray(rows, np.int64), None)
        self._changed(self.autosave)

    # ---- query (vector_chroma.py:204-253) ------------------------------------
    def _search(self, q: np.ndarray, where, top_k: int, include_embeddings: bool):
        if top_k is None or int(top_k) <= 0:
            raise ValueError(f"Expected n_results to be a positive integer, got {top_k}")
        self._ensure_loaded()
        if self._index is None:
            return None
        if where:  # device-evaluated filter
            allow, n_ok = engine.where_bits(self._meta, where, "chroma", self._index.device)
        else:
            allow, n_ok = None, self._index.live_count()
        k = min(int(top_k), n_ok)
        if k <= 0:
            return None
        # k beyond the fused kernels' lists (cm_max_topk) runs the full-order device path
        return self._index.search(q, k, allow, return_vectors=include_embeddings)

    def _items(self, dist, rows, vecs, i, include_documents, include_embeddings, copy=False) -> List[Dict[str, Any]]:
        out = []
        for j in range(rows.shape[1]):
            r = int(rows[i, j])
            if r < 0:
                break
            item = {"id": self._ids[r], "document": self._docs[r] if include_documents else None,
                    "metadata": self._meta.metas[r],
                    "distance": float(dist[i, j])}
            if include_embeddings:
                # query(): an independent array per item, as Chroma returns; query_batch(): a
                # read-only row view of the call's own (B, k, D) buffer (zero-copy for the MMR pool)
                item["embedding"] = np.array(vecs[i, j]) if copy else vecs[i, j]
            out.append(item)
        return out

    def query(self, *, query_embeddings: np.ndarray, where: Optional[Dict[str, Any]] = None, top_k: int = 8,
              include_documents: bool = True, include_embeddings: bool = False) -> List[Dict[str, Any]]:
        q = np.asarray(query_embeddings).astype("float32")
        if q.ndim == 1:
            q = q[None, :]
        res = self._search(q[:1], where, top_k, include_embeddings)   # row 0 only, like the reference
        if res is None:
            return []
        dist, rows = res[0], res[1]
        vecs = res[2] if include_embeddings else None
        return self._items(dist, rows, vecs, 0, include_documents, include_embeddings, copy=True)

    def query_batch(self, *, query_embeddings: np.ndarray, where: Optional[Dict[str, Any]] = None, top_k: int = 8,
                    include_documents: bool = True, include_embeddings: bool = False) -> List[List[Dict[str, Any]]]:
        q = np.atleast_2d(np.asarray(query_embeddings).astype("float32"))
        res = self._search(q, where, top_k, include_embeddings)
        if res is None:
            return [[] for _ in range(q.shape[0])]
        dist, rows = res[0], res[1]
        vecs = res[2] if include_embeddings else None
        if vecs is not None:
            vecs.setflags(write=False)   # the items share it: an in-place edit must not reach the others
        return [self._items(dist, rows, vecs, i, include_documents, include_embeddings) for i in range(q.shape[0])]

    # ---- admin ------------------------------------------------------------------
    def count(self) -> int:
        self._ensure_loaded()
        try:
            return 0 if self._index is None else self._index.live_count()
        except Exception:
            return 0

    def reset_collection(self) -> None:
        self._ensure_loaded()
        if self._index is not None:
            self._index.close()
        self._index = None
        self._version += 1
        self._ids, self._row, self._docs = [], {}, []
        self._meta = MetaIndex()
        d = self._dir
        if d is not None and d.exists():
            shutil.rmtree(d, ignore_errors=True)
        self._changed(True)

    @classmethod
    def from_config(cls) -> "GpuVectorStore":
        """Same settings as the reference (rag/config.py:75-76,179-180), read from the environment."""
        return cls(persist_dir=Path(os.getenv("CHROMA_PERSIST_DIRECTORY", "./indexes/chroma") or "./indexes/chroma"),
                   collection_name=os.getenv("CHROMA_COLLECTION_NAME", "classmate_rag") or "classmate_rag",
                   distance="cosine")

    # rows <-> ids for the batched device pipeline
    def id_of(self, row: int) -> Optional[str]:
        return self._ids[row]


ChromaVectorStore = GpuVectorStore
