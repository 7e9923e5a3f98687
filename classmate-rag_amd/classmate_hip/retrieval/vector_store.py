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
* ``meta.json`` -- ``{"format", "dim", "rows"}``, rewritten after every append;
* ``snapshot/`` -- the ids, each row's latest record offset in the log and the
  metadata filter columns, valid for a prefix of the log (same inode): a cold
  open reads it plus the records appended after it, and parses a row's
  document / metadata only when a result needs them (10M rows: seconds instead
  of a 10M-record JSON replay).

With ``autosave`` (the reference persists every ``upsert``/``delete``) a call
writes only its own rows and log records: O(batch), not O(collection); the
snapshot is refreshed once the log tail since it passes half the rows.
``save()`` writes everything from the device copy, compacts the log and writes
the snapshot.

Constructions on one directory in one process share the collection (``_State``:
the reference's per-call ``ChromaVectorStore.from_config()`` attaches to the
resident index while the directory is unchanged).

String ids, documents and metadata stay on the host; rows are assigned in
insertion order and re-upserting an id overwrites its row in place.
"""
from __future__ import annotations

import functools
import json
import os
import shutil
import threading
from collections import OrderedDict
from dataclasses import dataclass
from pathlib import Path
from typing import Any, Dict, List, Mapping, Optional, Sequence

import numpy as np

from .. import engine, multidev
from .filters import MetaIndex, next_uid, settle_loaded


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
        self.line_off = None        # per row: byte offset of its latest record in rows.log.jsonl
        self.tail = 0               # records appended since the last snapshot
        # serialises every use of the collection -- its host tables and its device handle (whose
        # search staging buffers and workspace are per handle) -- across the stores attached to it
        # and the threads using them (SURVEY §8(b) Threading)
        self.lock = threading.RLock()


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


def _locked(fn):
    """Run a GpuVectorStore method under its collection's lock (_State.lock, reentrant)."""
    @functools.wraps(fn)
    def run(self, *a, **kw):
        with self._st.lock:
            return fn(self, *a, **kw)
    return run


class _LazyRecords:
    """Parses row r's log record (the document and metadata of a row opened from the snapshot)
    on first access, by its byte offset in rows.log.jsonl."""

    def __init__(self, path: Path, st: "_State"):
        self.path, self.st, self.fh = path, st, None
        self._lock = threading.Lock()      # one file object: seek + readline as a unit

    def parse(self, r: int):
        with self._lock:
            if self.fh is None:
                self.fh = open(self.path, "rb")
            self.fh.seek(int(self.st.line_off[r]))
            line = self.fh.readline()
        rec = json.loads(line)
        live = rec.get("id") is not None
        return (rec.get("document") if live else None), (rec.get("metadata") if live else None)


_PENDING = object()
_SNAPSHOT_MIN_TAIL = 1 << 15   # log records appended since the snapshot before a refresh is considered
_SNAPSHOT_TAIL_FRAC = 0.5      # ... and their fraction of the rows


class _LazyList(list):
    """A row-aligned list whose first n0 entries are parsed from the log on first read (field 0:
    document, 1: metadata); writes and appends behave as a plain list's."""

    def __init__(self, n0: int, rec: _LazyRecords, field: int):
        super().__init__([_PENDING] * n0)
        self.rec, self.field = rec, field

    def __getitem__(self, r):
        v = list.__getitem__(self, r)
        if v is _PENDING:
            v = self.rec.parse(r)[self.field]
            list.__setitem__(self, r, v)
        return v


def _read_snapshot(d: Path, n: int):
    """(info, arrays, ids) of d/snapshot when it covers a prefix of the current log (same inode,
    the log at least as long) and of the rows, else None."""
    sd = d / "snapshot"
    try:
        info = json.loads((sd / "info.json").read_text(encoding="utf-8"))
        st = os.stat(d / "rows.log.jsonl")
        if (info.get("version") != 1 or info.get("log_ino") != st.st_ino or int(info["log_size"]) > st.st_size
                or int(info["ids_rows"]) > n):
            return None
        ids = json.loads((sd / "ids.json").read_text(encoding="utf-8"))
        arrays = {p.stem: np.load(p) for p in sd.glob("*.npy")}
    except (OSError, ValueError, KeyError):
        return None
    if len(ids) != int(info["ids_rows"]) or arrays["line_off"].shape[0] != len(ids):
        return None
    # rows past the metadata columns' prefix (never given metadata): pad the columns' view
    info["rows"] = len(ids) if int(info["rows"]) <= len(ids) else None
    if info["rows"] is None:
        return None
    for k in [k for k in arrays if k.endswith("_py") or k.endswith("_ty")]:
        a = arrays[k]
        if a.shape[0] < len(ids):
            arrays[k] = np.concatenate([a, np.full(len(ids) - a.shape[0], -1, np.int32)])
    if arrays["live"].shape[0] < len(ids):
        arrays["live"] = np.concatenate([arrays["live"], np.zeros(len(ids) - arrays["live"].shape[0], bool)])
    return info, arrays, ids


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
        key = (str(d.resolve()), dev, os.environ.get("CM_DEVICES", "") if self.device is None else "")
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

    @_locked
    def _ensure_loaded(self):
        if self._loaded:
            return
        self._loaded = True
        d = self._dir
        if d is not None and (d / "meta.json").exists():
            self._load_from(d)
            settle_loaded()

    def _load_from(self, d: Path):
        """Open the directory: from the snapshot + the log records appended after it when the
        snapshot matches the log (seconds at 10M rows: no per-row JSON parse or metadata insert --
        documents and metadata dicts are parsed when a result needs them), else by replaying the
        whole log.  Then the live rows' vectors stream to HBM."""
        meta = json.loads((d / "meta.json").read_text(encoding="utf-8"))
        if meta.get("format") != _FORMAT:
            raise ValueError(f"{d}: unsupported vector store format {meta.get('format')!r}")
        dim, n = int(meta["dim"]), int(meta["rows"])
        st = self._st
        log = d / "rows.log.jsonl"
        snap = _read_snapshot(d, n)
        if snap is not None:
            info, arrays, ids = snap
            n0 = int(info["rows"])
            st.line_off = np.full(max(n, 1), -1, np.int64)
            st.line_off[:n0] = arrays["line_off"][:n0]
            rec = _LazyRecords(log, st)
            st.ids = ids
            st.docs = _LazyList(n0, rec, 0)
            st.meta = MetaIndex.from_snapshot(info, arrays, _LazyList(n0, rec, 1))
            st.row = {i: r for r, i in enumerate(ids) if i is not None}
            start = int(info["log_size"])
        else:
            st.line_off = np.full(max(n, 1), -1, np.int64)
            start = 0
        # the log from `start`: every record after the snapshot (all of them without one)
        recs: Dict[int, tuple] = {}
        with open(log, "rb") as f:
            f.seek(start)
            off = start
            for line in f:
                if line.strip():
                    rec = json.loads(line)
                    if rec["row"] < n:   # records past meta.rows belong to an interrupted append
                        recs[rec["row"]] = (rec, off)
                off += len(line)
        ids_, row_, docs_, meta_ = st.ids, st.row, st.docs, st.meta
        while len(ids_) < n:
            ids_.append(None)
            docs_.append(None)
        for r in sorted(recs):
            rec, off = recs[r]
            _id = rec.get("id")
            old = ids_[r]
            if old is not None and row_.get(old) == r:
                del row_[old]
            ids_[r] = _id
            docs_[r] = rec.get("document") if _id is not None else None
            # the old metadata first: MetaIndex.set / remove read metas[r], which for a snapshot row
            # is parsed lazily through line_off[r] -- it must still point at the OLD record, or the
            # columns and tags only the old metadata had keep their codes on a live row
            if _id is not None:
                row_[_id] = r
                meta_.set(r, rec.get("metadata"))
            else:
                meta_.remove(r)
            st.line_off[r] = off
        self._index = multidev.new_dense_index(dim, device=self.device, capacity=max(n, 1))
        self._version += 1
        live = np.fromiter((i is not None for i in ids_), bool, count=n) if n else np.zeros(0, bool)
        if live.any():
            vecs = np.memmap(d / "vectors.f32", dtype=np.float32, mode="r", shape=(n, dim))
            slab = 1 << 16
            for s0 in range(0, n, slab):
                s1 = min(n, s0 + slab)
                lv = live[s0:s1]
                if lv.all():                 # contiguous: no gather copy
                    self._index.upsert(np.asarray(vecs[s0:s1], np.float32), np.arange(s0, s1, dtype=np.int64))
                elif lv.any():
                    part = np.nonzero(lv)[0] + s0
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

    def _line_off(self, n: int) -> np.ndarray:
        lo = self._st.line_off
        if lo is None or lo.shape[0] < n:
            new = np.full(max(n, 2 * (0 if lo is None else lo.shape[0]), 1024), -1, np.int64)
            if lo is not None:
                new[: lo.shape[0]] = lo
            self._st.line_off = lo = new
        return lo

    def _append(self, rows: np.ndarray, emb: Optional[np.ndarray]):
        """Autosave of one upsert (emb given) or delete: its rows' vectors and log records only.
        The snapshot is refreshed (no log rewrite) once the records appended since it outnumber
        half the rows, so a cold open replays at most that much of the log."""
        d = self._dir
        if d is None or self._index is None:
            return
        if not (d / "meta.json").exists():   # first write of this collection: the full layout
            self.save()
            return
        n = len(self._ids)
        if emb is not None:
            dim = self._index.dim
            with open(d / "vectors.f32", "r+b") as f:
                if f.seek(0, 2) < n * dim * 4:
                    f.truncate(n * dim * 4)
            mm = np.memmap(d / "vectors.f32", dtype=np.float32, mode="r+", shape=(n, dim))
            mm[rows] = emb
            mm.flush()
            del mm
        lo = self._line_off(n)
        blobs = [self._record(int(r)).encode("utf-8") for r in rows]
        with (d / "rows.log.jsonl").open("ab") as f:
            off = f.seek(0, 2)
            for r, b in zip(rows, blobs):
                lo[int(r)] = off
                off += len(b)
            f.write(b"".join(blobs))
        self._write_meta(d)
        self._st.tail += len(blobs)
        if self._st.tail > max(n * _SNAPSHOT_TAIL_FRAC, _SNAPSHOT_MIN_TAIL):
            self._write_snapshot(d)

    def _write_snapshot(self, d: Path):
        """snapshot/: ids, each row's latest log record offset and the metadata columns, valid for
        the log's first ``log_size`` bytes (same file: inode).  Skipped (and any old one removed)
        when the metadata cannot round-trip through JSON."""
        shutil.rmtree(d / "snapshot", ignore_errors=True)
        n = len(self._ids)
        ms = self._meta.snapshot()
        lo = self._line_off(n)
        if ms is None or (n and (lo[:n] < 0).any() and any(self._ids[r] is not None for r in np.nonzero(lo[:n] < 0)[0])):
            return
        info, arrays = ms
        if info["rows"] > n:   # (fewer: trailing rows never given metadata -- the load pads them)
            return
        st = os.stat(d / "rows.log.jsonl")
        info.update(version=1, log_size=st.st_size, log_ino=st.st_ino, ids_rows=n)
        arrays["line_off"] = lo[:n].copy()
        tmp = d / "snapshot.tmp"
        shutil.rmtree(tmp, ignore_errors=True)
        tmp.mkdir()
        for k, a in arrays.items():
            np.save(tmp / f"{k}.npy", a)
        (tmp / "ids.json").write_text(json.dumps(self._ids, ensure_ascii=False), encoding="utf-8")
        (tmp / "info.json").write_text(json.dumps(info, ensure_ascii=False), encoding="utf-8")
        os.replace(tmp, d / "snapshot")
        self._st.tail = 0

    @_locked
    def save(self):
        """Full write from the device copy + a compacted log (one record per row) + the snapshot."""
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
        del vecs
        os.replace(d / "vectors.tmp.f32", d / "vectors.f32")
        lo = self._line_off(n)
        off = 0
        with (d / "rows.tmp.jsonl").open("wb") as f:
            for r in range(n):
                b = self._record(r).encode("utf-8")
                lo[r] = off
                off += len(b)
                f.write(b)
        shutil.rmtree(d / "snapshot", ignore_errors=True)    # offsets of the old log
        os.replace(d / "rows.tmp.jsonl", d / "rows.log.jsonl")
        self._write_meta(d)
        self._write_snapshot(d)
        self._changed(True)

    # ---- upsert (vector_chroma.py:168-200) ---------------------------------
    @_locked
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
            self._index = multidev.new_dense_index(emb.shape[1], device=self.device, capacity=len(ids))
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

    @_locked
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

    @_locked
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

    @_locked
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
    @_locked
    def count(self) -> int:
        self._ensure_loaded()
        try:
            return 0 if self._index is None else self._index.live_count()
        except Exception:
            return 0

    @_locked
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

    def lock(self):
        """The collection's lock (reentrant): HybridRetriever holds it across a whole retrieve."""
        return self._st.lock

    # rows <-> ids for the batched device pipeline
    def id_of(self, row: int) -> Optional[str]:
        return self._ids[row]


ChromaVectorStore = GpuVectorStore
