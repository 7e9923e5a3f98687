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

Persistence: ``save`` writes the reference's JSONL catalog
unchanged (bm25.py:220-231) plus a binary sidecar ``<index_file>.cm/`` -- the
CSR term ids, document offsets, vocabulary and each record's byte offset in the
JSONL.  ``load`` checks the sidecar against the JSONL's size and mtime and, when
it matches, builds the device index straight from the memory-mapped CSR: no JSON
parsing, re-tokenisation or vocabulary mapping at open.  Records are parsed one
by one when a search returns them; metadata is parsed in full only when a
``where`` filter first needs it, and a mutation or ``save`` materializes every
record.  A missing or stale sidecar falls back to the reference's full parse.
"""
from __future__ import annotations

import contextlib
import dataclasses
import functools
import json
import os
import shutil
import threading
import weakref
from collections import OrderedDict
from dataclasses import dataclass
from pathlib import Path
from typing import Any, Dict, List, Mapping, Optional, Sequence

import numpy as np

from .. import engine, multidev
from .filters import MetaIndex, next_uid, settle_loaded
from .tokenize import _tokenize, detect_lang_tag


@dataclass
class _Entry:
    id: str
    text: str
    tokens: List[str]
    metadata: Dict[str, Any]
    term_ids: Optional[np.ndarray] = None


_SIDECAR_VERSION = 1


def _entry_of(rec: Mapping[str, Any]) -> _Entry:
    """bm25.py:240-245: one JSONL record -> _Entry."""
    return _Entry(id=rec["id"], text=rec.get("text", ""), tokens=list(rec.get("tokens", [])),
                  metadata=dict(rec.get("metadata", {})))


class _Catalog(dict):
    """id -> _Entry, in insertion order.  Opened from a sidecar, values start as JSONL line numbers
    and a record is parsed on first read (search results); ``values``/``items``/``materialize``
    parse every pending record in one sequential pass."""

    def __init__(self):
        super().__init__()
        self._src = None  # (jsonl path, line byte offsets, CSR term ids, doc offsets)
        self._fh = None
        self._lock = threading.Lock()   # the shared file object: seek + read as a unit

    def attach(self, path: Path, ids: Sequence[str], line_off, term_ids, doc_off) -> None:
        self._src = (path, line_off, term_ids, doc_off)
        for r, i in enumerate(ids):
            dict.__setitem__(self, i, r)

    @property
    def pending(self) -> bool:
        return self._src is not None

    def _finish(self, row: int, rec: Mapping[str, Any]) -> _Entry:
        _, _, terms, doc_off = self._src
        e = _entry_of(rec)
        e.term_ids = np.array(terms[int(doc_off[row]): int(doc_off[row + 1])], np.int32)
        return e

    def _parse(self, row: int) -> _Entry:
        path, line_off = self._src[0], self._src[1]
        with self._lock:
            if self._fh is None:
                self._fh = open(path, "rb")
            self._fh.seek(int(line_off[row]))
            blob = self._fh.read(int(line_off[row + 1] - line_off[row]))
        return self._finish(row, json.loads(blob))

    def __getitem__(self, key):
        v = dict.__getitem__(self, key)
        if type(v) is int:
            v = self._parse(v)
            dict.__setitem__(self, key, v)
        return v

    def get(self, key, default=None):
        return self[key] if key in self else default

    def pop(self, key, *default):
        v = dict.pop(self, key, *default)
        return self._parse(v) if type(v) is int and self._src is not None else v

    def materialize(self) -> None:
        if self._src is None:
            return
        pending = {v: k for k, v in dict.items(self) if type(v) is int}
        if pending:
            with open(self._src[0], "rb") as f:
                for row, line in enumerate(f):
                    key = pending.get(row)
                    if key is not None:
                        dict.__setitem__(self, key, self._finish(row, json.loads(line)))
        self.detach()

    def detach(self) -> None:
        with self._lock:
            if self._fh is not None:
                self._fh.close()
            self._src = self._fh = None

    def values(self):
        self.materialize()
        return dict.values(self)

    def items(self):
        self.materialize()
        return dict.items(self)

    def clear(self):
        self.detach()
        dict.clear(self)


class _BState:
    """One BM25 index's in-memory state (catalog, vocabulary, device index, metadata).  Instances
    loaded from one JSONL file share it while it matches the file (see BM25Store.load)."""

    def __init__(self):
        self.entries: Dict[str, _Entry] = _Catalog()
        self.id_list: List[str] = []
        self.vocab: Dict[str, int] = {}
        self.index: Optional[engine.BM25Index] = None
        self.meta = MetaIndex()
        self.dirty = True
        self.meta_dirty = True
        self.csr: Optional[tuple] = None   # persisted (term_ids, doc_off) to build from
        self.version = 0                   # bumped by every change of the document set
        self.uid = next_uid()              # identity in device caches (never reused)
        self.sig = None                    # the JSONL (+ sidecar) signature it was loaded from / saved to
        self.unsaved = False               # mutated since: private to its holder
        self.holders = weakref.WeakValueDictionary()   # id(store) -> store (dataclasses are unhashable)
        # the JSONL + sidecar this state last wrote or read (path, JSONL size / mtime, record count, line
        # and document offsets, term ids); while only new documents were appended since (append_only),
        # the next save appends their records instead of rewriting the file (same bytes either way)
        self.saved: Optional[dict] = None
        self.append_only = False
        # serialises the state's users (stores attached to it, threads): the device handle's search
        # staging and workspace are per handle (SURVEY §8(b) Threading)
        self.lock = threading.RLock()

    def clone(self) -> "_BState":
        """A private copy for a holder that mutates a shared state (the reference's instances are
        independent copies of the file): host tables copied, the device index and metadata rebuilt
        on demand."""
        st = _BState()
        cat = _Catalog()
        # the clone's own _Entry objects: term ids are filled in lazily against the holder's vocab
        # (_ensure_index / save), so shared entries would carry the other state's ids;
        # pending records (ints: not parsed yet) are parsed by each catalog on its own
        dict.update(cat, ((k, v if type(v) is int else dataclasses.replace(v))
                          for k, v in dict.items(self.entries)))
        cat._src = self.entries._src if isinstance(self.entries, _Catalog) else None
        st.entries = cat
        st.id_list = list(self.id_list)
        st.vocab = dict(self.vocab)
        st.csr = self.csr
        st.version = self.version
        return st


def _jsonl_sig(path) -> Optional[tuple]:
    try:
        s = os.stat(path)
        return (s.st_size, s.st_mtime_ns)
    except OSError:
        return None


def _file_sig(store) -> Optional[tuple]:
    out = []
    for p in (store.index_path, store.sidecar_dir / "meta.json"):
        try:
            s = os.stat(p)
            out.append((s.st_size, s.st_mtime_ns))
        except OSError:
            out.append(None)
    return tuple(out)


class _CatalogMetas(list):
    """MetaIndex.metas of a sidecar-opened store: row r's metadata dict, parsed from its JSONL
    record on first access (the same parse the catalog does for a search result)."""

    def __init__(self, n: int, cat: "_Catalog", ids: List[str]):
        super().__init__([None] * n)
        self.cat, self.ids, self.done = cat, ids, bytearray(n)

    def __getitem__(self, r):
        if isinstance(r, int) and r < len(self.done) and not self.done[r]:
            list.__setitem__(self, r, self.cat[self.ids[r]].metadata)
            self.done[r] = 1
        return list.__getitem__(self, r)

    def __setitem__(self, r, v):
        if isinstance(r, int) and r < len(self.done):
            self.done[r] = 1
        list.__setitem__(self, r, v)


def _load_meta_snapshot(side: Path, n: int, cat: "_Catalog", ids: List[str]) -> Optional[MetaIndex]:
    try:
        info = json.loads((side / "meta_info.json").read_text(encoding="utf-8"))
        arrays = {p.stem[len("meta_"):]: np.load(p) for p in side.glob("meta_*.npy")}
    except (OSError, ValueError):
        return None
    if int(info.get("rows", -1)) > n:
        return None
    m0 = int(info["rows"])
    if m0 < n:   # trailing documents without metadata columns: pad the arrays
        for k in [k for k in arrays if k.endswith("_py") or k.endswith("_ty")]:
            arrays[k] = np.concatenate([arrays[k], np.full(n - m0, -1, np.int32)])
        arrays["live"] = np.concatenate([arrays["live"], np.ones(n - m0, bool)])
        info["rows"] = n
    try:
        return MetaIndex.from_snapshot(info, arrays, _CatalogMetas(n, cat, ids))
    except (KeyError, ValueError):
        return None


_REGISTRY: "OrderedDict[tuple, _BState]" = OrderedDict()
_REGISTRY_MAX = 8
_REG_LOCK = threading.Lock()


def release_all() -> None:
    """Forget every registered BM25 state (freed once no store holds it)."""
    with _REG_LOCK:
        _REGISTRY.clear()


def _proxy(name: str):
    return property(lambda self: getattr(self._st, name), lambda self, v: setattr(self._st, name, v))


@contextlib.contextmanager
def _store_lock(store):
    """This store's lock, then its current state's: the first serialises the threads that use one
    BM25Store object (a copy on write swaps its state), the second the stores sharing a state."""
    with store._obj_lock:
        with store._st.lock:
            yield


def _locked(fn):
    @functools.wraps(fn)
    def run(self, *a, **kw):
        with _store_lock(self):
            return fn(self, *a, **kw)
    return run


@dataclass
class BM25Store:
    index_dir: Optional[Path] = Path("./indexes/bm25")
    index_file: str = "bm25_index.jsonl"
    device: Optional[int] = None

    _entries = _proxy("entries")
    _id_list = _proxy("id_list")
    _vocab = _proxy("vocab")
    _index = _proxy("index")
    _meta = _proxy("meta")
    _dirty = _proxy("dirty")
    _meta_dirty = _proxy("meta_dirty")
    _csr = _proxy("csr")
    _version = _proxy("version")
    _uid = _proxy("uid")

    def __post_init__(self):
        self._obj_lock = threading.RLock()
        self._st = _BState()
        self._st.holders[id(self)] = self

    def lock(self):
        """This store's locks as one context (HybridRetriever holds it across a whole retrieve)."""
        return _store_lock(self)

    def _set_state(self, st: "_BState") -> None:
        self._st.holders.pop(id(self), None)
        self._st = st
        st.holders[id(self)] = self

    def _registry_key(self):
        dev = engine.default_device() if self.device is None else int(self.device)
        return (str(Path(self.index_path).resolve()), dev, os.environ.get("CM_DEVICES", "") if self.device is None else "")

    def _mutating(self) -> None:
        """Before a change of the document set: a state other stores also hold is copied first."""
        if len(self._st.holders) > 1:
            self._set_state(self._st.clone())
        self._st.unsaved = True

    # ---------- core ops ----------
    def _term_ids(self, tokens: Sequence[str]) -> np.ndarray:
        v = self._vocab
        return np.fromiter((v.setdefault(t, len(v)) for t in tokens), dtype=np.int32, count=len(tokens))

    def _rebuild(self) -> None:
        """bm25.py:140-145: the reference rebuilds BM25Okapi here; it raises ZeroDivisionError when
        entries exist but every token list is empty.  We check that and defer the device build."""
        self._id_list = list(self._entries.keys())
        self._version += 1
        self._csr = None
        if self._entries and all(len(e.tokens) == 0 for e in self._entries.values()):
            raise ZeroDivisionError("float division by zero")
        self._dirty = self._meta_dirty = True

    def _ensure_index(self) -> None:
        if not self._dirty and self._index is not None:
            return
        if self._index is None:
            self._index = multidev.new_bm25_index(device=self.device)
        if self._csr is not None:  # opened from a sidecar: the persisted CSR is the index
            term_ids, doc_off = self._csr
            self._index.build(np.ascontiguousarray(term_ids), np.ascontiguousarray(doc_off),
                              max(len(self._vocab), 1))
            self._dirty = False
            return
        entries = [self._entries[i] for i in self._id_list]
        for e in entries:
            if e.term_ids is None:
                e.term_ids = self._term_ids(e.tokens)
        off = np.zeros(len(entries) + 1, np.int64)
        if entries:
            off[1:] = np.cumsum([e.term_ids.shape[0] for e in entries])
        flat = np.concatenate([e.term_ids for e in entries]) if off[-1] else np.zeros(0, np.int32)
        self._index.build(flat, off, max(len(self._vocab), 1))
        self._dirty = False

    def _ensure_meta(self) -> None:
        """Row-aligned metadata for where-filters (parses every record of a sidecar-opened store)."""
        if not self._meta_dirty:
            return
        self._meta = MetaIndex()
        for r, i in enumerate(self._id_list):
            self._meta.set(r, self._entries[i].metadata)
        self._meta_dirty = False

    @_locked
    def upsert_many(self, *, ids: Sequence[str], texts: Sequence[str], metadatas: Sequence[Mapping[str, Any]]) -> None:
        """bm25.py:147-166: language from metadata (or detected), tokenize, replace in place."""
        if not (len(ids) == len(texts) == len(metadatas)):
            raise ValueError("ids, texts, metadatas must have the same length")
        self._mutating()
        st = self._st
        n0 = len(self._entries)
        appended = []                  # (row, metadata) of documents new to the store, in insertion order
        for i, doc_id in enumerate(ids):
            text = texts[i] or ""
            meta = dict(metadatas[i] or {})
            lang = meta.get("language")
            if not lang or lang == "auto":
                lang = detect_lang_tag(text)
                meta["language"] = lang
            toks = _tokenize(text, lang_hint=lang)
            if doc_id in self._entries:  # replaced in place: the saved records are no longer a prefix
                st.append_only = False
                appended = None
            elif appended is not None:
                appended.append((n0 + len(appended), meta))
            self._entries[doc_id] = _Entry(id=doc_id, text=text, tokens=toks, metadata=meta)
        meta_ok = not self._meta_dirty
        self._rebuild()
        if meta_ok and appended is not None:   # the filter columns follow the appended rows
            for r, meta in appended:
                self._meta.set(r, meta)
            self._meta_dirty = False

    @_locked
    def delete_many(self, ids: Sequence[str]) -> None:
        self._mutating()
        self._st.append_only = False
        for doc_id in ids:
            self._entries.pop(doc_id, None)
        self._rebuild()

    # ---------- query ----------
    def _query_ids(self, query: str) -> List[int]:
        q_lang = detect_lang_tag(query)
        get = self._vocab.get          # (one proxy-property read, not one per token)
        return [get(t, -1) for t in _tokenize(query, lang_hint=q_lang)]

    def search(self, *, query: str, where: Optional[Mapping[str, Any]] = None, top_k: int = 8) -> List[Dict[str, Any]]:
        """bm25.py:175-212 on the GPU."""
        return self.search_batch(queries=[query], where=where, top_k=top_k)[0]

    @_locked
    def search_batch(self, *, queries: Sequence[str], where: Optional[Mapping[str, Any]] = None,
                     top_k: int = 8) -> List[List[Dict[str, Any]]]:
        """Many queries sharing one filter: one device launch (build-side addition)."""
        out: List[List[Dict[str, Any]]] = [[] for _ in queries]
        live = [i for i, q in enumerate(queries) if q.strip()]
        if not live or not self._entries:
            return out
        self._ensure_index()
        allow = None
        if where:  # device-evaluated filter; statistics follow it (Q2)
            self._ensure_meta()
            allow, n_cand = engine.where_bits(self._meta, where, "bm25", self._index.device)
        else:
            n_cand = len(self._id_list)
        if n_cand == 0:
            return out
        k = top_k if top_k >= 0 else n_cand + top_k      # python slice semantics of [:top_k]
        k = min(k, n_cand)
        if k <= 0:
            return out
        # k beyond the fused kernels' lists (cm_max_topk) runs the full-order device path
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

    @property
    def sidecar_dir(self) -> Path:
        return Path(self.index_dir) / (self.index_file + ".cm")

    @_locked
    def save(self) -> None:
        """bm25.py:220-231 (same JSONL records) + the binary sidecar of the device index."""
        if self.index_dir is None:
            return
        Path(self.index_dir).mkdir(parents=True, exist_ok=True)
        side = self.sidecar_dir
        if (side / "meta.json").exists():
            os.remove(side / "meta.json")  # the sidecar is invalid until rewritten below
        bs = self._st
        sv = bs.saved
        n_all = len(self._entries)
        append = (bs.append_only and sv is not None and sv["path"] == str(self.index_path)
                  and sv["n"] <= n_all and _jsonl_sig(self.index_path) == sv["sig"])
        r0 = sv["n"] if append else 0
        ids_new = self._id_list[r0:] if append else list(self._entries.keys())
        entries = [self._entries[i] for i in ids_new] if append else list(self._entries.values())
        line_off = np.zeros(len(entries) + 1, np.int64)
        doc_off = np.zeros(len(entries) + 1, np.int64)
        parts = []
        # the reference rewrites the whole JSONL (bm25.py:220-231); while only documents were appended
        # since this state's last save or load, the file is that file plus their records: append them
        with self.index_path.open("ab" if append else "wb") as f:
            base = f.tell() if append else 0
            for r, e in enumerate(entries):
                rec = {"id": e.id, "text": e.text, "tokens": e.tokens, "metadata": e.metadata}
                line = (json.dumps(rec, ensure_ascii=False) + "\n").encode("utf-8")
                f.write(line)
                line_off[r + 1] = line_off[r] + len(line)
                if e.term_ids is None:
                    e.term_ids = self._term_ids(e.tokens)
                parts.append(e.term_ids)
                doc_off[r + 1] = doc_off[r] + e.term_ids.shape[0]
        new_terms = np.concatenate(parts) if doc_off[-1] else np.zeros(0, np.int32)
        if append:
            line_off = np.concatenate([sv["line_off"], line_off[1:] + base])
            doc_off = np.concatenate([sv["doc_off"], doc_off[1:] + sv["doc_off"][-1]])
            terms = np.concatenate([np.asarray(sv["term_ids"], np.int32), new_terms])
            ids_all = self._id_list
        else:
            terms = new_terms
            ids_all = [e.id for e in entries]
        st = self.index_path.stat()
        tmp = Path(str(side) + ".tmp")
        shutil.rmtree(tmp, ignore_errors=True)
        tmp.mkdir(parents=True)
        np.save(tmp / "term_ids.npy", terms)
        np.save(tmp / "doc_off.npy", doc_off)
        np.save(tmp / "line_off.npy", line_off)
        vocab = [None] * len(self._vocab)
        for t, i in self._vocab.items():
            vocab[i] = t
        (tmp / "vocab.json").write_text(json.dumps(vocab, ensure_ascii=False), encoding="utf-8")
        (tmp / "ids.json").write_text(json.dumps(list(ids_all), ensure_ascii=False), encoding="utf-8")
        # the where-filter columns (filters.MetaIndex), so a sidecar open can filter without parsing
        # every record's metadata (10M records: ~100 s of JSON before the first filtered search)
        self._ensure_meta()
        ms = self._meta.snapshot()
        if ms is not None and ms[0]["rows"] <= len(ids_all):
            info, arrays = ms
            for k, a in arrays.items():
                np.save(tmp / f"meta_{k}.npy", a)
            (tmp / "meta_info.json").write_text(json.dumps(info, ensure_ascii=False), encoding="utf-8")
        (tmp / "meta.json").write_text(json.dumps({
            "version": _SIDECAR_VERSION, "docs": len(ids_all), "postings": int(doc_off[-1]),
            "jsonl_size": st.st_size, "jsonl_mtime_ns": st.st_mtime_ns}), encoding="utf-8")
        shutil.rmtree(side, ignore_errors=True)
        os.replace(tmp, side)
        del terms    # (the saved arrays are kept memory-mapped from the new sidecar, not in RAM)
        bs.saved = dict(path=str(self.index_path), sig=(st.st_size, st.st_mtime_ns), n=len(ids_all),
                        line_off=np.load(side / "line_off.npy", mmap_mode="r"),
                        doc_off=np.load(side / "doc_off.npy", mmap_mode="r"),
                        term_ids=np.load(side / "term_ids.npy", mmap_mode="r"))
        bs.append_only = True
        # the state matches the files again: later load()s of this index attach to it
        st = self._st
        st.sig, st.unsaved = _file_sig(self), False
        with _REG_LOCK:
            key = self._registry_key()
            _REGISTRY[key] = st
            _REGISTRY.move_to_end(key)
            while len(_REGISTRY) > _REGISTRY_MAX:
                _REGISTRY.popitem(last=False)

    def _sidecar_valid(self) -> Optional[dict]:
        try:
            meta = json.loads((self.sidecar_dir / "meta.json").read_text(encoding="utf-8"))
            st = self.index_path.stat()
        except (OSError, ValueError):
            return None
        if (meta.get("version") != _SIDECAR_VERSION or meta.get("jsonl_size") != st.st_size
                or meta.get("jsonl_mtime_ns") != st.st_mtime_ns):
            return None
        return meta

    def _load_sidecar(self, meta: dict) -> bool:
        side = self.sidecar_dir
        try:
            ids = json.loads((side / "ids.json").read_text(encoding="utf-8"))
            vocab = json.loads((side / "vocab.json").read_text(encoding="utf-8"))
            term_ids = np.load(side / "term_ids.npy", mmap_mode="r")
            doc_off = np.load(side / "doc_off.npy", mmap_mode="r")
            line_off = np.load(side / "line_off.npy", mmap_mode="r")
        except (OSError, ValueError):
            return False
        n = len(ids)
        if (n != meta["docs"] or doc_off.shape[0] != n + 1 or line_off.shape[0] != n + 1
                or term_ids.shape[0] != int(doc_off[-1]) or len(set(ids)) != n):
            return False
        if n and int(doc_off[-1]) == 0:
            raise ZeroDivisionError("float division by zero")  # bm25.py:145 on an all-empty corpus
        cat = _Catalog()
        cat.attach(self.index_path, ids, line_off, term_ids, doc_off)
        self._entries = cat
        self._vocab = {t: i for i, t in enumerate(vocab)}
        self._id_list = list(ids)
        self._version += 1
        self._csr = (term_ids, doc_off)
        self._dirty = self._meta_dirty = True
        self._st.saved = dict(path=str(self.index_path), sig=(meta["jsonl_size"], meta["jsonl_mtime_ns"]), n=n,
                              line_off=line_off, doc_off=doc_off, term_ids=term_ids)
        self._st.append_only = True
        meta = _load_meta_snapshot(side, n, cat, self._id_list)
        if meta is not None:   # filter columns restored; a row's metadata dict is parsed on demand
            self._meta, self._meta_dirty = meta, False
        return True

    @_locked
    def load(self) -> None:
        """bm25.py:233-248; through the sidecar when it matches the JSONL.  A state this process
        already holds for the same file -- loaded or saved by another BM25Store, unchanged since on
        disk and in memory -- is attached instead of re-read: the reference's per-call
        ``BM25Store.load_or_create`` (rag/pipeline/rag.py:532) then costs two stat() calls, not a
        corpus parse and index build."""
        if self.index_dir is None or not self.index_path.exists():
            self._set_state(_BState())
            self._rebuild()
            return
        key, sig = self._registry_key(), _file_sig(self)
        with _REG_LOCK:
            st = _REGISTRY.get(key)
            if st is not None and not st.unsaved and st.sig == sig:
                _REGISTRY.move_to_end(key)
                self._set_state(st)
                return
        self._set_state(_BState())
        meta = self._sidecar_valid()
        if not (meta is not None and self._load_sidecar(meta)):
            with self.index_path.open("r", encoding="utf-8") as f:
                for line in f:
                    if not line.strip():
                        continue
                    rec = json.loads(line)
                    self._entries[rec["id"]] = _entry_of(rec)
            self._rebuild()
        settle_loaded()
        st = self._st
        st.sig, st.unsaved = sig, False
        with _REG_LOCK:
            _REGISTRY[key] = st
            _REGISTRY.move_to_end(key)
            while len(_REGISTRY) > _REGISTRY_MAX:
                _REGISTRY.popitem(last=False)

    @classmethod
    def load_or_create(cls, index_dir: str | Path = "./indexes/bm25") -> "BM25Store":
        store = cls(index_dir=Path(index_dir))
        store.load()
        return store
