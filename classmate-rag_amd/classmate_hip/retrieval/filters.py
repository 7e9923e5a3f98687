"""Metadata where-filters evaluated into row bitmaps for the device kernels.

Two semantics, both from the reference:

* Chroma ``where`` (what ``build_where_filter``, rag/retrieval/vector_chroma.py:45-78,
  produces): typed equality per key (bool True != int 1), ``$and``/``$or``,
  ``$eq``/``$ne``/``$in``/``$nin``; a row lacking the key never matches.
* BM25 ``_matches_filter`` (rag/retrieval/bm25.py:79-107): Python equality of
  ``meta.get(f)`` for the six simple fields *whenever the key is present in
  where, even when its value is None* (quirk Q4), ``tags: {"$contains": ...}``
  over a ``tags`` list (returning before the simple fields are looked at), and
  ``$and`` recursion (ignoring sibling keys).

Metadata is kept column-wise (per key an int32 code array + value->code dicts).
``bm25_program`` / ``chroma_program`` compile a where clause into a postfix
``FilterProgram`` over those code columns that ``cm_filter_eval`` runs in HBM
(``engine.filter_bits``), one lane per row, straight into the
uint32 allow bitmap the scan kernels read.  Leaves the columns cannot express
-- BM25 ``tags.$contains`` row sets, ``$gt``-style comparisons, unhashable
values -- are evaluated here and enter the program as bitmaps.
``bm25_mask`` / ``chroma_mask`` are the same semantics in numpy (bool[n]).
"""
from __future__ import annotations

import itertools
import re
from typing import Any, Dict, List, Mapping, Optional

import numpy as np

SIMPLE_FIELDS = ("course", "unit", "language", "doc_type", "author", "semester")
_MISSING = -1
_UNHASHABLE = -2


def _slug_tag(t: str) -> str:
    s = re.sub(r"[^a-z0-9]+", "_", (t or "").lower().strip())
    return s.strip("_")


def _parse_tags(obj) -> List[str]:
    if not obj:
        return []
    vals = [str(x) for x in obj] if isinstance(obj, (list, tuple)) else str(obj).split(",")
    return [v.strip() for v in vals if v.strip()]


def build_where_filter(meta_like: Mapping[str, Any]) -> Optional[Dict[str, Any]]:
    """Chroma where from CLI-style filters (vector_chroma.py:45-78)."""
    if not meta_like:
        return None
    clauses: List[Dict[str, Any]] = []
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
        slug = _slug_tag(t)
        if slug:
            clauses.append({f"tag_{slug}": True})
    if not clauses:
        return None
    return clauses[0] if len(clauses) == 1 else {"$and": clauses}


def pack_bits(mask: np.ndarray) -> np.ndarray:
    """bool[n] -> uint32[ceil(n/32)], bit (r & 31) of word r >> 5 (little-endian)."""
    n = mask.shape[0]
    b = np.packbits(mask.astype(np.uint8), bitorder="little")
    pad = (-b.shape[0]) % 4
    if pad:
        b = np.concatenate([b, np.zeros(pad, np.uint8)])
    words = b.view("<u4").astype(np.uint32)
    need = (n + 31) // 32
    if words.shape[0] < need:
        words = np.concatenate([words, np.zeros(need - words.shape[0], np.uint32)])
    return words[:max(need, 1)] if need else np.zeros(1, np.uint32)


def _typed(v):
    return (type(v).__name__, v)


# identities of MetaIndex / BM25Store objects for device caches: never reused (id() of a freed
# object is, and a fresh MetaIndex restarts its version at 0 -- ADVICE r4)
_UIDS = itertools.count(1)


def next_uid() -> int:
    return next(_UIDS)


def settle_loaded() -> None:
    """After a cold open: move the objects it just built out of the young generations.  A 10M-row
    open creates a few 10M-entry id lists as single container allocations, too few to trigger a
    collection, so they sat in generation 0 until the first request's gen-0 collection traversed
    them: a one-time ~15 ms stall inside that request (the construct-then-retrieve p99 at 10M,
    bench.py's gc diagnostics).  One gen-1 collection here traverses them during the open instead
    and promotes them to the oldest generation."""
    import gc
    if gc.isenabled():
        gc.collect(1)


class _Column:
    __slots__ = ("py", "ty", "py_map", "ty_map", "n_odd")

    def __init__(self, cap: int):
        self.n_odd = 0  # rows holding an unhashable value (evaluated row by row)
        self.py = np.full(cap, _MISSING, np.int32)
        self.ty = np.full(cap, _MISSING, np.int32)
        self.py_map: Dict[Any, int] = {}
        self.ty_map: Dict[Any, int] = {}

    def grow(self, cap: int):
        if cap > self.py.shape[0]:
            for name in ("py", "ty"):
                old = getattr(self, name)
                new = np.full(cap, _MISSING, np.int32)
                new[: old.shape[0]] = old
                setattr(self, name, new)


class MetaIndex:
    """Row-aligned metadata with vectorised where-evaluation."""

    def __init__(self):
        self.metas: List[Optional[Mapping[str, Any]]] = []
        self.live = np.zeros(0, bool)
        self.cols: Dict[str, _Column] = {}
        self.tags: Dict[Any, set] = {}
        self._cap = 0
        self.version = 0          # bumped by every set/remove: device copies compare against it
        self.uid = next_uid()     # this object's identity in device caches (never reused)
        self._dev_cache = None    # engine.filter_bits' device copies of columns / live bits

    def __len__(self):
        return len(self.metas)

    def _ensure(self, n: int):
        if n > self._cap:
            cap = max(n, 2 * self._cap, 1024)
            live = np.zeros(cap, bool)
            live[: self.live.shape[0]] = self.live
            self.live = live
            for c in self.cols.values():
                c.grow(cap)
            self._cap = cap
        while len(self.metas) < n:
            self.metas.append(None)

    def set(self, row: int, meta: Optional[Mapping[str, Any]]):
        self._ensure(row + 1)
        if self.live[row]:
            self.remove(row)
        self.version += 1
        self.metas[row] = meta
        self.live[row] = True
        for key, v in (meta or {}).items():
            col = self.cols.get(key)
            if col is None:
                col = self.cols[key] = _Column(self._cap)
            try:
                col.py[row] = col.py_map.setdefault(v, len(col.py_map))
                col.ty[row] = col.ty_map.setdefault(_typed(v), len(col.ty_map))
            except TypeError:  # unhashable value: evaluated row by row
                col.py[row] = col.ty[row] = _UNHASHABLE
                col.n_odd += 1
        tags = (meta or {}).get("tags")
        if isinstance(tags, (list, tuple, set)):
            for t in tags:
                try:
                    self.tags.setdefault(t, set()).add(row)
                except TypeError:
                    pass

    # ---- snapshot (vector_store.py's cold open) ----------------------------
    _JSON_SCALARS = (str, int, float, bool, type(None))

    def snapshot(self):
        """(info, arrays) describing the columns, tags and live bits -- JSON-able info plus numpy
        arrays -- or None when a value cannot be restored exactly from JSON (map keys that are not
        JSON scalars).  Rows holding unhashable values keep their marker code; they are evaluated
        from ``metas`` row by row, as before."""
        n = len(self.metas)
        ok = self._JSON_SCALARS
        cols, arrays = [], {"live": np.asarray(self.live[:n], bool)}
        for i, (key, c) in enumerate(self.cols.items()):
            if not isinstance(key, str):
                return None
            if not all(type(v) in ok for v in c.py_map) or not all(type(t[1]) in ok for t in c.ty_map):
                return None
            cols.append({"key": key, "n_odd": c.n_odd, "py": [[v, code] for v, code in c.py_map.items()],
                         "ty": [[t[0], t[1], code] for t, code in c.ty_map.items()]})
            arrays[f"col{i}_py"] = np.asarray(c.py[:n], np.int32)
            arrays[f"col{i}_ty"] = np.asarray(c.ty[:n], np.int32)
        tags = []
        off = [0]
        rows = []
        for t, rs in self.tags.items():
            if type(t) not in ok:
                return None
            tags.append(t)
            rows.append(np.fromiter(sorted(rs), np.int64, count=len(rs)))
            off.append(off[-1] + len(rs))
        arrays["tag_off"] = np.asarray(off, np.int64)
        arrays["tag_rows"] = np.concatenate(rows) if rows else np.zeros(0, np.int64)
        return {"rows": n, "cols": cols, "tags": tags}, arrays

    @classmethod
    def from_snapshot(cls, info, arrays, metas) -> "MetaIndex":
        """The inverse of ``snapshot``; ``metas`` is the row-aligned metadata list (a lazily
        parsed one for a cold open)."""
        m = cls()
        n = int(info["rows"])
        cap = max(n, 1024)
        m._cap = cap
        m.metas = metas
        m.live = np.zeros(cap, bool)
        m.live[:n] = arrays["live"][:n]
        for i, c in enumerate(info["cols"]):
            col = _Column(cap)
            col.py[:n] = arrays[f"col{i}_py"][:n]
            col.ty[:n] = arrays[f"col{i}_ty"][:n]
            col.py_map = {v: code for v, code in c["py"]}
            col.ty_map = {(tn, v): code for tn, v, code in c["ty"]}
            col.n_odd = int(c.get("n_odd", 0))
            m.cols[c["key"]] = col
        off, rows = arrays["tag_off"], arrays["tag_rows"]
        for j, t in enumerate(info["tags"]):
            m.tags[t] = set(rows[off[j]: off[j + 1]].tolist())
        return m

    def remove(self, row: int):
        if row >= len(self.metas) or not self.live[row]:
            return
        self.version += 1
        meta = self.metas[row] or {}
        for key in meta:
            col = self.cols.get(key)
            if col is not None:
                if col.py[row] == _UNHASHABLE:
                    col.n_odd -= 1
                col.py[row] = col.ty[row] = _MISSING
        tags = meta.get("tags")
        if isinstance(tags, (list, tuple, set)):
            for t in tags:
                try:
                    self.tags.get(t, set()).discard(row)
                except TypeError:
                    pass
        self.metas[row] = None
        self.live[row] = False

    # ---- evaluation helpers --------------------------------------------
    def _n(self):
        return len(self.metas)

    def _slow(self, pred) -> np.ndarray:
        return np.array([bool(self.live[r]) and pred(self.metas[r] or {}) for r in range(self._n())], bool)

    def _eq_py(self, key: str, value) -> np.ndarray:
        """rows with meta.get(key) == value (Python equality; missing key == None)."""
        n = self._n()
        col = self.cols.get(key)
        if col is None:
            m = np.ones(n, bool) if value is None else np.zeros(n, bool)
            return m & self.live[:n]
        codes = col.py[:n]
        try:
            c = col.py_map.get(value, None)
        except TypeError:
            return self._slow(lambda meta: meta.get(key) == value)
        m = (codes == c) if c is not None else np.zeros(n, bool)
        if value is None:
            m = m | (codes == _MISSING)
        if col.n_odd:
            odd = np.nonzero(codes == _UNHASHABLE)[0]
            for r in odd:
                m[r] = (self.metas[r] or {}).get(key) == value
        return m & self.live[:n]

    def _eq_typed(self, key: str, value) -> np.ndarray:
        n = self._n()
        col = self.cols.get(key)
        if col is None:
            return np.zeros(n, bool)
        try:
            c = col.ty_map.get(_typed(value), None)
        except TypeError:
            return np.zeros(n, bool)
        if c is None:
            return np.zeros(n, bool)
        return (col.ty[:n] == c) & self.live[:n]

    def _has(self, key: str) -> np.ndarray:
        n = self._n()
        col = self.cols.get(key)
        if col is None:
            return np.zeros(n, bool)
        return (col.ty[:n] != _MISSING) & self.live[:n]

    # ---- public: BM25 semantics (bm25.py:79-107) ----------------------
    def bm25_mask(self, where: Optional[Mapping[str, Any]]) -> np.ndarray:
        n = self._n()
        if not where:
            return self.live[:n].copy()
        if "$and" in where:
            m = self.live[:n].copy()
            for clause in where["$and"]:
                m &= self.bm25_mask(clause)
            return m
        if "tags" in where and isinstance(where["tags"], dict) and "$contains" in where["tags"]:
            t = where["tags"]["$contains"]
            if not t:
                return self.live[:n].copy()
            want = {t} if isinstance(t, str) else set(t)
            m = self.live[:n].copy()
            for tag in want:
                rows = np.fromiter(self.tags.get(tag, ()), np.int64)
                hit = np.zeros(n, bool)
                hit[rows] = True
                m &= hit
            return m
        m = self.live[:n].copy()
        for f in SIMPLE_FIELDS:
            if f in where:
                m &= self._eq_py(f, where[f])
        return m

    # ---- public: Chroma semantics ---------------------------------------
    def chroma_mask(self, where: Optional[Mapping[str, Any]]) -> np.ndarray:
        n = self._n()
        m = self.live[:n].copy()
        if not where:
            return m
        for key, cond in where.items():
            if key == "$and":
                for c in cond:
                    m &= self.chroma_mask(c)
            elif key == "$or":
                acc = np.zeros(n, bool)
                for c in cond:
                    acc |= self.chroma_mask(c)
                m &= acc
            elif isinstance(cond, dict):
                if len(cond) != 1:
                    raise ValueError(f"Expected operator expression with one operator, got {cond}")
                (op, arg), = cond.items()
                if op == "$eq":
                    m &= self._eq_typed(key, arg)
                elif op == "$ne":
                    m &= self._has(key) & ~self._eq_typed(key, arg)
                elif op == "$in":
                    acc = np.zeros(n, bool)
                    for a in arg:
                        acc |= self._eq_typed(key, a)
                    m &= acc
                elif op == "$nin":
                    acc = self._has(key)
                    for a in arg:
                        acc &= ~self._eq_typed(key, a)
                    m &= acc
                elif op in ("$gt", "$gte", "$lt", "$lte"):
                    m &= self._slow(lambda meta, k=key, o=op, a=arg: _cmp(meta, k, o, a))
                else:
                    raise ValueError(f"Unsupported where operator {op}")
            else:
                m &= self._eq_typed(key, cond)
        return m


    # ---- compiled programs (same semantics, evaluated by cm_filter_eval) ----
    def _eq_py_prog(self, P: "FilterProgram", key: str, value) -> None:
        col = self.cols.get(key)
        if col is None:
            P.const(value is None)
            return
        try:
            c = col.py_map.get(value, None)
        except TypeError:
            P.mask(self._eq_py(key, value))
            return
        if col.n_odd:
            P.mask(self._eq_py(key, value))
            return
        if c is None and value is not None:
            P.const(False)
            return
        if c is not None:
            P.eq(key, "py", c)
        if value is None:
            P.eq(key, "py", _MISSING)
            if c is not None:
                P.op(FOP_OR)

    def _eq_typed_prog(self, P: "FilterProgram", key: str, value) -> None:
        col = self.cols.get(key)
        try:
            c = None if col is None else col.ty_map.get(_typed(value), None)
        except TypeError:
            c = None
        if c is None:
            P.const(False)
        else:
            P.eq(key, "ty", c)

    def _has_prog(self, P: "FilterProgram", key: str) -> None:
        if key not in self.cols:
            P.const(False)
        else:
            P.ne(key, "ty", _MISSING)

    def _bm25_prog(self, P: "FilterProgram", where) -> None:
        if not where:
            P.const(True)
            return
        if "$and" in where:
            P.const(True)
            for clause in where["$and"]:
                self._bm25_prog(P, clause)
                P.op(FOP_AND)
            return
        if "tags" in where and isinstance(where["tags"], dict) and "$contains" in where["tags"]:
            t = where["tags"]["$contains"]
            P.const(True)
            if t:
                n = self._n()
                for tag in ({t} if isinstance(t, str) else set(t)):
                    hit = np.zeros(n, bool)
                    hit[np.fromiter(self.tags.get(tag, ()), np.int64)] = True
                    P.mask(hit)
                    P.op(FOP_AND)
            return
        P.const(True)
        for f in SIMPLE_FIELDS:
            if f in where:
                self._eq_py_prog(P, f, where[f])
                P.op(FOP_AND)

    def _chroma_prog(self, P: "FilterProgram", where) -> None:
        P.const(True)
        if not where:
            return
        for key, cond in where.items():
            if key == "$and":
                P.const(True)
                for c in cond:
                    self._chroma_prog(P, c)
                    P.op(FOP_AND)
            elif key == "$or":
                P.const(False)
                for c in cond:
                    self._chroma_prog(P, c)
                    P.op(FOP_OR)
            elif isinstance(cond, dict):
                if len(cond) != 1:
                    raise ValueError(f"Expected operator expression with one operator, got {cond}")
                (op, arg), = cond.items()
                if op == "$eq":
                    self._eq_typed_prog(P, key, arg)
                elif op == "$ne":
                    self._has_prog(P, key)
                    self._eq_typed_prog(P, key, arg)
                    P.op(FOP_NOT)
                    P.op(FOP_AND)
                elif op == "$in":
                    P.const(False)
                    for a in arg:
                        self._eq_typed_prog(P, key, a)
                        P.op(FOP_OR)
                elif op == "$nin":
                    self._has_prog(P, key)
                    for a in arg:
                        self._eq_typed_prog(P, key, a)
                        P.op(FOP_NOT)
                        P.op(FOP_AND)
                elif op in ("$gt", "$gte", "$lt", "$lte"):
                    P.mask(self._slow(lambda meta, k=key, o=op, a=arg: _cmp(meta, k, o, a)))
                else:
                    raise ValueError(f"Unsupported where operator {op}")
            else:
                self._eq_typed_prog(P, key, cond)
            P.op(FOP_AND)

    def bm25_program(self, where: Optional[Mapping[str, Any]]) -> "FilterProgram":
        """bm25_mask as a device program: live AND the clause."""
        P = FilterProgram(self)
        P.live()
        self._bm25_prog(P, where)
        P.op(FOP_AND)
        return P

    def chroma_program(self, where: Optional[Mapping[str, Any]]) -> "FilterProgram":
        """chroma_mask as a device program: live AND the clause."""
        P = FilterProgram(self)
        P.live()
        self._chroma_prog(P, where)
        P.op(FOP_AND)
        return P


# cm_filter_eval opcodes (include/classmate_hip.h)
FOP_EQ, FOP_NE, FOP_BITS, FOP_TRUE, FOP_FALSE, FOP_AND, FOP_OR, FOP_NOT = range(1, 9)
MAX_OPS, MAX_SOURCES = 64, 16


class FilterProgram:
    """Postfix program for cm_filter_eval: ops (opcode, a, b); column slots name (key, "py"|"ty")
    code arrays of the MetaIndex, bitmap slots are the live bits ("live") or host-evaluated masks."""

    def __init__(self, meta: MetaIndex):
        self.meta = meta
        self.n = meta._n()
        self.ops: List[tuple] = []
        self.cols: List[tuple] = []
        self.bits: List[Any] = []
        self._depth = self.max_depth = 0

    def _push(self, op, a=0, b=0):
        self.ops.append((op, a, b))
        self._depth += 1
        self.max_depth = max(self.max_depth, self._depth)

    def op(self, op):
        self.ops.append((op, 0, 0))
        if op in (FOP_AND, FOP_OR):
            self._depth -= 1

    def _col(self, key, kind) -> int:
        if (key, kind) not in self.cols:
            self.cols.append((key, kind))
        return self.cols.index((key, kind))

    def eq(self, key, kind, code):
        self._push(FOP_EQ, self._col(key, kind), int(code))

    def ne(self, key, kind, code):
        self._push(FOP_NE, self._col(key, kind), int(code))

    def const(self, v: bool):
        self._push(FOP_TRUE if v else FOP_FALSE)

    def live(self):
        if "live" not in self.bits:
            self.bits.append("live")
        self._push(FOP_BITS, self.bits.index("live"))

    def mask(self, m: np.ndarray):
        self.bits.append(np.asarray(m, bool)[: self.n])
        self._push(FOP_BITS, len(self.bits) - 1)

    @property
    def fits_device(self) -> bool:
        return (len(self.ops) <= MAX_OPS and len(self.cols) <= MAX_SOURCES and len(self.bits) <= MAX_SOURCES
                and self.max_depth <= 32)

    def column(self, slot: int) -> np.ndarray:
        key, kind = self.cols[slot]
        return getattr(self.meta.cols[key], kind)[: self.n]

    def bitmap(self, slot: int) -> np.ndarray:
        b = self.bits[slot]
        return self.meta.live[: self.n] if isinstance(b, str) else b


def _cmp(meta, key, op, arg) -> bool:
    if key not in meta or not isinstance(meta[key], (int, float)) or isinstance(meta[key], bool):
        return False
    v = meta[key]
    return {"$gt": v > arg, "$gte": v >= arg, "$lt": v < arg, "$lte": v <= arg}[op]
