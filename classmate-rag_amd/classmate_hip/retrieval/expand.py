"""Neighbour expansion + per-document diversity cap — drop-in for ``rag/retrieval/expand.py``
 and ``rag.utils.ids.stable_chunk_id``.

The step after retrieval: every hit pulls in the chunks ``chunk_id ± r`` of the same page
of the same file, then a per-``source_path`` cap keeps breadth over depth.

Behaviour mirrored from the reference:

* neighbour ids are ``stable_chunk_id(source_path, page, chunk_id + d, course, unit)``
  — ``cm_`` + blake2b-128 of ``"<resolved path>|page|index|course|unit"`` (ids.py:17-29);
  hits without ``source_path``/``page``/``chunk_id`` (or non-integer ones) get none
  (expand.py:64-76);
* seeds keep their input order, empty and repeated ids are skipped; each seed's neighbours
  follow it in ``d = -r..-1, 1..r`` order, only when present in the catalog with non-blank
  text, at ``score - neighbor_penalty`` (expand.py:118-140);
* the cap counts ``str(metadata.get("source_path") or "")`` in output order (expand.py:143-151).

Difference in HOW, not WHAT: the reference re-parses the whole BM25 JSONL catalog on every
call (expand.py:36-56, O(corpus) per question).  Here the catalog is the ``BM25Store`` already
resident in the process (``catalog=store``): a neighbour is one dict probe into its id table and,
for a store opened from the binary sidecar, one seek+parse of that single JSONL line.  Without a
store the reference's file path is read, as the reference does.
"""
from __future__ import annotations

import json
import os
from hashlib import blake2b
from pathlib import Path
from typing import Any, Dict, List, Mapping, Optional, Sequence, Tuple

_BM25_JSONL = Path("./indexes/bm25/bm25_index.jsonl")


def stable_chunk_id(*, source_path, page: int, chunk_index: int, course: Optional[str] = None,
                    unit: Optional[str] = None, prefix: str = "cm_") -> str:
    """rag/utils/ids.py:17-29."""
    key = f"{Path(source_path).resolve()}|{page}|{chunk_index}|{course or ''}|{unit or ''}"
    return prefix + blake2b(key.encode("utf-8"), digest_size=16).hexdigest()


def _jsonl_catalog(path: Path) -> Dict[str, Tuple[str, Dict[str, Any]]]:
    """expand.py:36-56: id -> (text, metadata); malformed lines and empty ids are skipped."""
    out: Dict[str, Tuple[str, Dict[str, Any]]] = {}
    if not path.exists():
        return out
    with path.open("r", encoding="utf-8", errors="ignore") as f:
        for line in f:
            line = line.strip()
            if not line:
                continue
            try:
                rec = json.loads(line)
                cid = str(rec.get("id") or "")
                if cid:
                    out[cid] = (str(rec.get("text") or ""), dict(rec.get("metadata") or {}))
            except Exception:
                continue
    return out


class _StoreCatalog:
    """Lookup view over a live BM25Store (its _Catalog parses sidecar-backed rows lazily)."""

    def __init__(self, store):
        self._entries = store._entries

    def get(self, cid: str):
        e = self._entries.get(cid)
        if e is None:
            return None
        return str(e.text or ""), dict(e.metadata or {})


def _neighbor_ids(meta: Mapping[str, Any], *, radius: int) -> List[str]:
    """expand.py:59-89."""
    sp, page, cid = meta.get("source_path"), meta.get("page"), meta.get("chunk_id")
    if sp is None or page is None or cid is None:
        return []
    try:
        page, cid = int(page), int(cid)
    except Exception:
        return []
    course, unit = meta.get("course") or None, meta.get("unit") or None
    return [stable_chunk_id(source_path=str(sp), page=page, chunk_index=cid + d, course=course, unit=unit)
            for d in range(-radius, radius + 1) if d != 0]


def expand_with_neighbors(results: Sequence[Mapping[str, Any]], *, radius: int = 1,
                          max_per_doc: Optional[int] = None, neighbor_penalty: float = 0.001,
                          catalog=None) -> List[Dict[str, Any]]:
    """expand.py:92-153.  ``catalog``: a BM25Store (resident lookup), a JSONL path, or None for the
    reference's ``./indexes/bm25/bm25_index.jsonl``."""
    if catalog is None or isinstance(catalog, (str, os.PathLike)):
        table = _jsonl_catalog(Path(catalog) if catalog is not None else _BM25_JSONL)
    elif hasattr(catalog, "_entries"):
        table = _StoreCatalog(catalog)
    else:
        table = catalog  # any mapping id -> (text, metadata)

    seen = set()
    out: List[Dict[str, Any]] = []
    for r in results:
        rid = str(r.get("id") or "")
        if not rid or rid in seen:
            continue
        seen.add(rid)
        sc = float(r.get("score") or 0.0)
        meta = dict(r.get("metadata") or {})
        out.append({"id": rid, "document": str(r.get("document") or ""), "score": sc, "metadata": meta})
        if radius <= 0:
            continue
        for nid in _neighbor_ids(meta, radius=radius):
            if nid in seen:
                continue
            hit = table.get(nid)
            if hit is None:
                continue
            ntext, nmeta = hit
            if not (ntext or "").strip():
                continue
            out.append({"id": nid, "document": ntext, "score": sc - neighbor_penalty, "metadata": nmeta})
            seen.add(nid)

    if max_per_doc and max_per_doc > 0:
        counts: Dict[str, int] = {}
        kept = []
        for it in out:
            sp = str(it["metadata"].get("source_path") or "")
            if counts.get(sp, 0) < max_per_doc:
                kept.append(it)
                counts[sp] = counts.get(sp, 0) + 1
        out = kept
    return out


def apply_expansion_and_diversity(results: Sequence[Mapping[str, Any]], *, catalog=None,
                                  radius: Optional[int] = None, cap: Optional[int] = None,
                                  enable: Optional[bool] = None) -> List[Dict[str, Any]]:
    """rag/pipeline/rag.py:429-455: env knobs ENABLE_NEIGHBOR_EXPANSION (true), NEIGHBOR_RADIUS (1),
    DOC_DIVERSITY_CAP (3); explicit arguments stand in for the reference's config overrides.
    With expansion off the cap is still applied."""
    if enable is None:
        enable = os.getenv("ENABLE_NEIGHBOR_EXPANSION", "true").strip().lower() in {"1", "true", "yes"}
    radius = int(os.getenv("NEIGHBOR_RADIUS", "1")) if radius is None else int(radius)
    cap = int(os.getenv("DOC_DIVERSITY_CAP", "3")) if cap is None else int(cap)
    if enable and radius > 0:
        return expand_with_neighbors(results, radius=radius, max_per_doc=cap, catalog=catalog)
    return expand_with_neighbors(results, radius=0, max_per_doc=cap, catalog=catalog)
