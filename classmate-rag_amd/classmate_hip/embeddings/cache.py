"""Disk cache in front of an embedder — drop-in for ``rag/embeddings/cache.py``.

Same on-disk format as the reference so an existing ``indexes/emb_cache`` tree is reused
unchanged: one ``<root>/<model>/<mode>/<sha1(text.strip())>.npy`` fp32 vector per text,
``mode`` in {"query", "passage"} (cache.py:67-77).  Behaviour mirrored:

* root = ``cache_dir`` or ``$EMB_CACHE_DIR`` or ``./indexes/emb_cache`` (cache.py:48);
* model sub-directory from ``base.model.name_or_path`` else ``base.model_name`` else
  ``unknown-model``, sanitised to ``[A-Za-z0-9._-]`` (cache.py:52-59); a base embedder running
  below the reference's fp32 (``dtype`` bfloat16, the opt-in fast path) gets ``__bfloat16``
  appended, so its vectors never mix with fp32 ones under the same key.  fp32 (the default
  since round 2, and the reference's precision) keeps the reference's unsuffixed directory, so
  an existing reference cache is reused; a directory written by a round-1 build of this package
  (whose default was bf16, unsuffixed) must be cleared -- this build marks the directories it
  writes with ``.classmate_hip_dtype`` and refuses an unsuffixed directory marked otherwise;
* a file that fails to load is a miss (cache.py:100-106); write errors are swallowed (cache.py:136-141);
* all misses of one call go to the base embedder as ONE batch, in input order, duplicates
  included (cache.py:132-133) — with the HIP E5 path that is one padded forward + the K6
  mean-pool/L2 kernel instead of one forward per text;
* an empty input raises ``ValueError`` from ``np.vstack`` like the reference's ``_fill``
  (cache.py:116-124).
"""
from __future__ import annotations

import hashlib
import os
from pathlib import Path
from typing import Iterable, List, Optional, Tuple

import numpy as np

_MODES = ("query", "passage")


def _text_key(text: str) -> str:
    """cache.py:24-30: sha1 of the stripped UTF-8 text (undecodable characters dropped)."""
    return hashlib.sha1((text or "").strip().encode("utf-8", "ignore")).hexdigest()


def _model_dirname(base) -> str:
    """cache.py:52-59."""
    model = getattr(base, "model", None)
    if model is not None and hasattr(model, "name_or_path"):
        name = str(model.name_or_path)
    else:
        name = getattr(base, "model_name", "unknown-model")
    dt = str(getattr(base, "dtype", "") or "")
    if dt and not dt.endswith("float32"):          # e.g. torch.bfloat16 -> "__bfloat16"
        name = f"{name}__{dt.rsplit('.', 1)[-1]}"
    return "".join(c if (c.isalnum() or c in "-_.") else "_" for c in name)


class CachingEmbedder:
    """Wrap ``base`` (``encode_queries`` / ``encode_passages``) with the reference's .npy cache."""

    def __init__(self, base, cache_dir: Optional[str] = None) -> None:
        self.base = base
        root = cache_dir or os.getenv("EMB_CACHE_DIR") or "./indexes/emb_cache"
        self.root = Path(root).expanduser().resolve()
        self.model_dir = self.root / _model_dirname(base)
        self.model_dir.mkdir(parents=True, exist_ok=True)
        dt = str(getattr(base, "dtype", "") or "float32").rsplit(".", 1)[-1]
        marker = self.model_dir / ".classmate_hip_dtype"
        try:
            prev = marker.read_text().strip() if marker.exists() else None
            if prev is not None and prev != dt:
                raise ValueError(f"embedding cache {self.model_dir} holds {prev} vectors, this embedder is {dt}")
            if prev is None:
                marker.write_text(dt + "\n")
        except OSError:
            pass

    def _key_path(self, mode: str, text: str) -> Path:
        return self.model_dir / mode / f"{_text_key(text)}.npy"

    def _lookup(self, mode: str, items: List[str]) -> Tuple[List[Optional[np.ndarray]], List[int], List[Path]]:
        (self.model_dir / mode).mkdir(parents=True, exist_ok=True)
        hits: List[Optional[np.ndarray]] = []
        misses: List[int] = []
        paths: List[Path] = []
        for i, t in enumerate(items):
            fp = self._key_path(mode, t)
            vec = None
            if fp.exists():
                try:
                    vec = np.load(fp).astype(np.float32, copy=False)  # allow_pickle stays False
                except Exception:
                    vec = None
            hits.append(vec)
            if vec is None:
                misses.append(i)
                paths.append(fp)
        return hits, misses, paths

    def _encode(self, mode: str, texts: Iterable[str]) -> np.ndarray:
        assert mode in _MODES
        items = list(texts)
        hits, misses, paths = self._lookup(mode, items)
        if misses:
            fn = self.base.encode_queries if mode == "query" else self.base.encode_passages
            fresh = fn([items[i] for i in misses])
            for j, fp in enumerate(paths):
                try:
                    fp.parent.mkdir(parents=True, exist_ok=True)
                    np.save(fp, fresh[j])
                except Exception:
                    pass
            it = iter(fresh)
            hits = [next(it) if h is None else h for h in hits]
        # np.vstack([]) raises ValueError, as the reference does for an empty call
        return np.vstack(hits).astype(np.float32, copy=False)

    def encode_queries(self, queries: Iterable[str]) -> np.ndarray:
        return self._encode("query", queries)

    def encode_queries_dev(self, queries: Iterable[str]):
        """encode_queries with the result left on the device, for the device retrieval chain
        (retrieval/device_batch.py): hits come from their .npy files, the misses go to the base
        embedder's device path as ONE batch, as in ``_encode``.  The misses' files are written from a
        non-blocking device-to-host copy by ``flush_pending`` -- the chain calls it once its results
        are on the host, and the next call here flushes anything left -- so the query encode is not
        serialised behind a host round trip.  None when the base embedder has no device path."""
        import torch
        base_dev = getattr(self.base, "encode_queries_dev", None)
        if base_dev is None:
            return None
        self.flush_pending()
        items = list(queries)
        if not items:
            raise ValueError("need at least one array to concatenate")   # np.vstack([]), as _encode
        hits, misses, paths = self._lookup("query", items)
        if not misses:
            return torch.from_numpy(np.vstack(hits).astype(np.float32, copy=False)).to(self.base.device)
        fresh = base_dev([items[i] for i in misses])
        host = torch.empty(fresh.shape, dtype=torch.float32, pin_memory=True)
        host.copy_(fresh, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(fresh.device))
        self._pending.append((host, ev, paths))
        if len(misses) == len(items):
            return fresh
        out = torch.empty((len(items), fresh.shape[1]), dtype=torch.float32, device=fresh.device)
        out[torch.as_tensor(misses, device=fresh.device)] = fresh
        hit_idx = [i for i, h in enumerate(hits) if h is not None]
        out[torch.as_tensor(hit_idx, device=fresh.device)] = torch.from_numpy(
            np.vstack([hits[i] for i in hit_idx]).astype(np.float32, copy=False)).to(fresh.device)
        return out

    @property
    def _pending(self) -> list:
        return self.__dict__.setdefault("_pending_writes", [])

    def flush_pending(self) -> None:
        """Write the .npy files of encode_queries_dev's misses (errors swallowed, as ``_encode``)."""
        pend, self.__dict__["_pending_writes"] = self._pending, []
        for host, ev, paths in pend:
            ev.synchronize()
            arr = host.numpy()
            for j, fp in enumerate(paths):
                try:
                    fp.parent.mkdir(parents=True, exist_ok=True)
                    np.save(fp, arr[j])
                except Exception:
                    pass

    def encode_passages(self, texts: Iterable[str]) -> np.ndarray:
        return self._encode("passage", texts)
