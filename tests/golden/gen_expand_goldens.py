"""Generate golden fixtures for neighbour expansion and the embedding cache by running the
REFERENCE's own ``rag.retrieval.expand`` / ``rag.embeddings.cache`` / ``rag.utils.ids``.

Runs only in the build container (``/root/reference`` is absent on the GPU box); the same
``sys.modules`` stubs as ``gen_goldens.py``.  Outputs (data only: inputs, ids, scores, file
names) go to ``tests/golden/expand_cache.json``.

Usage:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_expand_goldens.py
"""
from __future__ import annotations

import json
import os
import sys
import tempfile
from pathlib import Path

sys.dont_write_bytecode = True
HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE))
sys.path.insert(0, str(HERE.parents[1]))

import numpy as np  # noqa: E402

from gen_goldens import REF, _install_stubs  # noqa: E402

FILES = ["/data/algebra/lecture01.pdf", "/data/algebra/lecture02.pdf", "/data/physics/notes.md"]


def _catalog(sid):
    """Synthetic BM25 JSONL catalog: 3 files x 2 pages x 6 chunks, a few blank texts."""
    recs = []
    for fi, sp in enumerate(FILES):
        course = ["algebra", "algebra", None][fi]
        unit = ["u1", None, None][fi]
        for page in (1, 2):
            for c in range(6):
                cid = sid(source_path=sp, page=page, chunk_index=c, course=course, unit=unit)
                text = "" if (fi, page, c) in {(0, 1, 3), (2, 2, 0)} else f"text {fi} {page} {c}"
                if (fi, page, c) == (1, 2, 4):
                    text = "   "
                meta = {"source_path": sp, "page": page, "chunk_id": c, "course": course, "unit": unit,
                        "language": "en"}
                recs.append({"id": cid, "text": text, "tokens": text.split(), "metadata": meta})
    return recs


def main():
    _install_stubs()
    sys.path.insert(0, str(REF))
    from rag.utils.ids import stable_chunk_id
    from rag.retrieval import expand as rexp
    from rag.embeddings.cache import CachingEmbedder

    recs = _catalog(stable_chunk_id)
    by_key = {(r["metadata"]["source_path"], r["metadata"]["page"], r["metadata"]["chunk_id"]): r for r in recs}

    def hit(sp, page, c, score, **over):
        r = by_key[(sp, page, c)]
        meta = dict(r["metadata"], **over)
        return {"id": r["id"], "document": r["text"], "score": score, "metadata": meta}

    results = [
        hit(FILES[0], 1, 2, 0.9), hit(FILES[0], 1, 4, 0.8), hit(FILES[1], 2, 5, 0.7),
        hit(FILES[2], 1, 0, 0.65), hit(FILES[0], 1, 2, 0.6),  # repeated seed
        {"id": "", "document": "x", "score": 0.5, "metadata": {}},  # empty id
        {"id": "cm_orphan", "document": "o", "score": 0.4, "metadata": {"source_path": FILES[2]}},  # no page
        hit(FILES[2], 2, 1, 0.35, chunk_id="one"),  # non-integer chunk_id
        hit(FILES[1], 1, 0, 0.3), hit(FILES[2], 2, 3, None),
        {"id": "cm_scores", "document": "s", "scores": {"fused": 0.1}, "metadata": {}},
    ]
    cases = []
    with tempfile.TemporaryDirectory() as td:
        cwd = os.getcwd()
        os.chdir(td)
        try:
            Path("indexes/bm25").mkdir(parents=True)
            with open("indexes/bm25/bm25_index.jsonl", "w", encoding="utf-8") as f:
                for r in recs:
                    f.write(json.dumps(r, ensure_ascii=False) + "\n")
                f.write("not json\n\n")
            for radius in (0, 1, 2):
                for cap in (None, 0, 1, 2, 3):
                    for pen in (0.001, 0.25):
                        out = rexp.expand_with_neighbors(results, radius=radius, max_per_doc=cap,
                                                         neighbor_penalty=pen)
                        cases.append({"radius": radius, "max_per_doc": cap, "neighbor_penalty": pen,
                                      "expected": out})
        finally:
            os.chdir(cwd)

    ids = [{"source_path": sp, "page": p, "chunk_index": c, "course": co, "unit": u,
            "id": stable_chunk_id(source_path=sp, page=p, chunk_index=c, course=co, unit=u)}
           for sp, p, c, co, u in [(FILES[0], 1, 0, None, None), (FILES[0], 1, -1, "algebra", "u1"),
                                   ("/x/ü ñ.pdf", 0, 7, "", "unit")]]

    # embedding cache: file layout and hit/miss behaviour
    class Base:
        model_name = "intfloat/multilingual-e5-base"
        calls = []

        def _enc(self, texts, off):
            Base.calls.append(list(texts))
            return np.stack([np.full(4, off + len(t), np.float32) for t in texts])

        def encode_queries(self, qs):
            return self._enc(qs, 1000.0)

        def encode_passages(self, ps):
            return self._enc(ps, 2000.0)

    texts = ["alpha", "  alpha  ", "beta", "ünïcode text", "alpha", ""]
    with tempfile.TemporaryDirectory() as td:
        ce = CachingEmbedder(Base(), cache_dir=td)
        q1 = ce.encode_queries(texts)
        q2 = ce.encode_queries(["beta", "gamma"])
        p1 = ce.encode_passages(["alpha"])
        files = sorted(str(p.relative_to(td)) for p in Path(td).rglob("*.npy"))
        model_dir = str(ce.model_dir.relative_to(Path(td).resolve()))
        try:
            ce.encode_queries([])
            empty = "ok"
        except Exception as e:  # noqa: BLE001
            empty = type(e).__name__
    cache = {"texts": texts, "q1": q1.tolist(), "q2": q2.tolist(), "p1": p1.tolist(), "files": files,
             "model_dir": model_dir, "base_calls": Base.calls, "empty_call": empty}

    out = {"catalog": recs, "results": results, "cases": cases, "stable_ids": ids, "cache": cache}
    (HERE / "expand_cache.json").write_text(json.dumps(out, indent=0, ensure_ascii=False))
    print("wrote", HERE / "expand_cache.json", len(cases), "expansion cases")


if __name__ == "__main__":
    main()
