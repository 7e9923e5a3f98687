"""Generate golden fixtures by running the REFERENCE's own retrieval code.

Runs only in the build container (``/root/reference`` does not exist on the GPU
box).  It imports ``rag.retrieval.bm25`` / ``rag.retrieval.fusion`` /
``rag.retrieval.vector_chroma`` from ``/root/reference`` with ``sys.modules``
stubs for the third-party packages that are not installed here
(SURVEY.md §8c): ``dotenv`` (no-op), ``sentence_transformers`` (dummy class),
``langdetect`` (``detect -> "en"``), ``rank_bm25`` (``BM25Okapi`` = the
published 0.2.2 algorithm restated in ``oracle/ref_semantics.py``).

Outputs (data only — ids, scores, orders — never reference source):
  tests/golden/hybrid_1k.json

Usage:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_goldens.py
"""
from __future__ import annotations

import json
import os
import sys
import types
from pathlib import Path

sys.dont_write_bytecode = True
os.environ["PYTHONDONTWRITEBYTECODE"] = "1"
HERE = Path(__file__).resolve().parent
REPO = HERE.parents[1]
REF = Path("/root/reference")
sys.path.insert(0, str(HERE))
sys.path.insert(0, str(REPO))

import numpy as np  # noqa: E402

from synth import make_corpus, make_queries  # noqa: E402
from oracle import ref_semantics as orc  # noqa: E402


def _install_stubs():
    dotenv = types.ModuleType("dotenv")
    dotenv.load_dotenv = lambda *a, **k: False
    dotenv.find_dotenv = lambda *a, **k: ""
    sys.modules["dotenv"] = dotenv
    st = types.ModuleType("sentence_transformers")

    class SentenceTransformer:  # never instantiated by the goldens
        def __init__(self, *a, **k):
            raise RuntimeError("stub")
    st.SentenceTransformer = SentenceTransformer
    sys.modules["sentence_transformers"] = st
    ld = types.ModuleType("langdetect")
    ld.detect = lambda text: "en"

    class DetectorFactory:
        seed = 0
    ld.DetectorFactory = DetectorFactory
    sys.modules["langdetect"] = ld
    rb = types.ModuleType("rank_bm25")
    rb.BM25Okapi = orc.BM25Okapi
    sys.modules["rank_bm25"] = rb


class PresetEmbedder:
    def __init__(self, table):
        self.table = table

    def encode_queries(self, qs):
        return np.stack([self.table[q] for q in qs]).astype(np.float32)


def main():
    _install_stubs()
    sys.path.insert(0, str(REF))
    from rag.retrieval.bm25 import BM25Store, _tokenize  # noqa: E402
    from rag.retrieval.fusion import HybridRetriever, _mmr_order, rrf_fuse  # noqa: E402
    from rag.retrieval.vector_chroma import build_where_filter  # noqa: E402

    cfg = dict(n=1000, dim=768, corpus_seed=1234, nq=16, query_seed=99, k=10, pool=24)
    ids, texts, metas, emb = make_corpus(cfg["n"], cfg["dim"], seed=cfg["corpus_seed"])
    qtexts, qvecs, targets = make_queries(texts, emb, nq=cfg["nq"], seed=cfg["query_seed"])

    store = BM25Store(index_dir=Path("/tmp/cm_golden_unused"))
    store.upsert_many(ids=ids, texts=texts, metadatas=metas)
    vstore = orc.ExactVectorStore(ids, texts, metas, emb)
    embedder = PresetEmbedder({q: v for q, v in zip(qtexts, qvecs)})
    retr = HybridRetriever(vector_store=vstore, bm25_store=store, embedder=embedder,
                           k_vector=cfg["k"], k_bm25=cfg["k"])

    # Filters: plain; a DocumentMetadata.to_dict()-shaped dict that keeps None keys (quirk Q4);
    # a tag filter (Chroma tag_<slug> vs BM25 ignoring list tags).
    filter_cases = {
        "none": None,
        "course_cs101": {"course": "cs101", "unit": None, "author": None, "semester": None,
                         "source_path": None, "created_at": None},
        "course_only": {"course": "math201"},
        "tags_exam": {"course": "cs101", "tags": ["exam"]},
        "lang_en_doctype": {"language": "en", "doc_type": "pptx"},
    }

    out = {"config": cfg, "tokenize": [], "bm25": {}, "dense": {}, "mmr": [], "rrf": [],
           "retrieve": {}, "where": {}, "misc": {}}
    # tokenizer cases
    tok_cases = ["Hello, World! the quick w123 brown fox", "È già l'università di Roma e la casa",
                 "a b c dd EE ff1gg", "", "ÀÖØöøÿ ×÷ naïve café"]
    for t in tok_cases:
        out["tokenize"].append({"text": t, "en": _tokenize(t, "en"), "it": _tokenize(t, "it")})

    for name, f in filter_cases.items():
        out["where"][name] = build_where_filter(f) if f else None
        out["bm25"][name] = []
        for q in qtexts:
            res = store.search(query=q, where=f, top_k=cfg["k"])
            out["bm25"][name].append([[r["id"], r["score"]] for r in res])
        out["retrieve"][name] = []
        for q in qtexts:
            res = retr.retrieve(question=q, filters=f, top_k=cfg["k"], hybrid=True)
            out["retrieve"][name].append([[r["id"], r["scores"]["fused"], r["scores"]["vector_distance"],
                                           r["scores"]["bm25_score"]] for r in res])
        cw = build_where_filter(f) if f else None
        out["dense"][name] = []
        for qv in qvecs:
            res = vstore.query(query_embeddings=qv, where=cw, top_k=cfg["pool"], include_embeddings=False)
            out["dense"][name].append([[r["id"], r["distance"]] for r in res])

    # hybrid=False and top_k larger than lists
    out["retrieve"]["none_vector_only"] = []
    for q in qtexts:
        res = retr.retrieve(question=q, filters=None, top_k=12, hybrid=False)
        out["retrieve"]["none_vector_only"].append(
            [[r["id"], r["scores"]["fused"], r["scores"]["vector_distance"], r["scores"]["bm25_score"]] for r in res])

    # MMR on each query's dense pool
    for qv in qvecs:
        res = vstore.query(query_embeddings=qv, top_k=cfg["pool"], include_embeddings=True)
        cids = [r["id"] for r in res]
        cand = np.stack([r["embedding"] for r in res])
        out["mmr"].append({"pool": cids, "order": _mmr_order(q=qv, cands=cand, ids=cids, k=cfg["k"])})

    # rrf_fuse cases
    rl = [["a", "b", "c", "d"], ["c", "e", "a"]]
    out["rrf"].append({"lists": rl, "weights": None, "rrf_k": 60, "out": rrf_fuse(rank_lists=rl)})
    out["rrf"].append({"lists": rl, "weights": [0.7, 1.3], "rrf_k": 10,
                       "out": rrf_fuse(rank_lists=rl, weights=[0.7, 1.3], rrf_k=10)})
    try:
        rrf_fuse(rank_lists=rl, weights=[1.0])
        out["misc"]["rrf_bad_weights"] = "no-error"
    except ValueError as e:
        out["misc"]["rrf_bad_weights"] = f"ValueError: {e}"

    # Edge cases
    out["misc"]["empty_query"] = store.search(query="   ", top_k=5)
    out["misc"]["stopword_only_query"] = [[r["id"], r["score"]] for r in store.search(query="the and of", top_k=5)]
    out["misc"]["topk_gt_n_filtered"] = [[r["id"], r["score"]] for r in
                                         store.search(query=qtexts[0], where={"course": "cs101", "unit": "u1",
                                                                              "doc_type": "pptx"}, top_k=500)]
    small = BM25Store(index_dir=Path("/tmp/cm_golden_unused"))
    try:
        small.upsert_many(ids=["x1", "x2"], texts=["the and", "12 34"], metadatas=[{"language": "en"}] * 2)
        out["misc"]["all_empty_docs"] = "no-error"
    except ZeroDivisionError as e:
        out["misc"]["all_empty_docs"] = f"ZeroDivisionError: {e}"
    small2 = BM25Store(index_dir=Path("/tmp/cm_golden_unused"))
    small2.upsert_many(ids=["a", "b", "c"], texts=["alpha beta", "beta gamma", "gamma delta"],
                       metadatas=[{"language": "en", "tags": ["x", "y"]}, {"language": "en", "tags": ["x"]},
                                  {"language": "en"}])
    small2.upsert_many(ids=["a"], texts=["alpha alpha zeta"], metadatas=[{"language": "en", "tags": ["y"]}])
    small2.delete_many(["b"])
    small2.upsert_many(ids=["b"], texts=["beta beta beta"], metadatas=[{"language": "en"}])
    out["misc"]["reorder_after_delete"] = [[r["id"], r["score"]] for r in small2.search(query="beta alpha gamma",
                                                                                        top_k=5)]
    out["misc"]["tags_contains"] = [[r["id"], r["score"]] for r in
                                    small2.search(query="alpha", where={"tags": {"$contains": "y"}}, top_k=5)]

    out["query_texts"] = qtexts
    out["query_targets"] = [int(t) for t in targets]
    # consistency: the oracle restatement must agree with the reference outputs
    path = HERE / "hybrid_1k.json"
    path.write_text(json.dumps(out, ensure_ascii=False, indent=0))
    print("wrote", path, path.stat().st_size, "bytes")


if __name__ == "__main__":
    main()
