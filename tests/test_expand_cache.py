"""Neighbour expansion (rag/retrieval/expand.py) and CachingEmbedder (rag/embeddings/cache.py)
against goldens produced by the reference itself (tests/golden/gen_expand_goldens.py)."""
import json
import os
from pathlib import Path

import numpy as np
import pytest

from classmate_hip.embeddings.cache import CachingEmbedder
from classmate_hip.retrieval.expand import apply_expansion_and_diversity, expand_with_neighbors, stable_chunk_id

GOLD = json.loads((Path(__file__).parent / "golden" / "expand_cache.json").read_text())


def _write_catalog(root: Path) -> Path:
    p = root / "indexes" / "bm25" / "bm25_index.jsonl"
    p.parent.mkdir(parents=True)
    with p.open("w", encoding="utf-8") as f:
        for r in GOLD["catalog"]:
            f.write(json.dumps(r, ensure_ascii=False) + "\n")
        f.write("not json\n\n")
    return p


def test_stable_chunk_id_matches_reference():
    for c in GOLD["stable_ids"]:
        got = stable_chunk_id(source_path=c["source_path"], page=c["page"], chunk_index=c["chunk_index"],
                              course=c["course"], unit=c["unit"])
        assert got == c["id"]


def test_expansion_default_catalog_path(tmp_path, monkeypatch):
    _write_catalog(tmp_path)
    monkeypatch.chdir(tmp_path)
    for c in GOLD["cases"]:
        got = expand_with_neighbors(GOLD["results"], radius=c["radius"], max_per_doc=c["max_per_doc"],
                                    neighbor_penalty=c["neighbor_penalty"])
        assert got == c["expected"], (c["radius"], c["max_per_doc"], c["neighbor_penalty"])


def test_expansion_missing_catalog_keeps_seeds(tmp_path, monkeypatch):
    monkeypatch.chdir(tmp_path)
    got = expand_with_neighbors(GOLD["results"], radius=2)
    zero = next(c for c in GOLD["cases"] if c["radius"] == 0 and c["max_per_doc"] is None)
    assert got == zero["expected"]


@pytest.mark.parametrize("reopen", [False, True])
def test_expansion_over_resident_bm25_store(tmp_path, reopen):
    """catalog=BM25Store: same output as the reference's JSONL re-read, incl. a sidecar-opened store."""
    from classmate_hip.retrieval import BM25Store
    recs = GOLD["catalog"]
    st = BM25Store(index_dir=str(tmp_path / "bm25"))
    st.upsert_many(ids=[r["id"] for r in recs], texts=[r["text"] for r in recs],
                   metadatas=[r["metadata"] for r in recs])
    if reopen:
        from classmate_hip.retrieval import bm25
        st.save()
        bm25.release_all()                  # a new process: the sidecar-opened store, not the attached state
        st = BM25Store.load_or_create(tmp_path / "bm25")
        assert st._entries.pending
    for c in GOLD["cases"]:
        got = expand_with_neighbors(GOLD["results"], radius=c["radius"], max_per_doc=c["max_per_doc"],
                                    neighbor_penalty=c["neighbor_penalty"], catalog=st)
        assert got == c["expected"]


def test_apply_expansion_env_knobs(tmp_path, monkeypatch):
    path = _write_catalog(tmp_path)
    want = {(c["radius"], c["max_per_doc"]): c["expected"] for c in GOLD["cases"] if c["neighbor_penalty"] == 0.001}
    monkeypatch.delenv("NEIGHBOR_RADIUS", raising=False)
    monkeypatch.delenv("DOC_DIVERSITY_CAP", raising=False)
    monkeypatch.delenv("ENABLE_NEIGHBOR_EXPANSION", raising=False)
    assert apply_expansion_and_diversity(GOLD["results"], catalog=path) == want[(1, 3)]
    monkeypatch.setenv("NEIGHBOR_RADIUS", "2")
    monkeypatch.setenv("DOC_DIVERSITY_CAP", "2")
    assert apply_expansion_and_diversity(GOLD["results"], catalog=path) == want[(2, 2)]
    monkeypatch.setenv("ENABLE_NEIGHBOR_EXPANSION", "no")
    assert apply_expansion_and_diversity(GOLD["results"], catalog=path) == want[(0, 2)]


class _Base:
    model_name = "intfloat/multilingual-e5-base"

    def __init__(self):
        self.calls = []

    def _enc(self, texts, off):
        self.calls.append(list(texts))
        return np.stack([np.full(4, off + len(t), np.float32) for t in texts])

    def encode_queries(self, qs):
        return self._enc(qs, 1000.0)

    def encode_passages(self, ps):
        return self._enc(ps, 2000.0)


def test_caching_embedder_matches_reference(tmp_path):
    g = GOLD["cache"]
    base = _Base()
    ce = CachingEmbedder(base, cache_dir=str(tmp_path))
    q1 = ce.encode_queries(g["texts"])
    q2 = ce.encode_queries(["beta", "gamma"])
    p1 = ce.encode_passages(["alpha"])
    assert q1.dtype == np.float32 and q1.tolist() == g["q1"]
    assert q2.tolist() == g["q2"] and p1.tolist() == g["p1"]
    assert base.calls == g["base_calls"]
    files = sorted(str(p.relative_to(tmp_path)) for p in tmp_path.rglob("*.npy"))
    assert files == g["files"]
    assert str(ce.model_dir.relative_to(tmp_path.resolve())) == g["model_dir"]
    with pytest.raises(ValueError):
        ce.encode_queries([])


def test_caching_embedder_corrupt_file_is_a_miss(tmp_path, monkeypatch):
    monkeypatch.delenv("EMB_CACHE_DIR", raising=False)
    monkeypatch.chdir(tmp_path)
    base = _Base()
    ce = CachingEmbedder(base)  # default root ./indexes/emb_cache
    assert ce.root == (tmp_path / "indexes" / "emb_cache").resolve()
    ce.encode_passages(["x"])
    fp = next(tmp_path.rglob("*.npy"))
    fp.write_bytes(b"garbage")
    out = ce.encode_passages(["x"])
    assert base.calls == [["x"], ["x"]] and out.tolist() == [[2001.0] * 4]
    monkeypatch.setenv("EMB_CACHE_DIR", str(tmp_path / "env"))
    assert CachingEmbedder(base).root == (tmp_path / "env").resolve()


def test_caching_embedder_model_dir_from_hf_model(tmp_path):
    class M:
        name_or_path = "/ckpt/e5 base@v2"

    class B(_Base):
        model = M()
    assert CachingEmbedder(B(), cache_dir=str(tmp_path)).model_dir.name == "_ckpt_e5_base_v2"
    assert CachingEmbedder(object(), cache_dir=str(tmp_path)).model_dir.name == "unknown-model"
    assert os.path.isdir(tmp_path / "unknown-model")
