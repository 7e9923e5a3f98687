"""Shared pytest setup: markers, import paths, fixture loading."""
import json
import os
import sys
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parents[1]
PKG_ROOT = REPO / "classmate-rag_amd"
for p in (str(REPO), str(PKG_ROOT), str(REPO / "tests" / "golden")):
    if p not in sys.path:
        sys.path.insert(0, p)
os.environ.setdefault("PYTHONDONTWRITEBYTECODE", "1")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")
    config.addinivalue_line("markers", "slow: larger CPU cases")


@pytest.fixture(scope="session")
def golden():
    return json.loads((REPO / "tests" / "golden" / "hybrid_1k.json").read_text())


@pytest.fixture(scope="session")
def corpus(golden):
    from synth import make_corpus, make_queries
    cfg = golden["config"]
    ids, texts, metas, emb = make_corpus(cfg["n"], cfg["dim"], seed=cfg["corpus_seed"])
    qtexts, qvecs, _ = make_queries(texts, emb, nq=cfg["nq"], seed=cfg["query_seed"])
    assert qtexts == golden["query_texts"], "synthetic generator drifted from the goldens"
    return dict(ids=ids, texts=texts, metas=metas, emb=emb, qtexts=qtexts, qvecs=qvecs)
