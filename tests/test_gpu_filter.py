"""GPU: cm_filter_eval bit-exact against the numpy masks (bm25_mask / chroma_mask,
which follow rag/retrieval/bm25.py:79-107 and Chroma's where semantics), ragged sizes included."""
import random

import numpy as np
import pytest

from test_filter_program import random_bm25_where, random_chroma_where, random_meta

pytestmark = pytest.mark.gpu


def _words(t):
    return t.cpu().numpy().view(np.uint32)


@pytest.mark.parametrize("n", [1, 31, 33, 64, 65, 257, 5000])
def test_filter_kernel_matches_masks(n):
    from classmate_hip import engine
    from classmate_hip.retrieval import filters as F
    rng = random.Random(n)
    mi = F.MetaIndex()
    for r in range(n):
        mi.set(r, random_meta(rng))
    for r in rng.sample(range(n), n // 10):
        mi.remove(r)
    for _ in range(40):
        for sem, w in (("bm25", random_bm25_where(rng)), ("chroma", random_chroma_where(rng))):
            mask = mi.bm25_mask(w) if sem == "bm25" else mi.chroma_mask(w)
            prog = mi.bm25_program(w) if sem == "bm25" else mi.chroma_program(w)
            bits, cnt = engine.filter_bits(prog)
            assert np.array_equal(_words(bits), F.pack_bits(mask)), (sem, w)
            assert cnt == int(mask.sum())


def test_filter_kernel_large_and_cache_refresh():
    from classmate_hip import engine
    from classmate_hip.retrieval import filters as F
    n = 2_000_003
    mi = F.MetaIndex()
    mi._ensure(n)
    rng = np.random.default_rng(0)
    col = F._Column(mi._cap)                      # bulk-load one column the way set() would
    col.py_map = {f"c{i}": i for i in range(50)}
    col.ty_map = {F._typed(f"c{i}"): i for i in range(50)}
    codes = rng.integers(0, 50, n).astype(np.int32)
    col.py[:n] = col.ty[:n] = codes
    mi.cols["course"] = col
    mi.live[:n] = True
    mi.metas = [None] * n
    for w in ({"course": "c7"}, {"course": {"$nin": ["c1", "c2"]}}, {"$or": [{"course": "c3"}, {"course": "c4"}]}):
        bits, cnt = engine.filter_bits(mi.chroma_program(w))
        mask = mi.chroma_mask(w)
        assert np.array_equal(_words(bits), F.pack_bits(mask)) and cnt == int(mask.sum())
    mi.set(5, {"course": "c7"})                   # metadata change -> device copies refreshed
    bits, cnt = engine.filter_bits(mi.chroma_program({"course": "c7"}))
    assert (_words(bits)[0] >> 5) & 1 and cnt == int(mi.chroma_mask({"course": "c7"}).sum())
