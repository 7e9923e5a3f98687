"""CPU: the where -> postfix program compiler against the numpy masks.

``run_program`` below is the cm_filter_eval kernel's semantics restated in numpy (test
infrastructure); every compiled program must reproduce ``bm25_mask`` / ``chroma_mask`` (which
follow rag/retrieval/bm25.py:79-107 and Chroma's where semantics) on random metadata, including
deletes, None values, unhashable values, tags and the slow comparison operators.
"""
import random

import numpy as np
import pytest

from classmate_hip.retrieval import filters as F


def run_program(P: F.FilterProgram) -> np.ndarray:
    st = []
    for op, a, b in P.ops:
        if op in (F.FOP_EQ, F.FOP_NE):
            col = P.column(a)
            st.append(col == b if op == F.FOP_EQ else col != b)
        elif op == F.FOP_BITS:
            st.append(P.bitmap(a).copy())
        elif op in (F.FOP_TRUE, F.FOP_FALSE):
            st.append(np.full(P.n, op == F.FOP_TRUE))
        elif op == F.FOP_NOT:
            st[-1] = ~st[-1]
        else:
            y, x = st.pop(), st.pop()
            st.append(x & y if op == F.FOP_AND else x | y)
    assert len(st) == 1 and P.fits_device
    return st[0]


VALUES = {"course": ["cs101", "math201", None], "unit": ["u1", "u2", None], "language": ["en", "it"],
          "doc_type": ["pdf", "pptx", "other"], "author": ["ann", None], "semester": [1, 2, True, "1"],
          "score": [0.5, 3, 7, True]}


def random_meta(rng):
    m = {}
    for k, vals in VALUES.items():
        if rng.random() < 0.7:
            m[k] = rng.choice(vals)
    tags = rng.sample(["exam", "lab", "notes"], rng.randint(0, 2))
    if rng.random() < 0.8:
        m["tags"] = tags
    for t in tags:
        m[f"tag_{t}"] = True
    if rng.random() < 0.05:
        m["unit"] = ["u1"]                       # unhashable value
    return m


def random_bm25_where(rng):
    r = rng.random()
    if r < 0.15:
        return {"tags": {"$contains": rng.choice(["exam", "lab", "", ["exam", "lab"]])}}
    if r < 0.3:
        return {"$and": [random_bm25_where(rng), random_bm25_where(rng)], "course": "ignored"}
    w = {f: rng.choice(VALUES[f] + ["zzz"]) for f in rng.sample(list(F.SIMPLE_FIELDS), rng.randint(1, 4))}
    if rng.random() < 0.1:
        w["unit"] = ["u1"]
    return w


def random_chroma_where(rng, depth=0):
    r = rng.random()
    if depth < 2 and r < 0.2:
        return {rng.choice(["$and", "$or"]): [random_chroma_where(rng, depth + 1) for _ in range(rng.randint(1, 3))]}
    key = rng.choice(list(VALUES) + ["tag_exam", "tag_lab", "nokey"])
    vals = VALUES.get(key, [True, False])
    op = rng.choice(["plain", "$eq", "$ne", "$in", "$nin", "$gt", "$lte"])
    if op == "plain":
        return {key: rng.choice(vals)}
    if op in ("$in", "$nin"):
        return {key: {op: rng.sample(vals, min(len(vals), 2))}}
    if op in ("$gt", "$lte"):
        return {key: {op: rng.choice([0, 2, 5])}}
    return {key: {op: rng.choice(vals)}}


@pytest.mark.parametrize("seed", range(4))
def test_programs_match_numpy_masks(seed):
    rng = random.Random(seed)
    mi = F.MetaIndex()
    n = 700
    for r in range(n):
        mi.set(r, random_meta(rng))
    for r in rng.sample(range(n), 60):
        mi.remove(r)
    for r in rng.sample(range(n), 30):
        mi.set(r, random_meta(rng))                # re-set in place
    for _ in range(150):
        w = random_bm25_where(rng)
        assert np.array_equal(run_program(mi.bm25_program(w)), mi.bm25_mask(w)), w
        c = random_chroma_where(rng)
        assert np.array_equal(run_program(mi.chroma_program(c)), mi.chroma_mask(c)), c
    for w in (None, {}):
        assert np.array_equal(run_program(mi.bm25_program(w)), mi.bm25_mask(w))
        assert np.array_equal(run_program(mi.chroma_program(w)), mi.chroma_mask(w))


def test_program_shapes_and_errors():
    mi = F.MetaIndex()
    mi.set(0, {"course": "a", "tags": ["x"]})
    mi.set(1, {"course": None})
    P = mi.bm25_program({"course": "a", "unit": None})
    assert [o[0] for o in P.ops] == [F.FOP_BITS, F.FOP_TRUE, F.FOP_EQ, F.FOP_AND, F.FOP_TRUE, F.FOP_AND, F.FOP_AND]
    assert P.cols == [("course", "py")] and P.bits == ["live"]
    with pytest.raises(ValueError):
        mi.chroma_program({"course": {"$eq": 1, "$ne": 2}})
    with pytest.raises(ValueError):
        mi.chroma_program({"course": {"$regex": "a"}})
    big = mi.chroma_program({"course": {"$in": [f"v{i}" for i in range(40)]}})
    assert not big.fits_device


def test_cm_filter_eval_rejects_bad_programs():
    """The C ABI validates the program before any device work (runs without a GPU)."""
    import ctypes as C
    from classmate_hip import _lib as L
    col = (C.c_void_p * 1)(1)
    none = (C.c_void_p * 1)(None)
    out = C.c_void_p(8)

    def run(ops, ncols=1, n=10):
        a = np.asarray(ops, np.int32).reshape(-1)
        return L.fn["cm_filter_eval"](L.ptr(a), len(ops), col, ncols, none, 0, n, out, None, None)

    assert run([(F.FOP_AND, 0, 0)]) == L.CM_EINVAL                           # stack underflow
    assert run([(F.FOP_TRUE, 0, 0), (F.FOP_TRUE, 0, 0)]) == L.CM_EINVAL     # two values left
    assert run([(F.FOP_EQ, 1, 0)]) == L.CM_EINVAL                            # column slot out of range
    assert run([(F.FOP_BITS, 0, 0)]) == L.CM_EINVAL                          # no bitmaps given
    assert run([(99, 0, 0)]) == L.CM_EINVAL                                  # unknown opcode
    assert run([(F.FOP_TRUE, 0, 0)] * 33 + [(F.FOP_AND, 0, 0)] * 32) == L.CM_EINVAL   # > 64 ops
    assert run([(F.FOP_TRUE, 0, 0)], n=-1) == L.CM_EINVAL
    assert "cm_filter_eval" in L.last_error()

