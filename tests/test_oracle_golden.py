"""Pin the CPU oracle (oracle/ref_semantics.py) against the reference-generated goldens.

The goldens were produced by running the reference's own code
(tests/golden/gen_goldens.py); if the oracle agrees bit-for-bit here it is a
trustworthy checker for the HIP path.
"""
import numpy as np
import pytest

from oracle import ref_semantics as orc


def _bm25_oracle(corpus):
    b = orc.BM25Oracle()
    b.upsert_many(corpus["ids"], corpus["texts"], corpus["metas"])
    return b


FILTERS = {
    "none": None,
    "course_cs101": {"course": "cs101", "unit": None, "author": None, "semester": None,
                     "source_path": None, "created_at": None},
    "course_only": {"course": "math201"},
    "tags_exam": {"course": "cs101", "tags": ["exam"]},
    "lang_en_doctype": {"language": "en", "doc_type": "pptx"},
}


def test_tokenize(golden):
    for case in golden["tokenize"]:
        assert orc.tokenize(case["text"], "en") == case["en"]
        assert orc.tokenize(case["text"], "it") == case["it"]


def test_where_filter(golden):
    for name, f in FILTERS.items():
        want = golden["where"][name]
        got = orc.build_where_filter(f) if f else None
        assert got == want


@pytest.mark.parametrize("fname", list(FILTERS))
def test_bm25_bit_exact(golden, corpus, fname):
    b = _bm25_oracle(corpus)
    for q, want in zip(corpus["qtexts"], golden["bm25"][fname]):
        got = [[r["id"], r["score"]] for r in b.search(q, FILTERS[fname], top_k=10)]
        assert got == want          # ids AND fp64 scores identical


def test_bm25_misc(golden, corpus):
    b = _bm25_oracle(corpus)
    m = golden["misc"]
    assert b.search("   ", top_k=5) == m["empty_query"]
    assert [[r["id"], r["score"]] for r in b.search("the and of", top_k=5)] == m["stopword_only_query"]
    got = [[r["id"], r["score"]] for r in
           b.search(corpus["qtexts"][0], {"course": "cs101", "unit": "u1", "doc_type": "pptx"}, top_k=500)]
    assert got == m["topk_gt_n_filtered"]
    small = orc.BM25Oracle()
    with pytest.raises(ZeroDivisionError):
        small.upsert_many(["x1", "x2"], ["the and", "12 34"], [{"language": "en"}] * 2)
    s2 = orc.BM25Oracle()
    s2.upsert_many(["a", "b", "c"], ["alpha beta", "beta gamma", "gamma delta"],
                   [{"language": "en", "tags": ["x", "y"]}, {"language": "en", "tags": ["x"]}, {"language": "en"}])
    s2.upsert_many(["a"], ["alpha alpha zeta"], [{"language": "en", "tags": ["y"]}])
    s2.delete_many(["b"])
    s2.upsert_many(["b"], ["beta beta beta"], [{"language": "en"}])
    assert [[r["id"], r["score"]] for r in s2.search("beta alpha gamma", top_k=5)] == m["reorder_after_delete"]
    assert [[r["id"], r["score"]] for r in s2.search("alpha", {"tags": {"$contains": "y"}}, top_k=5)] == \
        m["tags_contains"]


@pytest.mark.parametrize("fname", list(FILTERS))
def test_dense_exact(golden, corpus, fname):
    vs = orc.ExactVectorStore(corpus["ids"], corpus["texts"], corpus["metas"], corpus["emb"])
    cw = orc.build_where_filter(FILTERS[fname]) if FILTERS[fname] else None
    for qv, want in zip(corpus["qvecs"], golden["dense"][fname]):
        got = [[r["id"], r["distance"]] for r in vs.query(query_embeddings=qv, where=cw, top_k=24)]
        assert got == want


def test_mmr(golden, corpus):
    idx = {i: n for n, i in enumerate(corpus["ids"])}
    for qv, case in zip(corpus["qvecs"], golden["mmr"]):
        cand = corpus["emb"][[idx[i] for i in case["pool"]]]
        assert orc.mmr_order(qv, cand, case["pool"], 10) == case["order"]


def test_rrf(golden):
    for case in golden["rrf"]:
        got = orc.rrf_fuse(rank_lists=case["lists"], weights=case["weights"], rrf_k=case["rrf_k"])
        assert got == case["out"] and list(got) == list(case["out"])
    with pytest.raises(ValueError):
        orc.rrf_fuse(rank_lists=[["a"], ["b"]], weights=[1.0])


class _Emb:
    def __init__(self, table):
        self.t = table

    def encode_queries(self, qs):
        return np.stack([self.t[q] for q in qs])


@pytest.mark.parametrize("fname", list(FILTERS) + ["none_vector_only"])
def test_retrieve(golden, corpus, fname):
    vs = orc.ExactVectorStore(corpus["ids"], corpus["texts"], corpus["metas"], corpus["emb"])
    b = _bm25_oracle(corpus)
    emb = _Emb(dict(zip(corpus["qtexts"], corpus["qvecs"])))
    for q, want in zip(corpus["qtexts"], golden["retrieve"][fname]):
        if fname == "none_vector_only":
            res = orc.retrieve(vs, b, emb, question=q, filters=None, top_k=12, hybrid=False,
                               k_vector=10, k_bm25=10)
        else:
            res = orc.retrieve(vs, b, emb, question=q, filters=FILTERS[fname], top_k=10, hybrid=True,
                               k_vector=10, k_bm25=10)
        got = [[r["id"], r["scores"]["fused"], r["scores"]["vector_distance"], r["scores"]["bm25_score"]]
               for r in res]
        assert got == want
