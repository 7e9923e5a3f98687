"""The C oracle (oracle/cm_oracle.c, used at scales the Python oracle cannot
reach and as the timed CPU baseline) must agree bit-for-bit with the Python
oracle, which the reference-generated goldens pin."""
import numpy as np

from oracle import corc
from oracle import ref_semantics as orc


def _ids(tok_lists):
    vocab = {}
    arrs = [np.array([vocab.setdefault(t, len(vocab)) for t in toks], np.int32) for toks in tok_lists]
    off = np.zeros(len(arrs) + 1, np.int64)
    off[1:] = np.cumsum([len(a) for a in arrs])
    return np.concatenate(arrs), off, vocab


def _search(texts, queries, k):
    toks = [orc.tokenize(t, "en") for t in texts]
    flat, off, vocab = _ids(toks)
    csr = corc.build_csr(flat, off, len(vocab))
    idf, eps = corc.bm25_idf(csr["df"], csr["first_key"], len(texts))
    avgdl = off[-1] / len(texts)
    qs = [[vocab.get(t, -1) for t in orc.tokenize(q, "en")] for q in queries]
    return corc.bm25_topk(csr, idf, avgdl, qs, k)


def test_c_bm25_matches_python_oracle(corpus):
    b = orc.BM25Oracle()
    b.upsert_many(corpus["ids"], corpus["texts"], corpus["metas"])
    sc, rw = _search(corpus["texts"], corpus["qtexts"], 10)
    for i, q in enumerate(corpus["qtexts"]):
        want = [[r["id"], r["score"]] for r in b.search(q, None, 10)]
        assert [[corpus["ids"][r], s] for r, s in zip(rw[i], sc[i])] == want


def test_c_bm25_subset_and_negative_eps(corpus):
    sub = [t for i, t in enumerate(corpus["texts"]) if i % 7 == 0][:30]
    ids = [f"s{i}" for i in range(len(sub))]
    b = orc.BM25Oracle()
    b.upsert_many(ids, sub, [{"language": "en"}] * len(sub))
    qs = corpus["qtexts"] + ["lezione", "lezione lezione", "the"]
    sc, rw = _search(sub, qs, 12)
    for i, q in enumerate(qs):
        want = [[r["id"], r["score"]] for r in b.search(q, None, 12)]
        assert [[ids[r], s] for r, s in zip(rw[i], sc[i])] == want


def test_c_dense_matches_python_oracle(corpus):
    d, r = corc.dense_topk_f64(corpus["emb"], corpus["qvecs"], 24)
    rows, dists = orc.dense_topk_exact(corpus["emb"], corpus["qvecs"], 24)
    for i in range(len(rows)):
        assert r[i].tolist() == rows[i].tolist()
        np.testing.assert_allclose(d[i], dists[i], rtol=0, atol=1e-12)
