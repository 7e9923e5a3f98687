"""One corpus over several devices inside ONE process (classmate_hip/multidev.py; SURVEY §8(b)
Threading "multi-GPU inside the process", §8(e)).  The test box has one GPU, so the
shards are CM_DEVICES=0,0,0,0: four handles, four HIP streams, the same code path as four cards
(peer copies become same-device copies).  Bars:

* BM25 over 4 shards (global statistics installed at build; a where-filter's candidate statistics
  and epsilon floor summed over the shards) == the unsharded C oracle, bit for bit, host and device
  entries, k = 1 / 10 / 64 (incl. an epsilon-floor filter and the full-order k > cm_max_topk);
* dense over 4 shards == one index over the whole corpus (same distances, same rows);
* the drop-in classes with CM_DEVICES set reproduce the reference goldens (BM25, vector store,
  hybrid retrieve on the device chain and the host path, filtered cases);
* a 4 x 1M-row shard set at the bench's shape: dense top-24 within 1e-4 of the exact fp64 scan,
  BM25 top-10 bit-exact against the oracle built on the host from the tokens.
"""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from test_parallel_gloo import _corpus  # noqa: E402

from oracle import corc  # noqa: E402

pytestmark = pytest.mark.gpu
DEVS = [0, 0, 0, 0]


def _mask(nd):
    r = np.arange(nd)
    return (r % 3 == 0) | (r < 150)


def _words(mask):
    n = mask.shape[0]
    w = np.zeros(max((n + 31) // 32, 1), np.uint32)
    i = np.nonzero(mask)[0]
    np.bitwise_or.at(w, i >> 5, (np.uint32(1) << (i & 31).astype(np.uint32)))
    return w


def _oracle_bm25(toks, off, vocab, queries, k, mask=None):
    nd = off.shape[0] - 1
    if mask is None:
        csr = corc.build_csr(toks, off, vocab)
        idf, _ = corc.bm25_idf(csr["df"], csr["first_key"], nd)
        return corc.bm25_topk(csr, idf, float(off[-1]) / nd, queries, k)
    keep = np.nonzero(mask)[0]
    sub_toks = np.concatenate([toks[off[d]:off[d + 1]] for d in keep])
    sub_off = np.zeros(keep.shape[0] + 1, np.int64)
    sub_off[1:] = np.cumsum(off[keep + 1] - off[keep])
    csr = corc.build_csr(sub_toks, sub_off, vocab)
    idf, eps = corc.bm25_idf(csr["df"], csr["first_key"], keep.shape[0])
    sc, rw = corc.bm25_topk(csr, idf, float(sub_off[-1]) / keep.shape[0], queries, k)
    return sc, np.where(rw >= 0, keep[np.maximum(rw, 0)], -1), (idf == eps).any()


@pytest.mark.parametrize("block", [64, 1024])
def test_sharded_bm25_equals_unsharded_oracle(block):
    import torch
    from classmate_hip import multidev
    toks, off, vocab, queries = _corpus()
    nd = off.shape[0] - 1
    bm = multidev.ShardedBM25Index(DEVS, block=block)
    bm.build(toks, off, vocab)
    assert bm.num_docs == nd and all(sh.num_docs > 0 for sh in bm.shards)
    q_off = np.zeros(len(queries) + 1, np.int32)
    q_off[1:] = np.cumsum([len(x) for x in queries])
    qt = torch.from_numpy(np.concatenate([np.asarray(x, np.int32) for x in queries])).cuda()
    qo = torch.from_numpy(q_off).cuda()
    mask = _mask(nd)
    words = _words(mask)
    bm.prepare_filtered()
    for k in (1, 10, 64, 300):
        sc, rw = _oracle_bm25(toks, off, vocab, queries, k)
        S, R, nv = bm.search(queries, k)                          # host entry (any k)
        assert np.array_equal(R, rw) and np.array_equal(S, sc), k
        assert (nv == (rw >= 0).sum(1)).all()
        fsc, frw, eps_used = _oracle_bm25(toks, off, vocab, queries, k, mask)
        assert eps_used                                            # the epsilon floor is exercised
        S, R, _ = bm.search(queries, k, words)
        assert np.array_equal(R, frw) and np.array_equal(S, fsc), ("filtered host", k)
        if k <= 64:                                                # device entries (fused lists)
            S, R = bm.search_dev(qt, qo, k)
            assert np.array_equal(R.cpu().numpy(), rw) and np.array_equal(S.cpu().numpy(), sc), k
            allow = torch.from_numpy(words.view(np.int32)).cuda()
            S, R = bm.search_filtered(qt, qo, k, allow)
            assert np.array_equal(R.cpu().numpy(), frw) and np.array_equal(S.cpu().numpy(), fsc), ("filtered dev", k)
    # the global CSR the shards hold, on global rows, equals the oracle's build
    ocsr = corc.build_csr(toks, off, vocab)
    csr = bm.export()
    for key in ("term_off", "post_doc", "post_tf", "dl"):
        assert np.array_equal(csr[key], ocsr[key]), key
    bm.close()


@pytest.mark.parametrize("block", [64, 4096])
def test_sharded_dense_equals_one_index(block):
    import torch
    from classmate_hip import engine, multidev
    from test_gpu_scale import check_dense, exact_topk
    rng = np.random.default_rng(21)
    nd, D = 20_000, 768
    emb = rng.standard_normal((nd, D)).astype(np.float32)
    emb[nd // 2 + 3] = emb[11]                        # duplicates on different shards: tie by global row
    q = rng.standard_normal((40, D)).astype(np.float32)
    q[0] = emb[11]
    full = engine.DenseIndex(D, device=0, capacity=nd)
    full.upsert(emb, np.arange(nd, dtype=np.int64))
    sh = multidev.ShardedDenseIndex(D, DEVS, capacity=nd, block=block)
    for s0 in range(0, nd, 3000):                    # upserts that straddle blocks
        sh.upsert(emb[s0:s0 + 3000], np.arange(s0, min(nd, s0 + 3000), dtype=np.int64))
    assert sh.size == nd and sh.live_count() == nd
    drop = np.arange(5, nd, 97)
    full.delete(drop)
    sh.delete(drop)
    mask = np.ones(nd, bool)
    mask[1::4] = False
    w = _words(mask)
    live = np.ones(nd, bool)
    live[drop] = False
    for allow in (None, w):
        cand = np.nonzero(live & (mask if allow is not None else True))[0]
        o_d, o_r = exact_topk(emb[cand], q, 64 + 40)
        o_r = cand[o_r]
        qd = torch.from_numpy(q).cuda()
        al = None if allow is None else torch.from_numpy(allow.view(np.int32)).cuda()
        for k in (1, 10, 24, 64):
            d0, r0 = full.search(q, k, allow)
            d1, r1 = sh.search(q, k, allow)
            d2, r2 = sh.search_dev(qd, k, allow=al)
            for dd, rr in ((d0, r0), (d1, r1), (d2.cpu().numpy(), r2.cpu().numpy())):
                check_dense(dd, rr, o_d[:, :k + 40], o_r[:, :k + 40], k)
            np.testing.assert_allclose(d1, d0, rtol=0, atol=1e-6)
            assert np.array_equal(r1, r2.cpu().numpy()) and np.array_equal(d1, d2.cpu().numpy())
    d0, r0, v0 = full.search(q, 24, return_vectors=True)
    d1, r1, v1 = sh.search(q, 24, return_vectors=True)
    same = r0 == r1
    assert same.mean() > 0.99 and np.array_equal(v0[same], v1[same])
    rows = torch.from_numpy(np.concatenate([r0.reshape(-1), [-1, 0, nd - 1]])).cuda()
    assert torch.equal(sh.gather_dev(rows), full.gather_dev(rows))
    assert np.array_equal(sh.export(), full.export())
    e1, l1 = sh.export(1024, 9000, with_live=True)
    e0, l0 = full.export(1024, 9000, with_live=True)
    assert np.array_equal(e0, e1) and np.array_equal(l0, l1)
    full.close()
    sh.close()


FILTERS = {
    "none": None,
    "course_cs101": {"course": "cs101", "unit": None, "author": None, "semester": None,
                     "source_path": None, "created_at": None},
    "course_only": {"course": "math201"},
    "tags_exam": {"course": "cs101", "tags": ["exam"]},
    "lang_en_doctype": {"language": "en", "doc_type": "pptx"},
}


class _Preset:
    def __init__(self, qtexts, qvecs):
        self.t = dict(zip(qtexts, qvecs))

    def encode_queries(self, qs):
        return np.stack([self.t[q] for q in qs]).astype(np.float32)


def _rows(res):
    return [[r["id"], r["scores"]["fused"], r["scores"]["vector_distance"], r["scores"]["bm25_score"]] for r in res]


def _check(got, want):
    assert [g[0] for g in got] == [w[0] for w in want]
    for g, w in zip(got, want):
        assert g[1] == w[1] and g[3] == w[3]
        assert (g[2] is None) == (w[2] is None) and (w[2] is None or abs(g[2] - w[2]) <= 1e-4)


@pytest.mark.parametrize("path", ["device", "host"])
def test_dropin_classes_on_four_shards_match_goldens(corpus, golden, tmp_path, monkeypatch, path):
    from classmate_hip import multidev
    from classmate_hip.retrieval import BM25Store, GpuVectorStore, HybridRetriever, build_where_filter
    monkeypatch.setenv("CM_DEVICES", ",".join(map(str, DEVS)))
    monkeypatch.setenv("CM_SHARD_BLOCK", "64")           # 1000 chunks -> 16 blocks over 4 shards
    if path == "host":
        monkeypatch.setenv("CM_RETRIEVE_DEVICE", "0")
    ids, texts, metas, emb = corpus["ids"], corpus["texts"], corpus["metas"], corpus["emb"]
    vs = GpuVectorStore(persist_dir=tmp_path / "chroma")
    vs.upsert(ids=ids, documents=texts, metadatas=metas, embeddings=emb)
    bm = BM25Store.load_or_create(tmp_path / "bm25")
    bm.upsert_many(ids=ids, texts=texts, metadatas=metas)
    bm.save()
    assert isinstance(vs._index, multidev.ShardedDenseIndex)
    for fname, f in FILTERS.items():
        for q, want in zip(corpus["qtexts"], golden["bm25"][fname]):
            assert [[r["id"], r["score"]] for r in bm.search(query=q, where=f, top_k=10)] == want, fname
        cw = build_where_filter(f) if f else None
        for qv, want in zip(corpus["qvecs"], golden["dense"][fname]):
            got = vs.query(query_embeddings=qv, where=cw, top_k=24)
            assert [r["id"] for r in got] == [w[0] for w in want]
            np.testing.assert_allclose([r["distance"] for r in got], [w[1] for w in want], atol=1e-4)
    assert isinstance(bm._index, multidev.ShardedBM25Index)
    m = golden["misc"]
    got = [[r["id"], r["score"]] for r in bm.search(query=corpus["qtexts"][0],
                                                     where={"course": "cs101", "unit": "u1", "doc_type": "pptx"},
                                                     top_k=500)]
    assert got == m["topk_gt_n_filtered"]
    retr = HybridRetriever(vector_store=vs, bm25_store=bm, embedder=_Preset(corpus["qtexts"], corpus["qvecs"]),
                           k_vector=10, k_bm25=10)
    for fname, f in FILTERS.items():
        for q, want in zip(corpus["qtexts"], golden["retrieve"][fname]):
            _check(_rows(retr.retrieve(question=q, filters=f, top_k=10)), want)
        for got, want in zip(retr.retrieve_batch(questions=corpus["qtexts"], filters=f, top_k=10),
                             golden["retrieve"][fname]):
            _check(_rows(got), want)
    # reopened through the persisted files, still sharded: the same answers
    from classmate_hip.retrieval import bm25 as bm25_mod, vector_store as vs_mod
    bm25_mod.release_all()
    vs_mod.release_all()
    vs2 = GpuVectorStore(persist_dir=tmp_path / "chroma")
    bm2 = BM25Store.load_or_create(tmp_path / "bm25")
    retr2 = HybridRetriever(vector_store=vs2, bm25_store=bm2, embedder=retr.embedder, k_vector=10, k_bm25=10)
    for q, want in zip(corpus["qtexts"], golden["retrieve"]["course_cs101"]):
        _check(_rows(retr2.retrieve(question=q, filters=FILTERS["course_cs101"], top_k=10)), want)
    assert isinstance(vs2._index, multidev.ShardedDenseIndex)


def test_four_shards_of_1m_rows_at_the_bench_shape():
    """4 x 1M rows / documents (the bench generator): dense top-24 of 256 queries vs the exact fp64
    scan of all 4M rows; BM25 top-10 vs the oracle's own CSR of all 4M documents, bit for bit."""
    import torch
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    from classmate_hip import multidev
    from test_gpu_scale import check_dense, exact_topk_dev, mixed_queries
    N, D, B, K, P, V = 4_000_000, 768, 256, 10, 24, 1 << 20
    dense = multidev.ShardedDenseIndex(D, DEVS, capacity=N)
    g = torch.Generator(device="cuda").manual_seed(4242)
    C = np.empty((N, D), np.float32)
    for r0 in range(0, N, 1 << 20):
        m = min(1 << 20, N - r0)
        x = torch.randn(m, D, device="cuda", generator=g)
        x /= x.norm(dim=1, keepdim=True)
        C[r0:r0 + m] = x.cpu().numpy()
        dense.upsert(C[r0:r0 + m], np.arange(r0, r0 + m, dtype=np.int64))
    tokens, doc_off = bench.gen_tokens(N, V, 1.07, 120.0, seed=77)
    qt = bench.sample_query_terms(tokens, doc_off, B, 8, seed=78)
    tok_h, off_h = tokens.cpu().numpy(), doc_off.cpu().numpy()
    del tokens, doc_off
    torch.cuda.empty_cache()
    bm = multidev.ShardedBM25Index(DEVS)
    bm.build(tok_h, off_h, V)
    Q = mixed_queries(C, B, seed=79)
    q_dev = torch.from_numpy(Q).cuda()
    d, r = dense.search_dev(q_dev, P)
    q_off = (torch.arange(B + 1, device="cuda", dtype=torch.int32) * 8).contiguous()
    bs, br = bm.search_dev(qt.reshape(-1).contiguous(), q_off, K)
    torch.cuda.synchronize()
    o_d, o_r = exact_topk_dev(C, Q, P + 40)
    check_dense(d.cpu().numpy(), r.cpu().numpy(), o_d, o_r, P)
    ocsr = corc.build_csr(tok_h, off_h, V)
    idf, _ = corc.bm25_idf(ocsr["df"], ocsr["first_key"], N)
    o_sc, o_rw = corc.bm25_topk(ocsr, idf, float(ocsr["dl"].astype(np.int64).sum()) / N,
                                qt.cpu().numpy().tolist(), K)
    assert np.array_equal(br.cpu().numpy(), o_rw) and np.array_equal(bs.cpu().numpy(), o_sc)
    # rows of all four shards reach the merged lists
    own = (r.cpu().numpy() >> 16) % 4
    assert len(np.unique(own)) == 4
    dense.close()
    bm.close()
