"""SURVEY §8(b) Threading: the reference's ask_question builds its stores, embedder
and retriever on every call (rag/pipeline/rag.py:531-549); a server answering questions from
several threads therefore has threads that each construct their own ChromaVectorStore /
BM25Store on one directory -- and here those constructions attach to ONE resident collection
(one device handle, one search workspace).  The collection locks (vector_store._State.lock,
bm25._BState.lock + the per-store lock, held by HybridRetriever across a retrieve) must make
every concurrent answer equal the serial one, which equals the reference goldens.
"""
import random
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

FILTERS = {
    "none": None,
    "course_cs101": {"course": "cs101", "unit": None, "author": None, "semester": None,
                     "source_path": None, "created_at": None},
    "course_only": {"course": "math201"},
    "tags_exam": {"course": "cs101", "tags": ["exam"]},
}


class _Preset:
    def __init__(self, qtexts, qvecs):
        self.t = dict(zip(qtexts, qvecs))

    def encode_queries(self, qs):
        return np.stack([self.t[q] for q in qs]).astype(np.float32)


def _rows(res):
    return [[r["id"], r["scores"]["fused"], r["scores"]["vector_distance"], r["scores"]["bm25_score"]] for r in res]


def _run_threads(n, target):
    errors = []
    barrier = threading.Barrier(n)

    def wrap(t):
        try:
            barrier.wait(timeout=60)
            target(t)
        except BaseException as e:            # noqa: BLE001 -- re-raised in the main thread
            errors.append((t, e))

    threads = [threading.Thread(target=wrap, args=(t,), daemon=True) for t in range(n)]
    for th in threads:
        th.start()
    for th in threads:
        th.join(timeout=100)
    assert not any(th.is_alive() for th in threads), "a worker thread did not finish"
    if errors:
        raise errors[0][1]


def test_four_threads_construct_per_call_equal_serial_and_goldens(corpus, golden, tmp_path):
    from classmate_hip.retrieval import BM25Store, GpuVectorStore, HybridRetriever
    from classmate_hip.retrieval import bm25 as bm25_mod
    from classmate_hip.retrieval import vector_store as vs_mod
    bm25_mod.release_all()
    vs_mod.release_all()
    ids, texts, metas, emb = corpus["ids"], corpus["texts"], corpus["metas"], corpus["emb"]
    vs = GpuVectorStore(persist_dir=tmp_path / "chroma")
    vs.upsert(ids=ids, documents=texts, metadatas=metas, embeddings=emb)
    bm = BM25Store.load_or_create(tmp_path / "bm25")
    bm.upsert_many(ids=ids, texts=texts, metadatas=metas)
    bm.save()
    pe = _Preset(corpus["qtexts"], corpus["qvecs"])
    qtexts = corpus["qtexts"]

    def retriever():
        v = GpuVectorStore(persist_dir=tmp_path / "chroma")
        b = BM25Store.load_or_create(tmp_path / "bm25")
        return HybridRetriever(vector_store=v, bm25_store=b, embedder=pe, k_vector=10, k_bm25=10)

    jobs = [(i, fn) for i in range(len(qtexts)) for fn in FILTERS]
    serial = {(i, fn): _rows(retriever().retrieve(question=qtexts[i], filters=FILTERS[fn], top_k=10))
              for i, fn in jobs}
    for (i, fn), got in serial.items():                       # serial == the reference goldens
        want = golden["retrieve"][fn][i]
        assert [g[0] for g in got] == [w[0] for w in want], (i, fn)
        for g, w in zip(got, want):
            assert g[1] == w[1] and g[3] == w[3]
            assert (g[2] is None) == (w[2] is None) and (g[2] is None or abs(g[2] - w[2]) <= 1e-4)
    results = [[] for _ in range(4)]

    def worker(t):
        rng = random.Random(t)
        mine = jobs * 2
        rng.shuffle(mine)
        for n, (i, fn) in enumerate(mine):
            r = retriever()                                    # every call constructs (rag.py:531-545)
            if t == 3 and n % 3 == 0:                          # batched calls beside the single ones
                batch = r.retrieve_batch(questions=qtexts, filters=FILTERS[fn], top_k=10)
                results[t].extend(((j, fn), _rows(x)) for j, x in enumerate(batch))
            else:
                results[t].append(((i, fn), _rows(r.retrieve(question=qtexts[i], filters=FILTERS[fn], top_k=10))))

    _run_threads(4, worker)
    assert all(results)
    for t in range(4):
        for key, got in results[t]:
            assert got == serial[key], (t, key)
    # every construction attached to the one resident collection (the shared-handle case)
    assert retriever().vector_store._st is vs._st


def test_threads_share_one_store_object_and_mutate(corpus, tmp_path):
    """Threads using the SAME store objects: searches beside upserts / deletes through another
    thread.  Each search must see a consistent store (before or after a mutation, never a torn
    one): its ids must be live at the end or be among the rows mutated, and the final state must
    equal a serial replay."""
    from classmate_hip.retrieval import BM25Store, GpuVectorStore
    ids, texts, metas, emb = corpus["ids"], corpus["texts"], corpus["metas"], corpus["emb"]
    n0 = 800
    vs = GpuVectorStore(persist_dir=None)
    vs.upsert(ids=ids[:n0], documents=texts[:n0], metadatas=metas[:n0], embeddings=emb[:n0])
    bm = BM25Store(index_dir=None)
    bm.upsert_many(ids=ids[:n0], texts=texts[:n0], metadatas=metas[:n0])
    qv, qt = corpus["qvecs"], corpus["qtexts"]
    seen = [set() for _ in range(4)]

    def worker(t):
        if t == 0:                                             # the writer
            for s in range(n0, len(ids), 50):
                vs.upsert(ids=ids[s:s + 50], documents=texts[s:s + 50], metadatas=metas[s:s + 50],
                          embeddings=emb[s:s + 50])
                bm.upsert_many(ids=ids[s:s + 50], texts=texts[s:s + 50], metadatas=metas[s:s + 50])
            vs.delete(ids[:25])
            bm.delete_many(ids[:25])
            return
        for rep in range(6):
            for j in range(len(qt)):
                seen[t].update(r["id"] for r in vs.query(query_embeddings=qv[j], top_k=10))
                seen[t].update(r["id"] for r in bm.search(query=qt[j], top_k=10))

    _run_threads(4, worker)
    assert vs.count() == len(ids) - 25 and len(bm._id_list) == len(ids) - 25
    allowed = set(ids)
    for t in range(1, 4):
        assert seen[t] and seen[t] <= allowed
    # after the writer: the same answers as fresh single-threaded stores of the final content
    vs2 = GpuVectorStore(persist_dir=None)
    vs2.upsert(ids=ids[25:], documents=texts[25:], metadatas=metas[25:], embeddings=emb[25:])
    bm2 = BM25Store(index_dir=None)
    bm2.upsert_many(ids=ids[25:n0], texts=texts[25:n0], metadatas=metas[25:n0])
    bm2.upsert_many(ids=ids[n0:], texts=texts[n0:], metadatas=metas[n0:])
    for j in range(len(qt)):
        a = [(r["id"], r["distance"]) for r in vs.query(query_embeddings=qv[j], top_k=10)]
        b = [(r["id"], r["distance"]) for r in vs2.query(query_embeddings=qv[j], top_k=10)]
        assert a == b
        assert [(r["id"], r["score"]) for r in bm.search(query=qt[j], top_k=10)] == \
            [(r["id"], r["score"]) for r in bm2.search(query=qt[j], top_k=10)]


def test_e5_threads_share_the_model_and_its_graphs():
    """Four threads encoding through one E5 instance attached by name (its lean forward, K10 planes
    and small-batch hipGraphs are shared): every thread's embeddings equal the serial ones, bit for
    bit -- single queries (graph replays) and batches (eager forward)."""
    from classmate_hip.embeddings import E5MultilingualEmbedder
    e = E5MultilingualEmbedder.random_init(seed=0, num_layers=2).share_as("test/e5-threads")
    rng = random.Random(5)
    words = ["alpha", "beta", "gamma", "delta", "kappa", "omega", "sigma", "theta"]
    qs = [" ".join(rng.choice(words) for _ in range(3 + i % 9)) for i in range(24)]
    want_single = {q: E5MultilingualEmbedder(model_name="test/e5-threads", device="cuda").encode_queries([q])
                   for q in qs}
    want_batch = e.encode_queries(qs[:12])
    got = [[] for _ in range(4)]

    def worker(t):
        m = E5MultilingualEmbedder(model_name="test/e5-threads", device="cuda")
        assert m.model is e.model
        for rep in range(3):
            for q in qs[t::2]:
                got[t].append((q, m.encode_queries([q])))
            if t % 2 == 0:
                got[t].append(("__batch__", m.encode_queries(qs[:12])))

    try:
        _run_threads(4, worker)
    finally:
        E5MultilingualEmbedder.release_all()
    for t in range(4):
        assert got[t]
        for q, v in got[t]:
            assert np.array_equal(v, want_batch if q == "__batch__" else want_single[q]), (t, q)
