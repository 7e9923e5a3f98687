"""Drop-in API parity on the GPU: the classmate_hip.retrieval classes, used the
way rag/pipeline/rag.py and rag/admin/inspect.py use the reference classes,
must reproduce the reference-generated goldens (tests/golden/hybrid_1k.json).

Bars: BM25 ids + fp64 scores identical; RRF fused scores identical; vector
ids identical with distances within 1e-4 (exact brute force vs the reference's
HNSW-free exact stand-in); MMR orders identical.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

TOL = 1e-4
FILTERS = {
    "none": None,
    "course_cs101": {"course": "cs101", "unit": None, "author": None, "semester": None,
                     "source_path": None, "created_at": None},
    "course_only": {"course": "math201"},
    "tags_exam": {"course": "cs101", "tags": ["exam"]},
    "lang_en_doctype": {"language": "en", "doc_type": "pptx"},
}


def _new_process():
    """Forget this process's attached stores (registries): the next construction reads the files,
    as a new process would (without it a construction on the same directory attaches to the
    resident state -- the construct-per-call path, tests/test_registry.py)."""
    from classmate_hip.retrieval import bm25, vector_store
    bm25.release_all()
    vector_store.release_all()


class PresetEmbedder:
    def __init__(self, qtexts, qvecs):
        self.t = dict(zip(qtexts, qvecs))

    def encode_queries(self, qs):
        return np.stack([self.t[q] for q in qs]).astype(np.float32)


@pytest.fixture(scope="module")
def stores(corpus, tmp_path_factory):
    from classmate_hip.retrieval import BM25Store, GpuVectorStore
    d = tmp_path_factory.mktemp("idx")
    vs = GpuVectorStore(persist_dir=d / "chroma")
    vs.upsert(ids=corpus["ids"], documents=corpus["texts"], metadatas=corpus["metas"], embeddings=corpus["emb"])
    bm = BM25Store(index_dir=d / "bm25")
    bm.upsert_many(ids=corpus["ids"], texts=corpus["texts"], metadatas=corpus["metas"])
    return vs, bm, d


@pytest.mark.parametrize("fname", list(FILTERS))
def test_bm25store_search(stores, corpus, golden, fname):
    _, bm, _ = stores
    for q, want in zip(corpus["qtexts"], golden["bm25"][fname]):
        got = [[r["id"], r["score"]] for r in bm.search(query=q, where=FILTERS[fname], top_k=10)]
        assert got == want


def test_bm25store_misc(stores, corpus, golden):
    from classmate_hip.retrieval import BM25Store
    _, bm, _ = stores
    m = golden["misc"]
    assert bm.search(query="   ", top_k=5) == m["empty_query"]
    assert [[r["id"], r["score"]] for r in bm.search(query="the and of", top_k=5)] == m["stopword_only_query"]
    got = [[r["id"], r["score"]] for r in bm.search(query=corpus["qtexts"][0], where={"course": "cs101", "unit": "u1",
                                                                                   "doc_type": "pptx"}, top_k=500)]
    assert got == m["topk_gt_n_filtered"]
    s2 = BM25Store(index_dir=None)
    s2.upsert_many(ids=["a", "b", "c"], texts=["alpha beta", "beta gamma", "gamma delta"],
                   metadatas=[{"language": "en", "tags": ["x", "y"]}, {"language": "en", "tags": ["x"]},
                              {"language": "en"}])
    s2.upsert_many(ids=["a"], texts=["alpha alpha zeta"], metadatas=[{"language": "en", "tags": ["y"]}])
    s2.delete_many(["b"])
    s2.upsert_many(ids=["b"], texts=["beta beta beta"], metadatas=[{"language": "en"}])
    assert [[r["id"], r["score"]] for r in s2.search(query="beta alpha gamma", top_k=5)] == m["reorder_after_delete"]
    assert [[r["id"], r["score"]] for r in s2.search(query="alpha", where={"tags": {"$contains": "y"}}, top_k=5)] \
        == m["tags_contains"]


def test_bm25store_sidecar_reload_matches_goldens(stores, corpus, golden, tmp_path):
    """§8f-1: a store reopened through the binary sidecar (device index from the persisted CSR,
    records parsed on demand) returns the reference's results, before and after a mutation."""
    from classmate_hip.retrieval import BM25Store
    _, bm, _ = stores
    bm.index_dir = tmp_path
    bm.save()
    _new_process()
    again = BM25Store.load_or_create(tmp_path)
    assert again._entries.pending and again._csr is not None
    for fname in FILTERS:
        for q, want in zip(corpus["qtexts"], golden["bm25"][fname]):
            assert [[r["id"], r["score"]] for r in again.search(query=q, where=FILTERS[fname], top_k=10)] == want
    i0 = corpus["ids"][0]
    again.upsert_many(ids=[i0], texts=[corpus["texts"][0]], metadatas=[corpus["metas"][0]])   # same content
    assert again._csr is None and not again._entries.pending
    for q, want in zip(corpus["qtexts"], golden["bm25"]["course_cs101"]):
        assert [[r["id"], r["score"]] for r in again.search(query=q, where=FILTERS["course_cs101"], top_k=10)] == want


@pytest.mark.parametrize("fname", list(FILTERS))
def test_vector_store_query(stores, corpus, golden, fname):
    from classmate_hip.retrieval import build_where_filter
    vs, _, _ = stores
    f = FILTERS[fname]
    cw = build_where_filter(f) if f else None
    for qv, want in zip(corpus["qvecs"], golden["dense"][fname]):
        got = vs.query(query_embeddings=qv, where=cw, top_k=24)
        assert [r["id"] for r in got] == [w[0] for w in want]
        np.testing.assert_allclose([r["distance"] for r in got], [w[1] for w in want], atol=TOL)
        assert set(got[0]) == {"id", "document", "metadata", "distance"}


def test_vector_store_persistence_and_delete(stores, corpus):
    from classmate_hip.retrieval import GpuVectorStore
    vs, _, d = stores
    _new_process()
    again = GpuVectorStore(persist_dir=d / "chroma")          # a new process-style reload
    assert again.count() == len(corpus["ids"])
    q = corpus["qvecs"][0]
    a = vs.query(query_embeddings=q, top_k=5, include_embeddings=True)
    b = again.query(query_embeddings=q, top_k=5, include_embeddings=True)
    assert [r["id"] for r in a] == [r["id"] for r in b]
    assert all(np.array_equal(x["embedding"], y["embedding"]) for x, y in zip(a, b))
    again.delete([a[0]["id"]])
    assert again.count() == len(corpus["ids"]) - 1
    assert again.query(query_embeddings=q, top_k=1)[0]["id"] == a[1]["id"]
    again.reset_collection()
    assert again.count() == 0


def test_vector_store_incremental_log(corpus, tmp_path):
    """§8f-1: autosave appends only the call's rows (vectors in place + log records, tombstones for
    deletes); a reload replays the log; save() compacts it to one record per row."""
    import json
    from classmate_hip.retrieval import GpuVectorStore
    ids, emb = corpus["ids"][:300], corpus["emb"][:300]
    vs = GpuVectorStore(persist_dir=tmp_path)
    vs.upsert(ids=ids[:200], documents=corpus["texts"][:200], metadatas=corpus["metas"][:200], embeddings=emb[:200])
    vs.upsert(ids=ids[150:300], documents=["new"] * 150, metadatas=corpus["metas"][150:300], embeddings=emb[150:300])
    vs.delete(ids[:10])
    d = tmp_path / "classmate_rag"
    log = (d / "rows.log.jsonl").read_text().splitlines()
    assert len(log) == 200 + 150 + 10 and json.loads(log[-1])["id"] is None
    assert (d / "vectors.f32").stat().st_size == 300 * emb.shape[1] * 4
    _new_process()
    again = GpuVectorStore(persist_dir=tmp_path)
    assert again.count() == 290
    q = corpus["qvecs"][0]
    a = vs.query(query_embeddings=q, top_k=20, include_embeddings=True)
    b = again.query(query_embeddings=q, top_k=20, include_embeddings=True)
    assert [(r["id"], r["document"], r["metadata"]) for r in a] == [(r["id"], r["document"], r["metadata"]) for r in b]
    assert all(np.array_equal(x["embedding"], y["embedding"]) for x, y in zip(a, b))
    assert {r["document"] for r in b if r["id"] in ids[200:]} <= {"new"}
    again.save()
    assert len((d / "rows.log.jsonl").read_text().splitlines()) == 300
    _new_process()
    third = GpuVectorStore(persist_dir=tmp_path)
    assert [r["id"] for r in third.query(query_embeddings=q, top_k=20)] == [r["id"] for r in a]


def _rows(res):
    return [[r["id"], r["scores"]["fused"], r["scores"]["vector_distance"], r["scores"]["bm25_score"]] for r in res]


def _check(got, want):
    assert [g[0] for g in got] == [w[0] for w in want]
    for g, w in zip(got, want):
        assert g[1] == w[1]                                   # fused: bit-identical
        assert g[3] == w[3]                                   # bm25 score: bit-identical (or both None)
        if w[2] is None:
            assert g[2] is None
        else:
            assert abs(g[2] - w[2]) <= TOL


def _path_spy(monkeypatch, path):
    """path "device": count the device chain's answered calls; "host": CM_RETRIEVE_DEVICE=0."""
    from classmate_hip.retrieval import device_batch
    calls = []
    if path == "host":
        monkeypatch.setenv("CM_RETRIEVE_DEVICE", "0")
        return calls
    real = device_batch.retrieve_batch

    def spy(*a, **kw):
        out = real(*a, **kw)
        calls.append(out is not None)
        return out
    monkeypatch.setattr(device_batch, "retrieve_batch", spy)
    return calls


@pytest.mark.parametrize("path", ["device", "host"])
@pytest.mark.parametrize("fname", list(FILTERS) + ["none_vector_only"])
def test_hybrid_retrieve(stores, corpus, golden, fname, path, monkeypatch):
    """Single-query retrieve() against the reference-generated goldens, filtered cases included
    (course_cs101 is ask_question's DocumentMetadata.to_dict() shape with None keys, quirk Q4), on
    the device chain (retrieve_batch of one) and on the host per-stage path."""
    from classmate_hip.retrieval import HybridRetriever
    vs, bm, _ = stores
    retr = HybridRetriever(vector_store=vs, bm25_store=bm, embedder=PresetEmbedder(corpus["qtexts"], corpus["qvecs"]),
                           k_vector=10, k_bm25=10)
    calls = _path_spy(monkeypatch, path)
    for q, want in zip(corpus["qtexts"], golden["retrieve"][fname]):
        if fname == "none_vector_only":
            got = retr.retrieve(question=q, filters=None, top_k=12, hybrid=False)
        else:
            got = retr.retrieve(question=q, filters=FILTERS[fname], top_k=10)
        _check(_rows(got), want)
    if path == "device" and fname != "none_vector_only":
        assert calls and (all(calls) or fname not in ("none", "course_cs101"))   # the device chain answered


@pytest.mark.parametrize("path", ["device", "host"])
@pytest.mark.parametrize("fname", list(FILTERS))
def test_retrieve_batch_equals_retrieve(stores, corpus, golden, fname, path, monkeypatch):
    from classmate_hip.retrieval import HybridRetriever
    vs, bm, _ = stores
    retr = HybridRetriever(vector_store=vs, bm25_store=bm, embedder=PresetEmbedder(corpus["qtexts"], corpus["qvecs"]),
                           k_vector=10, k_bm25=10)
    calls = _path_spy(monkeypatch, path)
    batch = retr.retrieve_batch(questions=corpus["qtexts"], filters=FILTERS[fname], top_k=10)
    for got, want in zip(batch, golden["retrieve"][fname]):
        _check(_rows(got), want)
    if path == "device":
        assert calls == [True] or (len(calls) == 1 and fname not in ("none", "course_cs101"))


def test_mmr_and_rrf_public_functions(corpus, golden):
    from classmate_hip.retrieval import _mmr_order, rrf_fuse
    idx = {i: n for n, i in enumerate(corpus["ids"])}
    for qv, case in zip(corpus["qvecs"], golden["mmr"]):
        cand = corpus["emb"][[idx[i] for i in case["pool"]]]
        assert _mmr_order(qv, cand, case["pool"], 10) == case["order"]
    for case in golden["rrf"]:
        got = rrf_fuse(rank_lists=case["lists"], weights=case["weights"], rrf_k=case["rrf_k"])
        assert got == case["out"] and list(got) == list(case["out"])


def test_e5_graph_replay_matches_eager():
    """The hipGraph-captured query encode (bench.py's step) equals the eager device encode:
    same E5 forward (4-D boolean mask vs 2-D mask -> same attention), same HIP pooling."""
    import torch
    from classmate_hip.embeddings import E5MultilingualEmbedder
    emb = E5MultilingualEmbedder.random_init(seed=0, device="cuda", num_layers=2)
    B, S = 16, 24
    g = torch.Generator(device="cuda").manual_seed(5)
    ids = torch.randint(5, 250002, (B, S), device="cuda", generator=g)
    ids[:, 0] = 0
    ids[:, -1] = 2
    mask = torch.ones_like(ids)
    mask[3, 20:] = 0                                   # ragged rows: padding is masked out
    mask[7, 9:] = 0
    g_ids, g_mask, g_out, graph = emb.capture_graph(B, S)
    g_ids.copy_(ids)
    g_mask.copy_(mask)
    graph.replay()
    torch.cuda.synchronize()
    want = emb._encode_hf(ids, mask)
    torch.testing.assert_close(g_out, want, atol=2e-3, rtol=0)
    torch.testing.assert_close(emb.encode_token_ids(ids, mask), want, atol=2e-3, rtol=0)
    assert torch.allclose(g_out.norm(dim=1), torch.ones(B, device="cuda"), atol=1e-5)
    # unpadded batches: the maskless graph equals the eager encode
    mask.fill_(1)
    u_ids, u_mask, u_out, ugraph = emb.capture_graph(B, S, unpadded=True)
    u_ids.copy_(ids)
    u_mask.copy_(mask)
    ugraph.replay()
    torch.cuda.synchronize()
    torch.testing.assert_close(u_out, emb.encode_token_ids(ids, mask), atol=2e-3, rtol=0)
    # the bench's bf16 graph (same seeded weights, cast) against the fp32 HF forward: not a
    # self-comparison -- the stated bf16 bound (min cosine >= 0.9999; tests/test_gpu_scale.py holds
    # the 12-layer B = 32, S = 256 figure)
    emb_b = E5MultilingualEmbedder.random_init(seed=0, device="cuda", num_layers=2, dtype="bfloat16")
    b_ids, b_mask, b_out, bgraph = emb_b.capture_graph(B, S, unpadded=True)
    b_ids.copy_(ids)
    b_mask.copy_(mask)
    bgraph.replay()
    torch.cuda.synchronize()
    want32 = emb._encode_hf(ids, mask).float()
    cos = torch.nn.functional.cosine_similarity(b_out.float(), want32, dim=1)
    assert float(cos.min()) >= 0.9999, float(cos.min())


@pytest.mark.parametrize("top_k", [-3, 0, 1, 5])
def test_retrieve_slice_semantics_of_top_k(stores, corpus, top_k):
    """fused_list[:top_k] (rag/retrieval/fusion.py:167): negative and zero top_k slice the full
    fused order the way Python does, on the single and batched paths (oracle: the restatement of
    HybridRetriever.retrieve over the exact store)."""
    from oracle import ref_semantics as orc
    from classmate_hip.retrieval import HybridRetriever
    vs, bm, _ = stores
    emb = PresetEmbedder(corpus["qtexts"], corpus["qvecs"])
    retr = HybridRetriever(vector_store=vs, bm25_store=bm, embedder=emb, k_vector=10, k_bm25=10)
    ovs = orc.ExactVectorStore(corpus["ids"], corpus["texts"], corpus["metas"], corpus["emb"])
    obm = orc.BM25Oracle()
    obm.upsert_many(corpus["ids"], corpus["texts"], corpus["metas"])
    batch = retr.retrieve_batch(questions=corpus["qtexts"][:4], top_k=top_k)
    for i, q in enumerate(corpus["qtexts"][:4]):
        want = orc.retrieve(ovs, obm, emb, question=q, top_k=top_k, k_vector=10, k_bm25=10)
        w = _rows(want)
        _check(_rows(retr.retrieve(question=q, top_k=top_k)), w)
        _check(_rows(batch[i]), w)


def test_vector_store_save_after_trailing_deletes(corpus, tmp_path):
    """rows at the end of the store that were deleted before a reload never reach the
    device copy again; save() must still write meta.rows rows so the store reopens."""
    from classmate_hip.retrieval import GpuVectorStore
    ids, emb = corpus["ids"][:64], corpus["emb"][:64]
    vs = GpuVectorStore(persist_dir=tmp_path)
    vs.upsert(ids=ids, documents=corpus["texts"][:64], metadatas=corpus["metas"][:64], embeddings=emb)
    vs.delete(ids[40:])                                   # trailing tombstones
    _new_process()
    again = GpuVectorStore(persist_dir=tmp_path)
    assert again.count() == 40
    again.save()                                          # device copy holds 40 rows, meta says 64
    _new_process()
    third = GpuVectorStore(persist_dir=tmp_path)
    assert third.count() == 40
    q = corpus["qvecs"][0]
    assert [r["id"] for r in third.query(query_embeddings=q, top_k=10)] == \
        [r["id"] for r in vs.query(query_embeddings=q, top_k=10)]
    third.delete(ids[:40])                                # every row a tombstone
    _new_process()
    fourth = GpuVectorStore(persist_dir=tmp_path)
    assert fourth.count() == 0
    fourth.save()
    _new_process()
    assert GpuVectorStore(persist_dir=tmp_path).count() == 0
    fourth.upsert(ids=["new"], documents=["x"], metadatas=[{}], embeddings=emb[:1])
    _new_process()
    assert [r["id"] for r in GpuVectorStore(persist_dir=tmp_path).query(query_embeddings=emb[0], top_k=3)] == ["new"]


@pytest.mark.parametrize("top_k", [300, 999, 5000, -7])
def test_top_k_beyond_fused_lists(stores, corpus, top_k):
    """top_k above cm_max_topk() (256): the reference sorts every candidate (bm25.py:199) and passes
    any n_results to Chroma (vector_chroma.py:225-229); the device full-order path returns the
    same lists (BM25 bit-exact incl. zero-score padding; dense within 1e-4, exact-oracle order)."""
    from oracle import ref_semantics as orc
    vs, bm, _ = stores
    obm = orc.BM25Oracle()
    obm.upsert_many(corpus["ids"], corpus["texts"], corpus["metas"])
    for q in corpus["qtexts"][:3]:
        got = [[r["id"], r["score"]] for r in bm.search(query=q, top_k=top_k)]
        want = [[w["id"], w["score"]] for w in obm.search(q, None, top_k=top_k)]
        assert got == want
    got = [[r["id"], r["score"]] for r in bm.search(query=corpus["qtexts"][0], where=FILTERS["course_only"],
                                                     top_k=top_k)]
    assert got == [[w["id"], w["score"]] for w in obm.search(corpus["qtexts"][0], FILTERS["course_only"],
                                                             top_k=top_k)]
    if top_k > 0:
        ovs = orc.ExactVectorStore(corpus["ids"], corpus["texts"], corpus["metas"], corpus["emb"])
        for qv in corpus["qvecs"][:3]:
            got = vs.query(query_embeddings=qv, top_k=top_k, include_embeddings=True)
            want = ovs.query(query_embeddings=qv, top_k=top_k)
            assert len(got) == len(want) == min(top_k, len(corpus["ids"]))
            np.testing.assert_allclose([r["distance"] for r in got], [w["distance"] for w in want], atol=TOL)
            gd = np.array([w["distance"] for w in want])
            for j, (g, w) in enumerate(zip(got, want)):   # order exact wherever the oracle separates it
                if (j == 0 or gd[j] - gd[j - 1] > 1e-5) and (j == len(gd) - 1 or gd[j + 1] - gd[j] > 1e-5):
                    assert g["id"] == w["id"]
            idx = {i: n for n, i in enumerate(corpus["ids"])}
            assert all(np.array_equal(r["embedding"], corpus["emb"][idx[r["id"]]]) for r in got[:50])


@pytest.mark.parametrize("top_k", [10, 3, 0, -4])
def test_retrieve_batch_device_path_equals_host_path(corpus, monkeypatch, top_k):
    """The device-resident retrieve_batch (retrieval/device_batch.py) returns the same result dicts
    as the host path (CM_RETRIEVE_DEVICE=0), field by field, on stores that do not hold the same
    documents: ids only in the vector store, ids only in the BM25 store, a deleted vector row,
    documents / metadata present in one store only; plus a whitespace-only query (no BM25 list)."""
    from classmate_hip.retrieval import BM25Store, GpuVectorStore, HybridRetriever
    ids, texts, metas, emb = corpus["ids"], corpus["texts"], corpus["metas"], corpus["emb"]
    vs = GpuVectorStore(persist_dir=None)
    vs.upsert(ids=ids[:250], documents=[t if i % 7 else "" for i, t in enumerate(texts[:250])],
              metadatas=[m if i % 5 else {} for i, m in enumerate(metas[:250])], embeddings=emb[:250])
    vs.delete([ids[3], ids[120]])
    bm = BM25Store(index_dir=None)
    bm.upsert_many(ids=ids[40:], texts=texts[40:], metadatas=metas[40:])
    qtexts = list(corpus["qtexts"]) + ["   "]
    qvecs = np.concatenate([corpus["qvecs"], corpus["qvecs"][:1]])
    retr = HybridRetriever(vector_store=vs, bm25_store=bm, embedder=PresetEmbedder(qtexts, qvecs),
                           k_vector=8, k_bm25=8)
    from classmate_hip.retrieval import device_batch
    assert device_batch.applicable(retr, {}, True)
    got = retr.retrieve_batch(questions=qtexts, top_k=top_k)
    monkeypatch.setenv("CM_RETRIEVE_DEVICE", "0")
    want = retr.retrieve_batch(questions=qtexts, top_k=top_k)
    assert got == want
    # after a mutation the key map follows the stores
    monkeypatch.delenv("CM_RETRIEVE_DEVICE")
    bm.upsert_many(ids=[ids[0]], texts=["an extra lexical document " + texts[1]], metadatas=[{"course": "x"}])
    got = retr.retrieve_batch(questions=qtexts, top_k=top_k)
    monkeypatch.setenv("CM_RETRIEVE_DEVICE", "0")
    assert got == retr.retrieve_batch(questions=qtexts, top_k=top_k)
    # single queries and filtered batches: the same device chain, equal dicts
    for f in (None, FILTERS["course_cs101"], FILTERS["course_only"], {"course": "no-such-course"}):
        monkeypatch.delenv("CM_RETRIEVE_DEVICE")
        got1 = [retr.retrieve(question=q, filters=f, top_k=top_k) for q in qtexts]
        gotb = retr.retrieve_batch(questions=qtexts, filters=f, top_k=top_k)
        monkeypatch.setenv("CM_RETRIEVE_DEVICE", "0")
        assert got1 == [retr.retrieve(question=q, filters=f, top_k=top_k) for q in qtexts], f
        assert gotb == retr.retrieve_batch(questions=qtexts, filters=f, top_k=top_k), f


@pytest.mark.gpu
def test_retrieve_batch_device_bm25_only_items_take_bm25_fields(corpus, monkeypatch):
    """A BM25-only hit whose id the vector store also holds is built from the BM25 entry (document
    and metadata), as the reference's merge does (rag/retrieval/fusion.py:146-151): here the two
    stores hold different non-empty documents and metadata (the BM25 side without 'language', which
    BM25Store.upsert_many then detects), so the device path must not take the vector store's."""
    from classmate_hip.retrieval import BM25Store, GpuVectorStore, HybridRetriever, device_batch
    ids, texts, metas, emb = corpus["ids"], corpus["texts"], corpus["metas"], corpus["emb"]
    vs = GpuVectorStore(persist_dir=None)
    vs.upsert(ids=ids, documents=texts, metadatas=metas, embeddings=emb)
    bm = BM25Store(index_dir=None)
    bm.upsert_many(ids=ids, texts=[t + " bmside" for t in texts],
                   metadatas=[{"course": "bm25-" + str(m.get("course"))} for m in metas])
    retr = HybridRetriever(vector_store=vs, bm25_store=bm, embedder=PresetEmbedder(corpus["qtexts"], corpus["qvecs"]),
                           k_vector=8, k_bm25=8)
    assert device_batch.applicable(retr, {}, True)
    got = retr.retrieve_batch(questions=corpus["qtexts"], top_k=16)
    monkeypatch.setenv("CM_RETRIEVE_DEVICE", "0")
    want = retr.retrieve_batch(questions=corpus["qtexts"], top_k=16)
    assert got == want
    bm_only = [r for res in got for r in res if r["scores"]["vector_distance"] is None]
    assert bm_only and all(r["document"].endswith(" bmside") and r["metadata"]["course"].startswith("bm25-")
                           for r in bm_only)


@pytest.mark.parametrize("refresh", [False, True])
def test_vector_store_snapshot_cold_open(corpus, tmp_path, monkeypatch, refresh):
    """§8f-1 / VERDICT r4 #3: a reopened directory -- snapshot + the log records appended after it,
    and (snapshot removed) the full log replay -- returns the same ids, documents, metadata,
    filtered lists, distances and stored embeddings as the store that wrote it.  refresh: every
    autosave rewrites the snapshot (the tail threshold at 0) instead of leaving a tail."""
    import shutil
    from classmate_hip.retrieval import GpuVectorStore, build_where_filter
    from classmate_hip.retrieval import vector_store as VS
    if refresh:
        monkeypatch.setattr(VS, "_SNAPSHOT_MIN_TAIL", 0)
        monkeypatch.setattr(VS, "_SNAPSHOT_TAIL_FRAC", 0.0)
    _new_process()
    n = 600
    ids, emb, metas = corpus["ids"][:n], corpus["emb"][:n], corpus["metas"][:n]
    vs = GpuVectorStore(persist_dir=tmp_path)
    vs.upsert(ids=ids[:400], documents=corpus["texts"][:400], metadatas=metas[:400], embeddings=emb[:400])
    d = tmp_path / "classmate_rag"
    assert (d / "snapshot" / "info.json").exists()             # the first write is a full save
    vs.upsert(ids=ids[350:n], documents=["tail"] * (n - 350), metadatas=metas[350:n], embeddings=emb[350:n])
    vs.delete(ids[:20] + ids[390:395])
    info = __import__("json").loads((d / "snapshot" / "info.json").read_text())
    assert (info["ids_rows"] == n) == refresh                  # a tail past the snapshot, or none
    for mode in ("snapshot", "replay"):
        _new_process()
        if mode == "replay":
            shutil.rmtree(d / "snapshot")
        again = GpuVectorStore(persist_dir=tmp_path)
        assert again.count() == vs.count() == n - 25
        for f in FILTERS.values():
            cw = build_where_filter(f) if f else None
            for q in corpus["qvecs"][:4]:
                a = vs.query(query_embeddings=q, where=cw, top_k=10, include_embeddings=True)
                b = again.query(query_embeddings=q, where=cw, top_k=10, include_embeddings=True)
                assert [(r["id"], r["document"], r["metadata"], r["distance"]) for r in a] == \
                    [(r["id"], r["document"], r["metadata"], r["distance"]) for r in b], (mode, f)
                assert all(np.array_equal(x["embedding"], y["embedding"]) for x, y in zip(a, b))


def test_vector_store_cold_open_replaces_old_metadata(corpus, tmp_path):
    """rows re-upserted after the snapshot with metadata that has OTHER keys and
    tags must lose every old column code and tag on a cold open -- the replay has to resolve the
    old (snapshot) record before it moves the row's log offset to the new one."""
    from classmate_hip.retrieval import GpuVectorStore
    _new_process()
    n = 300
    ids, emb = corpus["ids"][:n], corpus["emb"][:n]
    old = [{"course": "cs101", "unit": "u1", "language": "en", "tags": ["exam", "old"], "tag_exam": True}
           for _ in range(n)]
    vs = GpuVectorStore(persist_dir=tmp_path)
    vs.upsert(ids=ids, documents=corpus["texts"][:n], metadatas=old, embeddings=emb)
    d = tmp_path / "classmate_rag"
    assert (d / "snapshot" / "info.json").exists()
    moved = ids[:100]
    new = [{"doc_type": "pdf", "tags": ["fresh"], "tag_fresh": True} for _ in moved]
    vs.upsert(ids=moved, documents=["moved"] * len(moved), metadatas=new, embeddings=emb[:100])
    info = __import__("json").loads((d / "snapshot" / "info.json").read_text())
    assert int(info["log_size"]) < (d / "rows.log.jsonl").stat().st_size   # the re-upserts are the tail
    wheres_chroma = [{"course": "cs101"}, {"tag_exam": True}, {"tag_fresh": True}, {"doc_type": "pdf"},
                     {"$and": [{"unit": "u1"}, {"language": "en"}]}]
    wheres_bm25 = [{"course": "cs101"}, {"tags": {"$contains": "exam"}}, {"tags": {"$contains": "fresh"}},
                   {"course": None}, {"doc_type": "pdf"}]
    _new_process()
    again = GpuVectorStore(persist_dir=tmp_path)
    again._ensure_loaded()
    for w in wheres_chroma:
        assert np.array_equal(again._meta.chroma_mask(w), vs._meta.chroma_mask(w)), w
    for w in wheres_bm25:
        assert np.array_equal(again._meta.bm25_mask(w), vs._meta.bm25_mask(w)), w
    assert not again._meta.chroma_mask({"course": "cs101"})[:100].any()
    assert sorted(again._meta.tags.get("exam", ())) == list(range(100, n))
    for w in wheres_chroma:
        for q in corpus["qvecs"][:3]:
            a = vs.query(query_embeddings=q, where=w, top_k=10)
            b = again.query(query_embeddings=q, where=w, top_k=10)
            assert [(r["id"], r["metadata"], r["distance"]) for r in a] == \
                [(r["id"], r["metadata"], r["distance"]) for r in b], w


def test_construct_per_call_attaches_and_sees_upserts(corpus, tmp_path):
    """the reference's ask_question builds its stores and embedder on every call
    (rag/pipeline/rag.py:531-545).  Constructions on the same directories / model attach to the
    resident state (no reload), retrieve exactly what the first instances retrieve, see upserts made
    through them (vector store: autosave; BM25: upsert_many + save, as ingest_file does,
    rag/pipeline/rag.py:410-413), and agree with a fresh process's reload."""
    from classmate_hip.embeddings import E5MultilingualEmbedder
    from classmate_hip.retrieval import BM25Store, GpuVectorStore, HybridRetriever
    _new_process()
    n0, n = 500, len(corpus["ids"])
    ids, texts, metas, emb = corpus["ids"], corpus["texts"], corpus["metas"], corpus["emb"]
    vs = GpuVectorStore(persist_dir=tmp_path / "chroma")
    vs.upsert(ids=ids[:n0], documents=texts[:n0], metadatas=metas[:n0], embeddings=emb[:n0])
    bm = BM25Store.load_or_create(tmp_path / "bm25")
    bm.upsert_many(ids=ids[:n0], texts=texts[:n0], metadatas=metas[:n0])
    bm.save()
    pe = PresetEmbedder(corpus["qtexts"], corpus["qvecs"])

    def ask(q, f):
        v = GpuVectorStore(persist_dir=tmp_path / "chroma")
        b = BM25Store.load_or_create(tmp_path / "bm25")
        r = HybridRetriever(vector_store=v, bm25_store=b, embedder=pe, k_vector=8, k_bm25=8, rrf_k=60)
        return v, b, _rows(r.retrieve(question=q, filters=f, top_k=8))

    first = HybridRetriever(vector_store=vs, bm25_store=bm, embedder=pe, k_vector=8, k_bm25=8, rrf_k=60)
    for q in corpus["qtexts"][:4]:
        for f in (None, FILTERS["course_cs101"]):
            v, b, got = ask(q, f)
            assert v._st is vs._st and b._st is bm._st                 # attached, not reloaded
            assert got == _rows(first.retrieve(question=q, filters=f, top_k=8))
    vs.upsert(ids=ids[n0:], documents=texts[n0:], metadatas=metas[n0:], embeddings=emb[n0:])
    bm.upsert_many(ids=ids[n0:], texts=texts[n0:], metadatas=metas[n0:])
    bm.save()
    v, b, _ = ask(corpus["qtexts"][0], None)
    assert v.count() == n and len(b._id_list) == n
    want = {}
    for q in corpus["qtexts"][:4]:
        want[q] = ask(q, FILTERS["course_cs101"])[2]
    _new_process()                                                       # a fresh process's reload
    for q in corpus["qtexts"][:4]:
        v, b, got = ask(q, FILTERS["course_cs101"])
        assert v._st is not vs._st and got == want[q]
    # the embedder: a construction by name attaches to the registered (here random-init) model
    e = E5MultilingualEmbedder.random_init(seed=0, num_layers=2).share_as("test/e5-registry")
    e2 = E5MultilingualEmbedder(model_name="test/e5-registry", device="cuda")
    assert e2.model is e.model
    assert np.array_equal(e2.encode_queries(["a b c"]), e.encode_queries(["a b c"]))
    E5MultilingualEmbedder.release_all()
