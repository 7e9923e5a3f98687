"""Host-side logic of the drop-in layer (no GPU): tokenizer, where-filters ->
row bitmaps, JSONL persistence format, error conventions.  Checked against
the reference-generated goldens and the pinned oracle."""
import json

import numpy as np
import pytest

from oracle import ref_semantics as orc
from classmate_hip.retrieval import filters as F
from classmate_hip.retrieval.tokenize import _tokenize

FILTERS = {
    "none": None,
    "course_cs101": {"course": "cs101", "unit": None, "author": None, "semester": None,
                     "source_path": None, "created_at": None},
    "course_only": {"course": "math201"},
    "tags_exam": {"course": "cs101", "tags": ["exam"]},
    "lang_en_doctype": {"language": "en", "doc_type": "pptx"},
}


def test_tokenizer_matches_reference_goldens(golden):
    for case in golden["tokenize"]:
        assert _tokenize(case["text"], "en") == case["en"]
        assert _tokenize(case["text"], "it") == case["it"]


def test_tokenizer_matches_oracle_on_corpus(corpus):
    for t in corpus["texts"][:200] + corpus["qtexts"]:
        assert _tokenize(t, "en") == orc.tokenize(t, "en")
        assert _tokenize(t, "it") == orc.tokenize(t, "it")


def test_build_where_filter_goldens(golden):
    for name, f in FILTERS.items():
        assert (F.build_where_filter(f) if f else None) == golden["where"][name]
    assert F.build_where_filter({"doc_type": "other", "tags": "a b, C-d"}) == \
        {"$and": [{"tag_a_b": True}, {"tag_c_d": True}]}
    assert F.build_where_filter({"course": "  "}) is None


def _index(metas):
    m = F.MetaIndex()
    for i, x in enumerate(metas):
        m.set(i, x)
    return m


@pytest.mark.parametrize("where", list(FILTERS.values()) + [
    {"$and": [{"course": "cs101"}, {"unit": "u2"}]}, {"tags": {"$contains": "x"}}, {"page": 3},
    {"course": None, "unit": "u1"}])
def test_bm25_mask_matches_matches_filter(corpus, where):
    metas = [dict(m, tags=["x"] if i % 6 == 0 else ["y"]) for i, m in enumerate(corpus["metas"])]
    got = _index(metas).bm25_mask(where)
    want = np.array([orc.bm25_matches_filter(m, where) for m in metas])
    assert np.array_equal(got, want)


@pytest.mark.parametrize("fname", list(FILTERS))
def test_chroma_mask_matches_oracle(corpus, fname):
    f = FILTERS[fname]
    cw = F.build_where_filter(f) if f else None
    got = _index(corpus["metas"]).chroma_mask(cw)
    want = np.array([orc.chroma_matches(m, cw) for m in corpus["metas"]])
    assert np.array_equal(got, want)


def test_chroma_typed_equality_and_operators():
    m = _index([{"a": 1}, {"a": True}, {"a": 1.0}, {"b": 2}, {"a": "1"}])
    assert m.chroma_mask({"a": 1}).tolist() == [True, False, False, False, False]
    assert m.chroma_mask({"a": True}).tolist() == [False, True, False, False, False]
    assert m.chroma_mask({"a": {"$ne": 1}}).tolist() == [False, True, True, False, True]
    assert m.chroma_mask({"$or": [{"a": 1}, {"b": 2}]}).tolist() == [True, False, False, True, False]
    assert m.chroma_mask({"a": {"$in": [1, "1"]}}).tolist() == [True, False, False, False, True]
    # BM25 semantics use Python equality: 1 == 1.0 == True
    assert m.bm25_mask({"course": None}).tolist() == [True] * 5
    m.remove(0)
    assert m.chroma_mask(None).tolist() == [False, True, True, True, True]


def test_pack_bits_layout():
    rng = np.random.default_rng(0)
    for n in (1, 31, 32, 33, 1000):
        mask = rng.random(n) < 0.4
        w = F.pack_bits(mask)
        assert w.dtype == np.uint32 and w.shape[0] == max((n + 31) // 32, 1)
        back = np.array([(w[i >> 5] >> (i & 31)) & 1 for i in range(n)], bool)
        assert np.array_equal(back, mask)


def test_bm25store_host_semantics(tmp_path):
    from classmate_hip.retrieval import BM25Store
    s = BM25Store(index_dir=tmp_path)
    with pytest.raises(ValueError):
        s.upsert_many(ids=["a"], texts=["x", "y"], metadatas=[{}])
    with pytest.raises(ZeroDivisionError):                       # quirk Q7, raised at upsert like _rebuild
        s.upsert_many(ids=["x1", "x2"], texts=["the and", "12 34"], metadatas=[{"language": "en"}] * 2)
    s2 = BM25Store(index_dir=tmp_path)
    s2.upsert_many(ids=["a", "b"], texts=["alpha beta", "gamma"], metadatas=[{"language": "en"}, {"language": "it"}])
    s2.upsert_many(ids=["a"], texts=["alpha alpha"], metadatas=[{"language": "auto"}])   # detected (fallback en)
    assert list(s2._entries) == ["a", "b"]                                               # in-place replace
    s2.save()
    lines = [json.loads(x) for x in (tmp_path / "bm25_index.jsonl").read_text().splitlines()]
    assert lines[0] == {"id": "a", "text": "alpha alpha", "tokens": ["alpha", "alpha"],
                        "metadata": {"language": "en"}}
    s3 = BM25Store.load_or_create(tmp_path)
    assert [e.tokens for e in s3._entries.values()] == [["alpha", "alpha"], ["gamma"]]
    assert s3.search(query="   ", top_k=3) == []
    assert BM25Store(index_dir=tmp_path / "none").search(query="alpha") == []


def test_bm25store_sidecar_roundtrip_lazy_and_stale(tmp_path):
    """save() writes the reference JSONL + a binary sidecar; load() opens through it
    without parsing records, falls back to the full parse when the JSONL changed."""
    from classmate_hip.retrieval import BM25Store
    s = BM25Store(index_dir=tmp_path)
    texts = ["alpha beta gamma", "gamma delta", "epsilon alpha alpha", "zeta eta theta"]
    metas = [{"language": "en", "course": c, "tags": ["x"]} for c in ("c1", "c2", "c1", None)]
    s.upsert_many(ids=[f"d{i}" for i in range(4)], texts=texts, metadatas=metas)
    s.delete_many(["d1"])
    s.save()
    side = tmp_path / "bm25_index.jsonl.cm"
    names = sorted(p.name for p in side.iterdir())
    assert [x for x in names if not x.startswith("meta_")] == ["doc_off.npy", "ids.json", "line_off.npy", "meta.json",
                                                               "term_ids.npy", "vocab.json"]
    assert "meta_info.json" in names and "meta_live.npy" in names    # the where-filter columns
    from classmate_hip.retrieval import bm25 as _bm25
    _bm25.release_all()              # a new process: open through the sidecar (no attached state)
    s2 = BM25Store.load_or_create(tmp_path)
    assert s2._entries.pending and s2._csr is not None and s2._id_list == ["d0", "d2", "d3"]
    assert s2._csr[1].tolist() == [0, 3, 6, 9]
    e = s2._entries["d2"]                                    # parsed on demand from its byte range
    assert (e.id, e.text, e.tokens, e.metadata) == ("d2", texts[2], ["epsilon", "alpha", "alpha"], metas[2])
    assert [s2._vocab.get(t) for t in e.tokens] == e.term_ids.tolist()
    assert dict.__getitem__(s2._entries, "d3") == 2           # still a line number: nothing else parsed
    # where-filters from the persisted columns, without parsing the records (quirk Q4 included)
    assert not s2._meta_dirty
    for w in ({"course": "c1"}, {"course": None, "unit": None}, {"tags": {"$contains": "x"}}, {"course": "c2"}):
        assert s2._meta.bm25_mask(w).tolist() == s._meta.bm25_mask(w).tolist(), w
    assert dict.__getitem__(s2._entries, "d3") == 2
    ref = {i: (x.text, x.tokens, x.metadata) for i, x in s._entries.items()}
    assert {i: (x.text, x.tokens, x.metadata) for i, x in s2._entries.items()} == ref   # materializes
    assert not s2._entries.pending
    # mutation after a sidecar open: ids keep their order, vocab ids stay consistent
    s3 = BM25Store.load_or_create(tmp_path)
    s3.upsert_many(ids=["d4"], texts=["alpha omega"], metadatas=[{"language": "en"}])
    assert s3._id_list == ["d0", "d2", "d3", "d4"] and s3._csr is None
    for x in s3._entries.values():
        ids = x.term_ids if x.term_ids is not None else s3._term_ids(x.tokens)
        assert [s3._vocab[t] for t in x.tokens] == list(ids)
    s3.save()
    assert BM25Store.load_or_create(tmp_path)._id_list == ["d0", "d2", "d3", "d4"]
    # a JSONL edited behind the sidecar's back: stale -> reference full parse
    with (tmp_path / "bm25_index.jsonl").open("a", encoding="utf-8") as f:
        f.write(json.dumps({"id": "d9", "text": "late", "tokens": ["late"], "metadata": {}}) + "\n")
    s4 = BM25Store.load_or_create(tmp_path)
    assert not s4._entries.pending and s4._csr is None and s4._id_list[-1] == "d9"
    # a corrupt sidecar is ignored too
    s3.save()
    (side / "ids.json").write_text("[1, 2", encoding="utf-8")
    _bm25.release_all()
    s5 = BM25Store.load_or_create(tmp_path)
    assert not s5._entries.pending and len(s5._id_list) == 4


def test_rrf_weights_error_before_device():
    from classmate_hip.retrieval import rrf_fuse
    with pytest.raises(ValueError):
        rrf_fuse(rank_lists=[["a"], ["b"]], weights=[1.0])
    assert rrf_fuse(rank_lists=[]) == {}


def test_vector_store_argument_errors(tmp_path):
    from classmate_hip.retrieval import GpuVectorStore
    vs = GpuVectorStore(persist_dir=tmp_path)
    with pytest.raises(ValueError):
        vs.upsert(ids=["a", "b"], documents=["x"], metadatas=[{}], embeddings=np.zeros((1, 4), np.float32))
    assert vs.count() == 0 and vs.query(query_embeddings=np.zeros(4, np.float32)) == []
    with pytest.raises(ValueError):
        GpuVectorStore(persist_dir=None, distance="l2")


def test_hash_tokenizer_memo_is_transparent():
    """The word -> id memo of the offline E5 tokenizer returns what the hash returns, across a
    memo reset (bounded memo), for repeated and new words."""
    import hashlib
    from classmate_hip.embeddings import HashTokenizer
    tok = HashTokenizer()
    tok._MEMO_MAX = 8                                  # force resets inside one batch

    def fresh(w):
        h = int.from_bytes(hashlib.blake2b(w.encode("utf-8"), digest_size=8).digest(), "little")
        return 5 + h % (tok.vocab_size - 5)

    texts = ["query: the cat sat on the mat, the cat!", "query: élan vital über alles", "", "a a a b b c"] * 3
    ids, mask = tok(texts)
    for i, t in enumerate(texts):
        want = [0] + [fresh(w) for w in tok._re.findall(t)] + [2]
        assert list(ids[i, :len(want)]) == want
        assert int(mask[i].sum()) == len(want)
    assert len(tok._memo) <= 8


def test_multidev_row_map_round_trip_and_word_split():
    """classmate_hip/multidev.py's block-round-robin row map (CM_DEVICES sharding, host side):
    global <-> (shard, local) is a bijection, local rows of a shard keep global order, local_count
    matches the map, and the allow words split into each shard's local words bit for bit."""
    import numpy as np
    import torch
    from classmate_hip.multidev import RowMap, _f32_key_np
    for G, B in ((4, 64), (3, 32), (2, 1 << 16), (8, 128)):
        m = RowMap(G, B)
        n = B * G * 3 + 17
        g = np.arange(n, dtype=np.int64)
        s, l = m.owner_local(g)
        back = np.empty_like(g)
        for sh in range(G):
            sel = s == sh
            assert np.all(np.diff(l[sel]) == 1) and (l[sel][:1] == 0).all()     # dense local rows
            back[sel] = m.to_global(sh, l[sel])
            assert m.local_count(sh, n) == sel.sum()
            tl = torch.from_numpy(l[sel])
            assert np.array_equal(m.to_global(sh, tl).numpy(), g[sel])
        assert np.array_equal(back, g)
        assert (m.to_global(1 % G, np.array([-1])) == -1).all()
        mask = (np.random.default_rng(G).random(n) < 0.4)
        words = np.packbits(mask, bitorder="little")
        words = np.concatenate([words, np.zeros((-len(words)) % 4, np.uint8)]).view(np.uint32)
        for kind in ("np", "torch"):
            w = words if kind == "np" else torch.from_numpy(words.view(np.int32))
            parts = m.split_words(w, G)
            for sh in range(G):
                p = parts[sh] if kind == "np" else parts[sh].numpy().view(np.uint32)
                bits = np.unpackbits(p.view(np.uint8), bitorder="little").astype(bool)
                loc = l[s == sh]
                assert np.array_equal(bits[loc], mask[s == sh])
                assert not bits[m.local_count(sh, n):].any()
    d = np.array([[0.5, 0.25, 0.25, -0.0, 0.0]], np.float32)
    r = np.array([[3, 9, 2, 7, -1]], np.int64)
    assert np.argsort(_f32_key_np(d, r), axis=1).tolist() == [[3, 2, 1, 0, 4]]
