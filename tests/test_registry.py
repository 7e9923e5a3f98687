"""Construct-per-call attach and the device-cache keys, host side.

The reference builds its stores on every ask_question call (rag/pipeline/rag.py:531-534):
``ChromaVectorStore.from_config()``, ``BM25Store.load_or_create("./indexes/bm25")``.  Here a
construction attaches to the state this process already holds for the same files when nothing
changed them since; the semantics must stay the reference's:

* BM25 (one JSONL file, each reference instance an independent copy of it): an attached instance
  sees exactly what ``load()`` from disk would give; an unsaved mutation through one instance is
  invisible to later ``load_or_create`` calls (they re-read the file) and to instances sharing the
  state (copy on write); ``save()`` makes the state attachable again.
* vector store (a Chroma collection, shared by every client of the directory): constructions on
  one directory share one collection.
* another writer of the files (size / mtime change) forces a re-read.

No GPU: BM25 mutations, save and load are host work (the device index is built on first search);
the vector-store part checks attach/refresh on directories without rows.
"""
import json
import os

import pytest

from classmate_hip.retrieval import bm25 as B
from classmate_hip.retrieval import device_batch as DB
from classmate_hip.retrieval import filters as F
from classmate_hip.retrieval import vector_store as VS


def _docs(n, tag):
    ids = [f"{tag}{i}" for i in range(n)]
    texts = [f"alpha{tag} beta gamma delta{i % 7} word{i}" for i in range(n)]
    metas = [{"language": "en", "course": f"C{i % 3}"} for i in range(n)]
    return ids, texts, metas


def test_bm25_attach_copy_on_write_and_save(tmp_path):
    B.release_all()
    d = tmp_path / "bm25"
    s1 = B.BM25Store.load_or_create(d)
    ids, texts, metas = _docs(20, "a")
    s1.upsert_many(ids=ids, texts=texts, metadatas=metas)
    s1.save()
    # attach: same state object, no parse
    s2 = B.BM25Store.load_or_create(d)
    assert s2._st is s1._st and s2._id_list == ids
    # an unsaved mutation through s1 copies the shared state first: s2 keeps the file's view
    ids2, texts2, metas2 = _docs(5, "b")
    s1.upsert_many(ids=ids2, texts=texts2, metadatas=metas2)
    assert s1._st is not s2._st
    assert s2._id_list == ids and s1._id_list == ids + ids2
    # a new load sees the file (not s1's unsaved rows) -- s2's clean state is still attachable
    s3 = B.BM25Store.load_or_create(d)
    assert s3._id_list == ids and s3._st is s2._st
    # after the save, the next construction attaches to s1's state and sees the upserts
    s1.save()
    s4 = B.BM25Store.load_or_create(d)
    assert s4._st is s1._st and s4._id_list == ids + ids2
    # a sole holder mutates in place (no copy), but the state stops being attachable until saved
    del s2, s3
    st = s4._st
    s4.delete_many([ids[0]])
    assert s4._st is st or len(st.holders) >= 1
    s5 = B.BM25Store.load_or_create(d)
    assert s5._id_list == ids + ids2                   # the file, not the unsaved delete


def test_bm25_external_writer_forces_reload(tmp_path):
    B.release_all()
    d = tmp_path / "bm25"
    s1 = B.BM25Store.load_or_create(d)
    ids, texts, metas = _docs(10, "x")
    s1.upsert_many(ids=ids, texts=texts, metadatas=metas)
    s1.save()
    # another process appends a record to the JSONL (the reference's format, bm25.py:220-231)
    with open(s1.index_path, "a", encoding="utf-8") as f:
        f.write(json.dumps({"id": "ext", "text": "external words here", "tokens": ["external", "words"],
                            "metadata": {"language": "en"}}) + "\n")
    s2 = B.BM25Store.load_or_create(d)
    assert s2._st is not s1._st and s2._id_list == ids + ["ext"]


def test_bm25_attached_state_searches_like_a_fresh_load(tmp_path):
    """The attached state and a from-disk load hold the same catalog in the same order (what the
    device index and the result dicts are built from)."""
    B.release_all()
    d = tmp_path / "bm25"
    s1 = B.BM25Store.load_or_create(d)
    ids, texts, metas = _docs(30, "q")
    s1.upsert_many(ids=ids, texts=texts, metadatas=metas)
    s1.save()
    s2 = B.BM25Store.load_or_create(d)
    B.release_all()
    s3 = B.BM25Store.load_or_create(d)                # forced re-read
    assert s3._st is not s2._st
    assert s2._id_list == s3._id_list
    assert [s2._entries[i].tokens for i in ids] == [s3._entries[i].tokens for i in ids]
    assert [s2._entries[i].metadata for i in ids] == [s3._entries[i].metadata for i in ids]


def test_bm25_clone_owns_its_entries(tmp_path):
    """a JSONL the reference wrote (no sidecar: term ids are assigned lazily
    against each state's vocabulary), two stores attached to it, one mutating before any search or
    save.  The copy on write must not share _Entry objects, or the first state to assign term ids
    writes them in its own vocabulary into the other's entries."""
    import numpy as np
    B.release_all()
    d = tmp_path / "bm25"
    d.mkdir()
    ids, texts, metas = _docs(12, "r")
    with open(d / "bm25_index.jsonl", "w", encoding="utf-8") as f:
        for i, t, m in zip(ids, texts, metas):
            f.write(json.dumps({"id": i, "text": t, "tokens": B._tokenize(t, lang_hint="en"), "metadata": m}) + "\n")
    s1 = B.BM25Store.load_or_create(d)
    s2 = B.BM25Store.load_or_create(d)
    assert s1._st is s2._st
    s1.delete_many([ids[0]])                     # s1's vocabulary now starts at the second document
    s1.upsert_many(ids=["new"], texts=["zeta eta theta"], metadatas=[{"language": "en"}])
    assert s1._st is not s2._st
    assert all(s1._entries[i] is not s2._entries[i] for i in ids[1:])
    for s, sub in ((s1, "a"), (s2, "b")):        # each state saves its own sidecar
        s.index_dir = tmp_path / sub
        s.save()
    for sub, want_ids in (("a", ids[1:] + ["new"]), ("b", ids)):
        side = tmp_path / sub / "bm25_index.jsonl.cm"
        vocab = json.loads((side / "vocab.json").read_text())
        tid, off = np.load(side / "term_ids.npy"), np.load(side / "doc_off.npy")
        recs = [json.loads(l) for l in open(tmp_path / sub / "bm25_index.jsonl", encoding="utf-8")]
        assert [r["id"] for r in recs] == want_ids
        for r, rec in enumerate(recs):
            assert [vocab[t] for t in tid[off[r]:off[r + 1]]] == rec["tokens"], (sub, r)


def test_vector_store_constructions_share_the_collection(tmp_path):
    VS.release_all()
    a = VS.GpuVectorStore(persist_dir=tmp_path / "chroma", collection_name="c1")
    b = VS.GpuVectorStore(persist_dir=tmp_path / "chroma", collection_name="c1")
    c = VS.GpuVectorStore(persist_dir=tmp_path / "chroma", collection_name="c2")
    assert a._st is b._st and a._st is not c._st
    assert a._uid == b._uid != c._uid
    # another writer creates files in the directory: the next construction starts a fresh state
    d = tmp_path / "chroma" / "c1"
    d.mkdir(parents=True)
    (d / "meta.json").write_text(json.dumps({"format": 2, "dim": 4, "rows": 0}))
    (d / "rows.log.jsonl").write_text("")
    e = VS.GpuVectorStore(persist_dir=tmp_path / "chroma", collection_name="c1")
    assert e._st is not a._st
    f = VS.GpuVectorStore(persist_dir=tmp_path / "chroma", collection_name="c1")
    assert f._st is e._st
    # in-memory stores (persist_dir=None) never share
    g, h = VS.GpuVectorStore(persist_dir=None), VS.GpuVectorStore(persist_dir=None)
    assert g._st is not h._st


def test_filter_cache_keys_are_typed_and_never_reused():
    """keys on a never-reused uid (a fresh MetaIndex restarts its version at 0
    and id() values are recycled) and on the typed clause (True, 1 and "1" differ)."""
    m1 = F.MetaIndex()
    k1 = DB._filter_key(m1, {"course": "C1"}, "bm25")
    uid1 = m1.uid
    del m1
    m2 = F.MetaIndex()
    assert m2.uid != uid1 and m2.version == 0
    assert DB._filter_key(m2, {"course": "C1"}, "bm25") != k1
    keys = {DB._filter_key(m2, {"week": v}, "chroma") for v in (True, 1, "1", 1.0)}
    assert len(keys) == 4
    assert DB._filter_key(m2, {"$and": [{"a": 1}, {"b": None}]}, "chroma") == \
        DB._filter_key(m2, {"$and": [{"a": 1}, {"b": None}]}, "chroma")
    assert DB._filter_key(m2, {"a": object()}, "chroma") is None


def test_meta_index_snapshot_round_trip():
    """The vector store's cold-open snapshot keeps the filter columns exact: typed maps (True, 1,
    1.0 stay distinct under Chroma semantics, merge under Python equality), tag row sets,
    unhashable-value rows (evaluated row by row from the metadata) and deleted rows."""
    m = F.MetaIndex()
    metas = [{"course": f"C{i % 3}", "week": [1, 1.0, True, "1"][i % 4], "flag": (i % 2 == 0),
              "tags": ["a", "b"] if i % 4 == 0 else ["c"]} for i in range(64)]
    for i, mm in enumerate(metas):
        m.set(i, mm)
    m.remove(7)
    m.set(9, None)
    snap = m.snapshot()
    assert snap is not None
    info, arrays = snap
    info = json.loads(json.dumps(info))                  # what the file round trip sees
    m2 = F.MetaIndex.from_snapshot(info, arrays, list(m.metas))
    assert m2.tags == m.tags and (m2.live[:64] == m.live[:64]).all()
    clauses = [{"course": "C1"}, {"week": 1}, {"week": True}, {"week": "1"}, {"week": 1.0}, {"flag": True},
               {"tags": {"$contains": "a"}}, {"course": None, "week": 1}, {"$and": [{"course": "C2"}, {"flag": False}]}]
    for w in clauses:
        for a, b in ((m2.chroma_mask, m.chroma_mask), (m2.bm25_mask, m.bm25_mask)):
            try:
                want = b(w)
            except ValueError:                               # e.g. $contains under Chroma semantics
                with pytest.raises(ValueError):
                    a(w)
                continue
            assert (a(w) == want).all(), w


def test_bm25_save_appends_when_only_documents_were_added(tmp_path):
    """ingest_file saves the whole BM25 catalog after every file (rag/pipeline/rag.py:413).  While a
    state only gained new documents since its last save (or sidecar load), save() appends their
    records: the JSONL and the sidecar must be byte-identical to a full rewrite of the same content
    (a fresh store saving everything once), and a replaced or deleted document forces the rewrite."""
    import numpy as np
    B.release_all()

    def files(d):
        side = d / "bm25_index.jsonl.cm"
        out = {"jsonl": (d / "bm25_index.jsonl").read_bytes()}
        for k in ("term_ids", "doc_off", "line_off"):
            out[k] = np.load(side / f"{k}.npy").tobytes()
        for k in ("ids.json", "vocab.json"):
            out[k] = (side / k).read_text()
        out["cols"] = {p.name: np.load(p).tobytes() for p in side.glob("meta_*.npy")}
        return out

    ids, texts, metas = _docs(60, "p")
    inc = B.BM25Store.load_or_create(tmp_path / "inc")
    for s0 in range(0, 60, 20):                         # three "files", saved after each
        inc.upsert_many(ids=ids[s0:s0 + 20], texts=texts[s0:s0 + 20], metadatas=metas[s0:s0 + 20])
        size_before = (tmp_path / "inc" / "bm25_index.jsonl").stat().st_size if s0 else 0
        inc.save()
        assert inc._st.append_only
    once = B.BM25Store.load_or_create(tmp_path / "once")
    once.upsert_many(ids=ids, texts=texts, metadatas=metas)
    once.save()
    a, b = files(tmp_path / "inc"), files(tmp_path / "once")
    assert a == b and size_before > 0
    # a sidecar-opened store (another process) appending: still identical
    B.release_all()
    more_ids, more_texts, more_metas = _docs(15, "q")
    again = B.BM25Store.load_or_create(tmp_path / "inc")
    assert again._st.append_only and again._st.saved["n"] == 60
    again.upsert_many(ids=more_ids, texts=more_texts, metadatas=more_metas)
    again.save()
    once.upsert_many(ids=more_ids, texts=more_texts, metadatas=more_metas)
    once.save()
    assert files(tmp_path / "inc") == files(tmp_path / "once")
    # a replaced document: the full rewrite (same bytes as the fresh store's)
    for s in (again, once):
        s.upsert_many(ids=[ids[3]], texts=["replaced words here"], metadatas=[{"language": "en", "course": "CX"}])
    assert not again._st.append_only
    again.save()
    once.save()
    assert files(tmp_path / "inc") == files(tmp_path / "once")
    # filters over the incrementally maintained metadata columns == a full rebuild's
    B.release_all()
    fresh = B.BM25Store.load_or_create(tmp_path / "inc")
    fresh._ensure_meta()
    again._meta_dirty = False
    for w in ({"course": "C1"}, {"course": "CX"}, {"course": None}):
        assert (again._meta.bm25_mask(w) == fresh._meta.bm25_mask(w)).all(), w


def test_cold_open_leaves_no_large_containers_in_the_young_generations(tmp_path):
    """A cold open's id lists (10M entries at the bench scale) are promoted to the oldest generation
    during the open (filters.settle_loaded), so the first request's gen-0 collection does not
    traverse them (the construct-then-retrieve p99 at 10M: one ~15 ms gen-0 collection)."""
    import gc
    B.release_all()
    d = tmp_path / "bm25"
    s1 = B.BM25Store.load_or_create(d)
    ids, texts, metas = _docs(3000, "g")
    s1.upsert_many(ids=ids, texts=texts, metadatas=metas)
    s1.save()
    B.release_all()
    s2 = B.BM25Store.load_or_create(d)                 # cold: sidecar path
    assert s2._id_list == ids
    young = [o for g in (0, 1) for o in gc.get_objects(g)]
    assert not any(isinstance(o, list) and len(o) >= 3000 for o in young)
