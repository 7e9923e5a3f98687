"""K1q -- the int8 coarse scan with per-row certified bounds (cm_dense_q8.inc) -- against the exact
fp64 oracle (the reference's cosine distance, rag/retrieval/vector_chroma.py:156 hnsw:space=cosine):
ids and distances within 1e-4 (set equality modulo oracle ties closer than 1e-5), no query sent to
the exact fallback, deletes and where-filters honoured, and the same lists as the f16 K1c and the
exact fp32 K1 on the same store."""
import numpy as np
import pytest

from test_gpu_scale import check_dense, exact_topk, exact_topk_dev, mixed_queries, unit_rows

pytestmark = pytest.mark.gpu

Q8, COARSE, F32, STREAM, Q8S = 5, 3, 1, 4, 6


@pytest.fixture(scope="module")
def store():
    from classmate_hip import engine
    C = unit_rows(1_000_000, 768, seed=21)
    idx = engine.DenseIndex(768, capacity=C.shape[0])
    idx.upsert(C, np.arange(C.shape[0], dtype=np.int64))
    yield C, idx
    idx.close()


def test_q8_kind_selection(store):
    """K1q is the automatic batched kind and K1q-s the automatic small-batch kind (CM_DENSE_Q8=0
    selects K1c / K1s); a forced set_path(Q8) takes the batched K1q for any batch, a forced Q8S the
    stream for nq <= 32."""
    import os
    _, idx = store
    off = os.environ.get("CM_DENSE_Q8", "") == "0"
    assert idx.search_kind(256, 24) == (COARSE if off else Q8) and idx.search_kind(64, 10) == (COARSE if off else Q8)
    for nq in (1, 16, 32):
        assert idx.search_kind(nq, 10) == (STREAM if off else Q8S)
    assert idx.search_kind(33, 10) == (COARSE if off else Q8)
    try:
        idx.set_path(Q8)
        assert idx.search_kind(256, 24) == Q8 and idx.search_kind(16, 24) == Q8
        idx.set_path(Q8S)
        assert idx.search_kind(16, 24) == Q8S and idx.search_kind(32, 10) == Q8S
        assert idx.search_kind(64, 10) == (COARSE if off else Q8)     # ineligible: the automatic rule
        idx.set_path(STREAM)
        assert idx.search_kind(16, 24) == STREAM
    finally:
        idx.set_path(0)


@pytest.mark.parametrize("nq", [1, 7, 16, 17, 32])
def test_q8s_matches_exact_fp64(store, nq):
    """K1q-s (the int8 per-wave stream, one or two 16-query tiles) against the exact fp64 scan, no
    query sent to the exact fallback, and the same lists as the batched K1q on the same queries (the
    two share the int8 plane, the bounds and the re-rank, so the distances are bit-identical)."""
    C, idx = store
    Q = mixed_queries(C, nq, seed=130 + nq)
    o_d, o_r = exact_topk(C, Q, 24 + 40)
    try:
        idx.set_path(0)
        assert idx.search_kind(nq, 24) == Q8S
        d, r = idx.search(Q, 24)
        assert idx.last_fallbacks() == 0
        idx.set_path(Q8)
        d8, r8 = idx.search(Q, 24)
    finally:
        idx.set_path(0)
    check_dense(d, r, o_d, o_r, 24)
    assert np.array_equal(r, r8) and np.array_equal(d, d8)


def test_q8_large_batch_keeps_row_groups(store):
    """A batch in the thousands (12 passes of 256 queries): every pass keeps >= 64 row groups and the
    seed sample >= 256, so the certificate holds as at B = 256 (the groups shrank to
    num_cus / n_pass, the seed went infinite below k sample groups and every (group, query) buffer
    overflowed into the exact pass).  Same check for the f16 K1c."""
    C, idx = store
    nq = 3000
    Q = mixed_queries(C, nq, seed=177)
    o_d, o_r = exact_topk_dev(C, Q, 24 + 40, chunk=1 << 18)
    try:
        for kind in (Q8, COARSE):
            idx.set_path(kind)
            d, r = idx.search(Q, 24)
            fb = idx.last_fallbacks()
            check_dense(d, r, o_d, o_r, 24)
            assert fb <= nq // 100, (kind, fb)
    finally:
        idx.set_path(0)


def test_q8s_gaussian_k10_deletes_filters_and_device_entry(store):
    """Random directions at k = 10 (the C2' shape), then deletes + an allow bitmap, and the device
    entry (search_dev, graph-capturable) equal to the host-array search, all on K1q-s."""
    import torch
    C, idx = store
    g = torch.Generator().manual_seed(15)
    Q = torch.randn(16, 768, generator=g).numpy().astype(np.float32)
    o_d, o_r = exact_topk(C, Q, 10 + 40)
    d, r = idx.search(Q, 10)
    assert idx.search_kind(16, 10) == Q8S and idx.last_fallbacks() == 0
    check_dense(d, r, o_d, o_r, 10)
    q = torch.from_numpy(Q).cuda()
    dd, rd = idx.search_dev(q, 10)
    torch.cuda.synchronize()
    assert np.array_equal(rd.cpu().numpy(), r) and np.array_equal(dd.cpu().numpy(), d)
    drop = np.unique(r[:, :3].ravel())
    allow = np.ones(C.shape[0], bool)
    allow[::3] = False
    words = np.packbits(allow, bitorder="little").view(np.uint32)
    idx.delete(drop)
    try:
        d2, r2 = idx.search(Q, 10, words)
        assert not np.isin(r2, drop).any() and (r2 % 3 != 0).all()
        keep = allow.copy()
        keep[drop] = False
        rows = np.nonzero(keep)[0]
        o_d2, o_r2 = exact_topk(C[rows], Q, 10 + 40)
        check_dense(d2, r2, o_d2, rows[o_r2], 10)
        assert idx.last_fallbacks() == 0
    finally:
        idx.upsert(C[drop], drop.astype(np.int64))       # restore the module store


@pytest.mark.parametrize("nq", [256, 100, 40])
def test_q8_matches_exact_fp64(store, nq):
    C, idx = store
    Q = mixed_queries(C, nq, seed=30 + nq)
    o_d, o_r = exact_topk(C, Q, 24 + 40)
    idx.set_path(Q8)
    d, r = idx.search(Q, 24)
    assert idx.last_fallbacks() == 0
    idx.set_path(0)
    check_dense(d, r, o_d, o_r, 24)


def test_q8_gaussian_queries_and_paths_agree(store):
    """Random directions (the widest bands of the analysis) on K1q, K1c and K1: same lists."""
    import torch
    C, idx = store
    g = torch.Generator().manual_seed(5)
    Q = torch.randn(256, 768, generator=g).numpy().astype(np.float32)
    o_d, o_r = exact_topk(C, Q[:64], 10 + 40)
    out = {}
    for kind in (Q8, COARSE, F32):
        idx.set_path(kind)
        out[kind] = idx.search(Q, 10)
        if kind != F32:
            assert idx.last_fallbacks() == 0, kind
    idx.set_path(0)
    for kind, (d, r) in out.items():
        check_dense(d[:64], r[:64], o_d, o_r, 10)
        np.testing.assert_allclose(d, out[F32][0], atol=1e-4)


def test_q8_deletes_and_filters(store):
    C, idx = store
    Q = mixed_queries(C, 64, seed=44)
    idx.set_path(Q8)
    _, r0 = idx.search(Q, 10)
    drop = np.unique(r0[:, :3].ravel())
    allow = np.ones(C.shape[0], bool)
    allow[1::2] = False
    words = np.packbits(allow, bitorder="little").view(np.uint32)
    idx.delete(drop)
    try:
        d, r = idx.search(Q, 10, words)
        assert not np.isin(r, drop).any() and (r % 2 == 0).all()
        keep = allow.copy()
        keep[drop] = False
        rows = np.nonzero(keep)[0]
        o_d, o_r = exact_topk(C[rows], Q, 10 + 40)
        check_dense(d, r, o_d, rows[o_r], 10)
        assert idx.last_fallbacks() == 0
    finally:
        idx.set_path(0)
        idx.upsert(C[drop], drop.astype(np.int64))       # restore the module store


def test_q8_device_search_and_workspace(store):
    """search_dev (the bench's entry, graph-capturable) on K1q equals the host-array search."""
    import torch
    C, idx = store
    Q = mixed_queries(C, 256, seed=77)
    idx.set_path(Q8)
    try:
        d_h, r_h = idx.search(Q, 24)
        q = torch.from_numpy(Q).cuda()
        d, r = idx.search_dev(q, 24)
        torch.cuda.synchronize()
    finally:
        idx.set_path(0)
    assert np.array_equal(r.cpu().numpy(), r_h)
    assert np.array_equal(d.cpu().numpy(), d_h)


def test_q8_band_overflow_takes_exact_fallback():
    """Near-duplicate chunks (real corpora hold them; the synthetic bench never does): 12 000 rows
    within 5e-4 of one base row put far more rows inside the int8 certificate than its 4096-row
    band holds, so the re-rank hands those queries to the wide re-rank (every band row's exact fp64
    distance from the complete candidate buffers; round 5) -- or, with it off, to the exact fp32 K1
    pass (fb_mask), whose merge writes only their rows.  Every list -- cluster and ordinary queries in one batch -- must
    still equal the exact fp64 oracle, on K1q and on K1c."""
    from classmate_hip import engine
    rng = np.random.default_rng(91)
    C = unit_rows(200_000, 768, seed=90)
    base = C[7].astype(np.float64)
    n_c = 12_000
    at = rng.choice(np.arange(8, C.shape[0]), n_c, replace=False)
    d_c = rng.permutation(np.linspace(1e-5, 5e-4, n_c))
    u = rng.standard_normal((n_c, 768))
    u -= np.outer(u @ base, base)                       # orthogonal to the base row
    u /= np.linalg.norm(u, axis=1, keepdims=True)
    t = np.sqrt(2.0 * d_c - d_c ** 2)                   # 1 - cos = d for x = cos.base + sin.u
    x = np.sqrt(1.0 - t ** 2)[:, None] * base + t[:, None] * u
    C[at] = x.astype(np.float32)
    n_near = 8
    Q = mixed_queries(C, 64, seed=92)
    Q[:n_near] = (base + 1e-4 * rng.standard_normal((n_near, 768)) / np.sqrt(768)).astype(np.float32)
    k, slack = 24, 600                                  # cluster gaps ~4e-8: the tie analysis needs a long tail
    o_d, o_r = exact_topk(C, Q, k + slack)
    idx = engine.DenseIndex(768, capacity=C.shape[0])
    try:
        idx.upsert(C, np.arange(C.shape[0], dtype=np.int64))
        for kind in (Q8, COARSE):
            idx.set_path(kind)
            d, r = idx.search(Q, k)
            fb = idx.last_fallbacks()
            check_dense(d, r, o_d, o_r, k)
            if kind == Q8:   # only the cluster queries leave the LDS re-rank; the wide re-rank finishes them
                wide = idx.last_wide_reranks()
                assert 1 <= fb + wide <= n_near and wide >= 1, (fb, wide)
        # the small-batch stream on the cluster queries + 8 ordinary ones: same certificate, same fallback
        idx.set_path(0)
        assert idx.search_kind(16, k) == Q8S
        d, r = idx.search(Q[:16], k)
        fb, wide = idx.last_fallbacks(), idx.last_wide_reranks()
        check_dense(d, r, o_d[:16], o_r[:16], k)
        assert 1 <= fb + wide <= n_near and wide >= 1, (fb, wide)
        # the exact scan as the only fallback (CM_K1Q_WIDE=0) gives the same lists
        import os
        os.environ["CM_K1Q_WIDE"] = "0"
        try:
            idx.set_path(Q8)
            d0, r0 = idx.search(Q, k)
            assert idx.last_wide_reranks() == 0 and 1 <= idx.last_fallbacks() <= n_near
            check_dense(d0, r0, o_d, o_r, k)
        finally:
            del os.environ["CM_K1Q_WIDE"]
            idx.set_path(0)
        # the deferred device entry: scan + re-rank, then the gated exact pass (what the bench step and
        # retrieve() enqueue behind the BM25 join) == the one-call search
        import torch
        q = torch.from_numpy(Q).cuda()
        idx.set_path(Q8)
        d1, r1 = idx.search_dev(q, k)
        out = idx.search_dev(q, k, defer_exact=True)
        idx.exact_fallback_dev(q, k, out)
        torch.cuda.synchronize()
        assert np.array_equal(out[1].cpu().numpy(), r1.cpu().numpy())
        assert np.array_equal(out[0].cpu().numpy(), d1.cpu().numpy())
    finally:
        idx.set_path(0)
        idx.close()


def test_q8_contiguous_cluster_rescans_overflowed_groups():
    """A contiguous run of near-duplicates (a re-ingested document): the queries on it overflow their
    128-slot (group, query) buffers -- an incomplete candidate set -- so the wide re-rank re-scans the
    overflowed groups' live and allowed rows on the f16 plane (rows with d_h - Eh <= kth_up) before the
    exact fp64 stage, instead of the exact scan of every row.  K1q and K1q-s, then deletes + an allow
    filter; every list equal to the fp64 oracle."""
    from classmate_hip import engine
    rng = np.random.default_rng(193)
    C = unit_rows(200_000, 768, seed=190)
    base = C[5].astype(np.float64)
    at = np.arange(100_000, 103_000)
    n_c = at.size
    d_c = rng.permutation(np.linspace(1e-5, 5e-4, n_c))
    u = rng.standard_normal((n_c, 768))
    u -= np.outer(u @ base, base)
    u /= np.linalg.norm(u, axis=1, keepdims=True)
    t = np.sqrt(2.0 * d_c - d_c ** 2)
    C[at] = (np.sqrt(1.0 - t ** 2)[:, None] * base + t[:, None] * u).astype(np.float32)
    Q = mixed_queries(C, 64, seed=194)
    Q[:8] = (base + 1e-4 * rng.standard_normal((8, 768)) / np.sqrt(768)).astype(np.float32)
    k = 24
    o_d, o_r = exact_topk(C, Q, k + 600)
    idx = engine.DenseIndex(768, capacity=C.shape[0])
    try:
        idx.upsert(C, np.arange(C.shape[0], dtype=np.int64))
        idx.set_path(Q8)
        d, r = idx.search(Q, k)
        check_dense(d, r, o_d, o_r, k)
        wide, fb = idx.last_wide_reranks(), idx.last_fallbacks()
        assert wide >= 8 and fb == 0, (wide, fb)          # the 8 cluster queries (+ any mixed query near it)
        idx.set_path(Q8S)
        d, r = idx.search(Q[:16], k)
        check_dense(d, r, o_d[:16], o_r[:16], k)
        assert idx.last_wide_reranks() + idx.last_fallbacks() >= 8
        # deletes inside the cluster + an allow bitmap: the re-scan honours both
        drop = at[::5]
        idx.delete(drop)
        allow = np.ones(C.shape[0], bool)
        allow[at[1::7]] = False
        allow[::11] = False
        words = np.packbits(allow, bitorder="little").view(np.uint32)
        keep = allow.copy()
        keep[drop] = False
        rows = np.nonzero(keep)[0]
        o_d2, o_r2 = exact_topk(C[rows], Q, k + 600)
        idx.set_path(Q8)
        d2, r2 = idx.search(Q, k, words)
        check_dense(d2, r2, o_d2, rows[o_r2], k)
        assert not np.isin(r2, drop).any() and allow[r2[r2 >= 0]].all()
    finally:
        idx.set_path(0)
        idx.close()
