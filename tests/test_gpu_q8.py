"""K1q -- the int8 coarse scan with per-row certified bounds (cm_dense_q8.inc) -- against the exact
fp64 oracle (the reference's cosine distance, rag/retrieval/vector_chroma.py:156 hnsw:space=cosine):
ids and distances within 1e-4 (set equality modulo oracle ties closer than 1e-5), no query sent to
the exact fallback, deletes and where-filters honoured, and the same lists as the f16 K1c and the
exact fp32 K1 on the same store."""
import numpy as np
import pytest

from test_gpu_scale import check_dense, exact_topk, mixed_queries, unit_rows

pytestmark = pytest.mark.gpu

Q8, COARSE, F32 = 5, 3, 1


@pytest.fixture(scope="module")
def store():
    from classmate_hip import engine
    C = unit_rows(1_000_000, 768, seed=21)
    idx = engine.DenseIndex(768, capacity=C.shape[0])
    idx.upsert(C, np.arange(C.shape[0], dtype=np.int64))
    yield C, idx
    idx.close()


def test_q8_kind_selection(store):
    """K1q is the automatic batched kind (CM_DENSE_Q8=0 selects K1c); a forced set_path(Q8) always
    takes it; K1s keeps the small batches below 4M rows (this store: 1M)."""
    import os
    _, idx = store
    auto = COARSE if os.environ.get("CM_DENSE_Q8", "") == "0" else Q8
    assert idx.search_kind(256, 24) == auto and idx.search_kind(64, 10) == auto
    assert idx.search_kind(16, 10) == 4
    idx.set_path(Q8)
    try:
        assert idx.search_kind(256, 24) == Q8
    finally:
        idx.set_path(0)


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
    within 5e-4 of one base row put far more rows inside the int8 certificate than its 8192-row
    band holds, so the re-rank hands those queries to the exact fp32 K1 pass (fb_mask) and the
    merge writes only their rows.  Every list -- cluster and ordinary queries in one batch -- must
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
            if kind == Q8:
                assert 1 <= fb <= n_near, fb             # only the cluster queries re-run exactly
    finally:
        idx.set_path(0)
        idx.close()
