"""The f16 plane as a seed-sample prefix (round 6; cm_dense.hip xh_rows_for): above 4M
rows -- or at any size with CM_DENSE_F16=prefix, as here -- a dim-768 store keeps only the first
1/16 of its rows in the f16 plane (the K1q seed pass reads nothing else), the re-rank ranks the
whole certified int8 band from the fp32 rows, and the wide re-rank filters overflowed groups on the
int8 plane.  Every list must equal the exact fp64 oracle and the full-plane store's lists bit for
bit (same fp64 arithmetic per row), with the same kinds, no exact re-runs on ordinary queries, and
~15/16 of the plane's bytes gone; growth re-planes the prefix's new rows from the fp32 data."""
import numpy as np
import pytest

from test_gpu_scale import check_dense, exact_topk, mixed_queries, unit_rows

pytestmark = pytest.mark.gpu

Q8, COARSE, F32, STREAM, Q8S = 5, 3, 1, 4, 6


def _index(monkeypatch, mode, C, cap=None, chunk=None):
    from classmate_hip import engine
    monkeypatch.setenv("CM_DENSE_F16", mode)
    idx = engine.DenseIndex(768, capacity=C.shape[0] if cap is None else cap)
    step = chunk or C.shape[0]
    for s in range(0, C.shape[0], step):
        idx.upsert(C[s:s + step], np.arange(s, min(C.shape[0], s + step), dtype=np.int64))
    monkeypatch.delenv("CM_DENSE_F16")
    return idx


@pytest.fixture(scope="module")
def data():
    return unit_rows(300_000, 768, seed=321)


def test_prefix_plane_lists_equal_full_plane_and_oracle(data, monkeypatch):
    C = data
    full = _index(monkeypatch, "full", C)
    pre = _index(monkeypatch, "prefix", C)
    try:
        mf, mp = full.mem_stats()["bytes"], pre.mem_stats()["bytes"]
        assert mf - mp >= 0.9 * C.shape[0] * 768 * 2, (mf, mp)        # ~15/16 of the f16 plane
        assert pre.search_kind(256, 24) == Q8 and pre.search_kind(16, 24) == Q8S
        for kind in (COARSE, STREAM):                                 # they read every plane row
            pre.set_path(kind)
            assert pre.search_kind(16, 24) in (Q8, Q8S) and pre.search_kind(64, 24) == Q8
        pre.set_path(0)
        for nq, k in ((256, 24), (100, 10), (16, 24), (1, 10)):
            Q = mixed_queries(C, nq, seed=400 + nq)
            o_d, o_r = exact_topk(C, Q, k + 40)
            d0, r0 = full.search(Q, k)
            d1, r1 = pre.search(Q, k)
            assert pre.last_fallbacks() == 0
            check_dense(d1, r1, o_d, o_r, k)
            assert np.array_equal(r0, r1) and np.array_equal(d0, d1), (nq, k)
        # deletes + a filter, and the device entry
        import torch
        Q = mixed_queries(C, 64, seed=471)
        _, r = pre.search(Q, 10)
        drop = np.unique(r[:, :2].ravel())
        allow = np.ones(C.shape[0], bool)
        allow[1::3] = False
        words = np.packbits(allow, bitorder="little").view(np.uint32)
        for idx in (full, pre):
            idx.delete(drop)
        d0, r0 = full.search(Q, 10, words)
        d1, r1 = pre.search(Q, 10, words)
        assert np.array_equal(r0, r1) and np.array_equal(d0, d1)
        assert not np.isin(r1, drop).any() and allow[r1[r1 >= 0]].all()
        q = torch.from_numpy(Q).cuda()
        dd, rd = pre.search_dev(q, 10)
        torch.cuda.synchronize()
        _, rh = pre.search(Q, 10)
        assert np.array_equal(rd.cpu().numpy(), rh)
    finally:
        full.close()
        pre.close()


def test_prefix_plane_growth_replanes_new_prefix_rows(data, monkeypatch):
    """Grown from a small capacity in chunks (every growth extends the prefix: its new rows are
    re-planed from the fp32 rows on the device) == one allocation of the final size."""
    C = data
    grown = _index(monkeypatch, "prefix", C, cap=1024, chunk=37_000)
    once = _index(monkeypatch, "prefix", C)
    try:
        for nq, k in ((256, 24), (16, 10)):
            Q = mixed_queries(C, nq, seed=500 + nq)
            d0, r0 = once.search(Q, k)
            d1, r1 = grown.search(Q, k)
            assert np.array_equal(r0, r1) and np.array_equal(d0, d1), nq
            assert grown.last_fallbacks() == 0
    finally:
        grown.close()
        once.close()


def test_prefix_plane_clusters_band_overflow_and_overflowed_groups(monkeypatch):
    """The two certificate overflows without a full f16 plane: a scattered 12k-row near-duplicate
    cluster (int8 band > 4096 rows: the wide re-rank from the candidate buffers) and a contiguous
    3k-row one (overflowed (group, query) buffers: their groups re-scanned on the int8 plane with the
    scan's per-row bound) -- lists equal to the fp64 oracle, finished by the wide re-rank."""
    rng = np.random.default_rng(93)
    C = unit_rows(200_000, 768, seed=94)
    base = C[7].astype(np.float64)

    def plant(at):
        n_c = at.size
        d_c = rng.permutation(np.linspace(1e-5, 5e-4, n_c))
        u = rng.standard_normal((n_c, 768))
        u -= np.outer(u @ base, base)
        u /= np.linalg.norm(u, axis=1, keepdims=True)
        t = np.sqrt(2.0 * d_c - d_c ** 2)
        C[at] = (np.sqrt(1.0 - t ** 2)[:, None] * base + t[:, None] * u).astype(np.float32)

    plant(rng.choice(np.arange(8, 100_000), 12_000, replace=False))
    plant(np.arange(150_000, 153_000))
    Q = mixed_queries(C, 64, seed=95)
    Q[:8] = (base + 1e-4 * rng.standard_normal((8, 768)) / np.sqrt(768)).astype(np.float32)
    k = 24
    o_d, o_r = exact_topk(C, Q, k + 900)
    idx = _index(monkeypatch, "prefix", C)
    try:
        for nq in (64, 16):
            d, r = idx.search(Q[:nq], k)
            check_dense(d, r, o_d[:nq], o_r[:nq], k)
            wide, fb = idx.last_wide_reranks(), idx.last_fallbacks()
            assert wide >= 1 and fb + wide <= 8 + 2, (nq, wide, fb)
    finally:
        idx.close()
