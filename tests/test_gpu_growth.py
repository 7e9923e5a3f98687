"""Ingest growth (VERDICT r2 "next" 8).

ChromaVectorStore.upsert (rag/retrieval/vector_chroma.py:168-200) grows the collection one batch at
a time.  cm_dense.hip dense_grow copies device to device when the new arrays fit next to the old
ones in free HBM (the automatic policy); under cm_dense_set_growth(1), or when they do not fit, a
store above 1 GiB grows through host memory: its rows go to the host (pinned bounce buffer), the
old arrays are freed, the new ones allocated and the rows copied back with the f16 plane recomputed
on the device -- so the device never holds the old and the new arrays together and the peak
footprint is the final allocation.
(An in-place growth through reserved address ranges, hipMemAddressReserve + hipMemMap, was tried
first and dropped: hipMemSetAccess rejects some chunk ranges on this ROCm, tools/vmm_probe.hip.)
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

D = 768


def _grow(index, batches, rows_per_batch, seed):
    """Upsert `batches` device batches of unit rows; returns (per-batch mem stats, the rows of a
    few probe indices as fp32 host arrays)."""
    import torch
    g = torch.Generator(device="cuda").manual_seed(seed)
    stats, probes = [], {}
    for b in range(batches):
        x = torch.randn(rows_per_batch, D, device="cuda", generator=g)
        x /= x.norm(dim=1, keepdim=True)
        index.upsert_dev(x, b * rows_per_batch)
        torch.cuda.synchronize()
        for j in (0, rows_per_batch // 2, rows_per_batch - 1):
            probes[b * rows_per_batch + j] = x[j].cpu().numpy()
        stats.append(index.mem_stats())
        del x
    return stats, probes


def _row_bytes(rows):
    """fp32 rows (4 B) + int8 plane (1 B) per element, the f16 plane (2 B) over every row -- or, above
    4M rows of dim 768, over the seed sample's prefix of 1/16 of them (round 6, cm_dense.hip
    xh_rows_for) -- invc + K1q {scale, bound} (12 B) and a live bit per row (dense_row_bytes)."""
    xh = rows if (D != 768 or rows <= 4 << 20) else min(rows, -(-(-(-rows // 16)) // 128) * 128)
    return rows * D * 5 + xh * D * 2 + rows * 12 + rows // 8


def _check_search(index, probes):
    rows = np.array(sorted(probes), dtype=np.int64)
    Q = np.stack([probes[r] for r in rows])
    dist, got = index.search(Q, 3)
    assert (got[:, 0] == rows).all()
    assert np.abs(dist[:, 0]).max() < 1e-5


def test_dense_growth_peak_is_final_size():
    import torch
    from classmate_hip import engine
    nb, per = 16, 125_000                                 # 0 -> 2M rows (9.2 GB) in 16 upserts
    idx = engine.DenseIndex(D, capacity=0)
    idx.set_growth(1)                                     # the peak-bounded policy
    stats, probes = _grow(idx, nb, per, seed=3)
    final = stats[-1]
    n = nb * per
    print(f"\nstaged growth: {final['bytes'] / 1e9:.2f} GB for {n} rows ({_row_bytes(n) / 1e9:.2f} GB of rows), "
          f"peak {final['peak_bytes'] / 1e9:.2f} GB, {final['staged_growths']} growths through the host")
    assert final["staged_growths"] >= 1
    assert final["peak_bytes"] <= 1.1 * final["bytes"]
    assert final["bytes"] <= 1.6 * _row_bytes(n)              # 1.5x growth steps
    assert idx.size == n and idx.live_count() == n
    _check_search(idx, probes)
    # searches after a staged growth: the recomputed f16 plane equals the upsert-written one
    # (K1c at B = 256 and K1s at B = 16 on the coarse plane, ids identical to the fp32 path)
    g = torch.Generator(device="cuda").manual_seed(9)
    q = torch.randn(256, D, device="cuda", generator=g)
    for nq in (256, 16):
        d1, r1 = idx.search_dev(q[:nq].contiguous(), 10)
        idx.set_path(1)
        d2, r2 = idx.search_dev(q[:nq].contiguous(), 10)
        idx.set_path(0)
        assert float((d1 - d2).abs().max()) < 1e-5          # a wrong plane would lose true neighbours
        assert float((r1 == r2).float().mean()) > 0.99
    # reserve() past the size: one more staged growth, nothing lost
    idx.reserve(3 * n)
    st = idx.mem_stats()
    assert st["peak_bytes"] <= 1.1 * st["bytes"] and st["bytes"] >= _row_bytes(3 * n)
    _check_search(idx, probes)
    idx.close()


def test_dense_small_store_copies_on_device():
    """Below 1 GiB the growth copies device to device (old + new together, at most ~2 GiB)."""
    from classmate_hip import engine
    idx = engine.DenseIndex(D, capacity=0)
    stats, probes = _grow(idx, 4, 50_000, seed=4)
    final = stats[-1]
    assert final["staged_growths"] == 0
    assert final["peak_bytes"] >= 1.5 * final["bytes"]              # old + new coexisted
    _check_search(idx, probes)
    idx.close()


def test_dense_large_store_auto_growth_stays_on_device():
    """with free HBM for old + new, the automatic policy copies a > 1 GiB store device to
    device (no host round trip); rows and searches are unchanged."""
    from classmate_hip import engine
    idx = engine.DenseIndex(D, capacity=0)
    with pytest.raises(ValueError):
        idx.set_growth(2)
    stats, probes = _grow(idx, 6, 125_000, seed=5)        # 0 -> 750k rows (3.5 GB): growths above 1 GiB
    final = stats[-1]
    assert final["bytes"] > 1 << 30
    assert final["staged_growths"] == 0
    assert final["peak_bytes"] > final["bytes"]           # old + new coexisted
    assert idx.size == 750_000 and idx.live_count() == 750_000
    _check_search(idx, probes)
    idx.close()
