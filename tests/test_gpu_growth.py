"""Ingest growth without double residency (VERDICT r2 "next" 8).

ChromaVectorStore.upsert (rag/retrieval/vector_chroma.py:168-200) grows the collection one batch at
a time.  The HBM store grows in place: its row arrays sit in reserved address ranges and a growth
maps more memory behind them (cm_common.h VmBuf), so the footprint never exceeds the final size by
more than the mapping slack, and the rows written earlier never move.  The hipMalloc + copy path
(CM_DENSE_VMM=0, kept for devices without virtual memory management) holds old + new at once.
"""
import os

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
    return rows * D * 6 + rows * 4 + rows // 8


def _check_search(index, probes):
    rows = np.array(sorted(probes), dtype=np.int64)
    Q = np.stack([probes[r] for r in rows])
    dist, got = index.search(Q, 3)
    assert (got[:, 0] == rows).all()
    assert np.abs(dist[:, 0]).max() < 1e-5


def test_dense_grows_in_place_within_10pct():
    import torch
    from classmate_hip import engine
    os.environ.pop("CM_DENSE_VMM", None)
    nb, per = 16, 125_000                                 # 0 -> 2M rows (9.2 GB) in 16 upserts
    idx = engine.DenseIndex(D, capacity=0)
    assert idx.mem_stats()["in_place"], "MI355X supports virtual memory management"
    free0 = torch.cuda.mem_get_info()[0]
    stats, probes = _grow(idx, nb, per, seed=3)
    final = stats[-1]
    used = free0 - torch.cuda.mem_get_info()[0]
    n = nb * per
    print(f"\nin place: {final['bytes'] / 1e9:.2f} GB mapped for {n} rows ({_row_bytes(n) / 1e9:.2f} GB), "
          f"peak {final['peak_bytes'] / 1e9:.2f} GB, device memory used {used / 1e9:.2f} GB")
    assert final["peak_bytes"] <= 1.1 * final["bytes"]
    assert final["bytes"] <= 1.1 * _row_bytes(n)
    assert used <= 1.15 * _row_bytes(n)
    assert idx.size == n and idx.live_count() == n
    _check_search(idx, probes)
    # a reserve() past the current size maps the rest without moving anything
    idx.reserve(3 * n)
    assert idx.mem_stats()["bytes"] >= _row_bytes(3 * n)
    _check_search(idx, probes)
    idx.close()


def test_dense_copy_growth_path_same_results():
    """CM_DENSE_VMM=0: the hipMalloc + copy growth (1.5x) gives the same rows and search results;
    its recorded peak holds the old and the new arrays together."""
    from classmate_hip import engine
    os.environ["CM_DENSE_VMM"] = "0"
    try:
        idx = engine.DenseIndex(D, capacity=0)
    finally:
        os.environ.pop("CM_DENSE_VMM", None)
    assert not idx.mem_stats()["in_place"]
    stats, probes = _grow(idx, 6, 50_000, seed=4)
    final = stats[-1]
    assert final["peak_bytes"] >= 1.5 * final["bytes"]              # old + new coexisted (1.5x steps)
    _check_search(idx, probes)
    idx.close()
