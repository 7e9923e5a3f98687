"""Multi-rank path on the GPU: two ranks (spawned processes, gloo for the
exchanges, both on cuda:0 because RCCL refuses two ranks per device) each own half of the
corpus in the HIP engines.  Sharded BM25 with the all-reduced statistics + the all-gather merge
must equal the unsharded oracle bit for bit, and the merged dense top-k must equal one HIP
index over the whole corpus — the same exchanges bench.py runs over RCCL at N > 1.
"""
import os
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from test_parallel_gloo import _corpus, _free_port  # noqa: E402

from oracle import corc  # noqa: E402

pytestmark = pytest.mark.gpu
WS = 2
DIM = 128


def _dense_data(nd):
    rng = np.random.default_rng(21)
    emb = rng.standard_normal((nd, DIM)).astype(np.float32)
    emb[nd // 2 + 3] = emb[11]                        # duplicate rows in different shards: tie by global row
    q = rng.standard_normal((9, DIM)).astype(np.float32)
    q[0] = emb[11]
    q[1] = emb[nd - 1] + 0.01 * q[1]
    return emb, q


def _worker(rank, port, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(WS))
    dist.init_process_group("gloo", rank=rank, world_size=WS)
    try:
        from classmate_hip import engine
        from classmate_hip import parallel as P
        toks, off, vocab, queries = _corpus()
        nd = off.shape[0] - 1
        row0, n = P.shard_range(nd, rank, WS)
        loc_off = off[row0:row0 + n + 1] - off[row0]
        loc_toks = toks[off[row0]:off[row0 + n]]
        bm = engine.BM25Index(device=0)
        bm.build(loc_toks, loc_off, vocab)
        df, fk = bm.term_stats()
        st = bm.stats()
        gdf, gfk, gn, gsum = P.allreduce_bm25_stats(df, fk, row0, st["n_live"], st["sum_len"])
        idf, eps = P.bm25_idf_table(gdf, gfk, gn)
        bm.set_stats(idf, gn, gsum, eps)
        res = {"rank": rank}
        for k in (1, 10, 64):
            sc, rw, _ = bm.search(queries, k)
            rg = np.where(rw >= 0, rw + row0, rw)
            S, R = P.merge_bm25_topk(torch.from_numpy(sc), torch.from_numpy(rg), k)
            res[f"bm25_{k}"] = (S.numpy(), R.numpy())
        emb, q = _dense_data(nd)
        dn = engine.DenseIndex(DIM, device=0, capacity=n)
        dn.upsert(emb[row0:row0 + n], np.arange(n, dtype=np.int64))
        d, r = dn.search(q, 16)
        rg = np.where(r >= 0, r + row0, r)
        D, R = P.merge_dense_topk(torch.from_numpy(d), torch.from_numpy(rg), 16)
        res["dense"] = (D.numpy(), R.numpy())
        out_q.put(res)
    finally:
        dist.destroy_process_group()


@pytest.fixture(scope="module")
def results():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, port, q)) for r in range(WS)]
    for p in procs:
        p.start()
    out = [q.get(timeout=240) for _ in range(WS)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return sorted(out, key=lambda r: r["rank"])


@pytest.mark.parametrize("k", [1, 10, 64])
def test_sharded_hip_bm25_equals_unsharded_oracle(results, k):
    toks, off, vocab, queries = _corpus()
    csr = corc.build_csr(toks, off, vocab)
    idf, _ = corc.bm25_idf(csr["df"], csr["first_key"], off.shape[0] - 1)
    sc, rw = corc.bm25_topk(csr, idf, float(off[-1]) / (off.shape[0] - 1), queries, k)
    for r in results:
        S, R = r[f"bm25_{k}"]
        assert np.array_equal(R, rw)
        assert np.array_equal(S, sc)


def test_sharded_hip_dense_equals_single_index(results):
    from classmate_hip import engine
    toks, off, _, _ = _corpus()
    nd = off.shape[0] - 1
    emb, q = _dense_data(nd)
    full = engine.DenseIndex(DIM, device=0, capacity=nd)
    full.upsert(emb, np.arange(nd, dtype=np.int64))
    d, r = full.search(q, 16)
    for res in results:
        D, R = res["dense"]
        assert np.array_equal(R, r)
        np.testing.assert_array_equal(D, d)
