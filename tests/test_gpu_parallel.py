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


def _filter_mask(nd):
    """Every third document plus a dense prefix: the candidates of term 0 exceed half of them
    (negative idf -> the epsilon floor's global exchange)."""
    r = np.arange(nd)
    return (r % 3 == 0) | (r < 150)


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
        # filtered (quirk Q2): candidate statistics all-reduced, device idf, all-gather merge
        mask = _filter_mask(nd)[row0:row0 + n]
        words = np.zeros((n + 31) // 32, np.uint32)
        idx = np.nonzero(mask)[0]
        np.bitwise_or.at(words, idx >> 5, (np.uint32(1) << (idx & 31).astype(np.uint32)))
        allow = torch.from_numpy(words.view(np.int32)).cuda()
        bm.prepare_filtered(nd)
        off_q = np.zeros(len(queries) + 1, np.int32)
        off_q[1:] = np.cumsum([len(x) for x in queries])
        qt = torch.from_numpy(np.concatenate([np.asarray(x, np.int32) for x in queries])).cuda()
        qo = torch.from_numpy(off_q).cuda()
        for k in (1, 10, 64):
            S, R = P.bm25_search_filtered_sharded(bm, qt, qo, k, allow, row0)
            res[f"filt_{k}"] = (S.cpu().numpy(), R.cpu().numpy())
        # uneven shards: rank 0 holds every document, rank 1 an empty index -- it joins every
        # exchange with zero statistics and empty lists (no hang, same results)
        if rank == 0:
            full = engine.BM25Index(device=0)
            full.build(toks, off, vocab)
            fm = _filter_mask(nd)
            fw = np.zeros((nd + 31) // 32, np.uint32)
            fi = np.nonzero(fm)[0]
            np.bitwise_or.at(fw, fi >> 5, (np.uint32(1) << (fi & 31).astype(np.uint32)))
            f_allow = torch.from_numpy(fw.view(np.int32)).cuda()
        else:
            full = engine.BM25Index(device=0)                 # never built: no documents
            f_allow = torch.zeros(1, dtype=torch.int32, device="cuda")
        full.prepare_filtered(nd)
        S, R = P.bm25_search_filtered_sharded(full, qt, qo, 10, f_allow, 0)
        res["filt_uneven_10"] = (S.cpu().numpy(), R.cpu().numpy())
        full.close()
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


@pytest.mark.parametrize("k", [1, 10, 64])
def test_sharded_hip_bm25_filtered_equals_unsharded_oracle(results, k):
    """Filtered BM25 across two shards (candidate statistics all-reduced, epsilon floor from the
    global first-occurrence order) == rank_bm25 over the filtered documents, bit for bit."""
    toks, off, vocab, queries = _corpus()
    nd = off.shape[0] - 1
    keep = np.nonzero(_filter_mask(nd))[0]
    sub_toks = np.concatenate([toks[off[d]:off[d + 1]] for d in keep])
    sub_off = np.zeros(keep.shape[0] + 1, np.int64)
    sub_off[1:] = np.cumsum(off[keep + 1] - off[keep])
    csr = corc.build_csr(sub_toks, sub_off, vocab)
    idf, eps = corc.bm25_idf(csr["df"], csr["first_key"], keep.shape[0])
    assert (idf == eps).any()                        # the epsilon floor is exercised
    sc, rw = corc.bm25_topk(csr, idf, float(sub_off[-1]) / keep.shape[0], queries, k)
    rw = np.where(rw >= 0, keep[np.maximum(rw, 0)], -1)
    for r in results:
        S, R = r[f"filt_{k}"]
        assert np.array_equal(R, rw)
        assert np.array_equal(S, sc)
        if k == 10:                                  # one shard empty (no hang)
            S, R = r["filt_uneven_10"]
            assert np.array_equal(R, rw)
            assert np.array_equal(S, sc)


@pytest.mark.gpu
@pytest.mark.parametrize("ws", [2, 3, 8])
def test_shard_merge_kernel_equals_torch_merge(ws):
    """the N > 1 step's merge of the packed all-gather runs as one hand-written kernel
    (cm_shard_merge_topk_dev); it must give exactly the torch merge's lists (parallel.merge_packed on
    host tensors, merge_dense_topk / merge_bm25_topk's rules): (distance, row) ascending; (score desc,
    row asc) with -0.0 == 0.0; -1 pads after every real entry -- incl. equal distances / scores
    across shards and shards with fewer live entries than the list length."""
    import torch
    from classmate_hip import parallel as Pl
    rng = np.random.default_rng(ws)
    B, P, K = 64, 24, 10
    packs = []
    for g in range(ws):
        d = np.sort(rng.choice(np.linspace(0.1, 0.9, 40), (B, P)).astype(np.float32), axis=1)   # ties
        r = rng.permutation(1_000_000)[: B * P].reshape(B, P).astype(np.int64) * ws + g         # unique rows
        d_key = np.lexsort((r, d), axis=1)
        d, r = np.take_along_axis(d, d_key, 1), np.take_along_axis(r, d_key, 1)
        s = -np.sort(-rng.choice([3.5, 2.25, 1.0, 0.0, -0.0, -0.5], (B, K)), axis=1)
        br = rng.permutation(1_000_000)[: B * K].reshape(B, K).astype(np.int64) * ws + g
        o = np.lexsort((br, -s), axis=1)
        s, br = np.take_along_axis(s, o, 1), np.take_along_axis(br, o, 1)
        npad = rng.integers(0, P // 2, B)                 # short shard lists: pads at the end
        for i in range(B):
            if npad[i]:
                d[i, P - npad[i]:], r[i, P - npad[i]:] = 0.0, -1
            m = min(npad[i], K)
            if m:
                s[i, K - m:], br[i, K - m:] = 0.0, -1
        dt = torch.from_numpy(d)
        packs.append(torch.cat([dt.view(torch.int32).to(torch.int64), torch.from_numpy(r),
                                torch.from_numpy(s).view(torch.int64), torch.from_numpy(br)], 1))
    allp = torch.stack(packs)                             # (ws, B, 2P + 2K)
    want = Pl.merge_packed(allp, P, K)
    got = Pl.merge_packed(allp.cuda(), P, K)
    torch.cuda.synchronize()
    for w, gt in zip(want, got):
        assert torch.equal(w, gt.cpu()), (w[:2], gt[:2])
