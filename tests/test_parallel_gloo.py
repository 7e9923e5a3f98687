"""World-size-2 and world-size-8 (gloo, CPU) tests of the multi-GPU exchange steps
in classmate_hip.parallel (8 = BASELINE configs[4]'s 8-way split):
sharded BM25 statistics must give the single-shard idf table / avgdl
bit-for-bit, and the all-gather top-k merges must give the unsharded oracle
top-k (ties by global row, zero-score padding).

Per-shard top-k here comes from the C oracle (no GPU); on the GPU the same merge
consumes the HIP shards' outputs (bench.py).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import corc

NQ = 8          # dense / packed-exchange queries: B = NQ splits into equal blocks at WS = 2 and 8


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _corpus(seed=3, nd=6000, vocab=700):
    rng = np.random.default_rng(seed)
    lens = np.maximum(rng.poisson(12, nd), 1)
    off = np.zeros(nd + 1, np.int64)
    off[1:] = np.cumsum(lens)
    p = 1.0 / np.arange(1, vocab + 1) ** 1.2
    toks = rng.choice(vocab, size=int(off[-1]), p=p / p.sum()).astype(np.int32)
    toks[toks == vocab - 1] = 0                      # term vocab-1 absent everywhere
    rare = int(vocab - 2)
    toks[np.isin(toks, [rare])] = 1
    toks[off[nd - 3]] = rare                         # rare term: a single doc, in the last shard
    queries = [rng.integers(0, 60, 5).tolist() for _ in range(12)] + [[rare], [rare, vocab - 1], [0, 0, 3]]
    return toks, off, vocab, queries


def _filter_mask(nd):
    r = np.arange(nd)
    return (r % 3 == 0) | (r < 150)


def _masked_csr(toks, off, vocab, mask):
    """CSR of a shard whose non-candidate documents are emptied: candidate df and first
    (local row, position) keys with the shard's own row numbering."""
    lens = np.where(mask, off[1:] - off[:-1], 0)
    keep = np.repeat(mask, off[1:] - off[:-1])
    moff = np.zeros(mask.shape[0] + 1, np.int64)
    moff[1:] = np.cumsum(lens)
    return corc.build_csr(toks[keep], moff, vocab)


def _filtered_shard_search(P, toks, off, vocab, queries, row0, n, k):
    import math
    mask = _filter_mask(off.shape[0] - 1)[row0:row0 + n]
    loc_off = off[row0:row0 + n + 1] - off[row0]
    loc_toks = toks[off[row0]:off[row0 + n]]
    mc = _masked_csr(loc_toks, loc_off, vocab, mask)
    flat = np.concatenate([np.asarray(q, np.int64) for q in queries])
    stats = torch.tensor([int(mask.sum()), int(mc["dl"].astype(np.int64).sum())], dtype=torch.int64)
    df = torch.from_numpy(np.where(flat >= 0, mc["df"][np.maximum(flat, 0)], 0).astype(np.int64))
    P.allreduce_filtered_stats(stats, df)
    nc, sl = int(stats[0]), int(stats[1])
    eps = P.filtered_eps_global(mc["df"], mc["first_key"], row0, nc)
    idf = np.zeros(vocab, np.float64)                       # per term: global filtered idf
    for t, d in zip(flat.tolist(), df.numpy().tolist()):
        if t >= 0 and d > 0:
            v = math.log(nc - d + 0.5) - math.log(d + 0.5)
            idf[t] = eps if v < 0 else v
    csr = corc.build_csr(loc_toks, loc_off, vocab)
    sc, rw = corc.bm25_topk(csr, idf, sl / nc, queries, k, allow=mask)
    S, R = P.merge_bm25_topk(torch.from_numpy(sc), torch.from_numpy(np.where(rw >= 0, rw + row0, rw)), k)
    return S.numpy(), R.numpy()


def _worker(rank, WS, port, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(WS))
    dist.init_process_group("gloo", rank=rank, world_size=WS)
    try:
        from classmate_hip import parallel as P
        toks, off, vocab, queries = _corpus()
        nd = off.shape[0] - 1
        row0, n = P.shard_range(nd, rank, WS)
        loc_off = off[row0:row0 + n + 1] - off[row0]
        loc_toks = toks[off[row0]:off[row0 + n]]
        csr = corc.build_csr(loc_toks, loc_off, vocab)
        df, fk, n_all, sum_len = P.allreduce_bm25_stats(csr["df"], csr["first_key"], row0, n,
                                                        int(loc_off[-1]))
        idf, eps = P.bm25_idf_table(df, fk, n_all)
        avgdl = sum_len / n_all
        res = {"rank": rank, "idf": idf, "eps": eps, "avgdl": avgdl, "n": n_all}
        # BM25: shard top-k with global statistics, then the all-gather merge
        for k in (1, 10, 64):
            sc, rw = corc.bm25_topk(csr, idf, avgdl, queries, k)
            S, R = P.merge_bm25_topk(torch.from_numpy(sc), torch.from_numpy(rw + row0), k)
            res[f"bm25_{k}"] = (S.numpy(), R.numpy())
        # dense: shard top-k (f32 distances) then merge
        rng = np.random.default_rng(8)
        emb = rng.standard_normal((nd, 32)).astype(np.float32)
        emb[5] = emb[4]                               # exact duplicate rows across the shard boundary region
        emb[nd // 2 + 1] = emb[4]
        q = rng.standard_normal((NQ, 32)).astype(np.float32)
        q[0] = emb[4]
        d, r = corc.dense_topk_f64(emb[row0:row0 + n], q, 16)
        D, R = P.merge_dense_topk(torch.from_numpy(d.astype(np.float32)), torch.from_numpy(r + row0), 16)
        res["dense"] = (D.numpy(), R.numpy())
        # pool assembly: owner contributes its rows
        rows = torch.tensor([[0, nd - 1, nd // 2, 7]])
        own = (rows >= row0) & (rows < row0 + n)
        local = torch.from_numpy(emb)[rows.clamp(0, nd - 1)] * own.unsqueeze(-1)
        res["pool"] = P.assemble_pool_vectors(rows, local, row0, n).numpy()
        res["max"] = P.max_over_ranks(float(rank) + 0.5)
        # the batched path's exchanges: ONE packed all-gather of both shard lists, then the pool
        # rows of this rank's query block fetched from their owners with one all-to-all
        sc, rw = corc.bm25_topk(csr, idf, avgdl, queries[:NQ], 10)
        d_m, r_m, s_m, b_m = P.exchange_topk(torch.from_numpy(d.astype(np.float32)), torch.from_numpy(r + row0),
                                             torch.from_numpy(sc), torch.from_numpy(np.where(rw >= 0, rw + row0, rw)))
        res["xchg"] = (d_m.numpy(), r_m.numpy(), s_m.numpy(), b_m.numpy())
        bq = NQ // WS
        shard_emb = torch.from_numpy(emb[row0:row0 + n])
        starts = [P.shard_range(nd, i, WS)[0] for i in range(WS)] + [nd]

        def gather_local(lr):          # cm_dense_gather_dev's contract: row < 0 -> a zero row
            return torch.where((lr >= 0)[:, None], shard_emb[lr.clamp(min=0)], torch.zeros(()))
        pool = P.fetch_pool_vectors(r_m, rank * bq, bq, gather_local, starts, 32)
        res["pool_block"] = pool.numpy()
        r_pad = r_m.clone()
        r_pad[:, -3:] = -1                                  # padded pools: zero rows
        res["pool_block_pad"] = P.fetch_pool_vectors(r_pad, rank * bq, bq, gather_local, starts, 32).numpy()
        try:                                                # uneven blocks are refused on every rank
            P.fetch_pool_vectors(r_m[:NQ - 1], rank * bq, bq, gather_local, starts, 32)
            res["uneven"] = None
        except ValueError:
            res["uneven"] = "ValueError"
        # filtered BM25 (quirk Q2): candidate statistics all-reduced, epsilon floor from the
        # global first-occurrence order -- the exchange bm25_search_filtered_sharded runs
        for k in (1, 10, 64):
            res[f"filt_{k}"] = _filtered_shard_search(P, toks, off, vocab, queries, row0, n, k)
        # a failure on one rank is raised on every rank (none is left blocked in a collective)
        try:
            P._raise_together(ValueError("shard failure") if rank == 1 else None)
            res["raise"] = None
        except Exception as e:  # noqa: BLE001
            res["raise"] = type(e).__name__
        # the epsilon exchange with an empty shard (no vocabulary): rank 0's candidates only
        if rank == 0:
            res["eps_uneven"] = P.filtered_eps_global(csr["df"], csr["first_key"], 0, n)
        else:
            res["eps_uneven"] = P.filtered_eps_global(np.zeros(0, np.int64), np.zeros(0, np.uint64), row0,
                                                      P.shard_range(nd, 0, WS)[1])   # the global count
        out_q.put(res)
    finally:
        dist.destroy_process_group()


@pytest.fixture(scope="module", params=[2, 8], ids=["ws2", "ws8"])
def results(request):
    WS = request.param
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, WS, port, q)) for r in range(WS)]
    for p in procs:
        p.start()
    out = [q.get(timeout=240) for _ in range(WS)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return sorted(out, key=lambda r: r["rank"])


def test_sharded_stats_equal_single_shard(results):
    toks, off, vocab, _ = _corpus()
    csr = corc.build_csr(toks, off, vocab)
    idf, eps = corc.bm25_idf(csr["df"], csr["first_key"], off.shape[0] - 1)
    for r in results:
        assert r["n"] == off.shape[0] - 1
        assert r["eps"] == eps
        assert np.array_equal(r["idf"][csr["df"] > 0], idf[csr["df"] > 0])
        assert r["avgdl"] == float(off[-1]) / (off.shape[0] - 1)


@pytest.mark.parametrize("k", [1, 10, 64])
def test_bm25_merge_equals_unsharded_oracle(results, k):
    toks, off, vocab, queries = _corpus()
    csr = corc.build_csr(toks, off, vocab)
    idf, _ = corc.bm25_idf(csr["df"], csr["first_key"], off.shape[0] - 1)
    sc, rw = corc.bm25_topk(csr, idf, float(off[-1]) / (off.shape[0] - 1), queries, k)
    for r in results:                                  # identical on every rank
        S, R = r[f"bm25_{k}"]
        assert np.array_equal(R, rw)
        assert np.array_equal(S, sc)


def test_dense_merge_equals_unsharded(results):
    rng = np.random.default_rng(8)
    toks, off, _, _ = _corpus()
    nd = off.shape[0] - 1
    emb = rng.standard_normal((nd, 32)).astype(np.float32)
    emb[5] = emb[4]
    emb[nd // 2 + 1] = emb[4]
    q = rng.standard_normal((NQ, 32)).astype(np.float32)
    q[0] = emb[4]
    d, r = corc.dense_topk_f64(emb, q, 16)
    for res in results:
        D, R = res["dense"]
        assert np.array_equal(R, r)                    # ties (duplicate rows) by ascending global row
        np.testing.assert_array_equal(D, d.astype(np.float32))


def test_pool_assembly_and_max(results):
    toks, off, _, _ = _corpus()
    nd = off.shape[0] - 1
    emb = np.random.default_rng(8).standard_normal((nd, 32)).astype(np.float32)
    want = emb[[0, nd - 1, nd // 2, 7]]
    for r in results:
        np.testing.assert_array_equal(r["pool"][0], want)
        assert r["max"] == len(results) - 0.5


@pytest.mark.parametrize("k", [1, 10, 64])
def test_filtered_bm25_exchange_equals_unsharded_oracle(results, k):
    """Sharded filtered BM25: the all-reduced candidate statistics and the global epsilon floor
    give rank_bm25 over the filtered documents bit for bit (rag/retrieval/bm25.py:184-191)."""
    toks, off, vocab, queries = _corpus()
    nd = off.shape[0] - 1
    keep = np.nonzero(_filter_mask(nd))[0]
    sub_toks = np.concatenate([toks[off[d]:off[d + 1]] for d in keep])
    sub_off = np.zeros(keep.shape[0] + 1, np.int64)
    sub_off[1:] = np.cumsum(off[keep + 1] - off[keep])
    csr = corc.build_csr(sub_toks, sub_off, vocab)
    idf, eps = corc.bm25_idf(csr["df"], csr["first_key"], keep.shape[0])
    assert (idf == eps).any()                           # the epsilon floor is exercised
    sc, rw = corc.bm25_topk(csr, idf, float(sub_off[-1]) / keep.shape[0], queries, k)
    rw = np.where(rw >= 0, keep[np.maximum(rw, 0)], -1)
    for r in results:
        S, R = r[f"filt_{k}"]
        assert np.array_equal(R, rw)
        assert np.array_equal(S, sc)


def test_packed_exchange_and_pool_fetch(results):
    """exchange_topk (one packed all-gather) == the two separate merges == the unsharded oracle;
    fetch_pool_vectors gives every rank exactly the embeddings of its query block's merged pool."""
    rng = np.random.default_rng(8)
    toks, off, vocab, queries = _corpus()
    nd = off.shape[0] - 1
    emb = rng.standard_normal((nd, 32)).astype(np.float32)
    emb[5] = emb[4]
    emb[nd // 2 + 1] = emb[4]
    q = rng.standard_normal((NQ, 32)).astype(np.float32)
    q[0] = emb[4]
    d, r = corc.dense_topk_f64(emb, q, 16)
    csr = corc.build_csr(toks, off, vocab)
    idf, _ = corc.bm25_idf(csr["df"], csr["first_key"], nd)
    sc, rw = corc.bm25_topk(csr, idf, float(off[-1]) / nd, queries[:NQ], 10)
    bq = NQ // len(results)
    for res in results:
        D, R, S, BR = res["xchg"]
        assert np.array_equal(R, r) and np.array_equal(D, d.astype(np.float32))
        assert np.array_equal(BR, rw) and np.array_equal(S, sc)
        blk = r[res["rank"] * bq:(res["rank"] + 1) * bq]
        np.testing.assert_array_equal(res["pool_block"], emb[blk])
        want = emb[blk].copy()
        want[:, -3:] = 0.0
        np.testing.assert_array_equal(res["pool_block_pad"], want)
        assert res["uneven"] == "ValueError"


def test_errors_raise_on_every_rank_and_empty_shard_eps(results):
    """a local failure must not leave the other ranks blocked in the next collective;
    an empty shard (no vocabulary) joins the epsilon exchange with padded arrays."""
    WS = len(results)
    assert [r["raise"] for r in results] == ["RuntimeError", "ValueError"] + ["RuntimeError"] * (WS - 2)
    toks, off, vocab, _ = _corpus()
    nd = off.shape[0] - 1
    _, n0 = shard_range_cpu(nd, 0, WS)
    csr0 = corc.build_csr(toks[:off[n0]], off[:n0 + 1], vocab)
    _, eps0 = corc.bm25_idf(csr0["df"], csr0["first_key"], n0)
    for r in results:
        assert r["eps_uneven"] == eps0


def shard_range_cpu(n_total, rank, ws):
    per = (n_total + ws - 1) // ws
    lo = min(rank * per, n_total)
    return lo, min(lo + per, n_total) - lo
