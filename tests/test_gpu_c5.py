"""C5 (BASELINE configs[4]): the 8-way corpus split, rehearsed with 8 ranks on the one GPU.

Eight spawned ranks (gloo exchanges, every rank on cuda:0 -- RCCL refuses two ranks per device;
the driver's 8-GPU runs use RCCL over the same code) each own a 1M-row dense shard and a
1M-document BM25 shard, and run bench.py's batched step:
  rank r encodes its block of B / 8 queries with the fp32 E5 (K10) -> all-gather of the (B, 768)
  query embeddings -> per-shard dense top-24 (K1c / K1s) and BM25 top-10 (K2a/K2b/K2 + K3, global
  statistics from the build-time all-reduce) -> ONE packed all-gather + merge (exchange_topk) ->
  the 8-owner pool all-to-all (fetch_pool_vectors) -> K4 MMR + K5 RRF on the rank's block ->
  all-gather of the fused top-10.
Checked against the unsharded references:
  BM25: the C oracle (oracle/cm_oracle.c, rank_bm25 0.2.2 restated) over all 8M documents, bit for
    bit;
  dense: the exact fp64 scan of all 8M rows (each rank scans its own rows on the host in fp64; a
    merge of exact per-shard lists is the exact global list), within 1e-4;
  pool vectors: the fp32 rows of their owners, bit for bit;
  fused top-10: the CPU restatement of HybridRetriever.retrieve (rag/retrieval/fusion.py:108-167;
    oracle/ref_semantics.py mmr_order / rrf_fuse) over the exact pools.
"""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

WS = 8
N_RANK = 1 << 20
B, K, P, D = 64, 10, 24, 768
SLACK = 40


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _bm25_queries(vocab):
    rng = np.random.default_rng(15)
    qs = [rng.integers(0, 3000, 8).tolist() for _ in range(B - 4)]
    return qs + [[0, 1], [vocab - 1], [4000, 4000, 17], [rng.integers(0, vocab)] * 3]


def _e5_token_ids(torch, dev):
    g = torch.Generator(device="cuda").manual_seed(21)
    ids = torch.randint(5, 250002, (B, 24), device=dev, generator=g)
    ids[:, 0], ids[:, -1] = 0, 2
    return ids


def _shard_exact(C, q, row0, kk):
    """Exact fp64 top-kk of this shard (global rows)."""
    from test_gpu_scale import exact_topk
    d, r = exact_topk(C, q, kk)
    return d, r + row0


def _worker(rank, port, out_q):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(WS))
    dist.init_process_group("gloo", rank=rank, world_size=WS)
    try:
        from test_gpu_scale import VOCAB, _bm25_docs, unit_rows
        from classmate_hip import engine
        from classmate_hip import parallel as Pl
        from classmate_hip.embeddings import E5MultilingualEmbedder
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(0)
        row0 = rank * N_RANK
        starts = [i * N_RANK for i in range(WS + 1)]
        # shards: BM25 with global statistics (build-time all-reduce), dense rows
        toks, off = _bm25_docs(row0, row0 + N_RANK)
        bm = engine.BM25Index(device=0)
        bm.build(toks, off, VOCAB)
        del toks, off
        df, fk = bm.term_stats()
        st = bm.stats()
        gdf, gfk, gn, gsum = Pl.allreduce_bm25_stats(df, fk, row0, st["n_live"], st["sum_len"])
        idf, eps = Pl.bm25_idf_table(gdf, gfk, gn)
        bm.set_stats(idf, gn, gsum, eps)
        C = unit_rows(N_RANK, D, seed=9, row0=row0)
        dn = engine.DenseIndex(D, device=0, capacity=N_RANK)
        dn.upsert(C, np.arange(N_RANK, dtype=np.int64))
        # the batched step
        bq, q_lo = B // WS, rank * (B // WS)
        e5 = E5MultilingualEmbedder.random_init(seed=0, device=str(dev), dtype="float32")
        ids = _e5_token_ids(torch, dev)
        q_local = e5.encode_token_ids(ids[q_lo:q_lo + bq], torch.ones_like(ids[q_lo:q_lo + bq]))
        q = Pl.all_gather_into(torch.empty((B, D), dtype=torch.float32, device=dev), q_local)
        qs = _bm25_queries(VOCAB)
        q_terms = torch.tensor([t for x in qs for t in x], dtype=torch.int32, device=dev)
        q_off = torch.tensor(np.concatenate([[0], np.cumsum([len(x) for x in qs])]), dtype=torch.int32, device=dev)
        d, r = dn.search_dev(q, P)
        bs, br = bm.search_dev(q_terms, q_off, K)
        rgl = torch.where(r >= 0, r + row0, r)
        brl = torch.where(br >= 0, br + row0, br)
        dm, rg, bsm, brg = Pl.exchange_topk(d, rgl, bs, brl)
        blk = slice(q_lo, q_lo + bq)
        vecs = Pl.fetch_pool_vectors(rg, q_lo, bq, lambda lr: dn.gather_dev(lr), starts, D)
        order = engine.mmr_dev(q[blk].contiguous(), vecs, K, 0.5)
        vk, vd, vn, bn = engine.rrf_pool_prep_dev(rg[blk].contiguous(), dm[blk].contiguous(), order,
                                                  brg[blk].contiguous())
        res = engine.rrf_merge_dev(vk, vd, vn, brg[blk].contiguous(), bsm[blk].contiguous(), bn,
                                   w_vec=1.0, w_bm25=1.0, rrf_k=60, top_k=K)
        keys = Pl.all_gather_into(torch.empty((B, K), dtype=res[0].dtype, device=dev), res[0])
        torch.cuda.synchronize()
        qh = q.cpu().numpy()
        rg_h = rg.cpu().numpy()
        mine = np.unique(rg_h[(rg_h >= row0) & (rg_h < row0 + N_RANK)])
        out = {"rank": rank, "q": qh, "dm": dm.cpu().numpy(), "rg": rg_h, "bsm": bsm.cpu().numpy(),
               "brg": brg.cpu().numpy(), "keys": keys.cpu().numpy(), "pool_block": vecs.cpu().numpy(),
               "own_rows": {int(x): C[x - row0].copy() for x in mine},
               "exact": _shard_exact(C, qh, row0, P + SLACK)}
        dn.close()
        bm.close()
        out_q.put(out)
    finally:
        dist.destroy_process_group()


def test_eight_rank_split_1m_rows_each():
    import torch.multiprocessing as mp
    from test_gpu_scale import TIE, VOCAB, _bm25_docs, check_dense
    from oracle import corc
    from oracle import ref_semantics as orc
    ctx = mp.get_context("spawn")
    qu = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, port, qu)) for r in range(WS)]
    for p in procs:
        p.start()
    # the unsharded BM25 oracle over all 8M documents, built while the ranks run
    toks, off = _bm25_docs(0, WS * N_RANK)
    csr = corc.build_csr(toks, off, VOCAB)
    idf, _ = corc.bm25_idf(csr["df"], csr["first_key"], WS * N_RANK)
    o_sc, o_rw = corc.bm25_topk(csr, idf, float(off[-1]) / (WS * N_RANK), _bm25_queries(VOCAB), K)
    del toks, off, csr
    out = sorted([qu.get(timeout=600) for _ in range(WS)], key=lambda x: x["rank"])
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    q = out[0]["q"]
    for res in out[1:]:                               # every rank holds the same merged lists
        for f in ("q", "dm", "rg", "bsm", "brg", "keys"):
            assert np.array_equal(res[f], out[0][f]), f
    # BM25: bit for bit against the unsharded oracle
    assert np.array_equal(out[0]["brg"], o_rw) and np.array_equal(out[0]["bsm"], o_sc)
    # dense: the exact fp64 list over all 8M rows (merge of the exact shard lists)
    ed = np.concatenate([r["exact"][0] for r in out], 1)
    er = np.concatenate([r["exact"][1] for r in out], 1)
    o = np.lexsort((er, ed), axis=1)[:, :P + SLACK]
    o_d, o_r = np.take_along_axis(ed, o, 1), np.take_along_axis(er, o, 1)
    check_dense(out[0]["dm"], out[0]["rg"], o_d, o_r, P)
    assert len(np.unique(o_r[:, :P] // N_RANK)) == WS      # the pools span every shard
    # pool vectors: each rank's block holds its merged pool rows, fetched from their owners
    rows = {}
    for res in out:
        rows.update(res["own_rows"])
    bq = B // WS
    for res in out:
        blk = out[0]["rg"][res["rank"] * bq:(res["rank"] + 1) * bq]
        want = np.stack([np.stack([rows[int(x)] for x in row]) for row in blk])
        assert np.array_equal(res["pool_block"], want), res["rank"]
    # fused top-10: the CPU restatement of retrieve() over the exact pools
    checked = 0
    for i in range(B):
        if o_d[i, P] - o_d[i, P - 1] <= TIE:                     # ambiguous pool boundary: skip
            continue
        pool = o_r[i, :P]
        cand = np.stack([rows[int(x)] for x in pool])
        ordr = orc.mmr_order(q[i], cand, list(range(P)), K, 0.5)
        vec_ids = [int(pool[j]) for j in ordr]
        bm_ids = [int(x) for x in o_rw[i] if x >= 0]
        fz = orc.rrf_fuse(rank_lists=[vec_ids, bm_ids], weights=[1.0, 1.0], rrf_k=60)
        vdist = {int(pool[j]): float(np.float32(o_d[i, j])) for j in ordr}
        items = list(dict.fromkeys(vec_ids + bm_ids))
        items.sort(key=lambda x: (fz[x], -vdist.get(x, 0.0)), reverse=True)
        assert [int(x) for x in out[0]["keys"][i] if x >= 0] == items[:K], i
        checked += 1
    assert checked >= B // 2
    print(f"\nC5 8-rank rehearsal: {WS} x {N_RANK} rows / docs, {B} queries, fused top-{K} checked on {checked}")
