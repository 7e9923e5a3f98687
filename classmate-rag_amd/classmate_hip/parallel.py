"""Multi-GPU sharding of the hybrid retrieval path.

One process per GPU (torch.distributed; backend "nccl" == RCCL over xGMI on
ROCm, "gloo" for the CPU tests).  The corpus is sharded by chunk: rank r owns
global rows [row0_r, row0_r + n_r).  Exchanges, and only these:

* build time — BM25 statistics: all-reduce SUM of df[V], N and total length,
  all-reduce MIN of each term's first (global row, position) key, so every rank
  computes the same idf table (including rank_bm25's epsilon floor, averaged in
  the reference's first-occurrence order) and avgdl;
* per query batch (``exchange_topk`` + ``fetch_pool_vectors``, the batched path):
  the B queries are encoded split across ranks (B / G each) and all-gathered;
  every shard's dense top-P (distance, global row) and BM25 top-k (score,
  global row) travel in ONE packed all-gather and are merged deterministically
  on every rank; rank r then fuses query block r only, so the MMR pool vectors
  move as one equal-split all-to-all in which each owner sends the pool entries
  it holds (zeros elsewhere) to the rank fusing that query -- fixed sizes, so
  no host synchronisation inside the step; a final all-gather assembles the
  fused top-k.  ``merge_dense_topk`` / ``merge_bm25_topk`` /
  ``assemble_pool_vectors`` remain for the host-API paths;
* per filtered BM25 batch (quirk Q2: rank_bm25's statistics over the filtered
  candidates, rag/retrieval/bm25.py:184-191) — one all-reduce SUM of the
  candidate count, their total length and the candidate df of the query terms,
  so every shard scores with the global filtered idf/avgdl; only when some idf
  is negative (a term in more than half of the candidates) a second exchange of
  every term's candidate df (SUM) and first-occurrence key (MIN) gives the
  epsilon floor in the global first-occurrence order.

The merges are torch ops so they run on either backend; the per-shard search is
the HIP path (classmate_hip.engine).
"""
from __future__ import annotations

import math
from typing import Optional, Tuple

import numpy as np

try:
    import torch
    import torch.distributed as dist
except Exception:  # pragma: no cover
    torch = None
    dist = None

EMPTY_U64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def world() -> Tuple[int, int]:
    if dist is not None and dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


# ---------------------------------------------------------------------------
# BM25 global statistics
# ---------------------------------------------------------------------------
def bm25_idf_table(df: np.ndarray, first_key: np.ndarray, n_live: int):
    """rank_bm25 idf for every term from global df and first-occurrence keys.

    Returns (idf[V] float64, eps).  Terms are visited in ascending first_key
    order (== the reference's dict insertion order) for the idf average; the
    logs are CPython's math.log (glibc), like rank_bm25."""
    present = np.nonzero(df > 0)[0]
    order = present[np.argsort(first_key[present], kind="stable")]
    idf = np.zeros(df.shape[0], np.float64)
    idf_sum = 0.0
    neg = []
    log = math.log
    for t in order.tolist():
        d = int(df[t])
        v = log(n_live - d + 0.5) - log(d + 0.5)
        idf[t] = v
        idf_sum += v
        if v < 0:
            neg.append(t)
    if len(order) == 0:
        raise ZeroDivisionError("float division by zero")
    eps = 0.25 * (idf_sum / len(order))
    if neg:
        idf[np.asarray(neg)] = eps
    return idf, eps


def allreduce_bm25_stats(df: np.ndarray, first_key: np.ndarray, row0: int, n_live: int, sum_len: int,
                         group=None):
    """Combine per-shard term statistics into the global ones (identity when world == 1)."""
    fk = first_key.astype(np.uint64).copy()
    present = fk != EMPTY_U64
    fk[present] += np.uint64(row0) << np.uint64(32)
    rank, ws = world()
    if ws == 1:
        return df.astype(np.int64), fk, int(n_live), int(sum_len)
    t_df = torch.from_numpy(df.astype(np.int64))
    # keys fit in int63 (rows < 2^31): compare as int64, absent = int64 max
    t_fk = torch.from_numpy(np.where(present, fk, np.uint64(2**63 - 1)).astype(np.int64))
    t_n = torch.tensor([n_live, sum_len], dtype=torch.int64)
    dev = _coll_device(group)
    t_df, t_fk, t_n = t_df.to(dev), t_fk.to(dev), t_n.to(dev)
    dist.all_reduce(t_df, op=dist.ReduceOp.SUM, group=group)
    dist.all_reduce(t_fk, op=dist.ReduceOp.MIN, group=group)
    dist.all_reduce(t_n, op=dist.ReduceOp.SUM, group=group)
    fk_g = t_fk.cpu().numpy().astype(np.uint64)
    fk_g[fk_g == np.uint64(2**63 - 1)] = EMPTY_U64
    n = t_n.cpu().numpy()
    return t_df.cpu().numpy(), fk_g, int(n[0]), int(n[1])


def _coll_device(group=None):
    backend = dist.get_backend(group)
    if backend == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


# ---------------------------------------------------------------------------
# Per-batch merges
# ---------------------------------------------------------------------------
def f32_order_key(dist_t, rows_t):
    """(dist f32, row i64) -> int64 sort key, ascending == (dist asc, row asc); -1 rows -> max."""
    b = dist_t.contiguous().view(torch.int32).to(torch.int64) & 0xFFFFFFFF
    neg = (b & 0x80000000) != 0
    ordered = torch.where(neg, (~b) & 0xFFFFFFFF, b | 0x80000000)
    # rows < 2^31; use 31 bits for the row, so the key stays a positive int64 when shifted by 31
    key = (ordered << 31) | (rows_t & 0x7FFFFFFF)
    return torch.where(rows_t < 0, torch.full_like(key, torch.iinfo(torch.int64).max), key)


def merge_dense_topk(dist_t, rows_t, k: int, group=None):
    """All-gather per-shard (B,k) (distance, global row) and keep the global top-k."""
    _, ws = world()
    if ws == 1:
        return dist_t[:, :k], rows_t[:, :k]
    dl = [torch.empty_like(dist_t) for _ in range(ws)]
    rl = [torch.empty_like(rows_t) for _ in range(ws)]
    dist.all_gather(dl, dist_t.contiguous(), group=group)
    dist.all_gather(rl, rows_t.contiguous(), group=group)
    D = torch.cat(dl, 1)
    R = torch.cat(rl, 1)
    key = f32_order_key(D, R)
    _, idx = torch.sort(key, dim=1)
    idx = idx[:, :k]
    return torch.gather(D, 1, idx), torch.gather(R, 1, idx)


def merge_bm25_topk(score_t, rows_t, k: int, group=None):
    """All-gather per-shard (B,k) (score f64, global row) -> global top-k by (score desc, row asc)."""
    _, ws = world()
    if ws == 1:
        return score_t[:, :k], rows_t[:, :k]
    sl = [torch.empty_like(score_t) for _ in range(ws)]
    rl = [torch.empty_like(rows_t) for _ in range(ws)]
    dist.all_gather(sl, score_t.contiguous(), group=group)
    dist.all_gather(rl, rows_t.contiguous(), group=group)
    S = torch.cat(sl, 1)
    R = torch.cat(rl, 1)
    big = torch.iinfo(torch.int64).max
    Rk = torch.where(R < 0, torch.full_like(R, big), R)
    S = S + 0.0                                   # -0.0 == 0.0 like Python
    Sk = torch.where(R < 0, torch.full_like(S, -math.inf), S)
    i1 = torch.argsort(Rk, dim=1, stable=True)   # row asc ...
    S1 = torch.gather(Sk, 1, i1)
    i2 = torch.argsort(-S1, dim=1, stable=True)  # ... then score desc (stable keeps row order)
    idx = torch.gather(i1, 1, i2)[:, :k]
    return torch.gather(S, 1, idx), torch.gather(R, 1, idx)


def allreduce_filtered_stats(stats_t, df_t, group=None):
    """Sum the shards' candidate statistics ({Nc, sum of lengths} and per-query-term df, int64
    tensors, in place; identity when world == 1).  Runs on the collective's device."""
    _, ws = world()
    if ws == 1:
        return stats_t, df_t
    dev = _coll_device(group)
    for t in (stats_t, df_t):
        x = t.to(dev)
        dist.all_reduce(x, op=dist.ReduceOp.SUM, group=group)
        if x.data_ptr() != t.data_ptr():
            t.copy_(x)
    return stats_t, df_t


def filtered_eps_global(df_v: np.ndarray, first_key: np.ndarray, row0: int, n_cand: int, group=None) -> float:
    """rank_bm25's epsilon over the global candidate set: every term's candidate df summed and its
    first (global row, position) key minimised over the shards, then the idf average in that
    first-occurrence order (bm25_idf_table).  A shard whose vocabulary is shorter (an empty shard
    has none) pads with absent terms."""
    df_v, first_key = np.asarray(df_v, np.int64), np.asarray(first_key, np.uint64)
    V = _max_flags([df_v.shape[0]], group)[0]
    if df_v.shape[0] < V:
        df_v = np.concatenate([df_v, np.zeros(V - df_v.shape[0], np.int64)])
        first_key = np.concatenate([first_key, np.full(V - first_key.shape[0], EMPTY_U64)])
    gdf, gfk, _, _ = allreduce_bm25_stats(df_v, first_key, row0, 0, 0, group=group)
    _, eps = bm25_idf_table(gdf, gfk, int(n_cand))
    return eps


def _max_flags(vals, group=None):
    """Element-wise MAX of small integers over the ranks (identity when world == 1)."""
    _, ws = world()
    if ws == 1:
        return [int(v) for v in vals]
    t = torch.tensor([int(v) for v in vals], dtype=torch.int64, device=_coll_device(group))
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return [int(v) for v in t.cpu().tolist()]


def _raise_together(err, group=None):
    """Every rank raises when any rank failed, so no rank is left blocked in the next collective:
    the failing rank re-raises its own exception, the others a RuntimeError naming it."""
    if _max_flags([err is not None], group)[0]:
        if err is not None:
            raise err
        raise RuntimeError("sharded BM25 search failed on another rank")


def bm25_search_filtered_sharded(bm, q_terms, q_off, k: int, allow, row0: int, group=None):
    """Filtered BM25 over a sharded corpus: local candidate statistics -> all-reduce -> every shard
    scores its allowed documents with the global statistics (device idf) -> all-gather merge.
    bm: this rank's engine.BM25Index (prepare_filtered(global docs) called); allow: this shard's
    device allow words.  Returns the global (scores, global rows) top-k, identical on all ranks.

    Every rank joins every exchange: a shard without documents contributes zero statistics and
    empty lists, and an error on one rank is raised on all of them (_raise_together)."""
    nq = q_off.numel() - 1
    dev = q_terms.device
    empty = bm.num_docs == 0
    err = stats = df = None
    try:
        if empty:
            stats = torch.zeros(2, dtype=torch.int64, device=dev)
            df = torch.zeros(max(q_terms.numel(), 1), dtype=torch.int64, device=dev)
        else:
            stats, df = bm.filter_stats_dev(allow, q_terms)
    except Exception as e:  # noqa: BLE001 -- re-raised below on every rank
        err = e
    _raise_together(err, group)
    allreduce_filtered_stats(stats, df, group)

    def local_search(eps_t=None):
        if empty:
            return (torch.zeros((nq, k), dtype=torch.float64, device=dev),
                    torch.full((nq, k), -1, dtype=torch.int64, device=dev), 0)
        s_, r_, st_ = bm.search_stats_dev(q_terms, q_off, k, allow, stats, df, eps=eps_t)
        return s_, r_, int(st_.item())

    s = r = None
    code = 0
    try:
        s, r, code = local_search()
    except Exception as e:  # noqa: BLE001
        err = e
    _raise_together(err, group)
    eps_missing = _max_flags([code & bm.FILT_EPS_MISSING], group)[0]
    if eps_missing:                         # global statistics: the epsilon floor over all shards
        try:
            if empty:
                dfv, fkv = np.zeros(0, np.int64), np.zeros(0, np.uint64)
            else:
                dfv_t, fkv_t = bm.filter_term_stats_dev(allow)
                dfv, fkv = dfv_t.cpu().numpy(), fkv_t.cpu().numpy().view(np.uint64)
        except Exception as e:  # noqa: BLE001
            err = e
        _raise_together(err, group)
        eps = filtered_eps_global(dfv, fkv, row0, int(stats[0].item()), group)
        eps_t = torch.tensor([eps], dtype=torch.float64, device=dev)
        try:
            s, r, code = local_search(eps_t)
        except Exception as e:  # noqa: BLE001
            err = e
        _raise_together(err, group)
    zero_div, other = _max_flags([code & bm.FILT_ZERO_DIV, code & ~(bm.FILT_ZERO_DIV | bm.FILT_EPS_MISSING)], group)
    if zero_div:
        raise ZeroDivisionError("float division by zero (candidate documents have no tokens)")
    if other:
        raise RuntimeError(f"filtered BM25 search status {other}")
    rg = torch.where(r >= 0, r + row0, r)
    return merge_bm25_topk(s, rg, k, group)


def assemble_pool_vectors(rows_t, local_vecs, row0: int, n_local: int, group=None):
    """Pool embeddings for global rows: owner rank contributes, others zeros; SUM all-reduce."""
    _, ws = world()
    own = (rows_t >= row0) & (rows_t < row0 + n_local)
    out = torch.where(own.unsqueeze(-1), local_vecs, torch.zeros_like(local_vecs))
    if ws > 1:
        dist.all_reduce(out, op=dist.ReduceOp.SUM, group=group)
    return out


def _host_staged(group=None) -> bool:
    """gloo (the CPU tests, and the one-GPU rehearsal of the N > 1 path) moves host tensors only;
    RCCL ("nccl") moves device tensors in place over xGMI."""
    return dist.get_backend(group) != "nccl"


def all_gather_into(out, t, group=None):
    """out (ws * n, ...) <- every rank's t (n, ...), rank order."""
    if _host_staged(group) and t.is_cuda:
        parts = [torch.empty_like(t, device="cpu") for _ in range(world()[1])]
        dist.all_gather(parts, t.cpu(), group=group)
        out.copy_(torch.cat(parts, 0))
    else:
        dist.all_gather_into_tensor(out, t.contiguous(), group=group)
    return out


def all_to_all(recv, send, recv_splits, send_splits, group=None):
    """All-to-all of rows (splits: row counts per rank, or None for equal splits)."""
    if _host_staged(group) and send.is_cuda:
        r = torch.empty_like(recv, device="cpu")
        dist.all_to_all_single(r, send.cpu(), output_split_sizes=recv_splits, input_split_sizes=send_splits,
                               group=group)
        recv.copy_(r)
    else:
        dist.all_to_all_single(recv, send.contiguous(), output_split_sizes=recv_splits,
                               input_split_sizes=send_splits, group=group)
    return recv


def _all_gather_cat(t, group=None):
    """(ws, *t.shape) stack of every rank's t (same shape on all ranks)."""
    _, ws = world()
    out = torch.empty((ws * t.shape[0],) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
    return all_gather_into(out, t.contiguous(), group).view((ws,) + tuple(t.shape))


def exchange_topk(d, r, bs, br, group=None):
    """Every shard's dense (B, P) (distance f32, global row) and BM25 (B, K) (score f64, global row)
    top lists -> the global ones, identical on every rank, through ONE all-gather of a packed int64
    tensor.  Merge order as merge_dense_topk (distance asc, row asc) and merge_bm25_topk (score
    desc, row asc; -1 pads last)."""
    _, ws = world()
    if ws == 1:
        return d, r, bs, br
    B, P = d.shape
    K = bs.shape[1]
    pack = torch.cat([d.contiguous().view(torch.int32).to(torch.int64), r.to(torch.int64),
                      bs.contiguous().view(torch.int64), br.to(torch.int64)], 1)
    allp = _all_gather_cat(pack, group)                                    # (ws, B, 2P + 2K)
    return merge_packed(allp, P, K)


def merge_packed(allp, P: int, K: int):
    """The merge of exchange_topk: allp (ws, B, 2P + 2K) int64 packed shard lists -> the global dense
    (B, P) and BM25 (B, K) lists.  Device tensors: the hand-written kernel (cm_shard_merge_topk_dev,
    one launch, stream-ordered); host tensors (the gloo CPU tests): the same order through torch
    sorts (merge_dense_topk / merge_bm25_topk's rules)."""
    ws, B = allp.shape[0], allp.shape[1]
    if allp.is_cuda:
        from . import _lib as L
        from .engine import _stream
        allp = allp.contiguous()
        d_m = torch.empty((B, P), dtype=torch.float32, device=allp.device)
        r_m = torch.empty((B, P), dtype=torch.int64, device=allp.device)
        s_m = torch.empty((B, K), dtype=torch.float64, device=allp.device)
        b_m = torch.empty((B, K), dtype=torch.int64, device=allp.device)
        L.check(L.fn["cm_shard_merge_topk_dev"](L.ptr(allp), ws, B, P, K, L.ptr(d_m), L.ptr(r_m), L.ptr(s_m),
                                                L.ptr(b_m), _stream(allp.device.index)), "cm_shard_merge_topk_dev")
        return d_m, r_m, s_m, b_m
    D = allp[:, :, :P].to(torch.int32).view(torch.float32).permute(1, 0, 2).reshape(B, ws * P)
    R = allp[:, :, P:2 * P].permute(1, 0, 2).reshape(B, ws * P)
    S = allp[:, :, 2 * P:2 * P + K].contiguous().view(torch.float64).permute(1, 0, 2).reshape(B, ws * K)
    BR = allp[:, :, 2 * P + K:].permute(1, 0, 2).reshape(B, ws * K)
    _, idx = torch.sort(f32_order_key(D, R), dim=1)
    idx = idx[:, :P]
    d_m, r_m = torch.gather(D, 1, idx), torch.gather(R, 1, idx)
    big = torch.iinfo(torch.int64).max
    Rk = torch.where(BR < 0, torch.full_like(BR, big), BR)
    S = S + 0.0                                   # -0.0 == 0.0 like Python
    Sk = torch.where(BR < 0, torch.full_like(S, -math.inf), S)
    i1 = torch.argsort(Rk, dim=1, stable=True)
    i2 = torch.argsort(-torch.gather(Sk, 1, i1), dim=1, stable=True)
    idx = torch.gather(i1, 1, i2)[:, :K]
    return d_m, r_m, torch.gather(S, 1, idx), torch.gather(BR, 1, idx)


_STARTS: dict = {}


def _starts_tensor(shard_starts, dev):
    key = (tuple(int(x) for x in shard_starts), str(dev))
    t = _STARTS.get(key)
    if t is None:
        if len(_STARTS) > 16:
            _STARTS.clear()
        t = _STARTS[key] = torch.as_tensor(list(key[0]), dtype=torch.int64, device=dev)
    return t


def fetch_pool_vectors(rows, q_lo: int, bq: int, gather_local, shard_starts, dim: int, group=None):
    """Embeddings of the merged MMR pool for THIS rank's query block [q_lo, q_lo + bq).

    rows: (B, P) merged global rows (-1 pad), identical on all ranks, B = bq x world and rank r's
    block = [r bq, (r + 1) bq); gather_local(local_rows int64 device tensor, -1 -> zero row) ->
    (n, D) fp32 rows of this rank's shard; shard_starts: G + 1 global row boundaries.

    Fixed-size exchange, no host synchronisation: every rank gathers the B x P pool entries it owns
    (zeros elsewhere) -- block-major, so the slice for peer p is exactly p's query block -- and ONE
    equal-split all-to-all of bq.P rows per peer delivers them; the receiver picks each entry from
    its owner's slice.  B.P.D.4 bytes per rank (G x the compacted exchange, 18.9 MB at B = 256,
    P = 24), in exchange for no data-dependent split sizes: the step stays stream-ordered on RCCL.
    The volume grows with the global batch (B = 2048: ~150 MB each way per rank, ~1 ms of xGMI at
    ~150 GB/s per link against the ~0.1 ms host round trip the compacted exchange's split sizes
    cost), so the equal split pays up to B ~ 512 at P = 24; larger global batches should be issued
    as several retrieval steps of <= 512 queries (the bench and the driver use B = 256 per rank).
    Returns (bq, P, D) fp32 (zeros for -1 pads)."""
    rank, ws = world()
    B, P = rows.shape
    dev = rows.device
    if ws == 1:
        return gather_local(rows.reshape(-1)).view(B, P, -1)
    if B != bq * ws or q_lo != rank * bq or len(shard_starts) != ws + 1:
        raise ValueError(f"fetch_pool_vectors: rows ({B}) must be {ws} equal query blocks of {bq} with this "
                         f"rank's block at {rank * bq} (got q_lo={q_lo}) and {ws + 1} shard boundaries")
    D = int(dim)
    lo, hi = int(shard_starts[rank]), int(shard_starts[rank + 1])
    mine = (rows >= lo) & (rows < hi)
    send = gather_local(torch.where(mine, rows - lo, torch.full_like(rows, -1)).reshape(-1)).reshape(B * P, D)
    recv = torch.empty((B * P, D), dtype=torch.float32, device=dev)
    all_to_all(recv, send, None, None, group)
    blk = rows[q_lo:q_lo + bq].reshape(-1)
    sizes = {int(shard_starts[i + 1]) - int(shard_starts[i]) for i in range(ws - 1)}
    if len(sizes) == 1 and int(shard_starts[0]) == 0 and min(sizes) > 0:
        # equal shards (the bench, weak scaling): the owner is a division, one elementwise kernel
        owner = torch.div(blk.clamp(min=0), min(sizes), rounding_mode="floor").clamp_(max=ws - 1)
    else:
        starts = _starts_tensor(shard_starts, dev)      # resident: no per-step host-to-device copy
        owner = (torch.searchsorted(starts, blk, right=True) - 1).clamp_(0, ws - 1)    # pads: any slice is zero
    pool = recv.view(ws, bq * P, D)[owner, torch.arange(bq * P, device=dev)]
    return pool.view(bq, P, D)


def max_over_ranks(x: float, device=None, group=None) -> float:
    _, ws = world()
    if ws == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())


def shard_range(n_total: int, rank: int, ws: int) -> Tuple[int, int]:
    per = (n_total + ws - 1) // ws
    lo = min(rank * per, n_total)
    return lo, min(lo + per, n_total) - lo


def init_from_env(backend: Optional[str] = None):
    """torch.distributed init for torchrun (MASTER_ADDR/PORT, RANK, WORLD_SIZE)."""
    import os
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    if ws <= 1 or dist.is_initialized():
        return world()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    if backend == "nccl":
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
    dist.init_process_group(backend=backend)
    return world()
