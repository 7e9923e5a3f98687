"""One corpus over several devices in ONE process (SURVEY §8(b) Threading, §8(e)).

The reference's caller is a single process (``ask_question``, rag/pipeline/rag.py:531-549) that
builds ``ChromaVectorStore`` / ``BM25Store`` and asks.  With ``CM_DEVICES=0,1,...`` (two or more
entries; repeats allowed: ``0,0,0,0`` puts four shards on one card, the GPU tests' rehearsal) the
drop-in stores create a ``ShardedDenseIndex`` / ``ShardedBM25Index`` instead of one handle, so one
process serves a corpus larger than one GPU's HBM (~40M rows per MI355X).

Row layout: the store's global rows are cut into blocks of ``CM_SHARD_BLOCK`` rows (default
65536, a power of two >= 32) dealt round-robin to the shards -- block b lives on shard b % G at
local block b // G -- so every shard holds contiguous runs of global rows, a growing store stays
balanced, and row maps are shifts and masks (no tables).  BM25 documents (the BM25 store's own
rows) are dealt the same way.

Per search:
* dense: every shard's handle searches on its own HIP stream (the launches are asynchronous, so one
  host thread drives every device; a where-filter's allow words are cut into the shards' local
  words on the device), the local top lists become (distance, global row) pairs, move to the first
  device (peer copy) and ``shard_merge_kernel`` (K3x, cm_shard_merge_topk_dev) merges them exactly
  like the reference's (distance, row) order;
* BM25: the statistics are global -- N, total length, df and the first-occurrence order summed /
  minimised over the shards at build, installed on every shard (cm_bm25_set_stats); a where-filter
  needs the filtered candidates' statistics of ALL shards (quirk Q2, rag/retrieval/bm25.py:184-191):
  per-shard candidate counts, lengths and query-term df are summed, and rank_bm25's epsilon floor,
  when some idf is negative, comes from the global candidate vocabulary in global first-occurrence
  order.  Every shard then scores with the global statistics and the lists merge by (score desc,
  row asc);
* MMR pool rows are gathered from their owners (peer copies of B x P rows).

Host-array searches (``search``) run shard by shard and merge on the host: exact for any k.
"""
from __future__ import annotations

import math
import os
from typing import List, Optional, Sequence

import numpy as np

from . import _lib as L
from . import engine, parallel

try:
    import torch
except Exception:  # pragma: no cover
    torch = None

BLOCK_DEFAULT = 1 << 16
_EMPTY = np.uint64(0xFFFFFFFFFFFFFFFF)


def shard_devices() -> Optional[List[int]]:
    """The devices of ``CM_DEVICES`` (comma separated), or None for a one-handle index."""
    env = os.environ.get("CM_DEVICES", "").strip()
    if not env:
        return None
    devs = [int(x) for x in env.split(",") if x.strip()]
    return devs if len(devs) > 1 else None


def _block_rows() -> int:
    b = int(os.environ.get("CM_SHARD_BLOCK", BLOCK_DEFAULT))
    if b < 32 or b & (b - 1):
        raise ValueError(f"CM_SHARD_BLOCK must be a power of two >= 32 (got {b})")
    return b


class RowMap:
    """global row g <-> (shard s, local row l): block g >> lb goes to shard (g >> lb) % G."""

    def __init__(self, G: int, block: int):
        self.G, self.B, self.lb = int(G), int(block), int(block).bit_length() - 1

    def owner_local(self, g):
        """numpy or torch int64 global rows (>= 0) -> (shard, local row)."""
        blk = g >> self.lb
        return blk % self.G, ((blk // self.G) << self.lb) | (g & (self.B - 1))

    def to_global(self, s: int, l):
        """local rows of shard s (numpy / torch int64; -1 stays -1) -> global rows."""
        g = (((l >> self.lb) * self.G + s) << self.lb) | (l & (self.B - 1))
        if torch is not None and isinstance(l, torch.Tensor):
            return torch.where(l >= 0, g, l)
        return np.where(l >= 0, g, l)

    def local_count(self, s: int, n: int) -> int:
        """Rows of [0, n) that shard s holds (its local high-water for a dense prefix)."""
        full, rem = divmod(int(n), self.B)
        cnt = ((full - s + self.G - 1) // self.G if full > s else 0) * self.B
        if rem and full % self.G == s:
            cnt += rem
        return cnt

    def split_words(self, words, n_shards: int):
        """Global allow words (numpy uint32 / torch int32, bit r & 31 of word r >> 5) -> a list of
        the shards' local words (same kind): block b's B / 32 words go to shard b % G."""
        W = self.B // 32
        nw = int(words.shape[0])
        nbp = -(-max(-(-nw // W), 1) // self.G) * self.G
        if torch is not None and isinstance(words, torch.Tensor):
            pad = torch.zeros(nbp * W, dtype=words.dtype, device=words.device)
            pad[:nw] = words
            v = pad.view(nbp // self.G, self.G, W).transpose(0, 1).contiguous().view(self.G, -1)
            return [v[s] for s in range(n_shards)]
        pad = np.zeros(nbp * W, words.dtype)
        pad[:nw] = words
        v = np.ascontiguousarray(pad.reshape(nbp // self.G, self.G, W).transpose(1, 0, 2).reshape(self.G, -1))
        return [v[s] for s in range(n_shards)]


def _f32_key_np(d: np.ndarray, r: np.ndarray) -> np.ndarray:
    """(distance f32, row) -> int64 key ordering like (distance asc, row asc); rows < 0 last."""
    b = np.ascontiguousarray(d, np.float32).view(np.uint32).astype(np.int64)
    ordered = np.where(b & 0x80000000, (~b) & 0xFFFFFFFF, b | 0x80000000)
    key = (ordered << 31) | (r & 0x7FFFFFFF)
    return np.where(r < 0, np.iinfo(np.int64).max, key)


def _pack(first, first_rows, second, second_rows):
    """One shard's lists in the packed layout cm_shard_merge_topk_dev reads: [dist f32 bits | rows |
    score f64 bits | rows] (int64)."""
    return torch.cat([first.contiguous().view(torch.int32).to(torch.int64), first_rows.to(torch.int64),
                      second.contiguous().view(torch.int64), second_rows.to(torch.int64)], 1)


class _Shards:
    def _streams(self):
        if self._st is None:
            self._st = [torch.cuda.Stream(device=d) for d in self.devices]
        return self._st

    def _fork(self):
        """An event on the caller's stream (primary device) every shard stream waits for."""
        cur = torch.cuda.current_stream(self.device)
        ev = torch.cuda.Event()
        ev.record(cur)
        return cur, ev

    def _to(self, t, s: int, st):
        """t (primary device) as seen from shard s's stream: itself (same device, recorded for the
        stream) or a stream-ordered peer copy."""
        if t is None:
            return None
        if self.devices[s] == t.device.index:
            t.record_stream(st)
            return t
        return t.to(torch.device("cuda", self.devices[s]), non_blocking=True)


class ShardedDenseIndex(_Shards):
    """engine.DenseIndex's interface over G handles (see the module docstring)."""

    sharded = True

    def __init__(self, dim: int, devices: Sequence[int], capacity: int = 0, block: Optional[int] = None):
        self.devices = [int(d) for d in devices]
        self.G = len(self.devices)
        self.map = RowMap(self.G, block or _block_rows())
        self.dim = int(dim)
        self.device = self.devices[0]
        self.shards = [engine.DenseIndex(dim, device=d, capacity=max(self.map.local_count(s, capacity), 0))
                       for s, d in enumerate(self.devices)]
        self._st = None

    def close(self):
        for sh in self.shards:
            sh.close()

    # -- mutation ---------------------------------------------------------
    def upsert(self, vecs: np.ndarray, rows: np.ndarray):
        v = np.ascontiguousarray(vecs, np.float32)
        r = np.ascontiguousarray(rows, np.int64)
        if v.ndim != 2 or v.shape[1] != self.dim or v.shape[0] != r.shape[0]:
            raise ValueError(f"expected ({r.shape[0]}, {self.dim}) embeddings, got {v.shape}")
        if (r < 0).any():
            raise ValueError("rows must be >= 0")
        s, l = self.map.owner_local(r)
        for i, sh in enumerate(self.shards):
            m = s == i
            if m.all():
                sh.upsert(v, l)
            elif m.any():
                sh.upsert(v[m], l[m])

    def delete(self, rows):
        r = np.ascontiguousarray(rows, np.int64)
        r = r[r >= 0]
        s, l = self.map.owner_local(r)
        for i, sh in enumerate(self.shards):
            m = s == i
            if m.any():
                sh.delete(l[m])

    def reserve(self, capacity: int):
        for s, sh in enumerate(self.shards):
            sh.reserve(self.map.local_count(s, capacity))

    def mem_stats(self) -> dict:
        st = [sh.mem_stats() for sh in self.shards]
        return {"bytes": sum(x["bytes"] for x in st), "peak_bytes": sum(x["peak_bytes"] for x in st),
                "staged_growths": sum(x["staged_growths"] for x in st), "per_shard": st}

    # -- queries ----------------------------------------------------------
    @property
    def size(self) -> int:
        n = 0
        for s, sh in enumerate(self.shards):
            ns = sh.size
            if ns > 0:
                n = max(n, int(self.map.to_global(s, np.array([ns - 1], np.int64))[0]) + 1)
        return n

    def live_count(self) -> int:
        return sum(sh.live_count() for sh in self.shards)

    def export(self, row0: int = 0, n: Optional[int] = None, with_live: bool = False):
        n = self.size - row0 if n is None else int(n)
        n = max(n, 0)
        out = np.zeros((n, self.dim), np.float32)
        live = np.zeros(n, bool)
        g = row0
        while g < row0 + n:
            end = min(((g >> self.map.lb) + 1) << self.map.lb, row0 + n)
            s, l = self.map.owner_local(np.array([g], np.int64))
            s, l = int(s[0]), int(l[0])
            sh = self.shards[s]
            avail = max(0, min(end - g, sh.size - l))
            if avail:
                part = sh.export(l, avail, with_live=with_live)
                if with_live:
                    out[g - row0:g - row0 + avail], live[g - row0:g - row0 + avail] = part
                else:
                    out[g - row0:g - row0 + avail] = part
            g = end
        return (out, live) if with_live else out

    def search_kind(self, nq: int, k: int) -> int:
        return self.shards[0].search_kind(nq, k)

    def _allow_parts(self, allow_bits):
        if allow_bits is None:
            return [None] * self.G
        return self.map.split_words(allow_bits, self.G)

    def search(self, q: np.ndarray, k: int, allow_bits=None, return_vectors: bool = False):
        """Host arrays: every shard's exact top-k, merged by (distance, global row)."""
        qq = np.ascontiguousarray(np.atleast_2d(q), np.float32)
        if qq.shape[1] != self.dim:
            raise ValueError(f"query dim {qq.shape[1]} != index dim {self.dim}")
        nq = qq.shape[0]
        parts = self._allow_parts(allow_bits)
        Ds, Rs, Vs = [], [], []
        for s, sh in enumerate(self.shards):
            ns = sh.size
            if ns == 0:
                continue
            a = parts[s]
            if a is not None:
                a = a[: max((ns + 31) // 32, 1)]
                if not hasattr(a, "data_ptr"):
                    a = np.ascontiguousarray(a, np.uint32)
                elif a.device.index != sh.device:
                    a = a.to(torch.device("cuda", sh.device))
                else:
                    a = a.contiguous()
            res = sh.search(qq, k, a, return_vectors=return_vectors)
            Ds.append(res[0])
            Rs.append(self.map.to_global(s, res[1]))
            if return_vectors:
                Vs.append(res[2])
        if not Ds:
            d = np.zeros((nq, k), np.float32)
            r = np.full((nq, k), -1, np.int64)
            return (d, r, np.zeros((nq, k, self.dim), np.float32)) if return_vectors else (d, r)
        D, R = np.concatenate(Ds, 1), np.concatenate(Rs, 1)
        o = np.argsort(_f32_key_np(D, R), axis=1, kind="stable")[:, :k]
        d, r = np.take_along_axis(D, o, 1), np.take_along_axis(R, o, 1)
        d = np.where(r < 0, np.float32(0), d).astype(np.float32)
        if not return_vectors:
            return d, r
        V = np.concatenate(Vs, 1)
        v = np.take_along_axis(V, o[:, :, None], 1)
        v[r < 0] = 0.0
        return d, r, v

    def search_dev(self, q, k: int, allow=None, out=None, workspace=None, defer_exact: bool = False):
        """Device tensors on the first device, torch's current stream there: every shard searches on
        its own stream, the lists merge in one cm_shard_merge_topk_dev launch.  (defer_exact is
        ignored: every shard completes its own certificate before the merge.)"""
        nq = q.shape[0]
        cur, ev = self._fork()
        parts = self._allow_parts(allow)
        packs = []
        for s, (sh, st) in enumerate(zip(self.shards, self._streams())):
            with torch.cuda.device(self.devices[s]), torch.cuda.stream(st):
                st.wait_event(ev)
                if sh.size == 0:
                    d = torch.zeros((nq, k), dtype=torch.float32, device=st.device)
                    r = torch.full((nq, k), -1, dtype=torch.int64, device=st.device)
                else:
                    qs = self._to(q, s, st)
                    a = self._to(parts[s], s, st)
                    if a is not None:
                        a = a[: max((sh.size + 31) // 32, 1)].contiguous()
                    d, r = sh.search_dev(qs, k, allow=a)
                pk = _pack(d, self.map.to_global(s, r), torch.zeros((nq, 1), dtype=torch.float64, device=d.device),
                           torch.full((nq, 1), -1, dtype=torch.int64, device=d.device))
                if pk.device.index != self.device:
                    pk = pk.to(torch.device("cuda", self.device), non_blocking=True)
                done = torch.cuda.Event()
                done.record(st)
            cur.wait_event(done)
            pk.record_stream(cur)
            packs.append(pk)
        d_m, r_m, _, _ = parallel.merge_packed(torch.stack(packs), k, 1)
        if out is not None:
            out[0].copy_(d_m)
            out[1].copy_(r_m)
            return out
        return d_m, r_m

    def exact_fallback_dev(self, q, k: int, out, workspace=None, allow=None):
        return out                                  # search_dev finished every shard's certificate

    def gather_dev(self, rows, out=None):
        """Global rows (device, first device; -1 -> zero row) -> (n, dim) fp32 from their owners."""
        n = rows.numel()
        res = out if out is not None else torch.zeros((n, self.dim), dtype=torch.float32, device=rows.device)
        if out is not None:
            res.zero_()
        if n == 0:
            return res
        own, loc = self.map.owner_local(rows.clamp(min=0))
        for s, sh in enumerate(self.shards):
            m = (own == s) & (rows >= 0)
            local = torch.where(m, loc, torch.full_like(loc, -1))
            dev_s = torch.device("cuda", self.devices[s])
            with torch.cuda.device(dev_s):
                g = sh.gather_dev(local.to(dev_s))
            res = torch.where(m[:, None], g.to(rows.device), res)   # exact (no zero-sign change)
        if out is not None and res.data_ptr() != out.data_ptr():
            out.copy_(res)
            return out
        return res


class ShardedBM25Index(_Shards):
    """engine.BM25Index's interface over G handles with global statistics (module docstring)."""

    sharded = True
    FILT_EPS_MISSING, FILT_ZERO_DIV, FILT_TABLE = 1, 2, 4

    def __init__(self, devices: Sequence[int], block: Optional[int] = None):
        self.devices = [int(d) for d in devices]
        self.G = len(self.devices)
        self.map = RowMap(self.G, block or _block_rows())
        self.device = self.devices[0]
        self.shards = [engine.BM25Index(device=d) for d in self.devices]
        self.vocab = 0
        self.ndocs = 0
        self.idf = np.zeros(0, np.float64)
        self.n_live = self.sum_len = 0
        self.eps = 0.0
        self._st = None

    def close(self):
        for sh in self.shards:
            sh.close()

    @property
    def num_docs(self) -> int:
        return self.ndocs

    @property
    def num_postings(self) -> int:
        return sum(sh.num_postings for sh in self.shards)

    def build(self, term_ids: np.ndarray, doc_off: np.ndarray, vocab: int, live: Optional[np.ndarray] = None):
        """Deal the documents' blocks to the shards, build each, then install the global statistics."""
        doc_off = np.asarray(doc_off, np.int64)
        N = doc_off.shape[0] - 1
        B, G = self.map.B, self.G
        for s, sh in enumerate(self.shards):
            spans = [(b * B, min((b + 1) * B, N)) for b in range(s, -(-N // B), G)]
            if spans:
                tids = np.concatenate([np.asarray(term_ids[doc_off[lo]:doc_off[hi]], np.int32) for lo, hi in spans])
                lens = np.concatenate([np.diff(doc_off[lo:hi + 1]) for lo, hi in spans])
                off = np.zeros(lens.shape[0] + 1, np.int64)
                np.cumsum(lens, out=off[1:])
                lv = None if live is None else np.concatenate([np.asarray(live[lo:hi]) for lo, hi in spans])
            else:
                tids, off, lv = np.zeros(0, np.int32), np.zeros(1, np.int64), None
            sh.build(tids, off, vocab, lv)
        self.vocab, self.ndocs = int(vocab), int(N)
        self._prepared = False
        self._install_global_stats()

    def _install_global_stats(self):
        V = self.vocab
        gdf = np.zeros(V, np.int64)
        gfk = np.full(V, _EMPTY, np.uint64)
        n = sl = 0
        for s, sh in enumerate(self.shards):
            if sh.num_docs == 0:
                continue
            df, fk = sh.term_stats()
            gdf += df.astype(np.int64)
            gfk = np.minimum(gfk, self._global_keys(s, fk))
            st = sh.stats()
            n += st["n_live"]
            sl += st["sum_len"]
        self.n_live, self.sum_len = int(n), int(sl)
        if n == 0 or not (gdf > 0).any():
            self.idf, self.eps = np.zeros(V, np.float64), 0.0
            return
        self.idf, self.eps = parallel.bm25_idf_table(gdf, gfk, n)
        for sh in self.shards:
            if sh.num_docs:
                sh.set_stats(self.idf, n, sl, self.eps)

    def _global_keys(self, s: int, fk: np.ndarray) -> np.ndarray:
        """Shard s's first-occurrence keys (local row << 32 | position, ~0 absent) on global rows."""
        fk = np.asarray(fk, np.uint64)
        present = fk != _EMPTY
        rows = (fk >> np.uint64(32)).astype(np.int64)
        g = self.map.to_global(s, rows).astype(np.uint64)
        key = (g << np.uint64(32)) | (fk & np.uint64(0xFFFFFFFF))
        return np.where(present, key, _EMPTY)

    def term_stats(self):
        """Global (df[V] int64, first_key[V] uint64 on global rows)."""
        gdf = np.zeros(self.vocab, np.int64)
        gfk = np.full(self.vocab, _EMPTY, np.uint64)
        for s, sh in enumerate(self.shards):
            if sh.num_docs:
                df, fk = sh.term_stats()
                gdf += df
                gfk = np.minimum(gfk, self._global_keys(s, fk))
        return gdf, gfk

    def stats(self):
        return dict(n_live=self.n_live, sum_len=self.sum_len,
                    avgdl=(self.sum_len / self.n_live) if self.n_live else 0.0, eps=self.eps)

    def export(self):
        """Host CSR of the whole corpus on global rows (tests): postings merged per term by row."""
        parts = [(s, sh.export()) for s, sh in enumerate(self.shards) if sh.num_docs]
        V, N = self.vocab, self.ndocs
        dl = np.zeros(N, np.int32)
        docs, tfs, poss, terms = [], [], [], []
        for s, c in parts:
            g = self.map.to_global(s, np.arange(c["dl"].shape[0], dtype=np.int64))
            dl[g] = c["dl"]
            cnt = np.diff(c["term_off"])
            terms.append(np.repeat(np.arange(V, dtype=np.int64), cnt))
            docs.append(self.map.to_global(s, c["post_doc"].astype(np.int64)))
            tfs.append(c["post_tf"])
            poss.append(c["post_pos"])
        if not parts:
            return dict(term_off=np.zeros(V + 1, np.int64), post_doc=np.zeros(0, np.int32),
                        post_tf=np.zeros(0, np.uint16), post_pos=np.zeros(0, np.uint32), dl=dl)
        t, d = np.concatenate(terms), np.concatenate(docs)
        o = np.lexsort((d, t))
        term_off = np.zeros(V + 1, np.int64)
        np.cumsum(np.bincount(t, minlength=V), out=term_off[1:])
        return dict(term_off=term_off, post_doc=d[o].astype(np.int32), post_tf=np.concatenate(tfs)[o],
                    post_pos=np.concatenate(poss)[o], dl=dl)

    def prepare_filtered(self, max_docs: int = 0):
        """Every shard's device log table for idf over the GLOBAL candidate count (up to ndocs)."""
        for sh in self.shards:
            if sh.num_docs:
                sh.prepare_filtered(max(int(max_docs), self.ndocs))
        self._prepared = True

    # -- statistics of a where-filter's candidates over all shards (quirk Q2) -------------------
    def _filtered_q_idf(self, flat: np.ndarray, parts_dev):
        """(q_idf[T] host, avgdl, n_cand) of the candidates the shards' allow words select, the
        global statistics rank_bm25 would build over them (bm25.py:184-191)."""
        T = int(flat.shape[0])
        nc = sl = 0
        df = np.zeros(max(T, 1), np.int64)
        for s, sh in enumerate(self.shards):
            if sh.num_docs == 0:
                continue
            dev_s = torch.device("cuda", self.devices[s])
            qt = torch.from_numpy(np.ascontiguousarray(flat if T else np.zeros(1, np.int32), np.int32)).to(dev_s)
            with torch.cuda.device(dev_s):
                st, d = sh.filter_stats_dev(parts_dev[s], qt[:T] if T else qt[:0])
            st = st.cpu().numpy()
            nc += int(st[0])
            sl += int(st[1])
            if T:
                df[:T] += d.cpu().numpy()[:T]
        q_idf = np.zeros(max(T, 1), np.float64)
        if nc == 0:
            return q_idf, 0.0, 0
        if sl == 0:
            raise ZeroDivisionError("float division by zero (candidate documents have no tokens)")
        avgdl = sl / nc
        log = math.log
        need_eps = False
        for i in range(T):
            t, d = int(flat[i]), int(df[i])
            if 0 <= t < self.vocab and d > 0:
                v = log((nc - d) + 0.5) - log(d + 0.5)
                q_idf[i] = v
                need_eps |= v < 0
        if need_eps:
            eps = self._filtered_eps(parts_dev, nc)
            q_idf = np.where(q_idf < 0, eps, q_idf)
        return q_idf, avgdl, nc

    def _filtered_eps(self, parts_dev, n_cand: int) -> float:
        gdf = np.zeros(self.vocab, np.int64)
        gfk = np.full(self.vocab, _EMPTY, np.uint64)
        for s, sh in enumerate(self.shards):
            if sh.num_docs == 0:
                continue
            with torch.cuda.device(self.devices[s]):
                d, fk = sh.filter_term_stats_dev(parts_dev[s])
            gdf += d.cpu().numpy()
            gfk = np.minimum(gfk, self._global_keys(s, fk.cpu().numpy().view(np.uint64)))
        return parallel.bm25_idf_table(gdf, gfk, int(n_cand))[1]

    def _parts_dev(self, allow_bits):
        """Global allow words (host or device) -> every shard's local words on its device."""
        if not hasattr(allow_bits, "data_ptr"):
            allow_bits = torch.from_numpy(np.ascontiguousarray(allow_bits, np.uint32).view(np.int32)).to(
                torch.device("cuda", self.device))
        out = []
        for s, (sh, w) in enumerate(zip(self.shards, self.map.split_words(allow_bits, self.G))):
            w = w[: max((sh.num_docs + 31) // 32, 1)]
            out.append(w.to(torch.device("cuda", self.devices[s])).contiguous())
        return out

    def search(self, queries: Sequence[Sequence[int]], k: int, allow_bits=None):
        """Host API (BM25Store.search_batch): every shard scores with the global statistics (the
        where-filter's candidate statistics over all shards when allow_bits is given) through
        cm_bm25_search_idf; the lists merge by (score desc, global row asc).  Any k."""
        nq = len(queries)
        off = np.zeros(nq + 1, np.int32)
        for i, q in enumerate(queries):
            off[i + 1] = off[i] + len(q)
        flat = np.ascontiguousarray(np.concatenate([np.asarray(q, np.int32) for q in queries])
                                    if off[-1] else np.zeros(1, np.int32), np.int32)
        T = int(off[-1])
        parts = None
        if allow_bits is None:
            q_idf = np.array([self.idf[t] if 0 <= t < self.vocab else 0.0 for t in flat[:T].tolist()] or [0.0],
                             np.float64)
            nc, avgdl = self.n_live, (self.sum_len / self.n_live if self.n_live else 0.0)
            if nc and self.sum_len == 0:
                raise ZeroDivisionError("float division by zero")
        else:
            parts = self._parts_dev(allow_bits)
            q_idf, avgdl, nc = self._filtered_q_idf(flat[:T], parts)
        Ss, Rs = [], []
        for s, sh in enumerate(self.shards):
            if sh.num_docs == 0:
                continue
            sc = np.empty((nq, k), np.float64)
            rw = np.empty((nq, k), np.int64)
            nv = np.empty(nq, np.int32)
            L.check(L.fn["cm_bm25_search_idf"](sh._h, L.ptr(flat), L.ptr(off), nq, int(k),
                                               L.ptr(parts[s]) if parts is not None else None,
                                               L.ptr(np.ascontiguousarray(q_idf, np.float64)), float(avgdl),
                                               int(nc), L.ptr(sc), L.ptr(rw), L.ptr(nv)), "cm_bm25_search_idf")
            Ss.append(sc)
            Rs.append(self.map.to_global(s, rw))
        if not Ss:
            return np.zeros((nq, k), np.float64), np.full((nq, k), -1, np.int64), np.zeros(nq, np.int32)
        S, R = np.concatenate(Ss, 1) + 0.0, np.concatenate(Rs, 1)
        big = np.iinfo(np.int64).max
        o = np.lexsort((np.where(R < 0, big, R), np.where(R < 0, np.inf, -S)), axis=1)[:, :k]
        sc, rw = np.take_along_axis(S, o, 1), np.take_along_axis(R, o, 1)
        sc = np.where(rw < 0, 0.0, sc)
        return sc, rw, (rw >= 0).sum(1).astype(np.int32)

    def _merge_dev(self, lists, k: int, cur):
        """[(scores f64, global rows) per shard on the first device] -> merged top-k (K3x)."""
        nq = lists[0][0].shape[0]
        packs = [_pack(torch.zeros((nq, 1), dtype=torch.float32, device=sc.device),
                       torch.full((nq, 1), -1, dtype=torch.int64, device=sc.device), sc, rw) for sc, rw in lists]
        _, _, s_m, r_m = parallel.merge_packed(torch.stack(packs), 1, k)
        return s_m, r_m

    def search_dev(self, q_terms, q_off, k: int, out=None, workspace=None, gate=None):
        """Unfiltered device search (first device, current stream): every shard on its own stream with
        the installed global statistics, then one merge launch."""
        nq = q_off.numel() - 1
        cur, ev = self._fork()
        if gate is not None:
            cur.wait_event(gate)
            ev = torch.cuda.Event()
            ev.record(cur)
        lists = []
        for s, (sh, st) in enumerate(zip(self.shards, self._streams())):
            with torch.cuda.device(self.devices[s]), torch.cuda.stream(st):
                st.wait_event(ev)
                if sh.num_docs == 0:
                    sc = torch.zeros((nq, k), dtype=torch.float64, device=st.device)
                    rw = torch.full((nq, k), -1, dtype=torch.int64, device=st.device)
                else:
                    sc, rw = sh.search_dev(self._to(q_terms, s, st), self._to(q_off, s, st), k)
                rw = self.map.to_global(s, rw)
                if sc.device.index != self.device:
                    sc = sc.to(torch.device("cuda", self.device), non_blocking=True)
                    rw = rw.to(torch.device("cuda", self.device), non_blocking=True)
                done = torch.cuda.Event()
                done.record(st)
            cur.wait_event(done)
            sc.record_stream(cur)
            rw.record_stream(cur)
            lists.append((sc, rw))
        s_m, r_m = self._merge_dev(lists, k, cur)
        if out is not None:
            out[0].copy_(s_m)
            out[1].copy_(r_m)
            return out
        return s_m, r_m

    def search_filtered(self, q_terms, q_off, k: int, allow):
        """Filtered device search with the candidates' statistics of all shards (quirk Q2): the
        global per-term idf (and epsilon) on the host, every shard scored through
        search_stats_dev with the summed statistics, one merge.  Synchronises (statistics)."""
        nq = q_off.numel() - 1
        if not getattr(self, "_prepared", False):
            self.prepare_filtered()
        parts = self._parts_dev(allow)
        T = int(q_terms.numel())
        # summed candidate statistics (device tensors per shard) and, when needed, epsilon
        stats = torch.zeros(2, dtype=torch.int64, device=q_terms.device)
        df = torch.zeros(max(T, 1), dtype=torch.int64, device=q_terms.device)
        per = []
        for s, sh in enumerate(self.shards):
            if sh.num_docs == 0:
                per.append(None)
                continue
            dev_s = torch.device("cuda", self.devices[s])
            with torch.cuda.device(dev_s):
                qt = q_terms.to(dev_s)
                st_s, df_s = sh.filter_stats_dev(parts[s], qt)
            per.append(qt)
            stats += st_s.to(q_terms.device)
            df[:max(T, 1)] += df_s.to(q_terms.device)[:max(T, 1)]
        nc = int(stats[0].item())
        if nc == 0:
            return (torch.zeros((nq, k), dtype=torch.float64, device=q_terms.device),
                    torch.full((nq, k), -1, dtype=torch.int64, device=q_terms.device))
        if int(stats[1].item()) == 0:
            raise ZeroDivisionError("float division by zero (candidate documents have no tokens)")
        eps_t = None
        lists = []
        for attempt in range(2):
            lists, code = [], 0
            for s, sh in enumerate(self.shards):
                if sh.num_docs == 0:
                    continue
                dev_s = torch.device("cuda", self.devices[s])
                with torch.cuda.device(dev_s):
                    sc, rw, status = sh.search_stats_dev(per[s], q_off.to(dev_s), k, parts[s], stats.to(dev_s),
                                                         df.to(dev_s), eps=None if eps_t is None else eps_t.to(dev_s))
                    code |= int(status.item())
                lists.append((sc.to(q_terms.device), self.map.to_global(s, rw).to(q_terms.device)))
            if code & self.FILT_EPS_MISSING and eps_t is None:
                eps_t = torch.tensor([self._filtered_eps(parts, nc)], dtype=torch.float64, device=q_terms.device)
                continue
            break
        if code & self.FILT_ZERO_DIV:
            raise ZeroDivisionError("float division by zero (candidate documents have no tokens)")
        if code & ~self.FILT_EPS_MISSING:
            raise RuntimeError(f"filtered BM25 search status {code}")
        return self._merge_dev(lists, k, torch.cuda.current_stream(self.device))


def new_dense_index(dim: int, device: Optional[int] = None, capacity: int = 0):
    """A DenseIndex, or a ShardedDenseIndex over CM_DEVICES when no device is named."""
    devs = shard_devices() if device is None else None
    if devs:
        return ShardedDenseIndex(dim, devs, capacity=capacity)
    return engine.DenseIndex(dim, device=device, capacity=capacity)


def new_bm25_index(device: Optional[int] = None):
    devs = shard_devices() if device is None else None
    if devs:
        return ShardedBM25Index(devs)
    return engine.BM25Index(device=device)
