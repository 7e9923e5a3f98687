#!/usr/bin/env python3
"""Hybrid-retrieval benchmark on MI355X — BASELINE.json's metric:
"hybrid queries/sec + recall@10 vs reference, 10M x 768 chunks, 1/2/4/8 GPU".

Workload (BASELINE.json configs[3]; weak scaling for configs[4]): every GPU
owns a shard of --docs-per-gpu synthetic chunks (default 10M): 768-d unit fp32
embeddings and BM25 postings (vocabulary 2^20, Zipf 1.07 term draws, chunk
length ~ Poisson(120)).  One step = one batch of B queries through the whole
hot path, inputs resident in HBM:

  E5-base query encode (PyTorch-ROCm bf16 forward replayed as one hipGraph,
  random-init weights + HIP mean-pool/L2, K6) -> dense cosine top-24 over the
  shard (K1c) -> MMR to 10 (K4) -> [N>1: RCCL all-gather of per-shard top-k +
  merge, pool embeddings all-reduce] -> RRF fusion (K5).  BM25 top-10 (K2a/K2b/K2,
  fp64) runs on a second HIP stream concurrently with the encode + dense search.

value = queries/s of the whole job (each query searches all N x shard chunks).
The CPU baseline is the oracle (oracle/) run on this host on a bounded sample
of the same queries over the same shard; recall@10 compares the GPU's final
top-10 with the oracle's.

  python bench.py [--gpus N --steps K --warmup W] [--mode hybrid|dense|ingest]
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent
for _p in (str(REPO), str(REPO / "classmate-rag_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

METRIC = "hybrid queries/sec + recall@10 vs reference, 10M×768 chunks, 1/2/4/8 GPU"
PEAK_F32_MFMA_TFLOPS = 157.3   # MI355X_MICROARCH.md: FP32 matrix (dense)
PEAK_F16_MFMA_TFLOPS = 2500.0  # MI355X_MICROARCH.md: BF16/F16 matrix, dense (no sparsity)
PEAK_HBM_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E spec
PEAK_I8_MFMA_TOPS = 5000.0     # cdna_hip_programming.md: i8 MFMA = 2x the bf16 rate (dense)
DENSE_KINDS = {1: "K1 fp32 MFMA (dense_topk_kernel)",
               3: "K1c dense_coarse_scan_kernel (f16 plane, MFMA, 256-query resident passes) + certified fp64 re-rank",
               4: "K1s dense_stream_scan_kernel (f16 plane, MFMA, per-wave HBM streams) + certified fp64 re-rank",
               5: "K1q dense_q8_scan_kernel (int8 plane + per-row bounds, i8 MFMA, 256-query resident passes) + "
                  "per-row certified fp64 re-rank",
               6: "K1q-s dense_q8_stream_kernel (int8 plane + per-row bounds, i8 MFMA, per-wave HBM streams) + "
                  "per-row certified fp64 re-rank"}


def parse_args():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--mode", choices=["hybrid", "dense", "ingest", "e2e"], default="hybrid")
    ap.add_argument("--docs-per-gpu", type=int, default=10_000_000)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--pool", type=int, default=24)
    ap.add_argument("--dim", type=int, default=768)
    ap.add_argument("--vocab", type=int, default=1 << 20)
    ap.add_argument("--zipf", type=float, default=1.07)
    ap.add_argument("--avg-len", type=float, default=120.0)
    ap.add_argument("--q-terms", type=int, default=8)
    ap.add_argument("--q-tokens", type=int, default=24)
    ap.add_argument("--e5-layers", type=int, default=12)
    ap.add_argument("--e5-dtype", choices=["bfloat16", "float32"], default="float32",
                    help="E5 forward dtype of the headline step: float32 = the reference's precision (K10 "
                         "split-precision MFMA GEMMs), the drop-in default")
    ap.add_argument("--e5-other-leg", type=int, default=1,
                    help="also time the step with the other E5 precision (reported as e5_bf16 / e5_fp32)")
    ap.add_argument("--dense-legs", type=int, default=1,
                    help="hybrid mode: also time the north_star dense configs -- C2' (this 10M shard, B=16, "
                         "k=10, the >=80%% HBM target) and C2 (a 1M-chunk shard, B=256, k=10)")
    ap.add_argument("--ingest-leg", type=int, default=1,
                    help="hybrid mode: also time BASELINE configs[2]'s passage encode at the reference's fp32 "
                         "(256 chunks x --seq-len tokens per step; reported as ingest_fp32 + rooflines.e5_ingest)")
    ap.add_argument("--varlen-chunks", type=int, default=4096,
                    help="hybrid mode with --ingest-leg: passages of S ~ U[64, 512] tokens through encode_passages "
                         "(SURVEY §8d C3's variable-length run; reported as ingest_varlen_fp32); 0 = off")
    ap.add_argument("--ingest-e2e-chunks", type=int, default=65536,
                    help="hybrid mode with --ingest-leg, N = 1: chunks through ingest_file's store path (encode_passages "
                         "-> upsert -> upsert_many -> save, files of 4096; reported as ingest_e2e); 0 = off")
    ap.add_argument("--ingest-e2e-file-chunks", type=int, default=4096,
                    help="chunks per ingested file in the ingest_e2e leg (the reference saves the whole BM25 JSONL "
                         "after every file, rag/pipeline/rag.py:413, so the leg's cost grows with files x corpus)")
    ap.add_argument("--no-e5", action="store_true", help="use perturbed corpus rows as query embeddings")
    ap.add_argument("--no-graph", action="store_true", help="run the E5 query encode eagerly (no hipGraph)")
    ap.add_argument("--serial", action="store_true", help="run BM25 on the main stream (no overlap with E5 + dense)")
    ap.add_argument("--bm25-priority", type=int, default=0, help="HIP stream priority of the BM25 stream (-1 = high)")
    ap.add_argument("--bm25-with-e5", dest="bm25_after_e5", action="store_false",
                    help="launch BM25 beside the E5 encode (the round-3 schedule); default: after the encode, "
                         "beside the dense search, whose seed / re-rank / fusion kernels leave CUs to it "
                         "(31.2k vs 30.5k q/s with K1q, profiles/r04b_sched_ab.txt)")
    ap.add_argument("--bm25-gate", type=int, default=1,
                    help="with BM25 after the encode: its query preparation (descriptors, postings bounds, seeded "
                         "threshold) starts beside the encode and only the scoring kernels wait for it "
                         "(cm_bm25_search_dev_gated); 0 = the whole search after the encode; 2 = the scoring "
                         "waits for the dense search's seed pass instead (cm_dense_set_seed_event)")
    ap.add_argument("--pipeline", type=int, default=0,
                    help="1 (2: on a high-priority stream) = encode batch i+1 (its own hipGraph + output buffer, its own stream) while batch i is "
                         "searched; every step still runs one whole encode and one whole search")
    ap.add_argument("--bm25-cus", default="", help="run the BM25 stream on a CU subset: 'first:N', 'stride:S' "
                    "(every S-th CU) or '' (all CUs)")
    ap.add_argument("--seq-len", type=int, default=256, help="ingest mode: tokens per chunk")
    ap.add_argument("--e2e-words", type=int, default=40, help="e2e mode: words per synthetic chunk")
    ap.add_argument("--e2e-latency-queries", type=int, default=32, help="e2e mode: single-query retrieve() calls timed")
    ap.add_argument("--e2e-construct", type=int, default=1,
                    help="e2e mode: also persist the stores and time ask_question's construct-then-retrieve "
                         "sequence (rag/pipeline/rag.py:531-554) and the cold open")
    ap.add_argument("--e2e-dir", default=None, help="e2e mode: directory for the persisted stores (default: a "
                                                  "fresh directory under $TMPDIR)")
    ap.add_argument("--e2e-ab-same-stream", type=int, default=0,
                    help="e2e mode: also time retrieve() with BM25 on the main stream (the pre-side-stream schedule)")
    ap.add_argument("--e2e-ab-env", default="",
                    help="e2e mode: ';'-separated env settings (NAME=V[,NAME=V]) under which retrieve_batch is "
                         "timed again right after the main measurement, alternating with the default (A/B)")
    ap.add_argument("--cpu-baseline", type=int, default=1)
    ap.add_argument("--cpu-queries", type=int, default=128)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--out", default=None, help="also write the JSON line to this file")
    return ap.parse_args()


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print("[bench]", *a, file=sys.stderr, flush=True)


# ---------------------------------------------------------------------------
# synthetic shard
# ---------------------------------------------------------------------------
def gen_dense(dense, n, dim, seed, chunk=1 << 20):
    import torch
    g = torch.Generator(device="cuda").manual_seed(seed)
    for r0 in range(0, n, chunk):
        m = min(chunk, n - r0)
        x = torch.randn(m, dim, device="cuda", generator=g)
        x /= x.norm(dim=1, keepdim=True)
        dense.upsert_dev(x, r0)
        del x
    torch.cuda.synchronize()


def gen_tokens(n, vocab, s, avg_len, seed, chunk=1 << 27):
    import torch
    g = torch.Generator(device="cuda").manual_seed(seed)
    lens = torch.poisson(torch.full((n,), float(avg_len), device="cuda"), generator=g).clamp_(min=1).to(torch.int64)
    doc_off = torch.zeros(n + 1, dtype=torch.int64, device="cuda")
    torch.cumsum(lens, 0, out=doc_off[1:])
    ntok = int(doc_off[-1].item())
    p = 1.0 / torch.arange(1, vocab + 1, dtype=torch.float64, device="cuda").pow(s)
    cdf = torch.cumsum(p, 0)
    cdf /= cdf[-1].clone()
    tokens = torch.empty(ntok, dtype=torch.int32, device="cuda")
    for t0 in range(0, ntok, chunk):
        m = min(chunk, ntok - t0)
        u = torch.rand(m, dtype=torch.float64, device="cuda", generator=g)
        tokens[t0:t0 + m] = torch.searchsorted(cdf, u).clamp_(max=vocab - 1).to(torch.int32)
        del u
    return tokens, doc_off


def sample_query_terms(tokens, doc_off, B, q_terms, seed):
    import torch
    g = torch.Generator(device="cuda").manual_seed(seed)
    n = doc_off.numel() - 1
    tgt = torch.randint(0, n, (B,), device="cuda", generator=g)
    lo = doc_off[tgt]
    ln = doc_off[tgt + 1] - lo
    pos = (torch.rand(B, q_terms, device="cuda", generator=g) * ln.unsqueeze(1)).long()
    return tokens[lo.unsqueeze(1) + pos].contiguous()           # (B, q_terms) int32


# ---------------------------------------------------------------------------
ABLATION_ENV = ("CM_DENSE_DEBUG", "CM_BM25_DEBUG")
KNOB_ENV = ("CM_DENSE_PATH", "CM_E5_FUSED_LN", "CM_E5_FUSED_ATTN", "CM_E5_TUNABLEOP", "CM_E5_DTYPE", "CM_E5_F16X3")


def main():
    args = parse_args()
    bad = [e for e in ABLATION_ENV if os.environ.get(e, "0") not in ("", "0")]
    if bad:   # timing ablations skip work; the product library ignores them, refuse anyway
        sys.exit(f"bench.py: refusing to run with ablation switches set: {bad}")
    import numpy as np
    import torch
    from classmate_hip import engine, parallel

    # CM_DIST_BACKEND=gloo + CM_BENCH_DEVICE=0: rehearse the N>1 path with every rank on one GPU
    # (RCCL refuses two ranks per device); the driver's multi-GPU runs use the defaults
    rank, ws = parallel.init_from_env(os.environ.get("CM_DIST_BACKEND") or None)
    local = int(os.environ.get("CM_BENCH_DEVICE", os.environ.get("LOCAL_RANK", "0")))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if args.gpus != ws:
        log(f"note: --gpus {args.gpus} but WORLD_SIZE={ws}; using {ws}")
    if args.mode == "ingest":
        return run_ingest(args, rank, ws, dev)
    if args.mode == "e2e":
        return run_e2e(args, rank, ws, dev)

    B, K, P, D = args.batch, args.k, args.pool, args.dim
    if args.mode == "dense":   # C2: plain cosine top-k (no MMR pool)
        P = K
    N = args.docs_per_gpu
    row0 = rank * N
    t_setup = time.perf_counter()
    dense = engine.DenseIndex(D, device=local, capacity=N)
    gen_dense(dense, N, D, seed=args.seed * 1000 + rank)
    log(f"dense shard {N}x{D} fp32 ready ({time.perf_counter() - t_setup:.1f}s)")

    bm25 = None
    tokens_host = None
    if args.mode == "hybrid":
        tokens, doc_off = gen_tokens(N, args.vocab, args.zipf, args.avg_len, seed=args.seed * 1000 + 500 + rank)
        bm25 = engine.BM25Index(device=local)
        bm25.build_dev(tokens, doc_off, args.vocab)
        torch.cuda.synchronize()
        if ws > 1:   # global statistics (df / N / length sums / first-occurrence order)
            df, fk = bm25.term_stats()
            st = bm25.stats()
            gdf, gfk, gn, gsum = parallel.allreduce_bm25_stats(df, fk, row0, st["n_live"], st["sum_len"])
            idf, eps = parallel.bm25_idf_table(gdf, gfk, gn)
            bm25.set_stats(idf, gn, gsum, eps)
        qt = sample_query_terms(tokens, doc_off, B, args.q_terms, seed=args.seed * 7 + 3)
        if ws > 1:
            torch.distributed.broadcast(qt, src=0)
        q_terms = qt.reshape(-1).contiguous()
        q_off = (torch.arange(B + 1, device=dev, dtype=torch.int32) * args.q_terms).contiguous()
        if args.cpu_baseline:    # the recall leg's oracle builds its own CSR from these
            tokens_host = (tokens.cpu().numpy(), doc_off.cpu().numpy())
        del tokens, doc_off
        torch.cuda.empty_cache()
        log(f"bm25 shard: {bm25.num_postings} postings, V={args.vocab} ({time.perf_counter() - t_setup:.1f}s)")

    # queries: every rank holds the same B queries (token ids / term ids); the E5 encode is split
    # across ranks -- rank r encodes block [q_lo, q_lo + bq) and the (B, D) embeddings are
    # all-gathered (at N = 1 the block is the whole batch)
    if B % ws:
        sys.exit(f"bench.py: --batch {B} must be divisible by the number of GPUs ({ws})")
    bq, q_lo = B // ws, rank * (B // ws)
    blk = slice(q_lo, q_lo + bq)
    use_e5 = not args.no_e5 and args.mode == "hybrid"
    if use_e5:
        from classmate_hip.embeddings import E5MultilingualEmbedder
        g = torch.Generator(device="cuda").manual_seed(args.seed * 13)
        ids = torch.randint(5, 250002, (B, args.q_tokens), device=dev, generator=g)
        ids[:, 0] = 0
        ids[:, -1] = 2
        mask = torch.ones_like(ids)

        def make_e5(dtype):
            """E5 query encoder of one dtype for this rank's block: dict(emb, graph or None, qbuf =
            output buffer, and the graph's input buffers, which must stay alive with the graph)."""
            m = E5MultilingualEmbedder.random_init(seed=0, device=str(dev), num_layers=args.e5_layers, dtype=dtype)
            if args.no_graph:
                return dict(emb=m, graph=None, qbuf=torch.empty((bq, D), dtype=torch.float32, device=dev),
                            dtype=dtype)
            # one hipGraph replay per batch instead of ~200 launches (fixed-length queries: lean forward)
            g_ids, g_mask, out_buf, gr = m.capture_graph(bq, args.q_tokens, unpadded=True)
            g_ids.copy_(ids[blk])
            g_mask.copy_(mask[blk])
            return dict(emb=m, graph=gr, qbuf=out_buf, ids=g_ids, mask=g_mask, dtype=dtype)

        e5 = make_e5(args.e5_dtype)
        if args.pipeline and e5["graph"] is not None:
            # the second batch slot: its own graph (own memory pool), inputs and output buffer
            g_ids, g_mask, out_buf, gr = e5["emb"].capture_graph(bq, args.q_tokens, unpadded=True)
            g_ids.copy_(ids[blk])
            g_mask.copy_(mask[blk])
            e5["slots"] = [dict(graph=e5["graph"], qbuf=e5["qbuf"]), dict(graph=gr, qbuf=out_buf, ids=g_ids,
                                                                          mask=g_mask)]
    else:
        g = torch.Generator(device="cuda").manual_seed(args.seed * 17)
        qfix = torch.randn(B, D, device=dev, generator=g)
        qfix /= qfix.norm(dim=1, keepdim=True)
    qfull = torch.empty((B, D), dtype=torch.float32, device=dev) if ws > 1 else None
    starts = [i * N for i in range(ws + 1)]            # global rows of the shards

    # buffers (allocated once: the step is allocation-free on our side at N = 1)
    dws = torch.empty(dense.workspace_bytes(B, P), dtype=torch.uint8, device=dev)
    dout = (torch.empty((B, P), dtype=torch.float32, device=dev), torch.empty((B, P), dtype=torch.int64, device=dev))
    vbuf = torch.empty((B * P, D), dtype=torch.float32, device=dev)
    obuf = torch.empty((bq, K), dtype=torch.int32, device=dev)
    pbuf = (torch.empty((bq, K), dtype=torch.int64, device=dev), torch.empty((bq, K), dtype=torch.float32, device=dev),
            torch.empty((bq,), dtype=torch.int32, device=dev), torch.empty((bq,), dtype=torch.int32, device=dev))
    if bm25 is not None:
        bws = torch.empty(bm25.workspace_bytes(B, q_terms.numel(), K), dtype=torch.uint8, device=dev)
        bout = (torch.empty((B, K), dtype=torch.float64, device=dev), torch.empty((B, K), dtype=torch.int64, device=dev))
    ev = []

    main = torch.cuda.current_stream(dev)
    side = (torch.cuda.Stream(device=dev, priority=args.bm25_priority)
            if (bm25 is not None and not args.serial) else main)
    if bm25 is not None and not args.serial and args.bm25_cus:
        n_cu = torch.cuda.get_device_properties(dev).multi_processor_count
        how, val = args.bm25_cus.split(":")
        cus = range(int(val)) if how == "first" else range(0, n_cu, int(val))
        side = engine.cu_masked_stream(local, list(cus))
        log(f"BM25 stream on {len(list(cus))} of {n_cu} CUs ({args.bm25_cus})")

    def run_bm25(e, gate=None):
        # BM25 needs only the query term ids: it runs on its own stream, overlapping the E5
        # encode and the dense search (joined before fusion)
        with torch.cuda.stream(side):
            if e:
                e["b0"].record()
            out = bm25.search_dev(q_terms, q_off, K, out=bout, workspace=bws, gate=gate)
            if e:
                e["b1"].record()
        return out

    pipe = dict(it=0, stream=None, ready=None)
    if use_e5 and "slots" in e5:
        # a stream of another priority gets its own hardware queue (same-priority streams may share
        # one of the GPU_MAX_HW_QUEUES = 4 round-robin queues and then run in submission order)
        pipe["stream"] = torch.cuda.Stream(device=dev, priority=-1 if args.pipeline == 2 else 0)
        pipe["ready"] = [torch.cuda.Event(), torch.cuda.Event()]

    def encode_pipelined(e):
        """--pipeline: replay the NEXT batch's graph on the encode stream (after the previous step's
        search, the last reader of that slot, has run on main), return THIS batch's embeddings."""
        es, it = pipe["stream"], pipe["it"]
        cur, nxt = it % 2, (it + 1) % 2
        es.wait_stream(main)
        with torch.cuda.stream(es):
            if it == 0:                      # first call: this batch's encode too
                e5["slots"][cur]["graph"].replay()
                pipe["ready"][cur].record(es)
            if e:
                e["e0"].record(es)
            e5["slots"][nxt]["graph"].replay()
            if e:
                e["e1"].record(es)
            pipe["ready"][nxt].record(es)
        main.wait_event(pipe["ready"][cur])
        pipe["it"] = it + 1
        q_local = e5["slots"][cur]["qbuf"]
        if ws == 1:
            return q_local
        return parallel.all_gather_into(qfull, q_local)

    def encode(e):
        """This rank's E5 block -> (B, D) query embeddings on the main stream."""
        if pipe["stream"] is not None:
            return encode_pipelined(e)
        if e:
            e["e0"].record()
        if e5["graph"] is not None:
            e5["graph"].replay()
            q_local = e5["qbuf"]
        else:
            q_local = e5["emb"].encode_token_ids(ids[blk], mask[blk], out=e5["qbuf"])
        if e:
            e["e1"].record()
        if ws == 1:
            return q_local
        return parallel.all_gather_into(qfull, q_local)

    last_lists = {}      # the last step's merged lists (recall diagnostics)
    gate_ev = torch.cuda.Event()
    if bm25 is not None and args.bm25_after_e5 and args.bm25_gate == 2 and side is not main:
        gate_ev.record(main)                # creates the event; K1q records it after each seed pass
        dense.set_seed_event(gate_ev)

    def step(record=False):
        e = {n: torch.cuda.Event(enable_timing=True) for n in ("e0", "e1", "d0", "d1", "b0", "b1")} if record else None
        gated = bm25 is not None and args.bm25_after_e5 and args.bm25_gate and side is not main
        if bm25 is not None and (not args.bm25_after_e5 or gated):
            side.wait_stream(main)          # previous step's fusion has read bout (not this encode)
        if bm25 is not None and not args.bm25_after_e5:
            bs, br = run_bm25(e)
        q = encode(e) if use_e5 else qfix
        # the certificate's exact pass (queries whose band overflowed; device-gated, normally none)
        # is deferred behind the BM25 join: its ~150 KiB-LDS grid would wait for the BM25 kernels'
        # CUs anyway and hold the stream's later work
        defer = bm25 is not None and side is not main
        seed_gate = gated and args.bm25_gate == 2
        if seed_gate:                       # dense first: it records gate_ev after its seed pass
            if record:
                e["d0"].record()
            d, r = dense.search_dev(q, P, out=dout, workspace=dws, defer_exact=defer)
            if record:
                e["d1"].record()
            bs, br = run_bm25(e, gate_ev)
        elif gated:                         # preparation beside the encode, scoring after it
            gate_ev.record(main)
            bs, br = run_bm25(e, gate_ev)
        elif bm25 is not None and args.bm25_after_e5:
            side.wait_stream(main)
            bs, br = run_bm25(e)
        if not seed_gate:
            if record:
                e["d0"].record()
            d, r = dense.search_dev(q, P, out=dout, workspace=dws, defer_exact=defer)
            if record:
                e["d1"].record()
        if args.mode == "dense":
            if record:
                ev.append(e)
            return r
        if defer:
            main.wait_stream(side)
            dense.exact_fallback_dev(q, P, dout, workspace=dws)
        if ws == 1:
            vecs = dense.gather_dev(r.reshape(-1), out=vbuf).view(B, P, D)
            order = engine.mmr_dev(q, vecs, K, 0.5, out=obuf)
            main.wait_stream(side)
            rg, dm, brg, bsm = r, d, br, bs
        else:
            # ONE packed all-gather of both shard lists (merged identically everywhere), then this
            # rank fuses its query block: its pool rows arrive from their owners in one all-to-all
            main.wait_stream(side)
            rgl = torch.where(r >= 0, r + row0, r)
            brl = torch.where(br >= 0, br + row0, br)
            dm, rg, bsm, brg = parallel.exchange_topk(d, rgl, bs, brl)
            vecs = parallel.fetch_pool_vectors(rg, q_lo, bq, lambda lr: dense.gather_dev(lr), starts, D)
            order = engine.mmr_dev(q[blk].contiguous(), vecs, K, 0.5, out=obuf)
        if record:
            ev.append(e)
        last_lists["pool"] = (rg, dm, brg, bsm, order, vecs)
        last_lists["q"] = q
        # MMR-ordered vector list + list counts in one device pass, then the fused merge
        vk, vd, vn, bn = engine.rrf_pool_prep_dev(rg[blk].contiguous(), dm[blk].contiguous(), order,
                                                  brg[blk].contiguous(), out=pbuf)
        res = engine.rrf_merge_dev(vk, vd, vn, brg[blk].contiguous(), bsm[blk].contiguous(), bn,
                                   w_vec=1.0, w_bm25=1.0, rrf_k=60, top_k=K)
        if ws > 1:   # the fused top-k of every block, on every rank
            keys = torch.empty((B, K), dtype=res[0].dtype, device=dev)
            res = (parallel.all_gather_into(keys, res[0]),) + tuple(res[1:])
        return res

    def timed(steps):
        """W untimed + `steps` timed steps between barriers; max over ranks."""
        for _ in range(args.warmup):
            step()
        torch.cuda.synchronize()
        if ws > 1:
            torch.distributed.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = None
        for _ in range(steps):
            out = step(record=True)
        torch.cuda.synchronize()
        if ws > 1:
            torch.distributed.barrier()
        return parallel.max_over_ranks(time.perf_counter() - t0, device=dev), out

    dense.timing(True)
    if bm25 is not None:
        bm25.timing(True)
    elapsed, res = timed(args.steps)
    # the recall check compares `res` with the oracle on the SAME step's inputs: keep this run's
    # query embeddings and merged lists before the side legs reuse the buffers (qfull at N > 1)
    q_main = ((qfull if ws > 1 else last_lists.get("q", e5["qbuf"])) if use_e5 else qfix).clone()
    lists_main = tuple(t.clone() for t in last_lists["pool"]) if "pool" in last_lists else None
    mean_ms = lambda a, b: sum(x[a].elapsed_time(x[b]) for x in ev) / len(ev)   # noqa: E731
    search_ms = mean_ms("d0", "d1")
    # gated: the search's scoring starts at the encode's end (e1); its preparation overlaps the encode
    gated_run = bm25 is not None and use_e5 and args.bm25_after_e5 and args.bm25_gate and side is not main
    bsearch_ms = (mean_ms("e1", "b1") if gated_run else mean_ms("b0", "b1")) if bm25 is not None else None
    e5_ms = mean_ms("e0", "e1") if use_e5 else None
    ev.clear()
    # scan-kernel launch times: HIP events the library records on the launch stream
    kt = dense.timing_drain()
    dense_ms = sum(kt) / len(kt)
    bm25_ms = bm25b_ms = None
    if bm25 is not None:
        bt = bm25.timing_drain()
        bm25_ms = sum(bt) / len(bt)
        btb = bm25.timing_drain_block()
        bm25b_ms = sum(btb) / len(btb) if btb else None
    dense.timing(False)
    if bm25 is not None:
        bm25.timing(False)
    kind = dense.search_kind(B, P)
    fallbacks = dense.workspace_fallbacks(B, P, dws)
    rescored = bm25.workspace_rescored(B, q_terms.numel(), K, bws) if bm25 is not None else None
    qps = B * args.steps / elapsed
    log(f"{args.steps} steps in {elapsed:.3f}s -> {qps:.1f} q/s; E5 ({args.e5_dtype}, {bq} queries/rank) "
        f"{e5_ms if e5_ms is not None else 0:.3f} ms; dense search {search_ms:.3f} ms (scan kernel {dense_ms:.3f} ms, "
        f"{DENSE_KINDS[kind]}, {fallbacks} exact re-runs)"
        + (f", bm25 search {bsearch_ms:.3f} ms{' after the encode' if gated_run else ''} (K2a tail pass {bm25_ms:.3f} ms, {rescored} (query, range) pairs "
           f"re-scored)" if bm25_ms is not None else ""))

    roofs = {"dense": _dense_roofline(kind, N, D, B, dense_ms,
                                      _pmc_traffic(args, {5: "dense_q8", 6: "dense_q8s"}.get(kind, "dense")))}
    if bm25 is not None:
        roofs["bm25"] = _bm25_roofline(bm25, q_terms, N, bm25_ms, _pmc_traffic(args, "bm25"), args.q_terms)
        if bm25b_ms is not None:
            roofs["bm25_block"] = _bm25_block_roofline(bm25, q_terms, bm25.workspace_items(B, q_terms.numel(), K, bws),
                                                       bm25b_ms, _pmc_traffic(args, "bm25b"), args.q_terms,
                                                       bm25.workspace_subblocks(B, q_terms.numel(), K, bws))
    # the headline roofline: the kernel with the most algorithmic work per step (K1q: 7.76 GB per launch
    # against K2a's 0.25 GB).  In-step launch times are not a fair ranking: the two run side by side and
    # whichever starts second is stretched by the other (rooflines.bm25 keeps K2a's line either way)
    dominant = max(roofs, key=lambda n: roofs[n].get("algorithmic_per_launch", {}).get("bytes", 0.0))
    roof = roofs[dominant]
    if use_e5:   # the whole encode (48 K10 GEMMs + attention + LayerNorms) against the MFMA peak
        roofs["e5"] = _e5_roofline(bq, args.q_tokens, args.e5_layers, e5_ms, args.e5_dtype)

    # side legs (not the headline): the other E5 precision, and the north_star dense configs
    legs = {}
    if use_e5 and args.e5_other_leg:
        other = "bfloat16" if args.e5_dtype == "float32" else "float32"
        main_e5, e5 = e5, make_e5(other)
        pipe_stream, pipe["stream"] = pipe["stream"], None     # the other precision's leg runs unpipelined
        el2, _ = timed(args.steps)
        pipe["stream"] = pipe_stream
        ev.clear()
        legs["e5_" + {"bfloat16": "bf16", "float32": "fp32"}[other]] = {
            "value": B * args.steps / el2, "unit": "queries/s", "ms_per_step": el2 / args.steps * 1e3,
            "e5_forward": other, "note": "same step with the other E5 forward precision (not the headline)"}
        log(f"{other} E5 leg: {B * args.steps / el2:.1f} q/s ({el2 / args.steps * 1e3:.3f} ms/step)")
        del e5
        e5 = main_e5
    if args.mode == "hybrid" and args.dense_legs:
        legs.update(dense_legs(args, dense, N, D, dev, ws, q_main, P))
        # the in-step launch shares its CUs with the BM25 stream (launched after the encode, beside
        # the dense search, since round 4), so its HIP-event time includes that time-sharing; the
        # same launch alone (the step's own queries, same shard) is the kernel's own roofline
        if "c4_dense_10m_b256" in legs:
            roof["standalone"] = legs["c4_dense_10m_b256"]["roofline"]
    if use_e5 and args.ingest_leg:
        e5_f32 = e5["emb"] if e5["dtype"] == "float32" else None
        legs["ingest_fp32"], roofs["e5_ingest"] = ingest_leg(args, e5_f32, dev, ws, rank)
        if args.varlen_chunks > 0:
            legs["ingest_varlen_fp32"] = varlen_ingest_leg(args, e5_f32, dev, ws, rank)
        if args.ingest_e2e_chunks > 0 and ws == 1:
            legs["ingest_e2e"] = ingest_e2e_leg(args, e5_f32, dev)

    out = {
        "metric": METRIC if args.mode == "hybrid" else f"dense cosine top-{K} queries/sec, {N}x{D} fp32",
        "value": qps, "unit": "queries/s", "n_gpus": ws, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None,
        "dtype": (("fp32-accurate E5 (K10 f16x3 MFMA) + " + ("int8/f16/f64" if kind in (5, 6) else "f16/f64")
                   + " dense + f64 BM25") if use_e5 and args.e5_dtype == "float32" else "f16+f64"),
        "dtypes": {"dense_knn": {1: "f32 (MFMA)", 3: "f16 coarse (MFMA) + fp64 exact re-rank of the certified band",
                                 4: "f16 coarse (MFMA) + fp64 exact re-rank of the certified band",
                                 5: "int8 coarse (i8 MFMA, 16-row group scales) -> certified int8 band -> "
                                    "certified f16 band -> fp64 exact re-rank",
                                 6: "int8 coarse (i8 MFMA, 16-row group scales) -> certified int8 band -> "
                                    "certified f16 band -> fp64 exact re-rank"}[kind],
                   "bm25": "f64", "fusion": "f64",
                   "e5_forward": ({"float32": "fp32 (K10: split-precision f16 hi/lo MFMA, fp32 accumulate)",
                                   "bfloat16": "bf16"}[args.e5_dtype] if use_e5 else None)},
        "data": "synthetic (seeded): unit-norm Gaussian chunk embeddings, Zipf BM25 postings, random-init "
                "E5-base weights (no checkpoint offline)",
        "config": {"workload": ("hybrid retrieve: E5 query encode + cosine top-24 + MMR-10 + BM25 top-10 + RRF "
                                "top-10" if args.mode == "hybrid" else "dense cosine top-k"),
                   "chunks_per_gpu": N, "chunks_total": N * ws, "dim": D, "global_batch": B, "k": K, "pool": P,
                   "bm25_vocab": args.vocab, "zipf_s": args.zipf, "chunk_len_mean": args.avg_len,
                   "query_terms": args.q_terms, "e5_query_tokens": args.q_tokens if use_e5 else None,
                   "e5_queries_per_rank": bq if use_e5 else None,
                   "parallelism": f"corpus-shard x{ws}",
                   "schedule": ("pipelined: batch i+1 encoded beside batch i's search" if pipe["stream"] is not None
                                else "serial: encode, then search")},
        "breakdown_ms": {"e5_encode": e5_ms, "dense_search": search_ms, "dense_scan_kernel": dense_ms,
                         "bm25_search": bsearch_ms, "bm25_tail_kernel": bm25_ms, "bm25_block_kernel": bm25b_ms},
        "dense_exact_reruns": fallbacks,
        "bm25_rescored_pairs": rescored,
        "roofline": roof,
        "rooflines": roofs,
        **legs,
        "env": {e: os.environ[e] for e in KNOB_ENV if e in os.environ},
    }
    if args.cpu_baseline and args.mode == "hybrid":
        cpu, recall = cpu_baseline_and_recall(args, dense, bm25, res, q_terms, q_main, rank, ws, row0, N,
                                              lists_main, tokens_host)
        tokens_host = None
        out["cpu_baseline"] = cpu
        out["recall_at_10"] = recall
    else:
        out["cpu_baseline"] = None
        out["recall_at_10"] = None
    if args.mode == "hybrid" and args.dense_legs and ws == 1:
        # last: it plants rows into the shard (after the recall check has read it)
        out["c4_dup_cluster_b256"] = dup_cluster_leg(args, dense, N, D, dev, q_main, P,
                                                     legs.get("c4_dense_10m_b256", {}).get("ms_per_step"))
    out["setup_s"] = time.perf_counter() - t_setup
    if rank == 0:
        line = json.dumps(out)
        print(line, flush=True)
        if args.out:
            Path(args.out).write_text(line + "\n")
    if ws > 1:
        torch.distributed.destroy_process_group()


def _roof(bytes_, flops, peak_tflops, ms):
    """Bound = the larger of the HBM and MFMA floors; achieved in that unit."""
    if flops / (peak_tflops * 1e12) >= bytes_ / (PEAK_HBM_GBS * 1e9):
        r = dict(bound="mfma", achieved=flops / (ms * 1e-3) / 1e12, peak=peak_tflops, unit="TFLOP/s")
    else:
        r = dict(bound="hbm", achieved=bytes_ / (ms * 1e-3) / 1e9, peak=PEAK_HBM_GBS, unit="GB/s")
    r["frac"] = r["achieved"] / r["peak"]
    return r


def _dense_roofline(kind, N, D, B, ms, traffic):
    """Algorithmic work of one scan launch: corpus bytes in the kernel's own
    storage format + live bitmap + query planes; flops as executed on the MFMA units."""
    if kind == 1:      # fp32 rows + invc
        bytes_, flops, peak = N * D * 4 + N * 4 + N / 8 + B * D * 4, 2.0 * N * D * B, PEAK_F32_MFMA_TFLOPS
    elif kind in (5, 6):   # K1q / K1q-s: the int8 plane once + per-row {scale, bound} + live bits + int8 queries
        bytes_, flops, peak = N * D + N * 8 + N / 8 + B * D, 2.0 * N * D * B, PEAK_I8_MFMA_TOPS
    else:              # K1c / K1s: the f16 plane once + live bits + the f16 queries
        bytes_, flops, peak = N * D * 2 + N / 8 + B * D * 2, 2.0 * N * D * B, PEAK_F16_MFMA_TFLOPS
    r = _roof(bytes_, flops, peak, ms)
    r.update(traffic=traffic, kernel=DENSE_KINDS[kind], avg_launch_ms=ms,
             algorithmic_per_launch=dict(bytes=bytes_, flops=flops, rows=N, queries=B, dim=D))
    # the other side of the same launch: at B = 256 the f16 scan's intensity (B flop/B = 256) sits
    # just under the nominal ridge (2.5 PF / 8 TB/s = 312), and under the chip's power limit the
    # MFMA clock drops, so the MFMA side is reported beside the HBM fraction
    r["mfma_side"] = dict(achieved=flops / (ms * 1e-3) / 1e12, peak=peak, unit="TOP/s" if kind in (5, 6) else "TFLOP/s",
                          frac=flops / (ms * 1e-3) / 1e12 / peak)
    return r


def _bm25_roofline(bm25, q_terms, N, ms, traffic, terms_per_query):
    """K2a (the pruned search's tail pass, its largest kernel) per launch, algorithmic bytes:
    every walked posting read once (4 B doc + 2 B tf) and, per posting, the candidate's doc
    length (4 B) and one tf byte per head term of its query.  Walked terms = non-head terms, or
    the rarest head term of a query that has none (bm25_qcand_kernel); head terms = the tiles (the
    num_head_terms highest-df terms, df > N/128 within 8 GiB by default)
    K2a is latency/issue-bound, so this fraction is low by nature."""
    import numpy as np
    df, _ = bm25.term_stats()
    nh = bm25.num_head_terms                       # the tiles: the nh highest-df terms
    head_df = np.sort(df)[::-1][nh - 1] if nh > 0 else np.iinfo(np.int64).max
    qt = q_terms.view(-1, terms_per_query).cpu().numpy()
    bytes_ = 0.0
    for row in qt:
        row = row[(row >= 0) & (row < df.shape[0])]
        d = df[row].astype(np.float64)
        head = d >= head_df
        walked = d[~head] if (~head).any() else (np.array([d[head].min()]) if head.any() else d[:0])
        n_post = float(walked.sum())
        bytes_ += n_post * (6.0 + 4.0 + float(head.sum()))
    r = _roof(bytes_, 0.0, 1.0, ms)
    r.update(traffic=traffic, kernel="K2a bm25_tail_kernel (pruned BM25 tail pass)", avg_launch_ms=ms,
             algorithmic_per_launch=dict(bytes=bytes_, queries=int(qt.shape[0]), docs=N))
    return r


def _bm25_block_roofline(bm25, q_terms, items, ms, traffic, terms_per_query, sub_masks=None):
    """K2b (bm25_block_kernel: the head-only documents of the planned 16-doc sub-blocks; 64-doc blocks
    before round 6) per launch, algorithmic bytes: every planned sub-block's 16 documents read once --
    one tf byte per head term of its query (the dense tiles) + the 4-B length -- plus 8 B of live /
    allow words per sub-block and the item's 16 B (range word + sub-block mask).  Planned items from
    the last timed step's workspace."""
    import numpy as np
    df, _ = bm25.term_stats()
    nh = bm25.num_head_terms
    head_df = np.sort(df)[::-1][nh - 1] if nh > 0 else np.iinfo(np.int64).max
    qt = q_terms.view(-1, terms_per_query).cpu().numpy()
    nh_q = np.array([int((df[row[(row >= 0) & (row < df.shape[0])]] >= head_df).sum()) for row in qt], np.int64)
    q = (items >> np.uint64(40)).astype(np.int64)
    nblk = np.array([bin(int(x)).count("1") for x in (items & np.uint64(0xFFFF)).tolist()], np.int64)
    if sub_masks is None or sub_masks.shape[0] != items.shape[0]:
        sub_masks = np.array([sum(0xF << (4 * b) for b in range(16) if (int(x) >> b) & 1)
                              for x in (items & np.uint64(0xFFFF)).tolist()], np.uint64)
    nsub = np.array([bin(int(x)).count("1") for x in sub_masks.tolist()], np.int64)
    bytes_ = float((nsub * (16 * (nh_q[q] + 4) + 8)).sum() + 16 * items.shape[0])
    r = _roof(bytes_, 0.0, 1.0, ms)
    r.update(traffic=traffic, kernel="K2b bm25_block_kernel (head-only documents of the planned 16-doc sub-blocks)",
             avg_launch_ms=ms, algorithmic_per_launch=dict(bytes=bytes_, items=int(items.shape[0]),
                                                           blocks=int(nblk.sum()), subblocks=int(nsub.sum()),
                                                           docs=int(nsub.sum()) * 16))
    return r


def _e5_roofline(bq, S, layers, ms, dtype):
    """The E5 query encode of one rank's block against the MFMA peak of the dtype it issues.
    Algorithmic (fp32-equivalent) flops per sequence: 12 x (24 S d^2 + 4 S^2 d).
    fp32 runs on K10: every product is three f16 MFMAs, so the issued f16 flops are 3x; bf16 issues
    the algorithmic flops once.  The encode is many kernels (48 GEMMs, attention, LayerNorms), timed
    as a whole with HIP events around the graph replay."""
    d = 768
    alg = float(bq) * layers * (24.0 * S * d * d + 4.0 * S * S * d)
    issued = 3.0 * alg if dtype == "float32" else alg
    tf = issued / (ms * 1e-3) / 1e12
    return {"bound": "mfma", "achieved": tf, "peak": PEAK_F16_MFMA_TFLOPS, "unit": "TFLOP/s",
            "frac": tf / PEAK_F16_MFMA_TFLOPS, "traffic": None, "avg_launch_ms": ms,
            "kernel": ("E5 encode (K10 split-precision f16 MFMA GEMMs x48 + f16x3 MFMA attention + K8 LayerNorm)"
                       if dtype == "float32" else "E5 encode (bf16, hipBLASLt GEMMs + K9 + K8)"),
            "algorithmic_per_launch": {"flops_fp32_equiv": alg, "flops_issued": issued, "queries": bq,
                                       "tokens": S, "layers": layers},
            "fp32_equiv_tflops": alg / (ms * 1e-3) / 1e12,
            "vs_fp32_mfma_peak": alg / (ms * 1e-3) / 1e12 / PEAK_F32_MFMA_TFLOPS}


def dense_legs(args, dense, N, D, dev, ws, q_step=None, pool=None):
    """north_star's dense configurations, timed in the same run (side fields, not the headline):
    C2' = this rank's 10M shard at B = 16, k = 10 (the HBM-bound case the >= 80 % target names; K1q
    since late round 4 -- the f16 K1s stream it replaced reached 0.84 of HBM on twice the bytes);
    C2 = a 1M-chunk shard (its own index), B = 256, k = 10 (queries: unit Gaussian); and the
    headline's dense search alone -- the step's own query embeddings and pool size on this shard,
    without the BM25 stream beside it."""
    import torch
    from classmate_hip import engine, parallel
    legs = {}

    def leg(index, n, b, name, q=None, kk=None):
        kk = kk or args.k
        if q is None:
            g = torch.Generator(device="cuda").manual_seed(args.seed * 31 + b)
            q = torch.randn(b, D, device=dev, generator=g)
            q /= q.norm(dim=1, keepdim=True)
        ws_buf = torch.empty(index.workspace_bytes(b, kk), dtype=torch.uint8, device=dev)
        o = (torch.empty((b, kk), dtype=torch.float32, device=dev),
             torch.empty((b, kk), dtype=torch.int64, device=dev))
        for _ in range(args.warmup):
            index.search_dev(q, kk, out=o, workspace=ws_buf)
        torch.cuda.synchronize()
        index.timing(True)
        if ws > 1:
            torch.distributed.barrier()
        t0 = time.perf_counter()
        steps = max(args.steps, 10)
        for _ in range(steps):
            index.search_dev(q, kk, out=o, workspace=ws_buf)
        torch.cuda.synchronize()
        if ws > 1:
            torch.distributed.barrier()
        el = parallel.max_over_ranks(time.perf_counter() - t0, device=dev)
        kt = index.timing_drain()
        index.timing(False)
        kind = index.search_kind(b, kk)
        r = _dense_roofline(kind, n, D, b, sum(kt) / len(kt),
                            _pmc_traffic(args, {5: "dense_q8", 6: "dense_q8s"}.get(kind, "dense"), b)
                            if n == args.docs_per_gpu else None)
        legs[name] = {"value": b * steps * ws / el, "unit": "queries/s", "ms_per_step": el / steps * 1e3,
                      "config": {"chunks_per_gpu": n, "batch": b, "k": kk, "dim": D},
                      "roofline": r}
        log(f"{name}: {b * steps * ws / el:.0f} q/s, scan {r['avg_launch_ms']:.3f} ms = {r['frac']:.3f} of {r['bound']}")

    if q_step is not None and q_step.shape[0] == args.batch:
        leg(dense, N, args.batch, "c4_dense_10m_b256", q=q_step.contiguous(), kk=pool)
    leg(dense, N, 16, "c2p_dense_10m_b16")
    n1 = min(1_000_000, N)
    d1 = engine.DenseIndex(D, device=dev.index, capacity=n1)
    gen_dense(d1, n1, D, seed=args.seed * 1000 + 77)
    leg(d1, n1, 256, "c2_dense_1m_b256")
    d1.close()
    del d1
    torch.cuda.empty_cache()
    return legs


def dup_cluster_leg(args, dense, N, D, dev, q_step, P, normal_ms):
    """the certificate's cliff, priced.  Real corpora hold near-duplicate chunks (the
    same file ingested under two courses: distinct ids, identical embeddings); a query that sits on
    a cluster wider than the int8 band's 8192 rows fails its certificate and is re-searched by the
    exact fp32 pass.  12 000 rows within 5e-4 (cosine distance) of one row are planted into the
    shard, and 8 of the step's 256 queries are put on that row: the whole dense search (pool 24,
    K1q + re-rank + the exact pass for the failing queries) timed like the c4 leg, with the number of
    exact re-runs.  Runs last (it changes the shard)."""
    import numpy as np
    import torch
    rng = np.random.default_rng(args.seed + 4242)
    n_c = 12_000
    base_row = 7
    base = dense.export(base_row, 1)[0].astype(np.float64)
    base /= np.linalg.norm(base)
    at = rng.choice(np.arange(base_row + 1, N), n_c, replace=False).astype(np.int64)
    d_c = rng.permutation(np.linspace(1e-5, 5e-4, n_c))
    u = rng.standard_normal((n_c, D))
    u -= np.outer(u @ base, base)
    u /= np.linalg.norm(u, axis=1, keepdims=True)
    t = np.sqrt(2.0 * d_c - d_c ** 2)
    x = (np.sqrt(1.0 - t ** 2)[:, None] * base + t[:, None] * u).astype(np.float32)
    dense.upsert(x, at)
    q = q_step.clone()
    near = torch.from_numpy((base + 1e-4 * rng.standard_normal((8, D)) / np.sqrt(D)).astype(np.float32)).to(dev)
    q[:8] = near
    B = q.shape[0]
    ws_buf = torch.empty(dense.workspace_bytes(B, P), dtype=torch.uint8, device=dev)
    o = (torch.empty((B, P), dtype=torch.float32, device=dev), torch.empty((B, P), dtype=torch.int64, device=dev))
    for _ in range(max(1, args.warmup)):
        dense.search_dev(q, P, out=o, workspace=ws_buf)
    torch.cuda.synchronize()
    steps = max(args.steps, 10)
    t0 = time.perf_counter()
    for _ in range(steps):
        dense.search_dev(q, P, out=o, workspace=ws_buf)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / steps * 1e3
    fb = dense.workspace_fallbacks(B, P, ws_buf)
    wide = dense.workspace_wide_reranks(B, P, ws_buf)
    rows = o[1][:8].cpu().numpy()
    on_cluster = float(np.isin(rows, np.concatenate([at, [base_row]])).mean())
    r = {"ms_per_step": ms, "queries/s": B / ms * 1e3, "exact_reruns": fb, "wide_reranks": wide, "cluster_rows": n_c,
         "cluster_queries": 8, "normal_batch_ms": normal_ms, "ratio_to_normal": (ms / normal_ms) if normal_ms else None,
         "cluster_queries_top24_on_cluster": on_cluster,
         "note": "dense search (pool 24) of the step's 256 queries with 8 moved onto a planted cluster of 12k rows "
                 "within 5e-4 of one row; their int8 bands overflow the re-rank's LDS and the wide re-rank "
                 "finishes them from the complete candidate buffers (exact fp64 distances of every band row); "
                 "the exact fp32 pass re-searches what it cannot take"}
    log(f"c4_dup_cluster_b256: {ms:.3f} ms per search ({wide} wide re-ranks, {fb} exact re-runs; normal batch "
        f"{normal_ms if normal_ms is None else round(normal_ms, 3)} ms)")
    return r


def ingest_leg(args, emb, dev, ws, rank):
    """BASELINE configs[2] beside the headline: the passage encode of 256 chunks x --seq-len tokens
    per step at the reference's fp32 (K10 GEMMs + attention + K8 + K6 pooling), chunks/s over all
    ranks (data-parallel replicas) and the encode against the f16 MFMA peak with the
    issued flops (3 x the fp32-equivalent 12 (24 S d^2 + 4 S^2 d) per chunk)."""
    import torch
    from classmate_hip import parallel
    from classmate_hip.embeddings import E5MultilingualEmbedder
    if emb is None:
        emb = E5MultilingualEmbedder.random_init(seed=0, device=str(dev), num_layers=args.e5_layers, dtype="float32")
    B, S = 256, args.seq_len
    g = torch.Generator(device="cuda").manual_seed(args.seed + 101 + rank)
    ids = torch.randint(5, 250002, (B, S), device=dev, generator=g)
    ids[:, 0] = 0
    ids[:, -1] = 2
    mask = torch.ones_like(ids)
    out = torch.empty((B, 768), dtype=torch.float32, device=dev)
    for _ in range(max(1, min(args.warmup, 2))):
        emb.encode_token_ids(ids, mask, out=out)
    steps = max(3, min(args.steps, 10))
    torch.cuda.synchronize()
    if ws > 1:
        torch.distributed.barrier()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record()
    for _ in range(steps):
        emb.encode_token_ids(ids, mask, out=out)
    e1.record()
    torch.cuda.synchronize()
    if ws > 1:
        torch.distributed.barrier()
    el = parallel.max_over_ranks(time.perf_counter() - t0, device=dev)
    ms = e0.elapsed_time(e1) / steps
    alg = float(B) * args.e5_layers * (24.0 * S * 768 ** 2 + 4.0 * S * S * 768)
    issued = 3.0 * alg
    leg = {"value": B * steps * ws / el, "unit": "chunks/s", "ms_per_step": el / steps * 1e3, "steps": steps,
           "config": {"workload": "E5-base passage encode (BASELINE configs[2] shape)", "chunks_per_step": B * ws,
                      "seq_len": S, "e5_forward": "fp32 (K10 f16x3)", "parallelism": f"replicas x{ws}"},
           "fp32_equiv_tflops": alg / (ms * 1e-3) / 1e12}
    roof = {"bound": "mfma", "achieved": issued / (ms * 1e-3) / 1e12, "peak": PEAK_F16_MFMA_TFLOPS,
            "unit": "TFLOP/s", "frac": issued / (ms * 1e-3) / 1e12 / PEAK_F16_MFMA_TFLOPS, "traffic": None,
            "avg_launch_ms": ms, "kernel": "E5 passage encode (K10 f16x3 GEMMs + attention + K8 + K6), whole forward",
            "algorithmic_per_launch": {"flops_fp32_equiv": alg, "flops_issued": issued, "chunks": B, "tokens": S,
                                       "layers": args.e5_layers}}
    log(f"ingest_fp32: {leg['value']:.0f} chunks/s ({ms:.2f} ms per {B} x {S} tokens, {roof['frac']:.3f} of f16 peak)")
    return leg, roof


def _zipf_texts(rng, n, lo, hi, zipf=1.07, vocab=1 << 16):
    """n synthetic chunks of U[lo, hi] letters-only words (Zipf draws from `vocab` words "zq" + 4
    letters): the BM25 tokenizer keeps every word, the E5 hash tokenizer maps each to one token."""
    import numpy as np
    p = 1.0 / np.arange(1, vocab + 1) ** zipf
    cdf = np.cumsum(p)
    cdf /= cdf[-1]
    alpha = np.frombuffer(b"abcdefghijklmnopqrstuvwxyz", np.uint8)
    wv = np.arange(vocab)
    vb = np.empty((vocab, 7), np.uint8)
    vb[:, 0], vb[:, 1], vb[:, 6] = ord("z"), ord("q"), ord(" ")
    for i in range(4):
        vb[:, 2 + i] = alpha[(wv // 26 ** i) % 26]
    lens = rng.integers(lo, hi + 1, n)
    words = np.minimum(np.searchsorted(cdf, rng.random(int(lens.sum()))), vocab - 1)
    blob = vb[words].tobytes()
    out, o = [], 0
    for ln in lens.tolist():
        out.append(blob[o * 7:(o + ln) * 7 - 1].decode("ascii"))
        o += ln
    return out, lens


def _e5_seq_flops(S, layers=12, d=768):
    """fp32-equivalent forward flops of one sequence of S real tokens (padding excluded)."""
    return float(layers) * (24.0 * S * d * d + 4.0 * S * S * d)


def varlen_ingest_leg(args, emb, dev, ws, rank):
    """SURVEY §8(d) C3's variable-length run: --varlen-chunks passages of S ~ U[64, 512] tokens
    (incl. <s>, "passage", ":" and </s>) through the drop-in ``encode_passages`` (sentence-
    transformers' length-sorted batches of 32, rag/embeddings/__init__.py:98-105), tokenization
    included, numpy fp32 out.  chunks/s over all ranks (replicas); the roofline counts the real
    tokens' flops only (no padding), 3x issued on K10."""
    import numpy as np
    import torch
    from classmate_hip import parallel
    from classmate_hip.embeddings import E5MultilingualEmbedder
    if emb is None:
        emb = E5MultilingualEmbedder.random_init(seed=0, device=str(dev), num_layers=args.e5_layers, dtype="float32")
    rng = np.random.default_rng(args.seed * 7 + 991 + rank)
    n = args.varlen_chunks
    texts, words = _zipf_texts(rng, n, 60, 508)
    S = words + 4
    emb.encode_passages(texts[: min(n, 256)])                       # kernels / first shapes
    torch.cuda.synchronize()
    if ws > 1:
        torch.distributed.barrier()
    t0 = time.perf_counter()
    out = emb.encode_passages(texts)
    torch.cuda.synchronize()
    if ws > 1:
        torch.distributed.barrier()
    el = parallel.max_over_ranks(time.perf_counter() - t0, device=dev)
    assert out.shape == (n, 768) and out.dtype == np.float32
    alg = sum(_e5_seq_flops(int(x), args.e5_layers) for x in S)
    tf = 3.0 * alg / el / 1e12
    leg = {"value": n * ws / el, "unit": "chunks/s", "seconds": el,
           "tokens_per_s": float(S.sum()) * ws / el,
           "config": {"workload": "encode_passages, S ~ U[64, 512] (BASELINE configs[2], SURVEY §8d C3 variable-length run)",
                      "chunks": n * ws, "mean_tokens": float(S.mean()), "min_tokens": int(S.min()),
                      "max_tokens": int(S.max()), "batching": "length-sorted batches of 32 (sentence-transformers)",
                      "includes": "host tokenization (offline hash tokenizer) + forward + K6 pooling + copy to numpy",
                      "e5_forward": "fp32 (K10 f16x3)", "parallelism": f"replicas x{ws}"},
           "roofline": {"bound": "mfma", "achieved": tf, "peak": PEAK_F16_MFMA_TFLOPS, "unit": "TFLOP/s",
                        "frac": tf / PEAK_F16_MFMA_TFLOPS, "traffic": None,
                        "algorithmic": {"flops_fp32_equiv": alg, "flops_issued": 3.0 * alg,
                                        "note": "real tokens only; padding to the batch maximum is wasted work"}}}
    log(f"ingest_varlen_fp32: {leg['value']:.0f} chunks/s ({n} chunks, mean S {S.mean():.0f}, {el:.2f} s, "
        f"{leg['roofline']['frac']:.3f} of f16 peak on real tokens)")
    return leg


def ingest_e2e_leg(args, emb, dev):
    """The reference's ingest of one file (rag/pipeline/rag.py:410-413) repeated over --ingest-e2e-chunks
    chunks in files of 4096: CachingEmbedder(E5).encode_passages -> ChromaVectorStore.upsert
    (persisted) -> BM25Store.upsert_many -> BM25Store.save, each file through the drop-in classes,
    then the first search's BM25 index build.  chunks/s end to end with the per-stage seconds.  Files of
    --ingest-e2e-file-chunks (4096 by default)."""
    import shutil
    import tempfile
    import numpy as np
    import torch
    from classmate_hip.embeddings import CachingEmbedder, E5MultilingualEmbedder
    from classmate_hip.retrieval.bm25 import BM25Store
    from classmate_hip.retrieval.vector_store import GpuVectorStore
    if emb is None:
        emb = E5MultilingualEmbedder.random_init(seed=0, device=str(dev), num_layers=args.e5_layers, dtype="float32")
    n, per_file = args.ingest_e2e_chunks, args.ingest_e2e_file_chunks
    rng = np.random.default_rng(args.seed * 11 + 5)
    root = Path(tempfile.mkdtemp(prefix="cm_ingest_", dir=os.environ.get("TMPDIR")))
    try:
        vs = GpuVectorStore(persist_dir=root / "chroma", device=dev.index)
        bm = BM25Store.load_or_create(root / "bm25")
        bm.device = dev.index
        cemb = CachingEmbedder(emb, cache_dir=str(root / "emb_cache"))
        warm, _ = _zipf_texts(rng, 64, 60, 508)
        emb.encode_passages(warm)
        torch.cuda.synchronize()
        st = dict(encode=0.0, vector_upsert=0.0, bm25_upsert=0.0, bm25_save=0.0, bm25_index_build=0.0, texts=0.0)
        tok = 0
        t_all = time.perf_counter()
        for f0 in range(0, n, per_file):
            m = min(per_file, n - f0)
            t = time.perf_counter()
            texts, words = _zipf_texts(rng, m, 60, 508)      # the chunker's output (not the path: untimed)
            st["texts"] += time.perf_counter() - t
            tok += int(words.sum()) + 4 * m
            ids = [f"f{f0 // per_file}:c{j}" for j in range(m)]
            metas = [{"course": f"C{(f0 + j) % 16}", "language": "en", "doc_type": "pdf", "week": (f0 + j) % 12}
                     for j in range(m)]
            t = time.perf_counter()
            e = cemb.encode_passages(texts)
            st["encode"] += time.perf_counter() - t
            t = time.perf_counter()
            vs.upsert(ids=ids, documents=texts, metadatas=metas, embeddings=e)
            st["vector_upsert"] += time.perf_counter() - t
            t = time.perf_counter()
            bm.upsert_many(ids=ids, texts=texts, metadatas=metas)
            st["bm25_upsert"] += time.perf_counter() - t
            t = time.perf_counter()
            bm.save()
            st["bm25_save"] += time.perf_counter() - t
            if per_file >= 16384 or (f0 // per_file) % 4 == 3 or f0 + m >= n:   # progress (long runs)
                log(f"ingest_e2e: {f0 + m} / {n} chunks ({time.perf_counter() - t_all:.1f} s)")
        t = time.perf_counter()
        bm._ensure_index()                                  # the first search after the ingest builds it
        torch.cuda.synchronize()
        st["bm25_index_build"] = time.perf_counter() - t
        total = time.perf_counter() - t_all - st["texts"]
        assert vs.count() == n and len(bm._id_list) == n
    finally:
        shutil.rmtree(root, ignore_errors=True)
    leg = {"value": n / total, "unit": "chunks/s", "seconds": total, "chunks": n, "tokens": tok,
           "breakdown_s": {k: v for k, v in st.items() if k != "texts"},
           "config": {"workload": "ingest_file's store path per file (rag/pipeline/rag.py:410-413): "
                                  "CachingEmbedder(E5 fp32).encode_passages -> ChromaVectorStore.upsert (persisted) -> "
                                  "BM25Store.upsert_many -> BM25Store.save; + the BM25 device index build",
                      "chunks_per_file": per_file,
                      "tokens_per_chunk": "U[64, 512]", "files": (n + per_file - 1) // per_file}}
    log(f"ingest_e2e: {leg['value']:.0f} chunks/s over {n} chunks ({total:.1f} s: "
        + ", ".join(f"{k} {v:.1f}" for k, v in leg["breakdown_s"].items()) + ")")
    return leg


def _pmc_traffic(args, which, batch=None):
    """HBM bytes per launch (FETCH_SIZE x 2, the gfx950 correction) from a committed rocprofv3
    --pmc summary of this config (profiles/pmc_traffic.json), or None."""
    p = REPO / "profiles" / "pmc_traffic.json"
    try:
        d = json.loads(p.read_text())
        return d.get(f"{which}_{args.docs_per_gpu}x{args.dim}_B{batch or args.batch}")
    except Exception:
        return None


# ---------------------------------------------------------------------------
def cpu_baseline_and_recall(args, dense, bm25, res, q_terms, q_dev, rank, ws, row0, N, gpu_lists=None,
                            tokens_host=None):
    """Time the CPU oracle on a bounded sample of the step's queries (its query embeddings) over
    every rank's shard (each rank scans its own, in parallel), merge the per-shard exact lists
    (a merge of exact per-shard top lists is the exact global list), run MMR + RRF on the merged
    pools, and compare with the GPU's final top-10: recall@10 at any N.  cpu_baseline.value is
    the rate of ONE host doing all shards' scans and the fusion (sum of the shard times)."""
    import numpy as np
    import torch
    from classmate_hip import parallel
    from oracle import corc
    from oracle import ref_semantics as orc

    Qc = min(args.cpu_queries, args.batch)
    K, P = args.k, args.pool
    qh = q_dev[:Qc].float().cpu().numpy()
    qt = q_terms.view(args.batch, -1)[:Qc].cpu().numpy()
    gpu_keys = res[0][:Qc].cpu().numpy()
    threads = max(corc.num_threads(), torch.get_num_threads())
    # BM25 statistics: global (build-time, not timed).  The oracle scores its OWN CSR, built on the
    # host from the shard's tokens (oracle/cm_oracle.c orc_build_csr), not the device index K7 built;
    # the device index is compared with it array for array first
    t = time.perf_counter()
    csr = bm25.export()
    if tokens_host is not None:
        ocsr = corc.build_csr(tokens_host[0], tokens_host[1], bm25.vocab)
        same = all(np.array_equal(csr[k], ocsr[k]) for k in ("term_off", "post_doc", "post_tf", "dl"))
        odf = np.diff(ocsr["term_off"])
        nz = odf > 0
        fp0 = ocsr["term_off"][:-1][nz]
        if same:
            same = np.array_equal(ocsr["first_key"][nz], (csr["post_doc"][fp0].astype(np.uint64) << np.uint64(32))
                                  | csr["post_pos"][fp0].astype(np.uint64))
        csr_source = ("oracle CSR built on the host from the shard's tokens; device index (K7) "
                      + ("== it, array for array" if same else "DIFFERS from it"))
        term_off, df, first = ocsr["term_off"], ocsr["df"], ocsr["first_key"]
        ccsr = dict(term_off=term_off, post_doc=ocsr["post_doc"], post_tf=ocsr["post_tf"], dl=ocsr["dl"],
                    vocab=int(df.shape[0]), ndocs=int(ocsr["dl"].shape[0]))
        del ocsr
    else:
        csr_source = "device index export (K7 build)"
        term_off = csr["term_off"]
        df = np.diff(term_off)
        first = np.full(df.shape[0], np.uint64(0xFFFFFFFFFFFFFFFF))
        nz = df > 0
        fp = term_off[:-1][nz]
        first[nz] = (csr["post_doc"][fp].astype(np.uint64) << np.uint64(32)) | csr["post_pos"][fp].astype(np.uint64)
        ccsr = dict(term_off=term_off, post_doc=csr["post_doc"], post_tf=csr["post_tf"], dl=csr["dl"],
                    vocab=int(df.shape[0]), ndocs=int(csr["dl"].shape[0]))
    del csr
    n_docs = ccsr["ndocs"]
    sum_len = int(ccsr["dl"].astype(np.int64).sum())
    if ws == 1:
        idf, _ = corc.bm25_idf(df, first, n_docs)
        gn, gsum = n_docs, sum_len
    else:
        gdf, gfk, gn, gsum = parallel.allreduce_bm25_stats(df, first, row0, n_docs, sum_len)
        idf, _ = parallel.bm25_idf_table(gdf, gfk, gn)
    avgdl = float(gsum) / gn
    log(f"cpu baseline: {csr_source}; global statistics ({time.perf_counter() - t:.1f}s)")

    # dense: exact fp64 top-P over this shard, chunk by chunk (fp32 BLAS scan for candidates, fp64
    # re-rank of 4P per chunk; export of each chunk not timed)
    t_dense = 0.0
    best_d = np.full((Qc, 0), np.inf)
    best_r = np.zeros((Qc, 0), np.int64)
    best_v = np.zeros((Qc, 0, qh.shape[1]), np.float32)
    qn = np.linalg.norm(qh.astype(np.float64), axis=1)
    chunk = 1 << 20
    for c0 in range(0, N, chunk):
        C = dense.export(c0, min(chunk, N - c0))
        t0 = time.perf_counter()
        sims = C @ qh.T                                        # (n, Qc)
        m = min(4 * P, C.shape[0])
        cand = np.argpartition(-sims, m - 1, axis=0)[:m].T     # (Qc, m)
        cv = C[cand].astype(np.float64)                        # (Qc, m, D)
        dd = 1.0 - np.einsum("qmd,qd->qm", cv, qh.astype(np.float64)) / np.linalg.norm(cv, axis=2) / qn[:, None]
        best_d = np.concatenate([best_d, dd], 1)
        best_r = np.concatenate([best_r, cand + c0 + row0], 1)
        best_v = np.concatenate([best_v, C[cand]], 1)
        o = np.lexsort((best_r, best_d), axis=1)[:, :P]
        best_d = np.take_along_axis(best_d, o, 1)
        best_r = np.take_along_axis(best_r, o, 1)
        best_v = np.take_along_axis(best_v, o[:, :, None], 1)
        t_dense += time.perf_counter() - t0
        del C, sims
    t1 = time.perf_counter()
    bs, br = corc.bm25_topk(ccsr, idf, avgdl, [list(x) for x in qt], K)
    t_bm25 = time.perf_counter() - t1
    br = np.where(br >= 0, br + row0, br)
    shard = dict(rank=rank, d=best_d, r=best_r, v=best_v, bs=bs, br=br, t_dense=t_dense, t_bm25=t_bm25)
    if ws > 1:
        allv = [None] * ws
        torch.distributed.all_gather_object(allv, shard)
    else:
        allv = [shard]
    # merge (exact per-shard lists -> exact global lists), then MMR + RRF (oracle semantics)
    D_ = np.concatenate([x["d"] for x in allv], 1)
    R_ = np.concatenate([x["r"] for x in allv], 1)
    V_ = np.concatenate([x["v"] for x in allv], 1)
    o = np.lexsort((R_, D_), axis=1)[:, :P]
    dense_dist, dense_rows = np.take_along_axis(D_, o, 1), np.take_along_axis(R_, o, 1)
    pool_v = np.take_along_axis(V_, o[:, :, None], 1)
    BS = np.concatenate([x["bs"] for x in allv], 1)
    BR = np.concatenate([x["br"] for x in allv], 1)
    t2 = time.perf_counter()
    cpu_keys = []
    for i in range(Qc):
        valid = BR[i] >= 0
        cand = sorted(zip(-BS[i][valid], BR[i][valid]))[:K]          # score desc, row asc
        bm_ids = [int(r_) for _, r_ in cand]
        order = orc.mmr_order(qh[i], pool_v[i], list(range(P)), K, 0.5)
        vec_ids = [int(dense_rows[i][j]) for j in order]
        fused = orc.rrf_fuse(rank_lists=[vec_ids, bm_ids], weights=[1.0, 1.0], rrf_k=60)
        vdist = {int(dense_rows[i][j]): float(np.float32(dense_dist[i][j])) for j in order}
        items = list(dict.fromkeys(vec_ids + bm_ids))
        items.sort(key=lambda x: (fused[x], -vdist.get(x, 0.0)), reverse=True)
        cpu_keys.append(items[:K])
    t_fuse = time.perf_counter() - t2
    recall = float(np.mean([len(set(cpu_keys[i]) & set(int(x) for x in gpu_keys[i] if x >= 0)) / K
                            for i in range(Qc)]))
    shown = 0
    for i in range(Qc):          # the first mismatching queries, for diagnosis
        g = [int(x) for x in gpu_keys[i] if x >= 0]
        if g != cpu_keys[i] and shown < 3:
            shown += 1
            log(f"recall mismatch q{i}: gpu {g} cpu {cpu_keys[i]}; pool rows {dense_rows[i][:P].tolist()} "
                f"dist {[round(float(x), 7) for x in dense_dist[i][:P]]}; bm25 {BR[i].tolist()} {BS[i].tolist()}")
            if gpu_lists is not None:
                rg, dm, brg, bsm, order, gv = (t.cpu().numpy() for t in gpu_lists)
                log(f"  gpu lists q{i}: pool rows {rg[i].tolist()} dist {[round(float(x), 7) for x in dm[i]]}; "
                    f"bm25 {brg[i].tolist()} {bsm[i].tolist()}")
                if i < order.shape[0]:   # rank 0's query block (rows of its MMR launch)
                    o_cpu = orc.mmr_order(qh[i], pool_v[i], list(range(P)), K, 0.5)
                    o_gv = orc.mmr_order(qh[i], gv[i], list(range(P)), K, 0.5)
                    log(f"  mmr q{i}: gpu {order[i].tolist()} oracle {o_cpu} oracle-on-gpu-pool {o_gv}; "
                        f"max |gpu pool - oracle pool| {float(np.abs(gv[i] - pool_v[i]).max()):.3e}")
    shard_s = [x["t_dense"] + x["t_bm25"] for x in allv]
    total = sum(shard_s) + t_fuse
    cpu = dict(value=Qc / total, unit="queries/s", cores=int(threads), kind="port",
               sample=f"{Qc} of the {args.batch} queries of one step over all {ws} x {N}-chunk shards (dense: numpy "
                      f"fp32 BLAS scan + fp64 re-rank per 1M-row chunk; BM25: oracle/cm_oracle.c OpenMP with the "
                      f"global statistics; MMR/RRF: oracle/ref_semantics.py; E5 encode excluded); value = one host "
                      f"doing every shard's scan in turn",
               seconds=total, per_shard_s=shard_s, bm25_csr=csr_source,
               breakdown_s=dict(dense=sum(x["t_dense"] for x in allv), bm25=sum(x["t_bm25"] for x in allv),
                                mmr_rrf=t_fuse))
    log(f"cpu baseline {cpu['value']:.2f} q/s ({threads} threads per shard, {ws} shards); recall@10 {recall:.4f}")
    return cpu, recall


# ---------------------------------------------------------------------------
def run_e2e(args, rank, ws, dev):
    """The drop-in API end to end: HybridRetriever.retrieve_batch over query STRINGS
    -> lists of result dicts, through GpuVectorStore / BM25Store / E5MultilingualEmbedder exactly as
    the reference's callers use them (rag/retrieval/fusion.py HybridRetriever.retrieve).  Corpus:
    --docs-per-gpu synthetic chunks of --e2e-words Zipf words (letters-only ids, as the BM25 tokenizer
    keeps letters only), metadata {course, week, language},
    random unit embeddings upserted with the texts (the passage encode is ingest mode's metric);
    queries are word samples of corpus chunks encoded by the random-init E5 (fp32, the drop-in
    default) with the offline hash tokenizer.  value = retrieve_batch queries/s (B per call);
    also single-query retrieve() latency p50 / p99."""
    import numpy as np
    import torch
    from classmate_hip.embeddings import E5MultilingualEmbedder
    from classmate_hip.retrieval import device_batch
    from classmate_hip.retrieval.bm25 import BM25Store
    from classmate_hip.retrieval.fusion import HybridRetriever
    from classmate_hip.retrieval.vector_store import GpuVectorStore
    if ws != 1:
        sys.exit("bench.py --mode e2e: single process (the drop-in API is one store per process)")
    N, B, K, D = args.docs_per_gpu, args.batch, args.k, args.dim
    rng = np.random.default_rng(args.seed)
    t_setup = time.perf_counter()
    V = 1 << 16
    p = 1.0 / np.arange(1, V + 1) ** args.zipf
    cdf = np.cumsum(p)
    cdf /= cdf[-1]
    W = args.e2e_words
    # word w = "zq" + 4 letters (letters only, as the BM25 tokenizer keeps letters only); texts are
    # cut from one byte image of N x W words (7 bytes with the separator) instead of a join per word
    alpha = np.frombuffer(b"abcdefghijklmnopqrstuvwxyz", np.uint8)
    wv = np.arange(V)
    vb = np.empty((V, 7), np.uint8)
    vb[:, 0], vb[:, 1], vb[:, 6] = ord("z"), ord("q"), ord(" ")
    for i in range(4):
        vb[:, 2 + i] = alpha[(wv // 26 ** i) % 26]
    texts = []
    for c0 in range(0, N, 1 << 20):
        c1 = min(N, c0 + (1 << 20))
        words = np.minimum(np.searchsorted(cdf, rng.random((c1 - c0) * W)), V - 1).astype(np.int32)
        blob = vb[words].tobytes()
        L = 7 * W
        texts.extend(blob[i * L:(i + 1) * L - 1].decode("ascii") for i in range(c1 - c0))
        del words, blob
    ids = [f"c{i}" for i in range(N)]
    # a quarter of the chunks carry no course: ask_question's filters.to_dict() keeps course=None, and
    # BM25's _matches_filter then admits exactly those (quirk Q4, rag/retrieval/bm25.py:103-106)
    metas = [({"course": f"C{i % 16}"} if i % 4 else {}) | {"week": int(i % 12), "language": "en"} for i in range(N)]
    log(f"e2e corpus: {N} chunks x {args.e2e_words} words ({time.perf_counter() - t_setup:.1f}s)")
    g = torch.Generator(device="cuda").manual_seed(args.seed * 1000)
    emb = torch.randn(N, D, device=dev, generator=g)
    emb /= emb.norm(dim=1, keepdim=True)
    emb = emb.cpu().numpy()
    vs = GpuVectorStore(persist_dir=None, device=dev.index)
    step = 1 << 18
    for i in range(0, N, step):
        vs.upsert(ids=ids[i:i + step], documents=texts[i:i + step], metadatas=metas[i:i + step],
                  embeddings=emb[i:i + step])
        if (i // step) % 8 == 7:
            log(f"vector store: {i + step} chunks ({time.perf_counter() - t_setup:.1f}s)")
    del emb
    bm = BM25Store(index_dir=None, device=dev.index)
    step = 1 << 20
    for i in range(0, N, step):       # one upsert_many per 1M chunks (progress lines; same store)
        bm.upsert_many(ids=ids[i:i + step], texts=texts[i:i + step], metadatas=metas[i:i + step])
        log(f"bm25 store: {min(N, i + step)} chunks tokenized ({time.perf_counter() - t_setup:.1f}s)")
    embedder = E5MultilingualEmbedder.random_init(seed=0, device=str(dev), num_layers=args.e5_layers)
    retr = HybridRetriever(vector_store=vs, bm25_store=bm, embedder=embedder)
    qsrc = rng.integers(0, N, B * (args.steps + args.warmup + 1))
    qs = [" ".join(texts[i].split()[j:j + 6]) for i, j in zip(qsrc, rng.integers(0, args.e2e_words - 6, qsrc.size))]
    log("first retrieve_batch: builds the BM25 device index")
    retr.retrieve_batch(questions=qs[:B], top_k=K)     # builds the BM25 index, first graph/kernels
    torch.cuda.synchronize()
    log(f"e2e stores ready: {vs.count()} vectors, {len(bm._id_list)} BM25 docs ({time.perf_counter() - t_setup:.1f}s)")
    for w in range(args.warmup):
        retr.retrieve_batch(questions=qs[(w + 1) * B:(w + 2) * B], top_k=K)
    torch.cuda.synchronize()
    prof = None
    if os.environ.get("CM_E2E_PROFILE"):              # host-side profile of the timed calls
        import cProfile
        prof = cProfile.Profile()
        prof.enable()
    t0 = time.perf_counter()
    n_res = 0
    for st in range(args.steps):
        o = (args.warmup + 1 + st) * B
        res = retr.retrieve_batch(questions=qs[o:o + B], top_k=K)
        n_res += sum(len(r) for r in res)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if prof is not None:
        import pstats
        prof.disable()
        pstats.Stats(prof, stream=sys.stderr).sort_stats("cumulative").print_stats(40)
    ab_env = {}
    if args.e2e_ab_env:                  # A/B knobs read at launch time (engine env_knob), alternating
        def timed_batches(tag):
            for w in range(2):
                retr.retrieve_batch(questions=qs[w * B:(w + 1) * B], top_k=K)
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            for st in range(args.steps):
                o = (args.warmup + 1 + st) * B
                retr.retrieve_batch(questions=qs[o:o + B], top_k=K)
            torch.cuda.synchronize()
            v = B * args.steps / (time.perf_counter() - t1)
            ab_env.setdefault(tag, []).append(round(v, 1))
            log(f"A/B retrieve_batch [{tag}]: {v:.1f} q/s")
        sets = [x for x in args.e2e_ab_env.split(";") if x]
        for _ in range(2):
            timed_batches("default")
            for spec in sets:
                kv = dict(item.split("=", 1) for item in spec.split(","))
                old_env = {k: os.environ.get(k) for k in kv}
                os.environ.update(kv)
                try:
                    timed_batches(spec)
                finally:
                    for k, v in old_env.items():
                        if v is None:
                            os.environ.pop(k, None)
                        else:
                            os.environ[k] = v
    # single-query retrieve() latency: unfiltered, and with ask_question's filters
    # (rag/pipeline/rag.py:548-554: DocumentMetadata(...).to_dict(), None keys kept -- quirk Q4)
    none_keys = {"course": None, "unit": None, "author": None, "semester": None, "source_path": None,
                 "created_at": None}
    shapes = {"unfiltered": None, "to_dict_default": none_keys, "to_dict_course": dict(none_keys, course="C3")}

    def latencies():
        lat_all, paths = {}, {}
        for name, f in shapes.items():
            calls = []
            real = device_batch.retrieve_batch

            def spy(*a, **kw):
                out = real(*a, **kw)
                calls.append(out is not None)
                return out
            device_batch.retrieve_batch = spy
            try:
                for i in range(3):                             # batch-1 shapes: first-call setup
                    retr.retrieve(question=qs[-1 - i], filters=f, top_k=K)
                lat = []
                lprof = None
                if os.environ.get("CM_E2E_PROFILE_LAT"):       # host-side profile of the single-query calls
                    import cProfile
                    lprof = cProfile.Profile()
                    lprof.enable()
                for i in range(args.e2e_latency_queries):
                    t1 = time.perf_counter()
                    retr.retrieve(question=qs[i], filters=f, top_k=K)
                    lat.append((time.perf_counter() - t1) * 1e3)
                if lprof is not None:
                    import pstats
                    lprof.disable()
                    print(f"---- host profile, retrieve() {name}", file=sys.stderr)
                    pstats.Stats(lprof, stream=sys.stderr).sort_stats("tottime").print_stats(25)
            finally:
                device_batch.retrieve_batch = real
            lat.sort()
            lat_all[name] = {"p50": lat[len(lat) // 2], "p99": lat[min(len(lat) - 1, int(len(lat) * 0.99))],
                             "n": len(lat), "filters": f}
            paths[name] = "device chain" if calls and all(calls) else "host (per-stage dicts)"
            log(f"retrieve() {name}: p50 {lat_all[name]['p50']:.2f} ms, p99 {lat_all[name]['p99']:.2f} ms ({paths[name]})")
        return lat_all, paths

    lat, paths = latencies()
    construct = construct_leg(args, vs, bm, embedder, qs, K, dev, none_keys, lat) if args.e2e_construct else None
    lat_same = None
    if args.e2e_ab_same_stream:       # A/B: BM25 on the main stream behind the dense search (the old schedule)
        os.environ["CLASSMATE_BM25_SAME_STREAM"] = "1"
        try:
            log("A/B: BM25 on the main stream")
            lat_same, _ = latencies()
        finally:
            del os.environ["CLASSMATE_BM25_SAME_STREAM"]
    qps = B * args.steps / elapsed
    log(f"{args.steps} retrieve_batch calls in {elapsed:.3f}s -> {qps:.1f} q/s")
    out = {
        "metric": f"drop-in HybridRetriever.retrieve_batch queries/sec (strings -> result dicts), {N} chunks",
        "value": qps, "unit": "queries/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "fp32 E5 + int8/f16/f64 dense + f64 BM25",
        "data": "synthetic (seeded): Zipf-word chunks, random unit embeddings, random-init E5-base weights",
        "config": {"workload": "drop-in retrieve_batch (E5 query encode + cosine pool 24 + MMR 8 + BM25 8 + RRF)",
                   "chunks": N, "words_per_chunk": args.e2e_words, "global_batch": B, "top_k": K, "dim": D},
        "retrieve_latency_ms": lat["unfiltered"],
        "retrieve_latency_ms_by_filter": lat,
        "retrieve_latency_ms_bm25_same_stream": lat_same,
        "retrieve_batch_env_ab_qps": ab_env or None,
        "construct_then_retrieve": construct,
        "retrieve_paths": paths,
        "results_returned": n_res, "setup_s": time.perf_counter() - t_setup,
        "retrieve_batch_path": ("device-resident (retrieval/device_batch.py)"
                                if os.environ.get("CM_RETRIEVE_DEVICE", "1") != "0" and device_batch.applicable(retr, {}, True)
                                else "host (per-stage dicts)"),
    }
    line = json.dumps(out)
    print(line, flush=True)
    if args.out:
        Path(args.out).write_text(line + "\n")


def construct_leg(args, vs, bm, embedder, qs, K, dev, none_keys, lat):
    """ask_question's real call pattern (rag/pipeline/rag.py:531-554): per question, construct
    ChromaVectorStore.from_config(), BM25Store.load_or_create(...), E5MultilingualEmbedder(...) and
    CachingEmbedder(...), a HybridRetriever over them, then retrieve(filters=to_dict()).  The stores
    are persisted first (vectors + log + snapshot; BM25 JSONL + sidecar), then opened cold in this
    process (timed: the first construction after start), and every later construction attaches to
    the resident state.  The random-init E5 stands in for the named checkpoint
    (share_as: no weights offline).  Reports p50 / p99 of the whole sequence beside the bare
    retrieve() p50 with the same filter."""
    import shutil
    import tempfile
    import threading
    import torch
    from classmate_hip.embeddings import CachingEmbedder, E5MultilingualEmbedder
    from classmate_hip.retrieval import bm25 as bm25_mod
    from classmate_hip.retrieval import vector_store as vs_mod
    from classmate_hip.retrieval.bm25 import BM25Store
    from classmate_hip.retrieval.fusion import HybridRetriever
    from classmate_hip.retrieval.vector_store import GpuVectorStore
    N, D = args.docs_per_gpu, args.dim
    root = Path(args.e2e_dir) if args.e2e_dir else Path(tempfile.mkdtemp(prefix="cm_e2e_", dir=os.environ.get("TMPDIR")))
    root.mkdir(parents=True, exist_ok=True)
    need = N * (D * 4 + 1600) * 1.2
    free = shutil.disk_usage(root).free
    if free < need:
        log(f"construct leg skipped: {free / 1e9:.1f} GB free under {root}, need ~{need / 1e9:.1f} GB")
        return {"skipped": f"{free / 1e9:.1f} GB free under {root}, need ~{need / 1e9:.1f} GB"}
    stop = threading.Event()

    def beat():                                       # progress while one long call runs
        t = time.perf_counter()
        while not stop.wait(45):
            log(f"construct leg: {time.perf_counter() - t:.0f}s")
    hb = threading.Thread(target=beat, daemon=True)
    hb.start()
    out = {"dir_free_gb": free / 1e9}
    try:
        t0 = time.perf_counter()
        vs.persist_dir, vs.collection_name = root / "chroma", "classmate_rag"
        vs.save()
        out["save_vector_store_s"] = time.perf_counter() - t0
        log(f"vector store saved ({out['save_vector_store_s']:.1f}s)")
        t0 = time.perf_counter()
        bm.index_dir = root / "bm25"
        bm.save()
        out["save_bm25_s"] = time.perf_counter() - t0
        log(f"bm25 store saved ({out['save_bm25_s']:.1f}s)")
        os.environ["CHROMA_PERSIST_DIRECTORY"] = str(root / "chroma")
        os.environ["CHROMA_COLLECTION_NAME"] = "classmate_rag"
        model = "intfloat/multilingual-e5-base"
        embedder.share_as(model)
        # cold open: nothing resident for these directories
        vs_mod.release_all()
        bm25_mod.release_all()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        v0 = GpuVectorStore.from_config()
        n_v = v0.count()
        torch.cuda.synchronize()
        out["cold_open_vector_store_s"] = time.perf_counter() - t0
        t0 = time.perf_counter()
        b0 = BM25Store.load_or_create(root / "bm25")
        b0._ensure_index()
        torch.cuda.synchronize()
        out["cold_open_bm25_s"] = time.perf_counter() - t0
        out["cold_open_s"] = out["cold_open_vector_store_s"] + out["cold_open_bm25_s"]
        log(f"cold open: vector store {out['cold_open_vector_store_s']:.1f}s ({n_v} rows), "
            f"bm25 {out['cold_open_bm25_s']:.1f}s ({len(b0._id_list)} docs)")
        cache_dir = root / "emb_cache"

        phase = {}

        def ask(q):
            t_a = time.perf_counter()
            v = GpuVectorStore.from_config()
            b = BM25Store.load_or_create(root / "bm25")
            base = E5MultilingualEmbedder(model_name=model, device=str(dev))
            emb = CachingEmbedder(base, cache_dir=str(cache_dir))
            r = HybridRetriever(vector_store=v, bm25_store=b, embedder=emb, k_vector=8, k_bm25=8, rrf_k=60,
                                weight_vector=1.0, weight_bm25=1.0)
            t_b = time.perf_counter()
            res = r.retrieve(question=q, filters=dict(none_keys), top_k=K)
            phase.update(construct_ms=(t_b - t_a) * 1e3, retrieve_ms=(time.perf_counter() - t_b) * 1e3)
            return res

        import gc
        gc_ms = []                                     # the tail's suspects: Python collections ...

        def gc_cb(ev, info, _t=[0.0]):
            if ev == "start":
                _t[0] = time.perf_counter()
            else:
                gc_ms.append((info.get("generation"), (time.perf_counter() - _t[0]) * 1e3))
        t0 = time.perf_counter()
        ask(qs[-10])                                   # the first question after the open: key map, filter columns
        torch.cuda.synchronize()
        out["first_retrieve_after_open_s"] = time.perf_counter() - t0
        log(f"first construct-then-retrieve after the cold open: {out['first_retrieve_after_open_s']:.2f}s")
        for i in range(2):
            ask(qs[-11 - i])
        torch.cuda.synchronize()
        ts, calls = [], []
        gc.callbacks.append(gc_cb)
        try:
            for i in range(args.e2e_latency_queries):
                n_gc = len(gc_ms)
                t1 = time.perf_counter()
                ask(qs[100 + i])                           # new questions: embedding-cache misses
                ts.append((time.perf_counter() - t1) * 1e3)
                calls.append(dict(ms=ts[-1], **phase, gc=[(g, round(m, 2)) for g, m in gc_ms[n_gc:]]))
        finally:
            gc.callbacks.remove(gc_cb)
        out["slowest_calls"] = sorted(calls, key=lambda c: -c["ms"])[:3]     # ... or the phase that grew
        ts.sort()
        out.update(p50_ms=ts[len(ts) // 2], p99_ms=ts[min(len(ts) - 1, int(len(ts) * 0.99))], n=len(ts),
                   bare_retrieve_p50_ms=lat["to_dict_default"]["p50"], filters="DocumentMetadata.to_dict() (None keys)",
                   sequence="from_config + load_or_create + E5(...) + CachingEmbedder + HybridRetriever + retrieve",
                   embedder="random-init E5-base registered under the model name (share_as; no weights offline)")
        out["overhead_vs_bare_ms"] = out["p50_ms"] - out["bare_retrieve_p50_ms"]
        log(f"construct-then-retrieve: p50 {out['p50_ms']:.2f} ms (bare retrieve {out['bare_retrieve_p50_ms']:.2f} ms), "
            f"p99 {out['p99_ms']:.2f} ms")
        # the tail's anatomy (a separate pass, so the introspection does not touch the timings above):
        # every collection's generation, duration, object count of the collected generations, largest
        # container in them and objects freed; then the same calls after gc.freeze() (the startup
        # objects moved to the permanent generation, as a serving process would do after warm-up)
        diag = []

        def gc_diag(ev, info, _s={}):
            if ev == "start":
                objs = [o for g in range(info["generation"] + 1) for o in gc.get_objects(g)]
                big = max(objs, key=lambda o: len(o) if isinstance(o, (list, dict, set, tuple)) else 0, default=None)
                _s["n"] = len(objs)
                _s["big"] = [type(big).__name__, len(big) if isinstance(big, (list, dict, set, tuple)) else 0]
                del objs, big
                _s["t"] = time.perf_counter()
            else:
                diag.append(dict(gen=info["generation"], ms=round((time.perf_counter() - _s["t"]) * 1e3, 2),
                                 objects=_s["n"], largest=_s["big"], collected=info["collected"]))
        gc.callbacks.append(gc_diag)
        try:
            for i in range(args.e2e_latency_queries):
                ask(qs[200 + i])
        finally:
            gc.callbacks.remove(gc_diag)
        out["gc_events"] = dict(n=len(diag), slowest=sorted(diag, key=lambda d: -d["ms"])[:4],
                                by_gen={g: sum(1 for d in diag if d["gen"] == g) for g in range(3)})
        gc.freeze()
        try:
            tf = []
            for i in range(args.e2e_latency_queries):
                t1 = time.perf_counter()
                ask(qs[300 + i])
                tf.append((time.perf_counter() - t1) * 1e3)
        finally:
            gc.unfreeze()
        tf.sort()
        out["after_gc_freeze"] = dict(p50_ms=tf[len(tf) // 2], p99_ms=tf[min(len(tf) - 1, int(len(tf) * 0.99))],
                                      n=len(tf), frozen_note="gc.freeze() after the warm-up (serving-process practice)")
        log(f"construct-then-retrieve gc: {out['gc_events']['n']} collections, slowest {out['gc_events']['slowest'][:2]}; "
            f"after gc.freeze(): p50 {out['after_gc_freeze']['p50_ms']:.2f} ms, p99 {out['after_gc_freeze']['p99_ms']:.2f} ms")
        del v0, b0
    finally:
        stop.set()
        if not args.e2e_dir:
            shutil.rmtree(root, ignore_errors=True)
    return out


def run_ingest(args, rank, ws, dev):
    """configs[2]: E5-base batch encode (forward in --e5-dtype + HIP mean-pool/L2), chunks/s."""
    import torch
    from classmate_hip import parallel
    from classmate_hip.embeddings import E5MultilingualEmbedder
    emb = E5MultilingualEmbedder.random_init(seed=0, device=str(dev), num_layers=args.e5_layers, dtype=args.e5_dtype)
    B, S = args.batch, args.seq_len
    g = torch.Generator(device="cuda").manual_seed(args.seed + rank)
    ids = torch.randint(5, 250002, (B, S), device=dev, generator=g)
    ids[:, 0] = 0
    ids[:, -1] = 2
    mask = torch.ones_like(ids)
    out = torch.empty((B, 768), dtype=torch.float32, device=dev)
    for _ in range(args.warmup):
        emb.encode_token_ids(ids, mask, out=out)
    torch.cuda.synchronize()
    if ws > 1:
        torch.distributed.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        emb.encode_token_ids(ids, mask, out=out)
    torch.cuda.synchronize()
    if ws > 1:
        torch.distributed.barrier()
    el = parallel.max_over_ranks(time.perf_counter() - t0, device=dev)
    flops_seq = args.e5_layers * (24 * S * 768 ** 2 + 4 * S * S * 768)
    val = B * ws * args.steps / el
    res = {"metric": "E5-base ingest encode chunks/sec (forward + HIP mean-pool/L2)", "value": val,
           "unit": "chunks/s", "n_gpus": ws, "steps": args.steps, "warmup": args.warmup,
           "ms_per_step": el / args.steps * 1e3, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
           "dtype": {"bfloat16": "bf16", "float32": "fp32"}[args.e5_dtype],
           "data": "synthetic token ids, random-init E5-base weights",
           "config": {"workload": "E5-base encode", "global_batch": B * ws, "seq_len": S,
                      "parallelism": f"replicas x{ws}"},
           "achieved_tflops": val * flops_seq / 1e12}
    if rank == 0:
        print(json.dumps(res), flush=True)
        if args.out:
            Path(args.out).write_text(json.dumps(res) + "\n")


if __name__ == "__main__":
    main()
