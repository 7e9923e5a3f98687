"""Ablation/profiling probe for the BM25 kernels at the bench's 10M shape (not a test).

python tools/bm25_probe.py [--docs N] [--batch B] [--reps R]
Env CM_BM25_DEBUG=1 (skip scoring) / 2 (skip range top-k) for ablations.
"""
import argparse
import os
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO), str(REPO / "classmate-rag_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from bench import gen_tokens, sample_query_terms  # noqa: E402
from classmate_hip import engine  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--docs", type=int, default=10_000_000)
ap.add_argument("--batch", type=int, default=256)
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--head-frac", type=float, default=1.0 / 128)
ap.add_argument("--head-bytes", type=int, default=8 << 30)
ap.add_argument("--paths", default="1,2", help="search strategies to time (1 full K2 scan, 2 pruned)")
ap.add_argument("--dbg", default="", help="comma list of CM_BM25_DEBUG values to sweep (ablation builds only)")
a = ap.parse_args()
tok, off = gen_tokens(a.docs, 1 << 20, 1.07, 120.0, seed=1500)
b = engine.BM25Index()
b.build_dev(tok, off, 1 << 20)
b.set_head_policy(a.head_frac, a.head_bytes)
qt = sample_query_terms(tok, off, a.batch, 8, seed=10)
q_terms = qt.reshape(-1).contiguous()
q_off = (torch.arange(a.batch + 1, device="cuda", dtype=torch.int32) * 8).contiguous()
df, _ = b.term_stats()
qh = qt.cpu().numpy()
qdf = df[qh].astype("int64")                                  # (B, 8)
head = qdf > a.docs * a.head_frac
print(f"workload: mean head terms/query {head.sum(1).mean():.2f}, mean head df sum/query {(qdf * head).sum(1).mean():.4g}, "
      f"mean tail df sum/query {(qdf * ~head).sum(1).mean():.4g}, distinct head terms in batch "
      f"{len(set(qh[head].tolist()))}, head tiles {b.num_head_terms}", flush=True)
ref = None
runs = [(int(p), None) for p in a.paths.split(",")]
if a.dbg:
    runs = [(int(a.paths.split(",")[-1]), d) for d in a.dbg.split(",")]
for path, dbgv in runs:
    if dbgv is not None:
        os.environ["CM_BM25_DEBUG"] = dbgv
    b.set_path(path)
    ws = torch.empty(b.workspace_bytes(a.batch, q_terms.numel(), 10), dtype=torch.uint8, device="cuda")
    out = b.search_dev(q_terms, q_off, 10, workspace=ws)
    torch.cuda.synchronize()
    ts = []
    b.timing(True)
    for _ in range(a.reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        b.search_dev(q_terms, q_off, 10, out=out, workspace=ws)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    kt = b.timing_drain()
    b.timing(False)
    res = (out[0].cpu(), out[1].cpu())
    same = "" if ref is None else f" identical_to_path{ref[2]}={bool(torch.equal(ref[0], res[0]) and torch.equal(ref[1], res[1]))}"
    if ref is None:
        ref = (res[0], res[1], path)
    nr = (a.docs + 1023) // 1024
    resc = b.workspace_rescored(a.batch, q_terms.numel(), 10, ws)
    if path == 2 and os.environ.get("BM25_ITEMS"):
        # K2b work: mirror bm_ws_layout (cm_bm25.hip) to read the planned items (diagnostic only)
        ru = lambda x: (x + 255) // 256 * 256
        nq, tt, k = a.batch, q_terms.numel(), 10
        off = ru(nq * 8) + ru(128 * 16 * 8) + ru(tt * 8) + ru(tt * (nr + 1) * 8) + ru(nq * nr * k * 8) + ru(nq * nr * k * 4)
        off_need = off
        off += ru(((nq + 3) // 4) * nr)
        off_items = off
        off += ru(nq * nr * 8)
        n_items = int(ws[off:off + 4].view(torch.int32).item())
        items = ws[off_items:off_items + 8 * n_items].view(torch.int64).cpu().numpy()
        masks = (items & 0xffff).astype(np.uint64)
        nblk = int(sum(bin(int(m)).count("1") for m in masks))
        need = ws[off_need:off_need + ((nq + 3) // 4) * nr].cpu().numpy()
        print(f"K2b items={n_items} blocks={nblk} ({nblk * 64} docs scored); K2 need pairs="
              f"{int(sum(bin(int(x)).count('1') for x in need))}", flush=True)
    print(f"docs={a.docs} B={a.batch} head_terms={b.num_head_terms} path={path} dbg={os.environ.get('CM_BM25_DEBUG', '0')} "
          f"search_ms={sorted(ts)[len(ts) // 2]:.3f} kernel_ms={sorted(kt)[len(kt) // 2]:.3f} rescored={resc}/{a.batch * nr}{same} "
          f"all={['%.2f' % t for t in ts]}", flush=True)
