"""Timing / profiling probe for the dense K1 kernel at the bench shape (not a test).

python tools/dense_probe.py [--docs N] [--batch B] [--k K] [--reps R]
"""
import argparse
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO), str(REPO / "classmate-rag_amd")]
import torch  # noqa: E402
from bench import gen_dense  # noqa: E402
from classmate_hip import engine  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--docs", type=int, default=10_000_000)
ap.add_argument("--dim", type=int, default=768)
ap.add_argument("--batch", type=int, default=256)
ap.add_argument("--k", type=int, default=24)
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--path", type=int, default=0, help="0 auto, 1 f32, 2 f16x3, 3 coarse")
a = ap.parse_args()
d = engine.DenseIndex(a.dim, capacity=a.docs)
gen_dense(d, a.docs, a.dim, seed=7)
d.set_path(a.path)
g = torch.Generator(device="cuda").manual_seed(3)
q = torch.randn(a.batch, a.dim, device="cuda", generator=g)
out = d.search_dev(q, a.k)
torch.cuda.synchronize()
d.timing(True)
ts = []
for _ in range(a.reps):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    d.search_dev(q, a.k, out=out)
    e1.record()
    torch.cuda.synchronize()
    ts.append(e0.elapsed_time(e1))
ms = sorted(ts)[len(ts) // 2]
kt = d.timing_drain()
fb = d.workspace_fallbacks(a.batch, a.k, d._ws)
flops = 2.0 * a.batch * a.docs * a.dim
print(f"docs={a.docs} B={a.batch} k={a.k} kind={d.search_kind(a.batch, a.k)} search_ms={ms:.3f} "
      f"scan_kernel_ms={sorted(kt)[len(kt) // 2]:.3f} fallbacks={fb} TFLOP/s={flops / ms / 1e9:.1f} "
      f"all={['%.2f' % t for t in ts]}", flush=True)
