"""Probe (not a test): batch-1 E5 query encode latency on the device (the single retrieve() path's
encode_queries_dev, small-batch hipGraph), random-init E5-base weights."""
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO), str(REPO / "classmate-rag_amd")]
import torch  # noqa: E402
from classmate_hip.embeddings import E5MultilingualEmbedder  # noqa: E402

emb = E5MultilingualEmbedder.random_init(seed=0, device="cuda:0", num_layers=12, dtype="float32")
qs = ["what is the deadline for the cs101 project report", "explain the rrf fusion formula"]
for b in (1, 8):
    for _ in range(5):
        emb.encode_queries_dev(qs[:1] * b)
    torch.cuda.synchronize()
    ts = []
    for i in range(30):
        t0 = time.perf_counter()
        q = emb.encode_queries_dev([qs[i % 2]] * b)
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) * 1e3)
    ts.sort()
    print(f"E5 encode_queries_dev B={b}: p50 {ts[len(ts) // 2]:.3f} ms, min {ts[0]:.3f} ms", flush=True)
