"""CPU: open time of a persisted BM25Store -- reference-style full JSONL parse vs the binary sidecar.

Both exclude the device upload (identical in both paths).  The full path includes mapping tokens to
term ids, which the device build needs; the sidecar path reads them memory-mapped.
  python tools/persist_bench.py --docs 200000
"""
import argparse
import shutil
import sys
import tempfile
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "classmate-rag_amd"))
from classmate_hip.retrieval import BM25Store  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--docs", type=int, default=200000)
    ap.add_argument("--len", type=int, default=120)
    a = ap.parse_args()
    rng = np.random.default_rng(0)
    letters = np.array(list("abcdefghijklmnopqrstuvwxyz"))
    vocab = ["".join(rng.choice(letters, size=int(rng.integers(4, 10)))) for _ in range(50000)]
    d = Path(tempfile.mkdtemp())
    s = BM25Store(index_dir=d)
    z = np.minimum(rng.zipf(1.1, size=(a.docs, a.len)), len(vocab)) - 1
    texts = [" ".join(vocab[t] for t in row) for row in z]
    metas = [{"language": "en", "course": f"c{i % 7}"} for i in range(a.docs)]
    t0 = time.perf_counter()
    s.upsert_many(ids=[f"d{i}" for i in range(a.docs)], texts=texts, metadatas=metas)
    s.save()
    t_save = time.perf_counter() - t0
    size = (d / "bm25_index.jsonl").stat().st_size

    t0 = time.perf_counter()
    fast = BM25Store.load_or_create(d)
    t_side = time.perf_counter() - t0
    assert fast._csr is not None
    shutil.rmtree(d / "bm25_index.jsonl.cm")
    t0 = time.perf_counter()
    slow = BM25Store.load_or_create(d)
    for e in slow._entries.values():  # the term-id mapping the device build needs
        e.term_ids = slow._term_ids(e.tokens)
    t_full = time.perf_counter() - t0
    print(f"docs={a.docs} jsonl_MB={size / 2**20:.1f} upsert+save_s={t_save:.2f} "
          f"open_full_parse_s={t_full:.3f} open_sidecar_s={t_side:.3f} speedup={t_full / t_side:.0f}x")
    shutil.rmtree(d)


if __name__ == "__main__":
    main()
