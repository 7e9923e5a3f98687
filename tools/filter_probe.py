"""GPU: where-filter cost at N rows -- numpy mask + pack_bits (host) vs cm_filter_eval (device).

Metadata: 6 simple fields with a few values each, tags; where = the reference ask pipeline's
BM25 filter (to_dict() with None keys, quirk Q4) and a Chroma $and of two equalities.
  python tools/filter_probe.py --rows 10000000
"""
import argparse
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "classmate-rag_amd"))
import torch  # noqa: E402
from classmate_hip import engine  # noqa: E402
from classmate_hip.retrieval import filters as F  # noqa: E402


def bulk_meta(n, rng):
    mi = F.MetaIndex()
    mi._ensure(n)
    vals = {"course": 40, "unit": 12, "language": 2, "doc_type": 4, "author": 30, "semester": 6}
    for key, nv in vals.items():
        col = F._Column(mi._cap)
        for i in range(nv):
            col.py_map[f"{key}{i}"] = i
            col.ty_map[F._typed(f"{key}{i}")] = i
        col.py_map[None] = nv
        col.ty_map[F._typed(None)] = nv
        codes = rng.integers(0, nv + 1, n).astype(np.int32)
        col.py[:n] = col.ty[:n] = codes
        mi.cols[key] = col
    mi.live[:n] = True
    mi.metas = [None] * n
    return mi


def timeit(fn, reps=7):
    fn()
    ts = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return 1e3 * float(np.median(ts))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=10_000_000)
    a = ap.parse_args()
    mi = bulk_meta(a.rows, np.random.default_rng(0))
    cases = {"bm25_q4": ("bm25", {"course": "course3", "unit": None, "author": None, "semester": None}),
             "chroma_and": ("chroma", {"$and": [{"course": "course3"}, {"language": "language1"}]})}
    for name, (sem, w) in cases.items():
        host_mask = (lambda: mi.bm25_mask(w)) if sem == "bm25" else (lambda: mi.chroma_mask(w))

        def host():
            m = host_mask()
            torch.from_numpy(F.pack_bits(m).view(np.int32)).to("cuda")
        prog = mi.bm25_program(w) if sem == "bm25" else mi.chroma_program(w)
        bits, cnt = engine.filter_bits(prog)
        assert np.array_equal(bits.cpu().numpy().view(np.uint32), F.pack_bits(host_mask()))
        t_host = timeit(host)
        t_dev = timeit(lambda: engine.filter_bits(mi.bm25_program(w) if sem == "bm25" else mi.chroma_program(w)))
        print(f"rows={a.rows} case={name} matches={cnt} host_mask_pack_upload_ms={t_host:.2f} "
              f"device_compile_eval_ms={t_dev:.3f} speedup={t_host / t_dev:.1f}x", flush=True)


if __name__ == "__main__":
    main()
