"""Timing probe for K10 (split-precision f16x3 linear) vs torch fp32 / bf16 GEMMs at the E5
shapes, and the E5 query encode (graph replay) in each precision mode (not a test)."""
import os
import sys
from pathlib import Path
REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO), str(REPO / "classmate-rag_amd")]
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402
from classmate_hip import engine  # noqa: E402

M = int(os.environ.get("K10_M", "6144"))


def timeit(fn, reps=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


tot = {"k10": 0.0, "f32": 0.0, "bf16": 0.0}
ONLY = os.environ.get("K10_ONLY")
for name, K, N, gelu in (("qkv", 768, 2304, False), ("o", 768, 768, False), ("up", 768, 3072, True),
                         ("down", 3072, 768, False)):
    if ONLY and name != ONLY:
        continue
    x = torch.randn(M, K, device="cuda")
    w = 0.02 * torch.randn(N, K, device="cuda")
    b = 0.1 * torch.randn(N, device="cuda")
    W = engine.F16x3Weight(w, b)
    out = torch.empty(M, N, device="cuda")
    xb, wb, bb = x.bfloat16(), w.bfloat16(), b.bfloat16()
    xp = engine.split_rows(x, 1.0)          # the producers emit planes: time the GEMM alone
    if gelu:
        t_k10 = timeit(lambda: engine.linear_f16x3(xp, W, gelu=True, planes_out=1.0))
    else:
        t_k10 = timeit(lambda: engine.linear_f16x3(xp, W, out=out))
    if ONLY:
        print(f"{name}: K10 {t_k10 * 1e3:.1f} us", flush=True)
        continue
    t_f32 = timeit(lambda: F.linear(x, w, b))
    t_b16 = timeit(lambda: F.linear(xb, wb, bb))
    fl = 2.0 * M * K * N
    tot["k10"] += t_k10
    tot["f32"] += t_f32
    tot["bf16"] += t_b16
    print(f"{name:5s} M={M} K={K} N={N}: K10 {t_k10 * 1e3:7.1f} us ({3 * fl / t_k10 / 1e9:6.0f} TF/s f16 issued, "
          f"{fl / t_k10 / 1e9:5.0f} TF/s fp32-equiv) | torch fp32 {t_f32 * 1e3:7.1f} us ({fl / t_f32 / 1e9:5.0f}) | "
          f"bf16 {t_b16 * 1e3:6.1f} us ({fl / t_b16 / 1e9:5.0f})", flush=True)
print(f"per layer: K10 {tot['k10'] * 1e3:.1f} us, fp32 {tot['f32'] * 1e3:.1f} us, bf16 {tot['bf16'] * 1e3:.1f} us",
      flush=True)

if os.environ.get("K10_E5", "1") == "1":
    from classmate_hip.embeddings import E5MultilingualEmbedder
    B, S = 256, 24
    g = torch.Generator(device="cuda").manual_seed(13)
    ids = torch.randint(5, 250002, (B, S), device="cuda", generator=g)
    for label, dt, env in (("fp32 K10", "float32", "1"), ("fp32 hipBLASLt", "float32", "0"), ("bf16", "bfloat16", "1")):
        os.environ["CM_E5_F16X3"] = env
        emb = E5MultilingualEmbedder.random_init(seed=0, device="cuda", dtype=dt)
        gi, gm, go, gr = emb.capture_graph(B, S, unpadded=True)
        gi.copy_(ids)
        print(f"E5 query encode B={B} S={S} {label}: {timeit(gr.replay, 20):.3f} ms", flush=True)
        del emb, gr
        torch.cuda.empty_cache()
