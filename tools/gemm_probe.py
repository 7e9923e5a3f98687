"""E5 query-encode GEMM shapes at the bench batch (256 x 24 tokens): TF/s per shape (not a test).
Run with PYTORCH_TUNABLEOP_* to compare hipBLASLt's default pick with a tuned one."""
import os
import torch
import torch.nn.functional as F

M = int(os.environ.get("GEMM_M", 6144))
shapes = [("qkv", 768, 2304), ("out", 768, 768), ("ffn_up", 768, 3072), ("ffn_down", 3072, 768)]
tot = 0.0
for name, k, n in shapes:
    x = torch.randn(M, k, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(n, k, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(n, device="cuda", dtype=torch.bfloat16)
    for _ in range(5):
        F.linear(x, w, b)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 50
    e0.record()
    for _ in range(reps):
        F.linear(x, w, b)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    tot += ms
    print(f"{name:9s} M={M} K={k} N={n}: {ms*1e3:7.1f} us  {2*M*k*n/ms/1e9:7.1f} TF/s", flush=True)
print(f"per layer {tot*1e3:.1f} us, x12 = {tot*12:.3f} ms", flush=True)
