"""Timing probe for the E5 query encode variants at the bench shape (not a test)."""
import sys
from pathlib import Path
REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO), str(REPO / "classmate-rag_amd")]
import torch  # noqa: E402
from classmate_hip.embeddings import E5MultilingualEmbedder  # noqa: E402

B, S = 256, 24
import os  # noqa: E402
emb = E5MultilingualEmbedder.random_init(seed=0, device="cuda", dtype=os.environ.get("E5_DTYPE", "bfloat16"))
g = torch.Generator(device="cuda").manual_seed(13)
ids = torch.randint(5, 250002, (B, S), device="cuda", generator=g)
mask = torch.ones_like(ids)


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


print("eager", round(timeit(lambda: emb.encode_token_ids(ids, mask)), 3), "ms", flush=True)
for unp in (False, True):
    gi, gm, go, gr = emb.capture_graph(B, S, unpadded=unp)
    gi.copy_(ids)
    gm.copy_(mask)
    print("graph unpadded=%s" % unp, round(timeit(gr.replay), 3), "ms", flush=True)
with torch.backends.cuda.sdp_kernel(enable_math=False):
    try:
        gi, gm, go, gr = emb.capture_graph(B, S, unpadded=True)
        gi.copy_(ids)
        print("graph unpadded, math off", round(timeit(gr.replay), 3), "ms", flush=True)
    except Exception as ex:  # noqa: BLE001
        print("graph unpadded, math off: failed", type(ex).__name__, str(ex)[:200])
