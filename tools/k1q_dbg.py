"""GPU debug probe (not a test): K1q on a small store, prints from a -DK1Q_PRINT variant library."""
import sys
from pathlib import Path
REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO), str(REPO / "classmate-rag_amd")]
import numpy as np
import torch
from classmate_hip import engine
rng = np.random.default_rng(1)
C = rng.standard_normal((200_000, 768)).astype(np.float32)
C /= np.linalg.norm(C, axis=1, keepdims=True)
idx = engine.DenseIndex(768, capacity=C.shape[0])
idx.upsert(C, np.arange(C.shape[0], dtype=np.int64))
Q = rng.standard_normal((256, 768)).astype(np.float32)
idx.set_path(5)
d, r = idx.search(Q, 24)
torch.cuda.synchronize()
print("fallbacks", idx.last_fallbacks(), flush=True)
