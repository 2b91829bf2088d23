"""Decode forward time of a random-weight 8B-shape engine at batch B and cache size max_ctx
(teacher-forced forwards after a T-token prefill; median of the timed steps).  For same-box A/B of
library builds (MTTS_LIB) on shapes the bench does not cover, e.g. a batch-32 step in the
engine's default 2,048-position cache.
  python scripts/decode_fwd_time.py B max_ctx [T] [layers]"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from moss_tts_amd.engine import Engine, EngineConfig  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
C = int(sys.argv[2]) if len(sys.argv) > 2 else 2048
T = int(sys.argv[3]) if len(sys.argv) > 3 else 181
L = int(sys.argv[4]) if len(sys.argv) > 4 else 36
steps = 10
e = Engine(EngineConfig(layers=L, max_batch=B, max_ctx=C, max_prefill_tokens=max(512, B * T)), 0)
e.init_random(seed=0)
rng = np.random.default_rng(0)
ids = torch.from_numpy(rng.integers(0, 1024, (B, T + steps, 33))).cuda()
mask = torch.ones(B, T + steps, dtype=torch.uint8, device="cuda")
e.forward(ids[:, :T], mask[:, :T], 0)
torch.cuda.synchronize()
ts = []
for s in range(steps):
    p = T + s
    t0 = time.perf_counter()
    e.forward(ids[:, p:p + 1], mask[:, :p + 1], p)
    torch.cuda.synchronize()
    ts.append(time.perf_counter() - t0)
print(f"lib {os.environ.get('MTTS_LIB', 'default')} B={B} max_ctx={C} T={T} layers={L}: "
      f"decode forward {np.median(ts[2:]) * 1e3:.3f} ms")
e.close()
