"""Batch-1 decode forward time (36 layers + heads, teacher-forced) of the persistent streaming
launch (pse.hip) against the per-op launches over the context length: where PSE stops paying."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def build(pse, max_ctx):
    from moss_tts_amd.engine import Engine, EngineConfig
    os.environ["MTTS_PSE"] = "1" if pse else "0"
    os.environ.setdefault("MTTS_PSE_CTX", "1000000")  # the kernel at every length (no gate)
    e = Engine(EngineConfig(max_batch=1, max_ctx=max_ctx, max_prefill_tokens=2048), 0)
    e.init_random(seed=0)
    return e


def run(e, T, steps=6):
    rng = np.random.default_rng(0)
    ids = torch.from_numpy(rng.integers(0, 1024, (1, T + steps, 33))).cuda()
    mask = torch.ones(1, T + steps, dtype=torch.uint8, device="cuda")
    e.forward(ids[:, :T], mask[:, :T], 0)
    torch.cuda.synchronize()
    ts = []
    for s in range(steps):
        p = T + s
        t0 = time.perf_counter()
        e.forward(ids[:, p:p + 1], mask[:, :p + 1], p)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts[1:])) * 1e3


Ts = [int(t) for t in (sys.argv[1] if len(sys.argv) > 1 else "200,400,600,800,1200,1600,2400,4000").split(",")]
mc = max(Ts) + 64
res = {}
for pse in (False, True):
    e = build(pse, mc)
    res[pse] = [run(e, T) for T in Ts]
    e.close()
for T, a, b in zip(Ts, res[False], res[True]):
    print(f"T={T:5d} per-op {a:.3f} ms  pse {b:.3f} ms  ratio {b / a:.3f}", flush=True)
