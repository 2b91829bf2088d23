"""Per-layer phase timeline of the batch-4 persistent decode launch (csrc/pse4.hip), 8B shape.

Random-weight engine with MTTS_PSE_TRACE=1, B = 4, a prefilled synthetic prompt, teacher-forced
decode forwards; prints each event's time (us from the layer's start; median over the 256
workgroups, steady-state layers) and the decode forward wall time with the launch on / off."""
import ctypes
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from moss_tts_amd import _native as N  # noqa: E402

NAMES = ["start", "qkv in", "qkv done", "att done", "o in", "o done", "gu in", "gu r01", "act0 (+gu2)",
         "act1 (+dn0-7)", "act2 (+dn8-15)", "down done", "L qkv", "L o", "L gu", "L down",
         "A q in", "A chunks + kv in", "A merged"]
B = 4


def build(on, layers):
    from moss_tts_amd.engine import Engine, EngineConfig
    os.environ["MTTS_PSE4"] = "1" if on else "0"
    os.environ["MTTS_PSE_TRACE"] = "1"
    e = Engine(EngineConfig(layers=layers, max_batch=B, max_ctx=512, max_prefill_tokens=1024), 0)
    e.init_random(seed=0)
    return e


def run(e, T, steps):
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
    return float(np.median(ts[2:])) * 1e3


layers = int(sys.argv[1]) if len(sys.argv) > 1 else 8
T = int(sys.argv[2]) if len(sys.argv) > 2 else 181
eb = build(False, layers)
print(f"per-op launches: decode forward {run(eb, T, 8):.3f} ms ({layers} layers, B={B})")
eb.close()
e = build(True, layers)
assert e.pse4_active()
print(f"pse4: decode forward {run(e, T, 8):.3f} ms ({layers} layers, B={B})")
EV = 28
n = layers * EV * 256
buf = (ctypes.c_uint64 * n)()
N.check(N.load().mtts_pse_trace(e._h, buf, n), "trace")
tr = np.frombuffer(buf, np.uint64).reshape(layers, EV, 256).astype(np.float64)
att = [255 - 7 * u for u in range(32)]
plain = [c for c in range(256) if c not in att and c + 1 not in att]
for name, cus in (("plain CUs", plain), ("attention CUs", att)):
    print(f"--- {name}: us after the layer's start (median over CUs, median over layers 1..{layers - 1})")
    rows = []
    for l in range(1, layers):
        t0 = np.median(tr[l, 0, cus])
        rows.append([np.median(tr[l, ev, cus]) - t0 if (tr[l, ev, cus] > 0).all() else np.nan for ev in range(19)])
    med = np.nanmedian(np.array(rows), axis=0) / 100
    print(" | ".join(f"{NAMES[ev]} {med[ev]:.1f}" for ev in range(19) if np.isfinite(med[ev])))
per = [np.median(tr[l, 11] - tr[l - 1, 11]) / 100 for l in range(1, layers)]
print("layer period (down done -> down done, median over CUs) us:", np.round(per, 1))
