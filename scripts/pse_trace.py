"""Per-layer event timeline of the persistent streaming decode launch (csrc/pse.hip), 8B shape, B=1.

Builds a random-weight engine with MTTS_PSE=1 MTTS_PSE_TRACE=1, prefills a synthetic prompt,
runs teacher-forced decode forwards, and prints, for a few layers, each event's time (us from the
launch's first stamp; median / max over the 256 workgroups) -- consumer events 0-9, loader
events 10-14 (see pse.hip) -- and the decode forward wall time with and without PSE."""
import ctypes
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from moss_tts_amd import _native as N  # noqa: E402

NAMES = ["layer", "qkv in", "qkv done", "att done", "o in", "o done", "gu in", "gu done", "down in", "down done",
         "L qkv", "L o", "L gu", "L down", "L end", "A qkv in", "A chunks", "A chunks done", "A parts in"]


def build(pse, layers):
    from moss_tts_amd.engine import Engine, EngineConfig
    os.environ["MTTS_PSE"] = "1" if pse else "0"
    if os.environ.get("PSE_NO_TRACE") != "1":
        os.environ["MTTS_PSE_TRACE"] = "1"
    e = Engine(EngineConfig(layers=layers, max_batch=1, max_ctx=512, max_prefill_tokens=512), 0)
    e.init_random(seed=0)
    return e


def run(e, T, steps):
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
    return float(np.median(ts[2:])) * 1e3


layers = int(sys.argv[1]) if len(sys.argv) > 1 else 8
T = int(sys.argv[2]) if len(sys.argv) > 2 else 181
eb = build(False, layers)
print(f"per-op launches: decode forward {run(eb, T, 8):.3f} ms ({layers} layers)")
eb.close()
e = build(True, layers)
print(f"pse: decode forward {run(e, T, 8):.3f} ms ({layers} layers)")
if os.environ.get("PSE_NO_TRACE") == "1":
    sys.exit(0)
EV = 28
n = layers * EV * 256
buf = (ctypes.c_uint64 * n)()
N.check(N.load().mtts_pse_trace(e._h, buf, n), "trace")
tr = np.frombuffer(buf, np.uint64).reshape(layers, EV, 256).astype(np.float64)
T2 = os.environ.get("PSE_T2") == "1"  # a PSE_TRACE2 build: events 10-14 are the input-norm h gather's
if T2:
    NAMES[10:15] = ["G issued", "G polled", "G cbar", "G sweeps", "G first take"]
t0 = tr[0, 0][tr[0, 0] > 0].min() if T2 else tr[0, 10][tr[0, 10] > 0].min()
for l in list(range(min(layers, 4))) + [layers - 1]:
    row = []
    for ev in range(19):
        v = tr[l, ev]
        v = v[v > 0]
        if v.size:
            row.append(f"{NAMES[ev]} {np.median((v - t0) / 100):.1f}/{np.max((v - t0) / 100):.1f}")
    print(f"L{l}: " + " | ".join(row))
lay = []
for l in range(1, layers):
    a0, a1 = tr[l - 1, 9], tr[l, 9]
    lay.append(np.median(a1 - a0) / 100)
print("median layer period (down done -> down done) us:", np.round(lay, 1))
# per-phase table over the steady-state layers (1 .. L-1): each phase = the median over CUs of
# its closing event minus the median of its opening event, then the median over layers
PH = [("h gather + input norm", 0, 1), ("q|k|v stream + publish", 1, 2), ("attention chain (q|k|v done -> o input)", 2, 4),
      ("o_proj stream + publish", 4, 5), ("h gather + post norm", 5, 6), ("gate|up stream + publish", 6, 7),
      ("act gather", 7, 8), ("down stream + publish", 8, 9)]
med = lambda l, ev: np.median(tr[l, ev][tr[l, ev] > 0]) / 100
rows = []
for name, a0, a1 in PH:
    d = [med(l, a1) - med(l, a0) for l in range(1, layers)]
    rows.append((name, float(np.median(d))))
# the attention CUs' own view of the chain
att = [("A: q|k|v gather", 2, 15), ("A: chunks", 16, 17), ("A: unit merge + publish", 17, 3)]
for name, a0, a1 in att:
    d = []
    for l in range(1, layers):
        v0, v1 = tr[l, a0], tr[l, a1]
        ok = (v0 > 0) & (v1 > 0)
        if ok.any():
            d.append(np.median(v1[ok] - v0[ok]) / 100)
    if d:
        rows.append((name, float(np.median(d))))
if T2:
    # the input-norm h gather, per CU then the median over CUs and layers (us); 'after the last
    # producer' = against the latest down-done stamp of the previous layer
    def st(f):
        return float(np.median([np.median(f(l)) for l in range(1, layers)]))
    g = lambda l, ev: tr[l, ev] / 100
    print("h gather (input norm), median over CUs and layers:")
    print(f"  enter -> first sweep issued      {st(lambda l: g(l, 10) - g(l, 0)):.2f} us")
    print(f"  first sweep issued -> taken       {st(lambda l: g(l, 14) - g(l, 10)):.2f} us")
    print(f"  poll loop after the first sweep   {st(lambda l: g(l, 11) - g(l, 14)):.2f} us")
    print(f"  sweeps                             {st(lambda l: tr[l, 13]):.1f}")
    print(f"  consumer barrier                   {st(lambda l: g(l, 12) - g(l, 11)):.2f} us")
    print(f"  norm (+ barrier)                   {st(lambda l: g(l, 1) - g(l, 12)):.2f} us")
    print(f"  last producer's down done -> polled {st(lambda l: g(l, 11) - g(l - 1, 9).max()):.2f} us")
    print(f"  last producer's down done -> normed {st(lambda l: g(l, 1) - g(l - 1, 9).max()):.2f} us")
    print(f"  own down done -> gather enter      {st(lambda l: g(l, 0) - g(l - 1, 9)):.2f} us")
    a = lambda l, e0, e1: [v for v in (tr[l, e1] - tr[l, e0]) / 100 if abs(v) < 1e4 and v != 0]
    print("attention CUs (median):")
    for nm, e0, e1 in (("chunks done -> k/v gathered", 17, 18), ("k/v norm, RoPE, append, partials + barrier", 18, 19),
                       ("merge + publish + barrier + return", 19, 3)):
        print(f"  {nm:44s} {st(lambda l: np.array(a(l, e0, e1) or [np.nan])):.2f} us")
    for nm, e0, e1 in (("own q|k|v done -> attention entry", 2, 25), ("entry -> q sweep issued", 25, 20),
                       ("q sweep issued -> taken", 20, 24), ("q poll loop", 24, 21), ("q barrier", 21, 22)):
        print(f"  {nm:44s} {st(lambda l: np.array(a(l, e0, e1) or [np.nan])):.2f} us")
    print(f"  last att done -> o input (median CU)    {st(lambda l: np.array([np.median(g(l, 4)) - g(l, 3)[tr[l, 3] > 0].max()])):.2f} us")
    print(f"  last q|k|v done -> A q|k|v gathered     {st(lambda l: np.array([np.median(g(l, 15)[tr[l, 15] > 0]) - g(l, 2).max()])):.2f} us")
    print(f"  spread of down done over CUs (max - median) {st(lambda l: np.array([g(l - 1, 9).max() - np.median(g(l - 1, 9))])):.2f} us")
print("| phase (steady-state layer, median) | us |")
print("|---|---|")
for name, v in rows:
    print(f"| {name} | {v:.2f} |")
print(f"| layer period | {float(np.median(lay)):.2f} |")
# stragglers: per CU, how far behind the median each op's completion runs (steady-state layers),
# attention CUs (pse_att_unit: 255 - c = 7 u, u < 8 PSE_AU) marked
att = set(255 - 7 * u for u in range(int(os.environ.get("PSE_AU", "4")) * 8))  # pse_att_unit
for name, ev in (("o done", 5), ("gu done", 7), ("down done", 9)):
    lag = np.stack([tr[l, ev] - np.median(tr[l, ev]) for l in range(1, layers)]) / 100  # [layer, CU] us
    mean_lag = lag.mean(0)
    worst = np.argsort(-mean_lag)[:12]
    print(f"{name}: mean lag behind the median, worst CUs: " +
          ", ".join(f"{c}{'*' if c in att else ''}:{mean_lag[c]:.1f}" for c in worst) +
          f" | attention CUs mean {np.mean([mean_lag[c] for c in att]):.2f}, others {np.mean([mean_lag[c] for c in range(256) if c not in att]):.2f}"
          + f" | by XCD (c % 8): " + " ".join(f"{x}:{np.mean(mean_lag[x::8]):.2f}" for x in range(8)))
e.close()
