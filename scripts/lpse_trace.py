"""Per-layer phase timeline of the MossTTSLocal persistent channel launch (csrc/lpse.hip).

MossTTSLocal-1.7B shape (depth stage exactly, a 2-layer backbone), random weights, B = 8,
MTTS_PSE_TRACE=1: a few greedy frames, then the stamps of the last channel launch; prints each
event's time (us from the layer's q|k|v input being ready; median over the CUs that stamp it) per
depth layer, and the frame time with the launch on / off (MTTS_LPSE)."""
import ctypes
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from moss_tts_amd import _native as N  # noqa: E402

NAMES = {0: "qkv input ready", 1: "normed", 2: "qkv done", 3: "att start", 4: "att done", 5: "o input in",
         6: "o done", 7: "gu input normed", 8: "gu r0 done", 9: "gu r1 done", 10: "gu r2 done",
         11: "gu r3 done (residual CUs)", 15: "down r3 in", 12: "down r0 in", 13: "down r1 in", 14: "down r2 in",
         16: "down done"}
B, EV = 8, 28


def build(on):
    from moss_tts_amd.engine import Engine, EngineConfig
    os.environ["MTTS_LPSE"] = "1" if on else "0"
    os.environ["MTTS_PSE_TRACE"] = "1"
    e = Engine(EngineConfig(hidden=2048, layers=2, n_heads=16, n_kv=8, head_dim=128, inter=6144, n_vq=32,
                            max_batch=B, max_ctx=256, max_prefill_tokens=1024, model_kind=1, local_hidden=1536,
                            local_layers=4, local_inter=8960, local_mlp_ffn=2048), 0)
    e.init_random(seed=0)
    return e


def frame_ms(e, frames=6):
    rng = np.random.default_rng(0)
    ids = np.full((B, 40, 33), 1024, np.int64)
    ids[..., 0] = rng.integers(200, 20000, (B, 40))
    ids[:, -1, 0] = 151652
    ids_d = torch.from_numpy(ids).cuda()
    e.local_generate_ids(ids_d, None, 2)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e.local_generate_ids(ids_d, None, frames + 1)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    e.local_generate_ids(ids_d, None, 1)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    return ((t1 - t0) - (t2 - t1)) / frames * 1e3


for on in (False, True):
    e = build(on)
    if on and not e.lpse_active():
        raise SystemExit("persistent channel launch unsupported")
    print(f"lpse={int(on)}: {frame_ms(e):.3f} ms per frame (2-layer backbone, B={B})")
    if on:
        LL = 4
        n = LL * EV * 256
        buf = (ctypes.c_uint64 * n)()
        N.check(N.load().mtts_pse_trace(e._h, buf, n), "trace")
        tr = np.frombuffer(buf, np.uint64).reshape(LL, EV, 256).astype(np.float64)
        for l in range(LL):
            t0 = tr[l, 0]
            row = []
            for ev, name in NAMES.items():
                v = tr[l, ev]
                ok = (v > 0) & (t0 > 0)
                if ok.sum() == 0:
                    continue
                row.append(f"{name} {np.median((v[ok] - t0[ok])) / 100:.1f}")
            print(f"layer {l}: " + " | ".join(row))
        print("layer periods (input ready -> next layer's input ready), us:",
              [round(float(np.median(tr[l + 1, 0] - tr[l, 0])) / 100, 1) for l in range(LL - 1)])
    e.close()
