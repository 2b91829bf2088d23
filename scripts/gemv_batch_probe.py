#!/usr/bin/env python3
"""Per-matrix GEMV timing vs batch rows (HIP events, back-to-back launches on layer 0)."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from moss_tts_amd import _native as N  # noqa: E402
from moss_tts_amd.engine import Engine, EngineConfig  # noqa: E402

e = Engine(EngineConfig(layers=8, max_batch=32, max_ctx=512, max_prefill_tokens=512), 0)
e.init_random(0)
names = ["qkv", "o", "gu", "down", "heads"]
for B in [int(x) for x in (sys.argv[1:] or ["1", "4", "16", "17", "32"])]:
    row = []
    for w in range(5):
        ms, nb = ctypes.c_float(), ctypes.c_uint64()
        N.check(N.load().mtts_engine_time_gemv(e._h, w, 0, B, 20, ctypes.byref(ms), ctypes.byref(nb)), "t")
        row.append(f"{names[w]} {ms.value * 1e3:7.1f}us {nb.value / ms.value / 1e6:6.0f}GB/s")
    print(f"B={B:2d}: " + " | ".join(row), flush=True)
