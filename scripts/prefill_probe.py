#!/usr/bin/env python3
"""Time generate_begin (prefill + step-0 sampling) at the 8B shape for a few prompt shapes."""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from moss_tts_amd import _native as N  # noqa: E402
from moss_tts_amd.engine import Engine, EngineConfig, sampling_params  # noqa: E402

shapes = [(1, 181), (1, 512), (4, 181), (32, 181), (1, 2048)]
if os.environ.get("PREFILL_SHAPES"):  # e.g. "1x181,4x181"
    shapes = [tuple(int(v) for v in t.split("x")) for t in os.environ["PREFILL_SHAPES"].split(",")]
# PREFILL_MAXCTX / PREFILL_CHUNK: the TTSD long form (e.g. 9,700 / 1,024: position-chunked prefill)
e = Engine(EngineConfig(max_batch=32, max_ctx=int(os.environ.get("PREFILL_MAXCTX", 2304)),
                        max_prefill_tokens=int(os.environ.get("PREFILL_CHUNK", 8192))), 0)
e.init_random(0)
sp = sampling_params(text_temperature=0, audio_temperature=0)
rng = np.random.default_rng(0)
for B, T in shapes:
    ids = torch.from_numpy(rng.integers(0, 1024, (B, T, 33))).cuda()
    ids[..., 0] = 151654
    mask = torch.ones(B, T, dtype=torch.uint8, device="cuda")
    ts = []
    for _ in range(4):
        torch.cuda.synchronize()
        a = time.perf_counter()
        N.check(N.load().mtts_generate_begin(e._h, ctypes.c_void_p(ids.data_ptr()), ctypes.c_void_p(mask.data_ptr()),
                                             B, T, 8, ctypes.byref(sp), None, None), "begin")
        N.check(N.load().mtts_generate_poll(e._h, None, None, None), "poll")
        ts.append((time.perf_counter() - a) * 1e3)
    print(f"B={B} T={T}: prefill {np.median(ts[1:]):.2f} ms ({B * T / np.median(ts[1:]) * 1e3:.0f} tok/s)", flush=True)
