#!/usr/bin/env python3
"""Per-launch time of each decode projection at one batch size, in isolation (the decode step's
own GEMV instances via mtts_engine_time_gemv: layers rotated, HIP events), 8B shape.
    python3 scripts/gemv_probe.py 32        # env knobs (MTTS_NW, MTTS_U, ...) apply"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from moss_tts_amd.engine import Engine, EngineConfig
    from moss_tts_amd import _native as N
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    eng = Engine(EngineConfig(max_batch=max(B, 1), max_ctx=512), 0)
    eng.init_random(0)
    out = []
    for which, name in enumerate(["qkv", "o", "gu", "down", "heads"]):
        ms, nb = ctypes.c_float(), ctypes.c_uint64()
        N.check(N.load().mtts_engine_time_gemv(eng._h, which, 0, B, 30, ctypes.byref(ms), ctypes.byref(nb)), "time")
        out.append(f"{name} {ms.value * 1e3:.2f}us {nb.value / ms.value / 1e9:.2f}TB/s")
    torch.cuda.synchronize()
    print(f"B={B} " + " | ".join(out), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
