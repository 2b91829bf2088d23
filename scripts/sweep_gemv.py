#!/usr/bin/env python3
"""GEMV tuning sweep on the GPU: every decode matrix shape x waves-per-block x fused norm,
timed with HIP events (torch.cuda.Event on the current stream, which the kernel uses)."""
import ctypes
import json
import sys

import torch

sys.path.insert(0, ".")
from moss_tts_amd import _native as N

N.load()
P = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None
dev = "cuda"
shapes = {"qkv": (6144, 4096, 0), "o": (4096, 4096, 1), "gu": (12288, 4096, 2), "down": (4096, 12288, 1),
          "heads": (184736, 4096, 0)}
res = []
for B in [int(b) for b in (sys.argv[1:] or ["1"])]:
    for name, (Nr, K, epi) in shapes.items():
        rows = 2 * Nr if epi == 2 else Nr
        w = torch.randn(rows * K // 16 * 16, dtype=torch.bfloat16, device=dev) * 0.02
        packed = torch.empty(N.load().mtts_k_packed_bytes(rows, K) // 2, dtype=torch.bfloat16, device=dev)
        N.call("mtts_k_pack", P(w), P(packed), rows, K, 0, 0, 0, None)
        del w
        x = torch.randn(B, K, dtype=torch.bfloat16, device=dev)
        y = torch.empty(B, Nr, dtype=torch.bfloat16, device=dev)
        ss = torch.rand(B, K // 16, dtype=torch.float32, device=dev)
        nw = torch.ones(K, dtype=torch.bfloat16, device=dev)
        sso = torch.empty(B, Nr // 16, dtype=torch.float32, device=dev)
        for norm in ([0, 1] if epi != 1 else [0]):
            for nw_ in (4, 8, 16):
                def run():
                    N.call("mtts_k_gemv_ex", P(packed), P(x), K, P(y), Nr, P(y) if epi == 1 else None, Nr, B, Nr, K,
                           epi, P(ss) if norm else None, K // 16, K // 16, P(nw) if norm else None,
                           ctypes.c_float(1e-6), P(sso) if epi == 1 else None, Nr // 16, nw_,
                           ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
                for _ in range(3):
                    run()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                it = 20
                e0.record()
                for _ in range(it):
                    run()
                e1.record()
                torch.cuda.synchronize()
                us = e0.elapsed_time(e1) / it * 1e3
                gbs = rows * K * 2 / (us * 1e-6) / 1e9
                r = dict(B=B, m=name, norm=norm, nw=nw_, us=round(us, 2), GBs=round(gbs))
                res.append(r)
                print(json.dumps(r), flush=True)
        del packed
        torch.cuda.empty_cache()
