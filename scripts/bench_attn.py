#!/usr/bin/env python3
"""Micro-timing of the decode attention kernel (back-to-back launches, HIP events).
Usage: bench_attn.py [pos ...]; MTTS_ATTN_PROBE selects a truncated variant (see kernels.h)."""
import ctypes
import os
import subprocess
import sys

if len(sys.argv) > 1 and sys.argv[1] == "--child":
    import torch
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from moss_tts_amd import _native as N
    L = N.load()
    B, Hq, Hkv, D, Cmax = int(sys.argv[3]), 32, 8, 128, int(os.environ.get("CMAX", "4096"))
    pos = int(sys.argv[2])
    P = lambda t: ctypes.c_void_p(t.data_ptr())
    qkv = torch.randn(B, (Hq + 2 * Hkv) * D, device="cuda").bfloat16()
    qn = torch.ones(D, device="cuda").bfloat16()
    cs = torch.randn(Cmax, D, device="cuda").bfloat16()
    kc = torch.randn(B, Hkv, Cmax, D, device="cuda").bfloat16()
    vc = torch.randn(B, Hkv, D, Cmax, device="cuda").bfloat16()
    mask = torch.ones(B, Cmax, dtype=torch.uint8, device="cuda")
    posd = torch.tensor([pos], dtype=torch.int32, device="cuda")
    out = torch.zeros(B, Hq * D, device="cuda").bfloat16()
    ws = torch.zeros(L.mtts_k_attn_decode_ws_bytes(B, Hq, Hkv, D, Cmax), dtype=torch.uint8, device="cuda")
    args = [P(qkv), P(qn), P(qn), P(cs), P(cs), P(kc), P(vc), P(mask), P(posd), P(out), P(ws), B, Hq, Hkv, D, Cmax,
            ctypes.c_float(1e-6), None]
    for _ in range(20):
        N.call("mtts_k_attn_decode", *args)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = 500
    e0.record()
    for _ in range(n):
        L.mtts_k_attn_decode(*args)
    e1.record()
    torch.cuda.synchronize()
    print(f"nwv={os.environ.get('MTTS_ATTN_NWV', '4')} probe={os.environ.get('MTTS_ATTN_PROBE', '0')} pos={pos} B={B}: {e0.elapsed_time(e1) / n * 1000:.2f} us/launch")
    sys.exit(0)

for pos in [int(x) for x in sys.argv[1:]] or [100, 389, 1000, 3000]:
  for nwv in os.environ.get("NWVS", "4,8,16").split(","):
    for B in [int(b) for b in os.environ.get("BS", "1,4").split(",")]:
        for probe in os.environ.get("PROBES", "3,0").split(","):
            env = dict(os.environ, MTTS_ATTN_PROBE=probe, MTTS_ATTN_NWV=nwv)
            r = subprocess.run([sys.executable, __file__, "--child", str(pos), str(B)], env=env, capture_output=True,
                               text=True, timeout=300)
            print(r.stdout.strip() or r.stderr[-500:], flush=True)
