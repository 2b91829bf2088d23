"""Diagnose GEMV tail: tiny shapes through mtts_k_gemv vs fp32 torch, NaN / mismatch census."""
import ctypes, os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from moss_tts_amd import _native as N
lib = N.load()
P = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None
torch.manual_seed(0)
for (B, N_, K, epi) in [(3, 4100, 64, 0), (3, 4100, 64, 3), (1, 64, 64, 0), (3, 300, 96, 0), (4, 512, 1536, 0), (8, 4096, 1536, 0), (3, 64, 128, 1)]:
    w = (torch.randn(N_, K) * K ** -0.5).to(torch.bfloat16).cuda()
    x = torch.randn(B, K).to(torch.bfloat16).cuda()
    wp = torch.zeros(lib.mtts_k_packed_bytes(N_, K) // 2, dtype=torch.bfloat16, device="cuda")
    N.check(lib.mtts_k_pack(P(w), P(wp), N_, K, 0, 0, 0, None), "pack")
    y = torch.full((B, N_), float("nan"), dtype=torch.bfloat16, device="cuda")
    res = torch.zeros(B, N_, dtype=torch.bfloat16, device="cuda") if epi == 1 else None
    N.check(lib.mtts_k_gemv(P(wp), P(x), K, P(y), N_, P(res), N_, B, N_, K, epi, N_ + 1 if epi == 3 else 0, 1, 0, None), "gemv")
    torch.cuda.synchronize()
    ref = (x.float() @ w.float().T)
    nan = torch.isnan(y.float())
    err = (y.float() - ref).abs()[~nan]
    print(B, N_, K, epi, "nan", int(nan.sum()), "of", y.numel(), "first nan", nan.nonzero()[:3].tolist(), "maxerr", float(err.max()) if err.numel() else None, flush=True)
