"""Reference point only (not used by the engine): torch.mm (hipBLASLt) bf16 timings for the
prefill GEMM shapes of the 8B backbone, to size the headroom of the hand-written GEMMs."""
import torch, time
shapes = {"qkv": (4096, 6144), "o_proj": (4096, 4096), "gate_up": (4096, 24576), "down": (12288, 4096)}
for M in (181, 2117):
    for name, (K, N) in shapes.items():
        x = torch.randn(M, K, dtype=torch.bfloat16, device="cuda")
        w = torch.randn(K, N, dtype=torch.bfloat16, device="cuda")
        for _ in range(3):
            y = x @ w
        torch.cuda.synchronize()
        n = 20
        t0 = time.perf_counter()
        for _ in range(n):
            y = x @ w
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / n
        print(f"M={M} {name} K={K} N={N}: {dt*1e6:.1f} us  {2*M*K*N/dt/1e12:.0f} TFLOP/s  {K*N*2/dt/1e12:.2f} TB/s(w)", flush=True)
