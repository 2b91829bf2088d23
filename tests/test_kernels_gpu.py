"""Kernel-level parity: each HIP kernel (called through the C ABI) against the
numpy oracle on the same seeded inputs.  bf16 tolerance: results within the
bf16 rounding band of the oracle (different fp32 summation order)."""
import ctypes
import os

import numpy as np
import pytest

from oracle import bf16 as B16
from oracle import moss_delay as O
from oracle import prng

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def N():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from moss_tts_amd import _native
    _native.load()
    return _native


def dev_bf16(a):
    """float32 numpy (bf16-representable) -> torch bf16 cuda"""
    return torch.from_numpy(np.ascontiguousarray(a, np.float32)).to(torch.bfloat16).cuda()


def host(t):
    return t.float().cpu().numpy()


def P(t):
    return ctypes.c_void_p(t.data_ptr())


def within_band(got, want, ulps=1.0, scale=None):
    """|got - want| <= ulps * ulp_bf16(scale) element-wise (scale defaults to |want|)"""
    from tests.parity_util import ulp_bf16
    s = np.abs(want) if scale is None else scale
    return np.abs(got - want) <= ulps * ulp_bf16(s) + 1e-30


def rand_bf16(rng, shape, scale=1.0):
    return B16.rnd(rng.standard_normal(shape).astype(np.float32) * np.float32(scale))


@pytest.mark.parametrize("B,Nr,K", [(1, 48, 64), (5, 4100, 256), (16, 96, 4096), (17, 64, 128), (32, 1040, 512),
                                    (40, 48, 96)])
def test_gemv_store(N, B, Nr, K):
    rng = np.random.default_rng(B * 1000 + Nr + K)
    W = rand_bf16(rng, (Nr, K), K ** -0.5)
    x = rand_bf16(rng, (B, K))
    wd = dev_bf16(W)
    packed = torch.zeros(N.load().mtts_k_packed_bytes(Nr, K) // 2, dtype=torch.bfloat16, device="cuda")
    N.call("mtts_k_pack", P(wd), P(packed), Nr, K, 0, 0, 0, None)
    xd = dev_bf16(x)
    y = torch.zeros(B, Nr, dtype=torch.bfloat16, device="cuda")
    N.call("mtts_k_gemv", P(packed), P(xd), K, P(y), Nr, None, 0, B, Nr, K, 0, 0, 1, 0, None)
    torch.cuda.synchronize()
    want = O.linear(O._Ctx("bf16"), x, W)
    got = host(y)
    rowscale = np.abs(want).max(axis=1, keepdims=True)
    assert within_band(got, want, 1.0, scale=np.maximum(np.abs(want), rowscale / 4)).all(), np.abs(got - want).max()
    assert np.mean(got == want) > 0.9


def test_gemv_epilogues(N):
    rng = np.random.default_rng(5)
    ctx = O._Ctx("bf16")
    B, H, I = 3, 256, 96
    x = rand_bf16(rng, (B, H))
    Wg, Wu = rand_bf16(rng, (I, H), H ** -0.5), rand_bf16(rng, (I, H), H ** -0.5)
    packed = torch.zeros(N.load().mtts_k_packed_bytes(2 * I, H) // 2, dtype=torch.bfloat16, device="cuda")
    wgd, wud = dev_bf16(Wg), dev_bf16(Wu)
    N.call("mtts_k_pack", P(wgd), P(packed), I, H, 0, 1, 0, None)
    N.call("mtts_k_pack", P(wud), P(packed), I, H, 0, 1, 1, None)
    y = torch.zeros(B, I, dtype=torch.bfloat16, device="cuda")
    xd = dev_bf16(x)
    N.call("mtts_k_gemv", P(packed), P(xd), H, P(y), I, None, 0, B, I, H, 2, 0, 1, 0, None)
    torch.cuda.synchronize()
    g, u = O.linear(ctx, x, Wg), O.linear(ctx, x, Wu)
    want = ctx.r(ctx.r(O.silu(g)) * u)
    got = host(y)
    assert within_band(got, want, 2.0, scale=np.abs(want).max()).all()
    # residual add, in place
    Wo = rand_bf16(rng, (H, I), I ** -0.5)
    po = torch.zeros(N.load().mtts_k_packed_bytes(H, I) // 2, dtype=torch.bfloat16, device="cuda")
    wod = dev_bf16(Wo)
    N.call("mtts_k_pack", P(wod), P(po), H, I, 0, 0, 0, None)
    res = rand_bf16(rng, (B, H))
    hd = dev_bf16(res)
    N.call("mtts_k_gemv", P(po), P(y), I, P(hd), H, P(hd), H, B, H, I, 1, 0, 1, 0, None)
    torch.cuda.synchronize()
    want2 = ctx.r(res + O.linear(ctx, got, Wo))
    assert within_band(host(hd), want2, 1.0, scale=np.abs(want2).max()).all()
    # logits: pad columns -inf
    Nr = 3 * 1025
    Wh = rand_bf16(rng, (Nr, H), H ** -0.5)
    ph = torch.zeros(N.load().mtts_k_packed_bytes(Nr, H) // 2, dtype=torch.bfloat16, device="cuda")
    whd = dev_bf16(Wh)
    N.call("mtts_k_pack", P(whd), P(ph), Nr, H, 0, 0, 0, None)
    lg = torch.zeros(B, Nr, dtype=torch.bfloat16, device="cuda")
    N.call("mtts_k_gemv", P(ph), P(xd), H, P(lg), Nr, None, 0, B, Nr, H, 3, 0, 1025, 1024, None)
    torch.cuda.synchronize()
    got = host(lg)
    assert np.isneginf(got[:, 1024::1025]).all()
    fin = np.isfinite(got)
    assert fin.sum() == B * (Nr - 3)


@pytest.mark.parametrize("B,Nr,K,epi", [(1, 4096, 4096, 0), (4, 6144, 4096, 0), (2, 512, 4096, 2), (5, 96, 1024, 0),
                                        (3, 4100, 512, 0), (8, 96, 512, 0), (12, 96, 64, 0), (16, 64, 128, 2)])
def test_gemv_fused_norm(N, B, Nr, K, epi):
    """Qwen3RMSNorm folded into the GEMV prologue (small decode batches): y = linear(rmsnorm(x)),
    r from per-16-column sums of squares as the residual epilogue writes them."""
    rng = np.random.default_rng(B * 7 + Nr + K)
    ctx = O._Ctx("bf16")
    x = rand_bf16(rng, (B, K), 2.0)
    nw = B16.rnd(1 + 0.25 * rng.standard_normal(K).astype(np.float32))
    ss = (x.astype(np.float32) ** 2).reshape(B, K // 16, 16).sum(-1).astype(np.float32)
    rows = 2 * Nr if epi == 2 else Nr
    W = rand_bf16(rng, (rows, K), K ** -0.5)
    packed = torch.zeros(N.load().mtts_k_packed_bytes(rows, K) // 2, dtype=torch.bfloat16, device="cuda")
    wd = dev_bf16(W)
    if epi == 2:
        wg, wu = dev_bf16(W[:Nr]), dev_bf16(W[Nr:])
        N.call("mtts_k_pack", P(wg), P(packed), Nr, K, 0, 1, 0, None)
        N.call("mtts_k_pack", P(wu), P(packed), Nr, K, 0, 1, 1, None)
    else:
        N.call("mtts_k_pack", P(wd), P(packed), Nr, K, 0, 0, 0, None)
    xd, nwd = dev_bf16(x), dev_bf16(nw)
    ssd = torch.from_numpy(ss).cuda()
    y = torch.zeros(B, Nr, dtype=torch.bfloat16, device="cuda")
    N.call("mtts_k_gemv_ex", P(packed), P(xd), K, P(y), Nr, None, 0, B, Nr, K, epi, P(ssd), K // 16, K // 16,
           P(nwd), ctypes.c_float(1e-6), None, 0, 0, None)
    torch.cuda.synchronize()
    xn = O.rmsnorm(ctx, x, nw, 1e-6)
    if epi == 2:
        want = ctx.r(ctx.r(O.silu(O.linear(ctx, xn, W[:Nr]))) * O.linear(ctx, xn, W[Nr:]))
    else:
        want = O.linear(ctx, xn, W)
    got = host(y)
    rowscale = np.abs(want).max(axis=1, keepdims=True)
    assert within_band(got, want, 2.0, scale=np.maximum(np.abs(want), rowscale / 4)).all(), np.abs(got - want).max()


@pytest.mark.parametrize("M,Nr,K,epi", [(181, 4100, 512, 0), (33, 96, 4096, 0), (300, 512, 256, 1), (181, 384, 1024, 2),
                                        (1000, 64, 128, 1)])
def test_gemm_prefill(N, M, Nr, K, epi):
    """Prefill GEMM (any token count) against the oracle linear + epilogues, including the
    residual epilogue's per-16-column sums of squares."""
    rng = np.random.default_rng(M + Nr + K + epi)
    ctx = O._Ctx("bf16")
    x = rand_bf16(rng, (M, K))
    rows = 2 * Nr if epi == 2 else Nr
    W = rand_bf16(rng, (rows, K), K ** -0.5)
    packed = torch.zeros(N.load().mtts_k_packed_bytes(rows, K) // 2, dtype=torch.bfloat16, device="cuda")
    keep = [dev_bf16(W[:Nr]), dev_bf16(W[Nr:]) if epi == 2 else None]
    if epi == 2:
        N.call("mtts_k_pack", P(keep[0]), P(packed), Nr, K, 0, 1, 0, None)
        N.call("mtts_k_pack", P(keep[1]), P(packed), Nr, K, 0, 1, 1, None)
    else:
        N.call("mtts_k_pack", P(keep[0]), P(packed), Nr, K, 0, 0, 0, None)
    xd = dev_bf16(x)
    res = rand_bf16(rng, (M, Nr))
    y = dev_bf16(res) if epi == 1 else torch.zeros(M, Nr, dtype=torch.bfloat16, device="cuda")
    nt = (Nr + 15) // 16
    ss = torch.zeros(M, nt, dtype=torch.float32, device="cuda")
    N.call("mtts_k_gemm", P(packed), P(xd), K, P(y), Nr, P(y) if epi == 1 else None, Nr, M, Nr, K, epi,
           P(ss) if epi == 1 else None, nt, None)
    torch.cuda.synchronize()
    lin = O.linear(ctx, x, W[:Nr])
    if epi == 0:
        want = lin
    elif epi == 1:
        want = ctx.r(res + lin)
    else:
        want = ctx.r(ctx.r(O.silu(lin)) * O.linear(ctx, x, W[Nr:]))
    got = host(y)
    rowscale = np.abs(want).max(axis=1, keepdims=True)
    assert within_band(got, want, 2.0, scale=np.maximum(np.abs(want), rowscale / 4)).all(), np.abs(got - want).max()
    if epi == 1:
        g2 = np.pad(got, ((0, 0), (0, nt * 16 - Nr))).reshape(M, nt, 16)
        want_ss = (g2.astype(np.float64) ** 2).sum(-1)
        assert np.allclose(ss.cpu().numpy(), want_ss, rtol=1e-5, atol=1e-6)


def xpk_indices(M, K):
    """u16 index of (token m, column k) in the packed prefill activations (kernels.h xpkT_index)."""
    T = (M + 15) // 16
    m = np.arange(M)[:, None]
    k = np.arange(K)[None, :]
    return (((((k >> 5) * T + (m >> 4)) * 64 + (m & 15) + 16 * ((k & 31) >> 3)) << 3) + (k & 7)), T


@pytest.mark.parametrize("M,Nr,K,epi", [(181, 6144, 4096, 0), (181, 4096, 4096, 1), (181, 12288, 4096, 2),
                                        (181, 4096, 12288, 1), (130, 1000, 512, 1), (192, 96, 1024, 2),
                                        (2048, 4096, 4096, 1), (2048, 1536, 2048, 2), (1024, 12288, 4096, 2),
                                        (2117, 4096, 4096, 1), (1500, 6144, 4096, 0), (3000, 1024, 512, 1),
                                        (2117, 12288, 4096, 2), (40, 4096, 4096, 1), (100, 6144, 4096, 0),
                                        (120, 12288, 4096, 2), (64, 4096, 12288, 1), (300, 4096, 4096, 1),
                                        (384, 12288, 4096, 2), (250, 6144, 4096, 0), (504, 4096, 12288, 1),
                                        (288, 12288, 4096, 2), (210, 4096, 12288, 1), (600, 6144, 2048, 2)])
def test_gemm_packed_prefill(N, M, Nr, K, epi):
    """Prefill GEMM on fragment-packed activations (the engine's >= 33-row prompts) at the 8B
    projections' shapes: 181 rows take gemm3's one-token-block form (split K for q|k|v, o_proj,
    down), 2,048 the 256 / 128-row blocks; the gate|up output packed for the down projection.
    Oracle linear + epilogues within 2 bf16 ulp (rows' scale / 4 floor), the residual epilogue's
    sums of squares to 1e-5."""
    rng = np.random.default_rng(M + Nr + K + epi)
    ctx = O._Ctx("bf16")
    x = rand_bf16(rng, (M, K))
    rows = 2 * Nr if epi == 2 else Nr
    W = rand_bf16(rng, (rows, K), K ** -0.5)
    packed = torch.zeros(N.load().mtts_k_packed_bytes(rows, K) // 2, dtype=torch.bfloat16, device="cuda")
    keep = [dev_bf16(W[:Nr]), dev_bf16(W[Nr:]) if epi == 2 else None]
    if epi == 2:
        N.call("mtts_k_pack", P(keep[0]), P(packed), Nr, K, 0, 1, 0, None)
        N.call("mtts_k_pack", P(keep[1]), P(packed), Nr, K, 0, 1, 1, None)
    else:
        N.call("mtts_k_pack", P(keep[0]), P(packed), Nr, K, 0, 0, 0, None)
    idx, T = xpk_indices(M, K)
    xp = np.zeros(T * 16 * K, np.uint16)
    xp[idx] = np.asarray(x, np.float32).view(np.uint32) >> 16
    xd = torch.from_numpy(xp.view(np.int16)).cuda().view(torch.bfloat16)
    res = rand_bf16(rng, (M, Nr))
    ypk = epi == 2
    y = dev_bf16(res) if epi == 1 else torch.zeros(M, Nr, dtype=torch.bfloat16, device="cuda")
    yp = torch.zeros(T * 16 * Nr, dtype=torch.bfloat16, device="cuda") if ypk else None
    nt = (Nr + 15) // 16
    ss = torch.zeros(M, nt, dtype=torch.float32, device="cuda")
    ws = torch.zeros(8 << 20, dtype=torch.float32, device="cuda")
    N.call("mtts_k_gemm_packed", P(packed), P(xd), P(yp if ypk else y), Nr, 1 if ypk else 0,
           P(y) if epi == 1 else None, Nr, M, Nr, K, epi, P(ss) if epi == 1 else None, nt, P(ws), ws.numel(), None)
    torch.cuda.synchronize()
    lin = O.linear(ctx, x, W[:Nr])
    if epi == 0:
        want = lin
    elif epi == 1:
        want = ctx.r(res + lin)
    else:
        want = ctx.r(ctx.r(O.silu(lin)) * O.linear(ctx, x, W[Nr:]))
    if ypk:
        oidx, _ = xpk_indices(M, Nr)
        flat = yp.view(torch.int16).cpu().numpy().view(np.uint16)
        got = (flat[oidx].astype(np.uint32) << 16).view(np.float32)
    else:
        got = host(y)
    rowscale = np.abs(want).max(axis=1, keepdims=True)
    assert within_band(got, want, 2.0, scale=np.maximum(np.abs(want), rowscale / 4)).all(), np.abs(got - want).max()
    if epi == 1:
        g2 = np.pad(got, ((0, 0), (0, nt * 16 - Nr))).reshape(M, nt, 16)
        want_ss = (g2.astype(np.float64) ** 2).sum(-1)
        assert np.allclose(ss.cpu().numpy(), want_ss, rtol=1e-5, atol=1e-6)


def test_gemm_packed_prefill_gemm3_forms():
    """The gemm3 (LDS-DMA-only) forms that MTTS_GEMM5=0 / MTTS_GEMM5_LONG=0 fall back to, pinned
    against the oracle by the same cases (the switches are read once per process, so
    they run in a child pytest)."""
    import subprocess
    import sys
    env = dict(os.environ, MTTS_GEMM5="0", MTTS_GEMM5_LONG="0")
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-p", "no:cacheprovider", "-m", "gpu",
                        os.path.abspath(__file__) + "::test_gemm_packed_prefill"],
                       env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, (r.stdout + r.stderr)[-3000:]
    assert " passed" in r.stdout and "failed" not in r.stdout, r.stdout[-2000:]


@pytest.mark.parametrize("B,Nr,K,splits", [(8, 1536, 8960, 0), (1, 1536, 8960, 3), (16, 1000, 4096, 2),
                                           (3, 64, 2048, 7)])
def test_gemv_splitk(N, B, Nr, K, splits):
    """Split-K residual GEMV (csrc/splitk.hip; MossTTSLocal's depth down_proj shape first, at
    the engine's own split choice) against the oracle linear + residual add, and its per-16-column
    sums of squares; run twice on the same workspace (tickets reset by the last arrival) with
    bit-identical results."""
    S = splits or N.load().mtts_k_gemv_splitk_splits(Nr, K, B)
    assert S >= 2
    rng = np.random.default_rng(B + Nr + K)
    ctx = O._Ctx("bf16")
    x = rand_bf16(rng, (B, K))
    W = rand_bf16(rng, (Nr, K), K ** -0.5)
    packed = torch.zeros(N.load().mtts_k_packed_bytes(Nr, K) // 2, dtype=torch.bfloat16, device="cuda")
    wd = dev_bf16(W)
    N.call("mtts_k_pack", P(wd), P(packed), Nr, K, 0, 0, 0, None)
    xd = dev_bf16(x)
    res = rand_bf16(rng, (B, Nr))
    nt = (Nr + 15) // 16
    ws = torch.zeros(N.load().mtts_k_gemv_splitk_ws_bytes(Nr, S), dtype=torch.uint8, device="cuda")
    outs = []
    for _ in range(2):
        y = dev_bf16(res)
        ss = torch.zeros(B, nt, dtype=torch.float32, device="cuda")
        N.call("mtts_k_gemv_splitk", P(packed), P(xd), K, P(y), Nr, P(y), Nr, B, Nr, K, S, P(ss), nt, P(ws), None)
        torch.cuda.synchronize()
        outs.append((host(y), ss.cpu().numpy()))
    got, ssg = outs[0]
    assert np.array_equal(outs[0][0], outs[1][0]) and np.array_equal(outs[0][1], outs[1][1])
    want = ctx.r(res + O.linear(ctx, x, W))
    rowscale = np.abs(want).max(axis=1, keepdims=True)
    assert within_band(got, want, 2.0, scale=np.maximum(np.abs(want), rowscale / 4)).all(), np.abs(got - want).max()
    g2 = np.pad(got, ((0, 0), (0, nt * 16 - Nr))).reshape(B, nt, 16)
    assert np.allclose(ssg, (g2.astype(np.float64) ** 2).sum(-1), rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("M,H", [(1, 64), (7, 4096), (3, 12288)])
def test_rmsnorm(N, M, H):
    rng = np.random.default_rng(M + H)
    x = rand_bf16(rng, (M, H), 3.0)
    w = B16.rnd(1 + 0.25 * rng.standard_normal(H).astype(np.float32))
    y = torch.zeros(M, H, dtype=torch.bfloat16, device="cuda")
    xd, wd = dev_bf16(x), dev_bf16(w)  # keep the device tensors alive across the call
    N.call("mtts_k_rmsnorm", P(xd), 0, H, P(wd), P(y), M, H, ctypes.c_float(1e-6), None)
    torch.cuda.synchronize()
    want = O.rmsnorm(O._Ctx("bf16"), x, w, 1e-6)
    got = host(y)
    assert within_band(got, want, 1.0).all()
    assert np.mean(got == want) > 0.99


@pytest.mark.parametrize("H,n_vq,M", [(64, 4, 6), (320, 32, 6), (4096, 32, 6), (320, 5, 100), (4096, 16, 70),
                                      (6144, 32, 64)])
def test_embed_exact(N, H, n_vq, M):
    """M >= 64 rows take the prompt form (norm_rope.hip embed_wide_kernel); bit-exact either way."""
    cfg = O.tiny_cfg(n_vq=n_vq)
    rng = np.random.default_rng(H + n_vq + M)
    et = rand_bf16(rng, (cfg.vocab, H))
    ea = rand_bf16(rng, (cfg.n_vq, 1025, H))
    ids = np.concatenate([rng.integers(0, cfg.vocab, (M, 1)), rng.integers(0, 1025, (M, cfg.n_vq))], 1).astype(np.int64)
    h = torch.zeros(M, H, dtype=torch.bfloat16, device="cuda")
    idd = torch.from_numpy(ids).cuda()
    etd, ead = dev_bf16(et), dev_bf16(ea)
    N.call("mtts_k_embed", P(idd), cfg.n_vq + 1, P(etd), P(ead), 1025, H, P(h), M, None)
    torch.cuda.synchronize()
    W = {"language_model.embed_tokens.weight": et}
    for j in range(cfg.n_vq):
        W[f"emb_ext.{j}.weight"] = ea[j]
    want = O.embed(O._Ctx("bf16"), W, cfg, ids)
    assert (host(h) == want).all()


def test_fill_uniform_matches_oracle_prng(N):
    n = 5000
    t = torch.zeros(n, dtype=torch.bfloat16, device="cuda")
    N.call("mtts_k_fill_uniform", P(t), n, 7, 123, ctypes.c_float(0.05), ctypes.c_float(1.0), None)
    torch.cuda.synchronize()
    want = B16.rnd(prng.tensor(7, 123, (n,), 0.05, 1.0))
    assert (host(t) == want).all()


def test_rope_table_matches_oracle():
    from moss_tts_amd import _native as Nn
    Nn.load()
    D, npos = 128, 4096
    cs = np.zeros((npos, D), np.uint16)
    sn = np.zeros((npos, D), np.uint16)
    Nn.call("mtts_rope_table", ctypes.c_float(1e6), D, npos, cs.ctypes.data_as(ctypes.c_void_p),
            sn.ctypes.data_as(ctypes.c_void_p))
    c, s = O.rope_cos_sin(O._Ctx("bf16"), O.Cfg(), np.arange(npos))
    assert np.mean(B16.from_bits(cs) == c) > 0.999
    assert np.abs(B16.from_bits(cs) - c).max() <= 2 ** -8


@pytest.mark.parametrize("S,past,D,Hq,Hkv", [(1, 10, 128, 32, 8), (5, 0, 16, 4, 2), (3, 300, 128, 8, 8), (40, 0, 128, 32, 8),
                                             (181, 0, 128, 32, 8), (100, 350, 64, 8, 2), (33, 17, 16, 8, 1)])
def test_qk_norm_rope_and_attention(N, S, past, D, Hq, Hkv):
    rng = np.random.default_rng(S * 7 + past)
    ctx = O._Ctx("bf16")
    B, Cmax = 2, 512
    M = B * S
    heads = Hq + 2 * Hkv
    qkv = rand_bf16(rng, (M, heads * D), 2.0)
    qn = B16.rnd(1 + 0.25 * rng.standard_normal(D).astype(np.float32))
    kn = B16.rnd(1 + 0.25 * rng.standard_normal(D).astype(np.float32))
    cfg = O.Cfg(head_dim=D, rope_theta=1e6)
    cos, sin = O.rope_cos_sin(ctx, cfg, np.arange(Cmax))
    # existing cache rows 0..past-1 (K [B,Hkv,Cmax,D]; V stored transposed [B,Hkv,D,Cmax])
    kc0 = rand_bf16(rng, (B, Hkv, Cmax, D))
    vc0 = rand_bf16(rng, (B, Hkv, D, Cmax))
    kc, vc = dev_bf16(kc0), dev_bf16(vc0)
    qo = torch.zeros(M, Hq * D, dtype=torch.bfloat16, device="cuda")
    pos = torch.tensor([past], dtype=torch.int32, device="cuda")
    keep = [dev_bf16(a) for a in (qkv, qn, kn, cos, sin)]  # alive across the call
    N.call("mtts_k_qk_norm_rope", P(keep[0]), P(qo), P(kc), P(vc), P(keep[1]), P(keep[2]),
           P(keep[3]), P(keep[4]), P(pos), M, S, Hq, Hkv, D, Cmax, ctypes.c_float(1e-6), None)
    torch.cuda.synchronize()
    x = qkv.reshape(B, S, heads, D)
    q = O.rmsnorm(ctx, x[:, :, :Hq], qn, 1e-6).transpose(0, 2, 1, 3)
    k = O.rmsnorm(ctx, x[:, :, Hq:Hq + Hkv], kn, 1e-6).transpose(0, 2, 1, 3)
    v = x[:, :, Hq + Hkv:].transpose(0, 2, 1, 3)
    q = O.apply_rope(ctx, q, cos[past:past + S], sin[past:past + S])
    k = O.apply_rope(ctx, k, cos[past:past + S], sin[past:past + S])
    gq = host(qo).reshape(B, S, Hq, D).transpose(0, 2, 1, 3)
    # r = rsqrt(mean(x^2)) sums in a different order than numpy, so a normed value can round
    # across a bf16 boundary before the rotation; the rotation (a difference of two products)
    # can cancel, so the band is taken against the head's scale (rare; > 98 % bit-equal)
    hscale = np.maximum(np.abs(q), np.abs(q).max(axis=-1, keepdims=True))
    ok = within_band(gq, q, 1.0, scale=hscale)
    bad = np.argwhere(~ok)
    assert ok.all() and np.mean(gq == q) > 0.98, (np.mean(gq == q), len(bad), bad[:4].tolist(),
                                                  [(float(gq[tuple(i)]), float(q[tuple(i)])) for i in bad[:4]])
    kcg, vcg = host(kc), host(vc).transpose(0, 1, 3, 2)
    assert within_band(kcg[:, :, past:past + S], k, 1.0).all()
    assert (vcg[:, :, past:past + S] == v).all()
    assert (kcg[:, :, :past] == kc0[:, :, :past]).all()
    # attention over the cache with a left-padding mask on row 1
    mask = np.ones((B, Cmax), np.uint8)
    mask[1, :3] = 0
    ctxlen = past + S
    for CH, n_split in ((64, (ctxlen + 63) // 64), (256, (ctxlen + 255) // 256), ("flash", 0)):
        out = torch.zeros(M, Hq * D, dtype=torch.bfloat16, device="cuda")
        md = torch.from_numpy(mask).cuda()
        if CH == "flash":  # the prefill path's MFMA flash kernel
            N.call("mtts_k_attention_prefill", P(qo), P(kc), P(vc), P(md), P(pos), P(out), M, S, Hq, Hkv, D, Cmax,
                   None)
        else:
            ws = torch.zeros(N.load().mtts_k_attention_ws_bytes(M, Hq, D, n_split) // 4 + 1, dtype=torch.float32,
                             device="cuda")
            N.call("mtts_k_attention", P(qo), P(kc), P(vc), P(md), P(pos), P(out), P(ws),
                   M, S, Hq, Hkv, D, Cmax, CH, n_split, None)
        torch.cuda.synchronize()
        K = kcg[:, :, :ctxlen]
        V = vcg[:, :, :ctxlen]
        want = O.attention(ctx, gq, K, V, mask[:, :ctxlen].astype(bool), np.arange(past, past + S), D ** -0.5)
        got = host(out).reshape(B, S, Hq, D).transpose(0, 2, 1, 3)
        err = np.abs(got - want)
        assert (err <= 4 * 2.0 ** -8 * np.maximum(np.abs(want), 1.0)).all(), (CH, err.max())


@pytest.mark.parametrize("S,past,B,Cmax,Hq", [(512, 0, 1, 512, 32), (600, 37, 2, 704, 32), (1100, 0, 1, 1152, 32),
                                             (777, 300, 1, 1088, 32), (181, 0, 1, 256, 32), (100, 29, 2, 192, 32),
                                             (64, 0, 1, 64, 32), (300, 0, 2, 320, 16), (130, 60, 1, 192, 16)])
def test_attention_prefill_long(N, S, past, B, Cmax, Hq):
    """Prompts of >= MTTS_ATTN_PF32_MIN = 64 query tokens take the 32-token LDS-staged flash kernel
    (attention.hip attn_prefill32_kernel, D = 128): ragged tail tiles, a cached prefix, left padding
    on row 1 and uninitialised (NaN) cache rows past the prompt.  Hq 32 / 16 over 8 KV heads: the 8B
    and the MossTTSLocal 1.7B backbone shapes (4 / 2 waves a block)."""
    rng = np.random.default_rng(S + past + Hq)
    ctx = O._Ctx("bf16")
    D, Hkv = 128, 8
    M = B * S
    q = rand_bf16(rng, (B, S, Hq, D), 2.0)
    kc0 = rand_bf16(rng, (B, Hkv, Cmax, D))
    vc0 = rand_bf16(rng, (B, Hkv, D, Cmax))
    end = past + S
    kc0[:, :, end:] = np.nan  # rows no query may read: must not leak through 0 * NaN
    vc0[:, :, :, end:] = np.nan
    mask = np.ones((B, Cmax), np.uint8)
    if B > 1:
        mask[1, :45] = 0
    qd, kc, vc = dev_bf16(q.reshape(M, Hq * D)), dev_bf16(kc0), dev_bf16(vc0)
    md = torch.from_numpy(mask).cuda()
    pos = torch.tensor([past], dtype=torch.int32, device="cuda")
    out = torch.zeros(M, Hq * D, dtype=torch.bfloat16, device="cuda")
    N.call("mtts_k_attention_prefill", P(qd), P(kc), P(vc), P(md), P(pos), P(out), M, S, Hq, Hkv, D, Cmax, None)
    torch.cuda.synchronize()
    want = O.attention(ctx, q.transpose(0, 2, 1, 3), kc0[:, :, :end], vc0.transpose(0, 1, 3, 2)[:, :, :end],
                       mask[:, :end].astype(bool), np.arange(past, end), D ** -0.5)
    got = host(out).reshape(B, S, Hq, D).transpose(0, 2, 1, 3)
    err = np.abs(got - want)
    assert np.isfinite(got).all()
    assert (err <= 4 * 2.0 ** -8 * np.maximum(np.abs(want), 1.0)).all(), err.max()


@pytest.mark.parametrize("past,D,Hq,Hkv,B", [(10, 128, 32, 8, 1), (0, 16, 4, 2, 3), (300, 128, 8, 2, 2), (700, 64, 4, 1, 2),
                                             (127, 128, 32, 8, 1), (128, 128, 32, 8, 2), (1023, 16, 8, 1, 1),
                                             (389, 128, 32, 8, 4), (3000, 128, 32, 8, 1), (8100, 64, 8, 2, 1)])
def test_attn_decode_fused(N, past, D, Hq, Hkv, B):
    """Fused decode step (norm + rope + append + attention) against the oracle ops; long
    contexts exercise the multi-block split and its combine."""
    rng = np.random.default_rng(past + D)
    ctx = O._Ctx("bf16")
    Cmax = max(1024, (past + 1 + 63) // 64 * 64)
    heads = Hq + 2 * Hkv
    qkv = rand_bf16(rng, (B, heads * D), 2.0)
    qn = B16.rnd(1 + 0.25 * rng.standard_normal(D).astype(np.float32))
    kn = B16.rnd(1 + 0.25 * rng.standard_normal(D).astype(np.float32))
    cos, sin = O.rope_cos_sin(ctx, O.Cfg(head_dim=D, rope_theta=1e6), np.arange(Cmax))
    kc0 = rand_bf16(rng, (B, Hkv, Cmax, D))
    vt0 = rand_bf16(rng, (B, Hkv, D, Cmax))
    kc, vc = dev_bf16(kc0), dev_bf16(vt0)
    mask = np.ones((B, Cmax), np.uint8)
    if B > 1:
        mask[1, :5] = 0
    md = torch.from_numpy(mask).cuda()
    pos = torch.tensor([past], dtype=torch.int32, device="cuda")
    out = torch.zeros(B, Hq * D, dtype=torch.bfloat16, device="cuda")
    keep = [dev_bf16(a) for a in (qkv, qn, kn, cos, sin)]
    ws = torch.zeros(N.load().mtts_k_attn_decode_ws_bytes(B, Hq, Hkv, D, Cmax), dtype=torch.uint8, device="cuda")
    N.call("mtts_k_attn_decode", P(keep[0]), P(keep[1]), P(keep[2]), P(keep[3]), P(keep[4]), P(kc), P(vc), P(md),
           P(pos), P(out), P(ws), B, Hq, Hkv, D, Cmax, ctypes.c_float(1e-6), None)
    torch.cuda.synchronize()
    x = qkv.reshape(B, 1, heads, D)
    q = O.apply_rope(ctx, O.rmsnorm(ctx, x[:, :, :Hq], qn, 1e-6).transpose(0, 2, 1, 3), cos[past:past + 1], sin[past:past + 1])
    k = O.apply_rope(ctx, O.rmsnorm(ctx, x[:, :, Hq:Hq + Hkv], kn, 1e-6).transpose(0, 2, 1, 3), cos[past:past + 1],
                     sin[past:past + 1])
    v = x[:, :, Hq + Hkv:].transpose(0, 2, 1, 3)
    kcg, vcg = host(kc), host(vc).transpose(0, 1, 3, 2)
    assert within_band(kcg[:, :, past:past + 1], k, 1.0).all()
    assert (vcg[:, :, past:past + 1] == v).all()
    assert (kcg[:, :, :past] == kc0[:, :, :past]).all()
    K = kcg[:, :, :past + 1]
    V = vcg[:, :, :past + 1]
    want = O.attention(ctx, q, K, V, mask[:, :past + 1].astype(bool), np.array([past]), D ** -0.5)
    got = host(out).reshape(B, 1, Hq, D).transpose(0, 2, 1, 3)
    err = np.abs(got - want)
    assert (err <= 4 * 2.0 ** -8 * np.maximum(np.abs(want), 1.0)).all(), err.max()
