"""17-32 row split-K GEMV (csrc/splitk.hip gemv_splitk2_kernel: two row tiles per workgroup
share the packed x fragments, K split in two): the B = 24 decode step's o_proj / down_proj at
the MossTTSDelay-8B layer shape (random weights, 3 layers) must give the logits of the one-tile
GEMV (MTTS_SK2=0) within the bf16 band (the K summation order differs), deterministically."""
import os

import numpy as np
import pytest

from tests.parity_util import ulp_bf16

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

B, T, STEPS = 24, 96, 4


def make(sk2):
    from moss_tts_amd.engine import Engine, EngineConfig
    os.environ["MTTS_SK2"] = sk2
    try:
        e = Engine(EngineConfig(layers=3, max_batch=B, max_ctx=256, max_prefill_tokens=4096), 0)
    finally:
        os.environ.pop("MTTS_SK2")
    e.init_random(seed=5)
    return e


def run(eng):
    rng = np.random.default_rng(11)
    ids = np.full((B, T + STEPS, 33), 1024, np.int64)
    ids[:, :, 0] = rng.integers(200, 20000, (B, T + STEPS))
    ids[:, :, 1:] = rng.integers(0, 1024, (B, T + STEPS, 32))
    mask = np.ones((B, T + STEPS), np.uint8)
    out = []
    eng.forward(torch.from_numpy(ids[:, :T].copy()), torch.from_numpy(mask[:, :T]), 0)
    for s in range(STEPS):
        lg = eng.forward(torch.from_numpy(ids[:, T + s:T + s + 1].copy()), torch.from_numpy(mask[:, :T + s + 1]), T + s)
        out.append(lg.float().cpu().numpy())
    return out


def test_splitk2_matches_one_tile_gemv():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ref, new = make("0"), make("2,2")
    try:
        want, got = run(ref), run(new)
        again = run(new)
    finally:
        ref.close()
        new.close()
    V, A = 151936, 1025
    for s, (w, g, g2) in enumerate(zip(want, got, again)):
        assert np.array_equal(g, g2), s
        for b in range(B):
            for j in (0, 1, 17, 32):
                sl = slice(0, V) if j == 0 else slice(V + (j - 1) * A, V + j * A)
                wr, gr = w[b, sl], g[b, sl]
                fin = np.isfinite(wr)
                assert (np.isfinite(gr) == fin).all(), (s, b, j)
                scale = np.abs(wr[fin]).max()
                assert np.abs(gr[fin] - wr[fin]).max() <= 8 * ulp_bf16(scale), (s, b, j)
