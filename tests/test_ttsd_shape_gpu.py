"""MOSS-TTSD long form at its real shape (BASELINE configs[4]): the batch-1 decode step at ~9,600
cached keys, n_vq 16, the MossTTSDelay-8B layer shape, against the oracle.

configs[4] decodes from 2,117 to 9,636 cached keys (`bench.py --config ttsd`); past 4,096 keys the
engine's batch-1 decode takes 16-wave (512-key) attention blocks (MTTS_ATTN_LONG), i.e. ~19 blocks
per KV head at 9,600 keys, whose (m, l, o) partials the last arriving block merges
(attn_body.h) -- or, by default since round 4, the persistent launch's long-context form
(pse.hip: every CU scores 1/32 of a KV head's cached keys, 64 merge units combine the slices).
Both are pinned here (MTTS_PSE_LONG 1 / 0).  The decode graphs of a TTSD generation capture exactly
these launches; here they run as teacher-forced forwards so every step's logits can be compared.

The cache of the long context is written directly (`mtts_engine_kv_write`, the same bf16 K / V
rows handed to the oracle's cache): the attention sees the same function of the past as after a
9,600-token prefill, which the numpy oracle could not run at this shape in a test's time.  A 37-key
left pad is masked out (positions include it, `TF/models/qwen3/modeling_qwen3.py:386-389`).

Oracle: `oracle.moss_delay` in bf16 emulation -- embed-sum (`modeling_moss_tts.py:196-213`), 3
Qwen3 decoder layers (`TF/.../modeling_qwen3.py:294-323`, SDPA `TF/integrations/sdpa_attention.py:
79-166`), final norm and the 1+16 heads (`modeling_moss_tts.py:279-300`).  Band: 8 bf16 ulps of
the row scale, argmax equal where the top-2 margin is clear."""
import os

import numpy as np
import pytest

from oracle import moss_delay as O
from tests.parity_util import margin_top2, ulp_bf16

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

LAYERS, NVQ = 3, 16
CFG = O.Cfg(layers=LAYERS, n_vq=NVQ)  # h 4096, 32 / 8 heads x 128, I 12288, V 151,936
V, A = CFG.vocab, CFG.audio_vocab + 1
T, STEPS, PAD = 9600, 4, 37


class DeviceRows:
    def __init__(self, t):
        self.t = t

    def __getitem__(self, ids):
        ids = np.asarray(ids)
        rows = self.t[torch.from_numpy(ids.reshape(-1)).to(self.t.device)].float().cpu().numpy()
        return rows.reshape(ids.shape + (rows.shape[-1],))


@pytest.fixture(scope="module")
def setup():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    assert int(os.environ.get("MTTS_ATTN_LONG", "4096")) < T
    g = torch.Generator(device="cuda").manual_seed(16)
    Wd = {}
    for name, shape, kind in O.weight_specs(CFG):
        sc, off = O.scale_for(kind, shape)
        Wd[name] = (off + sc * (2 * torch.rand(shape, generator=g, device="cuda") - 1)).to(torch.bfloat16)
    rng = np.random.default_rng(16)
    tile_lo = (min(CFG.im_end_token_id, CFG.audio_assistant_gen_slot_token_id,
                   CFG.audio_assistant_delay_slot_token_id) // 16) * 16
    sel = np.unique(np.concatenate([np.arange(tile_lo, V), rng.choice(tile_lo, 2048, replace=False)]))
    W = {}
    for name, t in Wd.items():
        if name == "language_model.embed_tokens.weight":
            W[name] = DeviceRows(t)
        elif name == "lm_heads.0.weight":
            text_rows = t[torch.from_numpy(sel).cuda()].float().cpu().numpy()
        else:
            W[name] = t.float().cpu().numpy()
    yield Wd, W, sel, text_rows


@pytest.mark.parametrize("pse_long", ["1", "0"])
def test_ttsd_long_context_decode_vs_oracle(setup, pse_long):
    from moss_tts_amd.engine import Engine, EngineConfig
    Wd, W, sel, text_rows = setup
    os.environ["MTTS_PSE_LONG"] = pse_long
    try:
        eng = Engine(EngineConfig(layers=LAYERS, n_vq=NVQ, max_batch=1, max_ctx=T + 64, max_prefill_tokens=1024), 0)
    finally:
        os.environ.pop("MTTS_PSE_LONG")
    try:
        eng.load_state_dict(Wd)
        if pse_long == "1" and not eng.pse_long_active():
            pytest.skip("persistent launch unsupported on this device")
        assert pse_long == "1" or not eng.pse_long_active()
        run_ttsd(eng, W, sel, text_rows)
        eng.pse_check()
    finally:
        eng.close()


def run_ttsd(eng, W, sel, text_rows):
    rng = np.random.default_rng(9600)
    ctx = O._Ctx("bf16")
    cache = O.KVCache(LAYERS)
    eng.kv_fill(0x7FC0)  # rows past the context stay NaN: none may reach a result
    for l in range(LAYERS):
        k = torch.randn(CFG.n_kv, T, CFG.head_dim, generator=torch.Generator().manual_seed(100 + l)).to(torch.bfloat16)
        v = torch.randn(CFG.n_kv, T, CFG.head_dim, generator=torch.Generator().manual_seed(200 + l)).to(torch.bfloat16)
        eng.kv_write(l, 0, 0, k, v)
        cache.k[l] = k.float().numpy()[None]
        cache.v[l] = v.float().numpy()[None]
    ids = np.full((1, T + STEPS, NVQ + 1), CFG.audio_pad_code, np.int64)
    ids[0, :, 0] = rng.integers(200, 20000, T + STEPS)
    ids[0, :, 1:] = rng.integers(0, 1024, (T + STEPS, NVQ))
    mask = np.ones((1, T + STEPS), np.uint8)
    mask[0, :PAD] = 0
    for s in range(STEPS):
        p = T + s
        pos = np.array([p])
        cos, sin = O.rope_cos_sin(ctx, CFG, pos)
        h = O.embed(ctx, W, CFG, ids[:, p:p + 1])
        for i in range(LAYERS):
            h = O.decoder_layer(ctx, W, CFG, i, h, cos, sin, cache, mask[:, :p + 1].astype(bool), pos)
        h = O.rmsnorm(ctx, h[:, -1:], W["language_model.norm.weight"], CFG.eps)[:, 0]
        want = [O.linear(ctx, h, text_rows)[0]]
        for j in range(NVQ):
            lg = O.linear(ctx, h, W[f"lm_heads.{j + 1}.weight"])[0]
            lg[-1] = -np.inf
            want.append(lg)
        lg = eng.forward(torch.from_numpy(ids[:, p:p + 1].copy()), torch.from_numpy(mask[:, :p + 1]), p)
        lg = lg.float().cpu().numpy()[0]
        got = [lg[sel]] + [lg[V + j * A:V + (j + 1) * A] for j in range(NVQ)]
        for j, (gr, wr) in enumerate(zip(got, want)):
            fin = np.isfinite(wr)
            assert (np.isfinite(gr) == fin).all(), (s, j)
            scale = np.abs(wr[fin]).max()
            err = np.abs(gr[fin] - wr[fin]).max()
            assert err <= 8 * ulp_bf16(scale), (s, j, float(err), float(scale))
            if margin_top2(wr) > 16 * float(ulp_bf16(scale)):
                assert int(np.argmax(np.where(fin, gr, -np.inf))) == int(np.argmax(np.where(fin, wr, -np.inf))), (s, j)
