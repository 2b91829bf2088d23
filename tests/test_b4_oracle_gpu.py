"""BASELINE configs[2]'s per-GPU batch (MossTTSDelay B = 4) at the 8B layer shape (h 4096,
32 / 8 heads x 128, I 12288, n_vq 32; 3 layers, random bf16 weights) against the oracle
(`oracle.moss_delay`, bf16 emulation: `TF/models/qwen3/modeling_qwen3.py:241-280, 294-323`, heads
`modeling_moss_tts.py:279-300`).

At this shape the decode step runs the per-op launches with the fused input / post-attention
RMSNorm prologues (four rows at K 4096) and the attention writing its rows itself (one
256-key block per (row, KV head) up to 256 cached keys, a self-merged pair of blocks beyond;
o_proj a plain GEMV: `gemv_attn_preload`).  Teacher-forced decode steps with ragged left padding
(positions count the pads, `modeling_moss_tts.py:453,475,513`) crossing 256 cached keys; every
row's audio heads and a 1,300-row slice of the text head within 8 bf16 ulps of the row scale,
argmax equal on a clear top-2 margin."""

import numpy as np
import pytest

from oracle import moss_delay as O
from tests.test_pse_oracle_gpu import CFG, LAYERS, V, A, DeviceRows, band, weights_on_device

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

B = 4


class BModel:
    """the oracle at B rows: embed-sum, LAYERS decoder layers, final norm, the heads of the last
    position (text at the selected rows, audio with the pad column at -inf)"""

    def __init__(self, Wd, sel):
        self.sel = sel
        self.W = {}
        for name, t in Wd.items():
            if name == "language_model.embed_tokens.weight":
                self.W[name] = DeviceRows(t)
            elif name == "lm_heads.0.weight":
                self.text_rows = t[torch.from_numpy(sel).cuda()].float().cpu().numpy()
            else:
                self.W[name] = t.float().cpu().numpy()

    def step(self, ctx, ids, mask, cache):
        S = ids.shape[1]
        pos = np.arange(S) + cache.length()
        cos, sin = O.rope_cos_sin(ctx, CFG, pos)
        h = O.embed(ctx, self.W, CFG, ids)
        km = np.asarray(mask, bool)
        for i in range(LAYERS):
            h = O.decoder_layer(ctx, self.W, CFG, i, h, cos, sin, cache, km, pos)
        h = O.rmsnorm(ctx, h[:, -1:], self.W["language_model.norm.weight"], CFG.eps)[:, 0]
        text = O.linear(ctx, h, self.text_rows)
        audio = []
        for j in range(CFG.n_vq):
            lg = O.linear(ctx, h, self.W[f"lm_heads.{j + 1}.weight"])
            lg[:, -1] = -np.inf
            audio.append(lg)
        return text, np.stack(audio, 1)


def prompt(T, steps, seed, pads):
    rng = np.random.default_rng(seed)
    ids = np.full((B, T + steps, 33), 1024, np.int64)
    ids[:, :, 0] = rng.integers(200, 20000, (B, T + steps))
    ids[:, :, 1:] = rng.integers(0, 1024, (B, T + steps, 32))
    mask = np.ones((B, T + steps), np.uint8)
    for b, p in enumerate(pads):
        ids[b, :p, 0] = CFG.pad_token_id
        ids[b, :p, 1:] = CFG.audio_pad_code
        mask[b, :p] = 0
    return ids, mask


def test_b4_decode_logits_vs_oracle():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from moss_tts_amd.engine import Engine, EngineConfig
    T, steps = 250, 10  # cached keys 250 .. 259: one attention block per head, then two
    ids, mask = prompt(T, steps, 44, [0, 9, 23, 61])
    Wd = weights_on_device(19)
    eng = Engine(EngineConfig(layers=LAYERS, max_batch=B, max_ctx=512, max_prefill_tokens=2048), 0)
    try:
        eng.load_state_dict(Wd)
        rng = np.random.default_rng(5)
        tile_lo = (min(CFG.im_end_token_id, CFG.audio_assistant_gen_slot_token_id,
                       CFG.audio_assistant_delay_slot_token_id) // 16) * 16
        sel = np.unique(np.concatenate([np.arange(tile_lo, V), rng.choice(tile_lo, 1024, replace=False)]))
        M = BModel(Wd, sel)
        del Wd
        eng.forward(torch.from_numpy(ids[:, :T].copy()), torch.from_numpy(mask[:, :T].copy()), 0)
        got = []
        for s in range(steps):
            p = T + s
            lg = eng.forward(torch.from_numpy(ids[:, p:p + 1].copy()), torch.from_numpy(mask[:, :p + 1].copy()), p)
            got.append(lg.float().cpu().numpy())
    finally:
        eng.close()
        torch.cuda.empty_cache()
    ctx = O._Ctx("bf16")
    cache = O.KVCache(LAYERS)
    M.step(ctx, ids[:, :T], mask[:, :T], cache)
    for s in range(steps):
        p = T + s
        text, audio = M.step(ctx, ids[:, p:p + 1], mask[:, :p + 1], cache)
        for b in range(B):
            band(got[s][b][sel], text[b], (s, b, "text"))
            for j in range(CFG.n_vq):
                band(got[s][b][V + j * A:V + (j + 1) * A], audio[b, j], (s, b, j))
