"""BASELINE configs[2]'s per-GPU batch (MossTTSDelay B = 4) at the 8B layer shape (h 4096,
32 / 8 heads x 128, I 12288, n_vq 32; 3 layers, random bf16 weights) against the oracle
(`oracle.moss_delay`, bf16 emulation: `TF/models/qwen3/modeling_qwen3.py:241-280, 294-323`, heads
`modeling_moss_tts.py:279-300`).

Both decode paths of B = 4 are pinned:
  * the persistent batch-4 launch (pse4.hip, round 4, the default within the PSE context range):
    the whole decoder stack per step, 32 attention units (row, KV head);
  * the per-op launches (MTTS_PSE4=0) with the fused input / post-attention RMSNorm prologues
    (four rows at K 4096) and the attention writing its rows itself (one 256-key block per (row,
    KV head) up to 256 cached keys, a self-merged pair of blocks beyond; o_proj a plain GEMV).
Teacher-forced decode steps with ragged left padding (positions count the pads,
`modeling_moss_tts.py:453,475,513`) crossing 256 cached keys; every row's audio heads and a
1,300-row slice of the text head within 8 bf16 ulps of the row scale, argmax equal on a clear
top-2 margin.  `poison`: every KV cache row starts NaN (rows past pos never reach a result)."""

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


T_B4, STEPS_B4 = 250, 10  # cached keys 250 .. 259: one attention block per head, then two


@pytest.fixture(scope="module")
def b4_oracle():
    """the oracle's logits of every teacher-forced step (computed once for every engine variant)"""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ids, mask = prompt(T_B4, STEPS_B4, 44, [0, 9, 23, 61])
    Wd = weights_on_device(19)
    rng = np.random.default_rng(5)
    tile_lo = (min(CFG.im_end_token_id, CFG.audio_assistant_gen_slot_token_id,
                   CFG.audio_assistant_delay_slot_token_id) // 16) * 16
    sel = np.unique(np.concatenate([np.arange(tile_lo, V), rng.choice(tile_lo, 1024, replace=False)]))
    M = BModel(Wd, sel)
    ctx = O._Ctx("bf16")
    cache = O.KVCache(LAYERS)
    M.step(ctx, ids[:, :T_B4], mask[:, :T_B4], cache)
    want = []
    for s in range(STEPS_B4):
        p = T_B4 + s
        want.append(M.step(ctx, ids[:, p:p + 1], mask[:, :p + 1], cache))
    yield Wd, ids, mask, sel, want
    del Wd
    torch.cuda.empty_cache()


@pytest.mark.parametrize("pse4,poison", [("1", False), ("1", True), ("0", False)])
def test_b4_decode_logits_vs_oracle(b4_oracle, pse4, poison):
    import os
    from moss_tts_amd.engine import Engine, EngineConfig
    Wd, ids, mask, sel, want = b4_oracle
    os.environ["MTTS_PSE4"] = pse4
    try:
        eng = Engine(EngineConfig(layers=LAYERS, max_batch=B, max_ctx=512, max_prefill_tokens=2048), 0)
    finally:
        os.environ.pop("MTTS_PSE4")
    try:
        if pse4 == "1" and not eng.pse4_active():
            pytest.skip("batch-4 persistent launch unsupported on this device")
        assert pse4 == "1" or not eng.pse4_active()
        eng.load_state_dict(Wd)
        if poison:
            eng.kv_fill(0x7FC0)
        eng.forward(torch.from_numpy(ids[:, :T_B4].copy()), torch.from_numpy(mask[:, :T_B4].copy()), 0)
        got = []
        for s in range(STEPS_B4):
            p = T_B4 + s
            lg = eng.forward(torch.from_numpy(ids[:, p:p + 1].copy()), torch.from_numpy(mask[:, :p + 1].copy()), p)
            got.append(lg.float().cpu().numpy())
        eng.pse_check()
    finally:
        eng.close()
    for s in range(STEPS_B4):
        text, audio = want[s]
        for b in range(B):
            band(got[s][b][sel], text[b], (s, b, "text"))
            for j in range(CFG.n_vq):
                band(got[s][b][V + j * A:V + (j + 1) * A], audio[b, j], (s, b, j))


def test_b4_generate_persistent_matches_launches(b4_oracle):
    """generate() at B = 4 through the batch-4 launch (hipGraph steps) vs the per-op launches:
    ids equal, or the first divergence on a bf16 near-tie (checked on the per-op run's logits)"""
    import os
    from moss_tts_amd.engine import Engine, EngineConfig, sampling_params
    Wd, ids, mask, sel, want = b4_oracle
    T, steps = 140, 40
    pr, pm = prompt(T, 0, 77, [0, 5, 17, 33])
    pr[:, -1, 0] = CFG.audio_start_token_id
    forced = torch.full((steps,), CFG.audio_assistant_gen_slot_token_id, dtype=torch.int32)
    sp = sampling_params(text_temperature=0, audio_temperature=0)
    outs = []
    for flag in ("1", "0"):
        os.environ["MTTS_PSE4"] = flag
        try:
            eng = Engine(EngineConfig(layers=LAYERS, max_batch=B, max_ctx=512, max_prefill_tokens=2048), 0)
        finally:
            os.environ.pop("MTTS_PSE4")
        try:
            if flag == "1" and not eng.pse4_active():
                pytest.skip("batch-4 persistent launch unsupported on this device")
            eng.load_state_dict(Wd)
            outs.append(eng.generate_ids(torch.from_numpy(pr), torch.from_numpy(pm.astype(bool)), steps, sp,
                                         forced_text=forced).cpu().numpy())
        finally:
            eng.close()
    a, b = outs
    assert a.shape == b.shape
    if np.array_equal(a, b):
        return
    # first differing step: a near-tie of the per-op run's own logits there
    diff = np.nonzero((a != b).any(axis=(0, 2)))[0]
    r = int(diff[0])
    assert r > T
    os.environ["MTTS_PSE4"] = "0"
    try:
        ref = Engine(EngineConfig(layers=LAYERS, max_batch=B, max_ctx=512, max_prefill_tokens=2048), 0)
    finally:
        os.environ.pop("MTTS_PSE4")
    try:
        ref.load_state_dict(Wd)
        traj = b
        lg = ref.forward(torch.from_numpy(traj[:, :T].copy()), torch.from_numpy(pm), 0)
        full = np.concatenate([pm, np.ones((B, r - T), np.uint8)], 1)
        for p in range(T, r):
            lg = ref.forward(torch.from_numpy(traj[:, p:p + 1].copy()), torch.from_numpy(full[:, :p + 1].copy()), p)
        lg = lg.float().cpu().numpy()
    finally:
        ref.close()
    from tests.parity_util import ulp_bf16
    for row in range(B):
        for j in np.nonzero(a[row, r] != b[row, r])[0]:
            x = lg[row, :V] if j == 0 else lg[row, V + (j - 1) * A: V + j * A - 1]
            top = np.sort(x[np.isfinite(x)])[-2:]
            assert top[1] - top[0] <= 8 * ulp_bf16(np.abs(top[1])), (r, row, int(j), top)
