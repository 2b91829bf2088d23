"""The batch-1 persistent streaming decode launch (csrc/pse.hip, the default B=1 decode path and
the bench's dominant kernel) pinned DIRECTLY to the oracle at the MossTTSDelay-8B layer shape
(h 4096, 32/8 heads x 128, I 12288, n_vq 32; 3 layers, random bf16 weights).

The oracle is `oracle.moss_delay` in bf16 emulation -- embed-sum (`modeling_moss_tts.py:196-213`),
Qwen3 decoder layers (`TF/models/qwen3/modeling_qwen3.py:294-323`), final norm and the 1+n_vq
heads with the audio pad column at -inf (`modeling_moss_tts.py:279-300`) -- on the same weights.
Teacher-forced decodes at 150 and 611 cached keys and with a 37-token left pad; every step's
audio heads and a 2,148-row slice of the text head (the special-id tiles + random rows) must
sit within 8 bf16 ulps of the row scale, with the argmax equal wherever the top-2 margin is
clear.  A greedy generate() through the launch must follow the oracle's trajectory; a first
divergence, if any, must sit on a bf16 near-tie of the oracle's own logits."""
import os

import numpy as np
import pytest

from oracle import moss_delay as O
from tests.parity_util import margin_top2, ulp_bf16

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

LAYERS = 3
CFG = O.Cfg(layers=LAYERS)  # the 8B shape: h 4096, 32 / 8 heads x 128, I 12288, V 151,936, n_vq 32
V, A = CFG.vocab, CFG.audio_vocab + 1


class DeviceRows:
    """embedding table kept on the device; the oracle gathers only the rows it indexes"""

    def __init__(self, t):
        self.t = t

    def __getitem__(self, ids):
        ids = np.asarray(ids)
        rows = self.t[torch.from_numpy(ids.reshape(-1)).to(self.t.device)].float().cpu().numpy()
        return rows.reshape(ids.shape + (rows.shape[-1],))


def weights_on_device(seed):
    """random bf16 weights by reference name (uniform, variance 1/K for matrices, 1 +- 0.25 for
    norms, unit-scale embeddings), generated on the GPU"""
    g = torch.Generator(device="cuda").manual_seed(seed)
    out = {}
    for name, shape, kind in O.weight_specs(CFG):
        sc, off = O.scale_for(kind, shape)
        t = torch.rand(shape, generator=g, device="cuda", dtype=torch.float32)
        out[name] = (off + sc * (2 * t - 1)).to(torch.bfloat16)
    return out


class Model:
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
        """oracle forward of ids [1, S, 33] after the cached positions: (text logits at sel,
        audio logits [n_vq, 1025]) of the last position"""
        S = ids.shape[1]
        pos = np.arange(S) + cache.length()
        cos, sin = O.rope_cos_sin(ctx, CFG, pos)
        h = O.embed(ctx, self.W, CFG, ids)
        km = np.asarray(mask, bool)
        for i in range(LAYERS):
            h = O.decoder_layer(ctx, self.W, CFG, i, h, cos, sin, cache, km, pos)
        h = O.rmsnorm(ctx, h[:, -1:], self.W["language_model.norm.weight"], CFG.eps)[:, 0]
        text = O.linear(ctx, h, self.text_rows)[0]
        audio = []
        for j in range(CFG.n_vq):
            lg = O.linear(ctx, h, self.W[f"lm_heads.{j + 1}.weight"])[0]
            lg[-1] = -np.inf
            audio.append(lg)
        return text, np.stack(audio)


@pytest.fixture(scope="module")
def setup():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from moss_tts_amd.engine import Engine, EngineConfig
    os.environ["MTTS_PSE"] = "1"
    os.environ["MTTS_PSE_CTX"] = str(1 << 20)  # the kernel itself at every context tested
    try:
        eng = Engine(EngineConfig(layers=LAYERS, max_batch=1, max_ctx=768, max_prefill_tokens=1024), 0)
    finally:
        os.environ.pop("MTTS_PSE")
        os.environ.pop("MTTS_PSE_CTX")
    if not eng.pse_active():
        eng.close()
        pytest.skip("persistent streaming decode unsupported on this device")
    Wd = weights_on_device(11)
    eng.load_state_dict(Wd)
    rng = np.random.default_rng(11)
    # the text-head tiles holding the special ids (what a decode step always evaluates) + 2,048 others
    tile_lo = (min(CFG.im_end_token_id, CFG.audio_assistant_gen_slot_token_id,
                   CFG.audio_assistant_delay_slot_token_id) // 16) * 16
    sel = np.unique(np.concatenate([np.arange(tile_lo, V), rng.choice(tile_lo, 2048, replace=False)]))
    model = Model(Wd, sel)
    del Wd
    torch.cuda.empty_cache()
    yield eng, model
    eng.close()


def prompt(T, steps, seed, pad=0):
    rng = np.random.default_rng(seed)
    ids = np.full((1, T + steps, 33), 1024, np.int64)
    ids[0, :, 0] = rng.integers(200, 20000, T + steps)
    ids[0, :, 1:] = rng.integers(0, 1024, (T + steps, 32))
    ids[0, :pad, 0] = CFG.pad_token_id
    ids[0, :pad, 1:] = CFG.audio_pad_code
    mask = np.ones((1, T + steps), np.uint8)
    mask[0, :pad] = 0
    return ids, mask


def band(got, want, what):
    fin = np.isfinite(want)
    assert (np.isfinite(got) == fin).all(), what
    scale = np.abs(want[fin]).max()
    err = np.abs(got[fin] - want[fin]).max()
    assert err <= 8 * ulp_bf16(scale), (what, float(err), float(scale))
    if margin_top2(want) > 16 * float(ulp_bf16(scale)):
        assert int(np.argmax(np.where(fin, got, -np.inf))) == int(np.argmax(np.where(fin, want, -np.inf))), what


@pytest.mark.parametrize("T,steps,pad,poison", [(150, 10, 0, False), (611, 14, 0, False), (300, 8, 37, False),
                                                (201, 9, 5, True)])
def test_pse_decode_logits_vs_oracle(setup, T, steps, pad, poison):
    """poison: every KV cache row starts as NaN (kv_fill), so rows past the decode position
    -- the V^T fragment holding pos reads 8 keys at once -- must never reach a result"""
    eng, M = setup
    if poison:
        eng.kv_fill(0x7FC0)
    ids, mask = prompt(T, steps, T + pad, pad)
    ctx = O._Ctx("bf16")
    cache = O.KVCache(LAYERS)
    M.step(ctx, ids[:, :T], mask[:, :T], cache)  # prefill (oracle)
    eng.forward(torch.from_numpy(ids[:, :T].copy()), torch.from_numpy(mask[:, :T]), 0)  # prefill (GEMM path)
    for s in range(steps):
        p = T + s
        text, audio = M.step(ctx, ids[:, p:p + 1], mask[:, :p + 1], cache)
        lg = eng.forward(torch.from_numpy(ids[:, p:p + 1].copy()), torch.from_numpy(mask[:, :p + 1]), p)
        lg = lg.float().cpu().numpy()[0]
        band(lg[M.sel], text, (T, s, "text"))
        for j in range(CFG.n_vq):
            band(lg[V + j * A:V + (j + 1) * A], audio[j], (T, s, j))
    assert eng.pse_active(), "the launch must not have fallen back"


def test_pse_greedy_trajectory_vs_oracle(setup):
    """generate() (hipGraph steps through the persistent launch; forced gen-slot schedule) vs the
    oracle's greedy decide_step loop on its own logits"""
    from moss_tts_amd.engine import sampling_params
    eng, M = setup
    T, steps = 120, 36
    ids, mask = prompt(T, 0, 23)
    ids[0, -1, 0] = CFG.audio_start_token_id  # continuation: the model decodes audio frames
    forced = np.full(steps, CFG.audio_assistant_gen_slot_token_id, np.int32)
    out = eng.generate_ids(torch.from_numpy(ids), torch.from_numpy(mask.astype(bool)), steps,
                           sampling_params(text_temperature=0, audio_temperature=0),
                           forced_text=torch.from_numpy(forced)).cpu().numpy()
    ctx = O._Ctx("bf16")
    cache = O.KVCache(LAYERS)
    st = O.init_state(CFG, ids)
    sp = dict(text_temperature=0, text_top_p=1.0, text_top_k=50, audio_temperature=0, audio_top_p=1.0,
              audio_top_k=0, audio_repetition_penalty=1.0)
    gen, cur, mk = ids.copy(), ids, mask.astype(bool)
    for step in range(steps):
        text, audio = M.step(ctx, cur, mk, cache)
        full = np.full((1, V), -np.inf, np.float32)
        full[0, M.sel] = text
        nt, na = O.decide_step(ctx, CFG, [full] + [audio[j][None] for j in range(CFG.n_vq)], step, st, gen, sp,
                               forced_text=forced)
        cur = np.concatenate([nt[:, None, None], na[:, None, :]], axis=2)
        row = out[0, T + step]
        if not np.array_equal(row, cur[0, 0]):
            # the first divergence must be a bf16 near-tie of the oracle's logits in that channel
            for j in np.nonzero(row[1:] != cur[0, 0, 1:])[0]:
                r = audio[j][:1024]
                assert margin_top2(r) <= 8 * float(ulp_bf16(np.abs(r).max())), (step, int(j))
            assert row[0] == cur[0, 0, 0], step
            return
        mk = np.concatenate([mk, (~st["is_stopping"])[:, None]], axis=1)
        gen = np.concatenate([gen, cur], axis=1)
    assert out.shape[1] == T + steps


@pytest.fixture(scope="module")
def setup_coop(setup):
    """the same weights on an engine that launches the persistent kernel cooperatively
    (MTTS_PSE_COOP=1, hipLaunchCooperativeKernel: the runtime refuses a grid whose workgroups
    cannot all be resident instead of relying on the bounded waits)"""
    from moss_tts_amd.engine import Engine, EngineConfig
    os.environ.update(MTTS_PSE="1", MTTS_PSE_CTX=str(1 << 20), MTTS_PSE_COOP="1")
    try:
        eng = Engine(EngineConfig(layers=LAYERS, max_batch=1, max_ctx=768, max_prefill_tokens=1024), 0)
    finally:
        for k in ("MTTS_PSE", "MTTS_PSE_CTX", "MTTS_PSE_COOP"):
            os.environ.pop(k)
    eng.load_state_dict(weights_on_device(11))
    torch.cuda.empty_cache()
    yield eng, setup[0], setup[1]
    eng.close()


def test_pse_cooperative_launch(setup_coop):
    """the cooperative launch of the batch-1 persistent kernel, teacher-forced
    against the oracle (T=150, as test_pse_decode_logits_vs_oracle) and bit-identical to the
    ordinary launch; then generate() (the launch captured into the step's hipGraph) gives the
    ordinary launch's ids."""
    from moss_tts_amd.engine import sampling_params
    coop, eng, M = setup_coop
    T, steps = 150, 4
    ids, mask = prompt(T, steps, T, 0)
    ctx = O._Ctx("bf16")
    cache = O.KVCache(LAYERS)
    M.step(ctx, ids[:, :T], mask[:, :T], cache)
    for e in (coop, eng):
        e.forward(torch.from_numpy(ids[:, :T].copy()), torch.from_numpy(mask[:, :T]), 0)
    for s in range(steps):
        p = T + s
        text, audio = M.step(ctx, ids[:, p:p + 1], mask[:, :p + 1], cache)
        lc, lo = [e.forward(torch.from_numpy(ids[:, p:p + 1].copy()), torch.from_numpy(mask[:, :p + 1]), p)
                  .float().cpu().numpy()[0] for e in (coop, eng)]
        assert np.array_equal(lc, lo), s
        band(lc[M.sel], text, (T, s, "text"))
        for j in range(CFG.n_vq):
            band(lc[V + j * A:V + (j + 1) * A], audio[j], (T, s, j))
    assert coop.pse_active()
    gp, gm = prompt(120, 0, 23)
    gp[0, -1, 0] = CFG.audio_start_token_id
    forced = torch.full((24,), CFG.audio_assistant_gen_slot_token_id, dtype=torch.int32)
    sp = sampling_params(text_temperature=0, audio_temperature=0)
    a, b = [e.generate_ids(torch.from_numpy(gp), torch.from_numpy(gm.astype(bool)), 24, sp, forced_text=forced)
            .cpu().numpy() for e in (coop, eng)]
    assert np.array_equal(a, b)
    assert coop.pse_active()
