"""MossTTSLocal on the GPU engine against the oracle (oracle/moss_local.py) and the golden
vectors made by the reference's own modules (tests/golden/make_golden_local.py).

Tolerances: logits within 12 bf16 ulps of the row's max |logit| (the oracle-vs-reference
band of tests/test_oracle_local.py), argmax equal where the top-2 margin is clear; greedy
ids identical, except that a divergence must sit on a near-tie (top-2 margin <= 24 ulps)."""
import json
import os

import numpy as np
import pytest

from oracle import moss_local as L
from tests.parity_util import margin_top2, ulp_bf16

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


@pytest.fixture(scope="module")
def gl():
    g = np.load(os.path.join(HERE, "golden", "golden_local.npz"))
    cases = json.load(open(os.path.join(HERE, "golden", "cases_local.json")))
    return g, cases


def make_local_engine(cfg, W=None, max_batch=4, max_ctx=128, seed=None):
    from moss_tts_amd.engine import Engine, EngineConfig
    e = Engine(EngineConfig(hidden=cfg.hidden, layers=cfg.layers, n_heads=cfg.n_heads, n_kv=cfg.n_kv,
                            head_dim=cfg.head_dim, inter=cfg.inter, vocab=cfg.vocab, n_vq=cfg.n_vq,
                            rope_theta=cfg.rope_theta, rms_eps=cfg.eps, max_batch=max_batch, max_ctx=max_ctx,
                            max_prefill_tokens=512, model_kind=1, local_hidden=cfg.local_hidden,
                            local_layers=cfg.local_layers, local_inter=cfg.local_inter, local_mlp_ffn=cfg.mlp_ffn,
                            eos_token_id=cfg.eos_token_id, audio_pad_code=cfg.audio_pad_code,
                            audio_start_token_id=cfg.audio_start_token_id), 0)
    if W is not None:
        e.load_state_dict({k: torch.from_numpy(v) for k, v in W.items()})
    else:
        e.init_random(seed)
    return e


def lcase(gl, name):
    g, cases = gl
    c = cases[name]
    cfg = L.tiny_lcfg(n_vq=c["n_vq"])
    W = L.make_weights(cfg, c["seed"], dtype="bf16", eos_boost=c["eos_boost"])
    return g, c, cfg, W


def band_check(got, want, k):
    fin = np.isfinite(want)
    assert (np.isfinite(got) == fin).all(), k
    scale = np.max(np.abs(np.where(fin, want, 0)), axis=-1, keepdims=True)
    u = ulp_bf16(np.broadcast_to(scale, want.shape))
    err = np.abs(got - np.where(fin, want, 0))[fin]
    assert (err <= 12 * u[fin]).all(), (k, float(err.max()), float(u.max()))
    srt = np.sort(np.where(fin, want, -np.inf), axis=-1)
    clear = (srt[:, -1] - srt[:, -2]) > 24 * u[:, 0]
    assert (np.argmax(got, -1) == np.argmax(want, -1))[clear].all(), k


def frame_logits(eng, ids_all, T, frames, n_vq_inf, prompt_mask=None):
    """teacher-forced logits of `frames` frames: frame 0 from the prompt, frame f from frame f-1
    (prompt_mask [B, T]: left pads; generated columns are unmasked)"""
    B = ids_all.shape[0]
    out = []
    for f in range(frames):
        if f == 0:
            x, past = ids_all[:, :T], 0
        else:
            x, past = ids_all[:, T + f - 1:T + f], T + f - 1
        mask = np.ones((B, past + x.shape[1]), np.uint8)
        if prompt_mask is not None:
            mask[:, :T] = prompt_mask
        lg = eng.local_forward(torch.from_numpy(np.ascontiguousarray(x)), torch.from_numpy(mask), past,
                               torch.from_numpy(np.ascontiguousarray(ids_all[:, T + f])), n_vq_inf)
        out += [t.float().cpu().numpy() for t in lg]
    return out


def case_mask(g, name):
    return g[name + "/attention_mask"] if name + "/attention_mask" in g.files else None


@pytest.mark.parametrize("name", ["l_nvq4_bf16", "l_nvq8_clone_bf16", "l_nvq8_depth4_bf16", "l_nvq8_ragged_bf16"])
def test_local_teacher_forced_logits_vs_reference(gpu, gl, name):
    """Every channel's logits of the first two frames against the reference's own modules;
    l_nvq8_ragged_bf16 is a left-padded batch whose reference forward got GenerationMixin's
    position ids (pads excluded: the engine's per-row RoPE offsets)."""
    g, c, cfg, W = lcase(gl, name)
    ids, ref = g[name + "/input_ids"], g[name + "/out"]
    eng = make_local_engine(cfg, W)
    got = frame_logits(eng, ref, ids.shape[1], 2, c["n_vq_inf"], case_mask(g, name))
    eng.close()
    assert len(got) == c["n_logits"]
    for k in range(c["n_logits"]):
        band_check(got[k], g[f"{name}/logit{k}"], k)


def test_local_ragged_fp32_teacher_forced_vs_reference(gpu, gl):
    """l_nvq4_ragged_fp32 against the reference's OWN fp32 logits (its generate case below runs on
    the bf16 oracle's trajectory, since the engine is bf16): the engine on the bf16-rounded weights,
    teacher-forced along the reference's fp32 frames, every channel's logits of the first two frames
    within 8 % of the row scale (the bf16 oracle on the same weights sits at <= 5.8 %,
    measured on this fixture: weight rounding dominates at the tiny shape), argmax equal where the
    reference's top-2 margin exceeds 16 % of the row scale."""
    name = "l_nvq4_ragged_fp32"
    g, c, cfg, W = lcase(gl, name)
    ids, ref = g[name + "/input_ids"], g[name + "/out"]
    eng = make_local_engine(cfg, W)
    got = frame_logits(eng, ref, ids.shape[1], 2, c["n_vq_inf"], case_mask(g, name))
    eng.close()
    assert len(got) == c["n_logits"]
    n_clear = 0
    for k in range(c["n_logits"]):
        want = g[f"{name}/logit{k}"]
        fin = np.isfinite(want)
        assert (np.isfinite(got[k]) == fin).all(), k
        scale = np.max(np.abs(np.where(fin, want, 0)), axis=-1, keepdims=True)
        err = np.abs(np.where(fin, got[k] - np.where(fin, want, 0), 0))
        assert (err <= 0.08 * scale).all(), (k, float((err / scale).max()))
        srt = np.sort(np.where(fin, want, -np.inf), axis=-1)
        clear = (srt[:, -1] - srt[:, -2]) > 0.16 * scale[:, 0]
        n_clear += int(clear.sum())
        assert (np.argmax(got[k], -1) == np.argmax(want, -1))[clear].all(), k
    assert n_clear >= 3  # (4 rows of this fixture clear the margin)


def check_trajectory(cfg, W, ids, got, want, n_vq_inf, mask=None):
    """ids equal, or the first divergence is a near-tie of the oracle's teacher-forced logits"""
    T = ids.shape[1]
    n = min(got.shape[1], want.shape[1])
    diff = np.argwhere((got[:, :n] != want[:, :n]))
    if diff.size == 0:
        assert got.shape == want.shape
        return
    f = int(diff[:, 1].min()) - T
    assert f >= 0, "prompt rows differ"
    n_ch = min(ids.shape[2], 1 + n_vq_inf)
    trace = []
    L.generate(W, cfg, ids, attention_mask=mask, max_new_tokens=f + 1, n_vq_for_inference=n_vq_inf, dtype="bf16",
               trace=trace, forced=want[:, T:T + f + 1])
    rows = diff[diff[:, 1] == T + f]
    for b in np.unique(rows[:, 0]):
        i = int(rows[rows[:, 0] == b, 2].min())  # later channels of the frame are conditioned on this one
        assert i < n_ch, "channels beyond n_vq_for_inference must be 0 / pad"
        lg = trace[f * n_ch + i][b]
        u = float(ulp_bf16(np.abs(lg[np.isfinite(lg)]).max()))
        assert margin_top2(lg) <= 24 * u, f"frame {f} row {b} channel {i}: divergence without a near tie"


@pytest.mark.parametrize("name", ["l_nvq4_bf16", "l_nvq8_clone_bf16", "l_nvq8_depth4_bf16", "l_nvq8_ragged_bf16",
                                  "l_nvq4_ragged_fp32"])
def test_local_generate_vs_reference(gpu, gl, name):
    """greedy ids against the reference's own trajectory (ragged cases: left-padded batches);
    the fp32 ragged case runs on bf16 weights' engine only as far as its ids go (the engine is
    bf16), so it is checked with the same near-tie rule against the bf16 oracle"""
    g, c, cfg, W = lcase(gl, name)
    ids, ref = g[name + "/input_ids"], g[name + "/out"]
    mask = case_mask(g, name)
    if c["dtype"] == "fp32":  # (lcase's weights are the bf16-rounded ones)
        rows = L.generate(W, cfg, ids, attention_mask=mask, max_new_tokens=c["steps"], n_vq_for_inference=c["n_vq_inf"],
                          dtype="bf16")
        T = ids.shape[1]
        ref = np.stack([np.concatenate([ids[b, :T - r[0] - 1], r[1]], 0) for b, r in enumerate(rows)])
    eng = make_local_engine(cfg, W)
    out = eng.local_generate_ids(torch.from_numpy(ids), None if mask is None else torch.from_numpy(mask), c["steps"],
                                 c["n_vq_inf"]).cpu().numpy()
    eng.close()
    assert out.shape[2] == ids.shape[2] and np.array_equal(out[:, :ids.shape[1]], ids)
    check_trajectory(cfg, W, ids, out, ref, c["n_vq_inf"], mask)


def test_local_generate_stop_matches_oracle(gpu):
    """eos on channel 0 stops a row; finished rows emit eos / pad; the loop ends when every
    row has stopped (_sample :425-446).  bf16 oracle trajectory with a boosted eos row."""
    cfg = L.tiny_lcfg(n_vq=4)
    W = L.make_weights(cfg, 31, dtype="bf16", eos_boost=10.0)  # rows stop at frames 2, 2, 1
    rng = np.random.default_rng(31)
    C = cfg.n_vq + 1
    ids = np.full((3, 14, C), cfg.audio_pad_code, np.int64)
    ids[..., 0] = rng.integers(200, 20000, (3, 14))
    ids[:, -1, 0] = cfg.audio_start_token_id
    want_rows = L.generate(W, cfg, ids, max_new_tokens=40, dtype="bf16")
    T = ids.shape[1]
    want = np.stack([np.concatenate([ids[b, :T - r[0] - 1], r[1]], 0) for b, r in enumerate(want_rows)])
    eng = make_local_engine(cfg, W)
    out = eng.local_generate_ids(torch.from_numpy(ids), None, 40).cpu().numpy()
    eng.close()
    assert want.shape[1] < T + 40, "fixture must stop before max_new_tokens"
    check_trajectory(cfg, W, ids, out, want, cfg.n_vq)
    if np.array_equal(out, want):
        fin = out[:, T:, 0] == cfg.eos_token_id
        assert fin[:, -1].all()


def test_local_init_random_matches_oracle_weights(gpu, gl):
    """mtts_engine_init_random == oracle.moss_local.make_weights (same names, order, scales)."""
    name = "l_nvq4_bf16"
    g, c, cfg, W = lcase(gl, name)
    ids, ref = g[name + "/input_ids"], g[name + "/out"]
    a = make_local_engine(cfg, W)
    b = make_local_engine(cfg, None, seed=c["seed"])
    la = frame_logits(a, ref, ids.shape[1], 1, c["n_vq_inf"])
    lb = frame_logits(b, ref, ids.shape[1], 1, c["n_vq_inf"])
    a.close()
    b.close()
    for x, y in zip(la, lb):
        assert np.array_equal(x, y)


def test_moss_rmsnorm_kernel(gpu):
    """bf16 MossTTSRMSNorm kernel vs the oracle's op-by-op bf16 restatement"""
    import ctypes
    from moss_tts_amd import _native as N
    from oracle.moss_delay import _Ctx
    rng = np.random.default_rng(5)
    for M, H in [(1, 64), (3, 2048), (5, 520), (2, 4096), (2, 6000)]:  # register-cached form up to 4096, then the general one
        x = (rng.standard_normal((M, H)) * rng.uniform(0.1, 30)).astype(np.float32)
        w = rng.uniform(0.5, 1.5, H).astype(np.float32)
        xt = torch.from_numpy(x).to(torch.bfloat16)
        wt = torch.from_numpy(w).to(torch.bfloat16)
        want = L.moss_rmsnorm_bf16(_Ctx("bf16"), xt.float().numpy(), wt.float().numpy(), 1e-6)
        xd, wd = xt.cuda(), wt.cuda()
        y = torch.empty_like(xd)
        N.check(N.load().mtts_k_moss_rmsnorm(ctypes.c_void_p(xd.data_ptr()), ctypes.c_void_p(wd.data_ptr()),
                                             ctypes.c_void_p(y.data_ptr()), M, H, 1e-6, None), "moss_rmsnorm")
        torch.cuda.synchronize()
        got = y.float().cpu().numpy()
        u = ulp_bf16(want)
        assert (np.abs(got - want) <= u).all(), (M, H)


def test_local_generate_sampling_readme_config(gpu, gl):
    """README generation_config (text 1.5/50/1.0; audio penalty 1.1, 1.0/50/0.95): valid ids,
    the audio pad code never drawn, same seed -> same trajectory, new seed -> a new one."""
    from moss_tts_amd.engine import sampling_params
    name = "l_nvq8_clone_bf16"
    g, c, cfg, W = lcase(gl, name)
    ids = g[name + "/input_ids"]
    eng = make_local_engine(cfg, W)
    sp = lambda seed: sampling_params(text_temperature=1.5, text_top_k=50, text_top_p=1.0, audio_temperature=1.0,
                                      audio_top_k=50, audio_top_p=0.95, audio_repetition_penalty=1.1, seed=seed)
    a = eng.local_generate_ids(torch.from_numpy(ids), None, 12, sampling=sp(1)).cpu().numpy()
    b = eng.local_generate_ids(torch.from_numpy(ids), None, 12, sampling=sp(1)).cpu().numpy()
    d = eng.local_generate_ids(torch.from_numpy(ids), None, 12, sampling=sp(2)).cpu().numpy()
    eng.close()
    T = ids.shape[1]
    assert np.array_equal(a, b)
    assert not np.array_equal(a, d)
    gen = a[:, T:]
    live = np.cumsum(gen[:, :, 0] == cfg.eos_token_id, axis=1) == 0  # frames before a row's eos
    assert ((gen[..., 0] >= 0) & (gen[..., 0] < cfg.vocab)).all()
    assert ((gen[..., 1:] >= 0) & (gen[..., 1:] < cfg.audio_pad_code))[live].all()


def build_local_model(cfg, W):
    from transformers import Qwen3Config
    from moss_tts_amd.local import MossTTSDelayConfig, MossTTSDelayModel
    lc = Qwen3Config(vocab_size=cfg.vocab, hidden_size=cfg.hidden, intermediate_size=cfg.inter,
                     num_hidden_layers=cfg.layers, num_attention_heads=cfg.n_heads, num_key_value_heads=cfg.n_kv,
                     head_dim=cfg.head_dim, rope_theta=cfg.rope_theta, rms_norm_eps=cfg.eps)
    model = MossTTSDelayModel(MossTTSDelayConfig(language_config=lc, n_vq=cfg.n_vq, local_hidden_size=cfg.local_hidden,
                                                 local_num_layers=cfg.local_layers, local_ffn_hidden_size=cfg.local_inter,
                                                 additional_mlp_ffn_hidden_size=cfg.mlp_ffn))
    sd = model.state_dict()
    for k, v in W.items():
        assert k in sd, k
        sd[k].copy_(torch.from_numpy(v))
    return model.to("cuda", torch.bfloat16).eval()


def test_local_model_generate_dropin(gpu, gl):
    """reference-shaped model + generation_config (greedy, n_vq_for_inference) -> the
    reference's output contract, ids equal to the engine run"""
    from transformers import GenerationConfig
    name = "l_nvq8_depth4_bf16"
    g, c, cfg, W = lcase(gl, name)
    ids = torch.from_numpy(g[name + "/input_ids"]).cuda()
    model = build_local_model(cfg, W)
    gc = GenerationConfig(max_new_tokens=c["steps"], eos_token_id=cfg.eos_token_id)
    gc.n_vq_for_inference = c["n_vq_inf"]
    gc.do_samples = [False] * (cfg.n_vq + 1)
    gc.layers = [{}] * (cfg.n_vq + 1)
    out = model.generate(input_ids=ids, attention_mask=torch.ones(ids.shape[:2], dtype=torch.bool, device="cuda"),
                         generation_config=gc)
    eng = make_local_engine(cfg, W)
    want = eng.local_generate_ids(ids, None, c["steps"], c["n_vq_inf"]).cpu()
    eng.close()
    T = ids.shape[1]
    starts = L.find_last_equal_C(g[name + "/input_ids"][..., 0], cfg.audio_start_token_id)
    assert len(out) == c["B"]
    for b, (start_len, rows) in enumerate(out):
        assert int(start_len) == T - int(starts[b]) - 1
        assert torch.equal(rows.cpu(), want[b, int(starts[b]):])
    # README sampling layout runs through the same entry point
    gc.do_samples = [True] * (cfg.n_vq + 1)
    gc.layers = [{"repetition_penalty": 1.0, "temperature": 1.5, "top_p": 1.0, "top_k": 50}] + \
        [{"repetition_penalty": 1.1, "temperature": 1.0, "top_p": 0.95, "top_k": 50}] * cfg.n_vq
    out = model.generate(input_ids=ids, generation_config=gc)
    assert out[0][1].shape[1] == cfg.n_vq + 1


def test_local_per_channel_processors(gpu, gl):
    """generation_config.do_samples / layers set per channel (`:356-368`): every channel takes
    its own processor set.  (1) sampled channels with top_k = 1 (any temperature / top_p) equal
    the argmax, so a table alternating greedy and top-1 channels reproduces the greedy run; (2) one
    sampled channel with a wide top_k changes that channel only from there on: the channels before
    it in the first frame stay the greedy ones, and two seeds draw differently."""
    from transformers import GenerationConfig
    name = "l_nvq8_depth4_bf16"
    g, c, cfg, W = lcase(gl, name)
    ids = torch.from_numpy(g[name + "/input_ids"]).cuda()
    model = build_local_model(cfg, W)
    C = cfg.n_vq + 1
    steps = 6

    def run(do, layers, seed=0):
        gc = GenerationConfig(max_new_tokens=steps, eos_token_id=cfg.eos_token_id)
        gc.n_vq_for_inference = cfg.n_vq
        gc.do_samples, gc.layers = do, layers
        torch.manual_seed(seed)
        return [r.cpu() for _, r in model.generate(input_ids=ids, generation_config=gc)]

    greedy = run([False] * C, [{}] * C)
    # (power-of-two temperatures: bf16(s / T) keeps every order.  HF's top-k keeps every score tied
    # with the k-th -- random bf16 logits often tie at the top of 1,025 codes -- and top_p 0.3 then
    # drops all but one of a tie: the HIGHEST index, torch.sort's ascending order dropping the lower
    # ones first (test_local_sampling.py::test_device_pick_greedy_and_top1), where argmax takes the
    # first -- so the top-1 channels are deterministic, and equal the greedy run where no tie occurs)
    top1 = [{"temperature": 2.0 ** (i % 3 - 1), "top_k": 1, "top_p": 0.3, "repetition_penalty": 1.0} for i in range(C)]
    mixed = run([i % 2 == 1 for i in range(C)], top1)
    assert all(torch.equal(a, b) for a, b in zip(mixed, run([i % 2 == 1 for i in range(C)], top1, seed=7)))
    assert all(a.shape == b.shape for a, b in zip(greedy, mixed))
    # generate-level: each row equals the greedy run up to its first difference, and that
    # difference is a tie at the top of that channel's logits (teacher-forced along the greedy
    # prefix on a bare engine with the same weights): the top-1 channel took the highest tied
    # index, argmax the lowest.  Where the margin is clear the two runs agree.
    T = ids.shape[1]
    starts = L.find_last_equal_C(g[name + "/input_ids"][..., 0], cfg.audio_start_token_id)
    eng = make_local_engine(cfg, W)
    try:
        n_same = 0
        for r in range(len(greedy)):
            f0 = T - int(starts[r])
            diff = (greedy[r] != mixed[r]).nonzero()
            if len(diff) == 0:
                n_same += 1
                continue
            f, j = int(diff[0, 0]), int(diff[0, 1])
            assert f >= f0, (r, f, j)
            prefix = torch.cat([ids[r, :int(starts[r])].cpu(), greedy[r][:f]], 0)[None]
            lg = eng.local_forward(prefix, torch.ones(prefix.shape[:2], dtype=torch.bool), 0, greedy[r][f][None],
                                   cfg.n_vq)[j][0].float().cpu().numpy()
            top = lg.max()
            assert lg[int(greedy[r][f, j])] == top and lg[int(mixed[r][f, j])] == top, (r, f, j)
            assert (lg == top).sum() >= 2, (r, f, j)
    finally:
        eng.close()
    j0 = 3
    layers = [{}] * C
    layers[j0] = {"temperature": 2.0, "top_k": 1000, "top_p": 1.0}
    do = [i == j0 for i in range(C)]
    a, b = run(do, layers, 1), run(do, layers, 2)
    for r in range(len(greedy)):
        f0 = T - int(starts[r])  # first generated row of this row's output
        assert torch.equal(a[r][f0, :j0], greedy[r][f0, :j0]) and torch.equal(b[r][f0, :j0], greedy[r][f0, :j0])
    assert any(not torch.equal(x[:, j0], y[:, j0]) for x, y in zip(a, b))


def test_local_mask_must_be_left_padded(gpu):
    """the backbone's RoPE offsets are the rows' pad counts, which equal GenerationMixin's
    cumsum(mask) - 1 positions only for left padding -- an interior or right pad is refused
    (MTTS_E_INVALID -> ValueError) by the teacher-forced forward and by generate, not decoded with
    shifted positions; a left-padded mask still runs"""
    cfg = L.tiny_lcfg(n_vq=4)
    eng = make_local_engine(cfg, None, seed=3)
    try:
        rng = np.random.default_rng(3)
        C = cfg.n_vq + 1
        ids = np.full((2, 10, C), cfg.audio_pad_code, np.int64)
        ids[..., 0] = rng.integers(200, 20000, (2, 10))
        ids[:, -1, 0] = cfg.audio_start_token_id
        frame = np.zeros((2, C), np.int64)
        for bad in ([1] * 4 + [0] + [1] * 5, [1] * 9 + [0]):  # interior pad, right pad
            mask = np.ones((2, 10), np.uint8)
            mask[1] = bad
            with pytest.raises(ValueError, match="left-padded"):
                eng.local_forward(torch.from_numpy(ids), torch.from_numpy(mask), 0, torch.from_numpy(frame))
            with pytest.raises(ValueError, match="left-padded"):
                eng.local_generate_ids(torch.from_numpy(ids), torch.from_numpy(mask), 2)
        mask = np.ones((2, 10), np.uint8)
        mask[1, :3] = 0
        eng.local_forward(torch.from_numpy(ids), torch.from_numpy(mask), 0, torch.from_numpy(frame))
    finally:
        eng.close()
