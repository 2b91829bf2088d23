"""Sampled MossTTSDelay decode on the GPU (generate() samples by default:
`modeling_moss_tts.py:392-405`, text T=1.5 / top_k=50, audio T=1.7 / top_p=0.8 / top_k=25).

The engine's draws are Philox(seed; step, row, channel) uniforms fed through torch's bf16
sample_token arithmetic (`inference_utils.py:111-145`).  Parity is checked step by step on the
logits the device itself drew from (`GenerateSession.logits`, the `mtts_generate_logits` hook):
the oracle's `decide_step` (text schedule + masks `modeling_moss_tts.py:451-509`, batch-wide
repetition penalty `inference_utils.py:79-88`, `topk_candidates` + `torch_draw` with the same
uniforms) must choose the same text token and the same audio codes at every step."""
import numpy as np
import pytest

from oracle import moss_delay as O

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

# (case, sampling kwargs): README / generate() defaults with a penalty, the CLI's top_k
# ceiling (clis/moss_tts_app.py:476-480: top_k up to 200), no audio top-k filter, top-p on text
PARAMS = [
    ("g_nvq4_bf16", dict(text_temperature=1.5, text_top_p=1.0, text_top_k=50, audio_temperature=1.7,
                         audio_top_p=0.8, audio_top_k=25, audio_repetition_penalty=1.1), 5),
    ("g_nvq16_bf16", dict(text_temperature=1.5, text_top_p=0.9, text_top_k=200, audio_temperature=1.0,
                          audio_top_p=0.95, audio_top_k=200, audio_repetition_penalty=1.3), 7),
    ("g_nvq4_stop_fp32", dict(text_temperature=0.8, text_top_p=0.7, text_top_k=1000, audio_temperature=1.2,
                              audio_top_p=1.0, audio_top_k=0, audio_repetition_penalty=0.9), 3),
    ("g_nvq32_bf16", dict(text_temperature=0.0, text_top_p=1.0, text_top_k=50, audio_temperature=1.7,
                          audio_top_p=0.8, audio_top_k=25, audio_repetition_penalty=1.0), 11),
    # wide text candidate sets (key-bin sampler, topk.h block_wide_draw): no top-k filter
    # (inference_utils.py:136), with and without top-p, and a top_k above the sorted form's 2,048
    ("g_nvq4_bf16", dict(text_temperature=1.5, text_top_p=1.0, text_top_k=0, audio_temperature=1.7,
                         audio_top_p=0.8, audio_top_k=25, audio_repetition_penalty=1.0), 13),
    ("g_nvq16_bf16", dict(text_temperature=1.0, text_top_p=0.9, text_top_k=-1, audio_temperature=1.0,
                          audio_top_p=0.95, audio_top_k=0, audio_repetition_penalty=1.1), 17),
    ("g_nvq4_stop_fp32", dict(text_temperature=0.8, text_top_p=0.95, text_top_k=5000, audio_temperature=1.2,
                              audio_top_p=1.0, audio_top_k=50, audio_repetition_penalty=1.0), 19),
]


@pytest.fixture(scope="module")
def gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _case(golden, name):
    g, cases = golden
    c = cases[name]
    cfg = O.tiny_cfg(n_vq=c["n_vq"])
    W = O.make_weights(cfg, c["seed"], dtype="bf16", special_boost=c["special_boost"])
    return g, c, cfg, W


def _engine(cfg, W):
    from moss_tts_amd.engine import Engine, EngineConfig
    e = Engine(EngineConfig(hidden=cfg.hidden, layers=cfg.layers, n_heads=cfg.n_heads, n_kv=cfg.n_kv,
                            head_dim=cfg.head_dim, inter=cfg.inter, vocab=cfg.vocab, n_vq=cfg.n_vq,
                            rope_theta=cfg.rope_theta, max_batch=4, max_ctx=256, max_prefill_tokens=512), 0)
    e.load_state_dict({k: torch.from_numpy(v) for k, v in W.items()})
    return e


def _heads(lg, cfg):
    A = cfg.audio_vocab + 1
    return [lg[:, :cfg.vocab]] + [lg[:, cfg.vocab + j * A: cfg.vocab + (j + 1) * A] for j in range(cfg.n_vq)]


@pytest.mark.parametrize("name,kw,seed", PARAMS, ids=[f"{p[0]}-k{p[1]['text_top_k']}" for p in PARAMS])
def test_sampled_steps_match_oracle(gpu, golden, name, kw, seed):
    from moss_tts_amd.engine import GenerateSession, sampling_params
    g, c, cfg, W = _case(golden, name)
    ids, mask = g[name + "/input_ids"], g[name + "/mask"]
    B, T, C = ids.shape
    eng = _engine(cfg, W)
    sess = GenerateSession(eng, torch.from_numpy(ids), torch.from_numpy(mask), c["steps"], sampling_params(**kw, seed=seed))
    ctx = O._Ctx("bf16")
    st = O.init_state(cfg, ids)
    rng = O.PhiloxDraw(seed)
    hist = ids.copy()
    sampled_text = sampled_audio = free_text = 0
    for step in range(c["steps"]):
        if step:
            if sess.finished:
                break
            sess.decode(1)
        lg = sess.logits().float().cpu().numpy()
        rows = sess.fetch().cpu().numpy()
        assert rows.shape[1] == T + step + 1
        samp_text = ~st["is_stopping"] & (st["delayed"] > cfg.n_vq)
        free_text += int((samp_text & ~st["is_audio"]).sum())  # text mode: the full masked row
        nt, na = O.decide_step(ctx, cfg, _heads(lg, cfg), step, st, hist, kw, rng=rng)
        got = rows[:, T + step]
        assert np.array_equal(got[:, 0], nt), (step, got[:, 0], nt)
        assert np.array_equal(got[:, 1:], na), (step, got[:, 1:], na)
        sampled_text += int(samp_text.sum())
        sampled_audio += int((na != cfg.audio_pad_code).sum())
        hist = rows
    eng.close()
    assert sampled_audio > 0 and sampled_text > 0
    if kw["text_temperature"] > 0 and not 0 < kw["text_top_k"] <= 2048:
        assert free_text > 0, "the wide text sampler was never exercised"


def test_sampled_generate_properties(gpu, golden):
    """same seed -> same ids; another seed -> other ids; sampled audio codes never the pad
    code; step-0 never emits delay_slot, steps <= n_vq never im_end (:461-464)."""
    from moss_tts_amd.engine import sampling_params
    name = "g_nvq4_bf16"
    g, c, cfg, W = _case(golden, name)
    ids, mask = torch.from_numpy(g[name + "/input_ids"]), torch.from_numpy(g[name + "/mask"])
    T = ids.shape[1]
    eng = _engine(cfg, W)
    sp = lambda s: sampling_params(audio_repetition_penalty=1.2, seed=s)  # generate() defaults otherwise
    a = eng.generate_ids(ids, mask, 40, sp(1)).cpu().numpy()
    b = eng.generate_ids(ids, mask, 40, sp(1)).cpu().numpy()
    d = eng.generate_ids(ids, mask, 40, sp(2)).cpu().numpy()
    eng.close()
    assert np.array_equal(a, b)
    assert not np.array_equal(a, d)
    gen = a[:, T:]
    assert (gen[:, 0, 0] != cfg.audio_assistant_delay_slot_token_id).all()
    assert (gen[:, :cfg.n_vq + 1, 0] != cfg.im_end_token_id).all()
    assert ((gen[..., 1:] >= 0) & (gen[..., 1:] <= cfg.audio_pad_code)).all()


def test_top_k_range(gpu, golden):
    """every top_k the reference accepts runs (inference_utils.py:136: <= 0 = no filter, any k
    up to the vocab): text 0 / -1 / 2,048 / 4,096 / the whole vocab, audio 0 / 5,000; sampled
    ids stay inside the vocab"""
    from moss_tts_amd.engine import sampling_params
    name = "g_nvq4_bf16"
    g, c, cfg, W = _case(golden, name)
    ids, mask = torch.from_numpy(g[name + "/input_ids"]), torch.from_numpy(g[name + "/mask"])
    eng = _engine(cfg, W)
    for tk, ak in ((0, 25), (-1, 0), (2048, 5000), (4096, 25), (cfg.vocab, 25)):
        out = eng.generate_ids(ids, mask, 6, sampling_params(text_top_k=tk, audio_top_k=ak)).cpu().numpy()
        assert out.shape[1] >= ids.shape[1] + 1
        assert ((out[..., 0] >= 0) & (out[..., 0] < cfg.vocab)).all()
    eng.close()
