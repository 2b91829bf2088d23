"""Engine-level parity on the GPU: the HIP generate() loop and teacher-forced
forwards against the oracle (bf16 emulation) on the golden tiny models, and
against the reference's own golden trajectories."""
import numpy as np
import pytest

from oracle import moss_delay as O
from tests.parity_util import first_divergence, margin_top2, ulp_bf16

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

CASES = ["g_nvq4_fp32", "g_nvq4_stop_fp32", "g_nvq16_bf16", "g_nvq32_bf16", "g_nvq4_pen_fp32", "g_nvq4_b1_fp32"]


def make_engine(cfg, W, max_batch=4, max_ctx=256, max_prefill_tokens=512):
    from moss_tts_amd.engine import Engine, EngineConfig
    e = Engine(EngineConfig(hidden=cfg.hidden, layers=cfg.layers, n_heads=cfg.n_heads, n_kv=cfg.n_kv,
                            head_dim=cfg.head_dim, inter=cfg.inter, vocab=cfg.vocab, n_vq=cfg.n_vq,
                            rope_theta=cfg.rope_theta, max_batch=max_batch, max_ctx=max_ctx,
                            max_prefill_tokens=max_prefill_tokens), 0)
    e.load_state_dict({k: torch.from_numpy(v) for k, v in W.items()})
    return e


def case(golden, name):
    g, cases = golden
    c = cases[name]
    cfg = O.tiny_cfg(n_vq=c["n_vq"])
    W = O.make_weights(cfg, c["seed"], dtype="bf16", special_boost=c["special_boost"])
    return g, c, cfg, W


def margin_ok(tr, step, B, n_vq):
    tl, al = tr.text_logits[step], tr.audio_logits[step]
    slack = []
    for b in range(B):
        for r in [tl[b]] + [al[b, j, :1024] for j in range(n_vq)]:
            f = r[np.isfinite(r)]
            if f.size:
                slack.append(margin_top2(r) - 8 * float(ulp_bf16(np.abs(f).max())))
    return min(slack) <= 0


@pytest.fixture(scope="module")
def gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


@pytest.mark.parametrize("name,prefill_cap", [(n, 512) for n in CASES] + [("g_nvq16_bf16", 8), ("g_nvq4_b1_fp32", 8)])
def test_generate_matches_oracle(gpu, golden, name, prefill_cap):
    """prefill_cap < prompt length exercises the position-chunked prefill (long-form path)."""
    generate_vs_oracle(golden, name, prefill_cap)


def test_generate_long_form_attention_graphs(gpu, golden):
    """The batch-1 decode graphs past the long-context threshold (16-wave attention blocks;
    MTTS_ATTN_LONG lowered to 8 so every decode step takes them) follow the oracle's greedy run."""
    import os
    os.environ["MTTS_ATTN_LONG"] = "8"
    try:
        generate_vs_oracle(golden, "g_nvq4_b1_fp32", 512)
    finally:
        os.environ.pop("MTTS_ATTN_LONG")


def generate_vs_oracle(golden, name, prefill_cap):
    from moss_tts_amd.engine import sampling_params
    g, c, cfg, W = case(golden, name)
    ids, mask = g[name + "/input_ids"], g[name + "/mask"]
    tr = O.StepTrace()
    ref = O.generate(W, cfg, ids, mask, max_new_tokens=c["steps"], text_temperature=0, audio_temperature=0,
                     audio_repetition_penalty=c["penalty"], dtype="bf16", trace=tr)
    eng = make_engine(cfg, W, max_prefill_tokens=prefill_cap)
    assert prefill_cap >= 512 or ids.shape[1] > max(prefill_cap, 4), "case must exceed the chunk"
    out = eng.generate_ids(torch.from_numpy(ids), torch.from_numpy(mask), c["steps"],
                           sampling_params(text_temperature=0, audio_temperature=0,
                                           audio_repetition_penalty=c["penalty"]))
    out = out.cpu().numpy()
    eng.close()
    T = ids.shape[1]
    starts = O.find_last_equal_C(ids[..., 0], cfg.im_start_token_id) + 3
    n_steps = len(tr.text_logits)
    divs = []
    for b in range(c["B"]):
        got = out[b, starts[b]:]
        want = ref[b][1]
        d = first_divergence(got, want)
        if d is not None:
            divs.append(min(max(d - (want.shape[0] - n_steps), 0), n_steps - 1))
    if divs:
        step = min(divs)
        assert step > 0 or margin_ok(tr, 0, c["B"], c["n_vq"]), "step-0 divergence without a near tie"
        assert margin_ok(tr, step, c["B"], c["n_vq"]), f"divergence at step {step} without a near tie"
    assert out.shape[1] >= T + 1


@pytest.mark.parametrize("name", ["g_nvq4_bf16", "g_nvq32_bf16"])
def test_teacher_forced_logits(gpu, golden, name):
    """Feed the oracle trajectory step by step; every step's logits stay within
    the bf16 band of the oracle's, and argmax agrees where the margin is clear."""
    g, c, cfg, W = case(golden, name)
    ids, mask = g[name + "/input_ids"], g[name + "/mask"]
    tr = O.StepTrace()
    ref = O.generate(W, cfg, ids, mask, max_new_tokens=12, text_temperature=0, audio_temperature=0,
                     dtype="bf16", trace=tr)
    B, T, C = ids.shape
    # rebuild the full generation_ids of the oracle run
    starts = O.find_last_equal_C(ids[..., 0], cfg.im_start_token_id) + 3
    gen = np.stack([np.concatenate([ids[b, :starts[b]], ref[b][1]], 0) for b in range(B)])
    eng = make_engine(cfg, W)
    full_mask = np.concatenate([mask, np.ones((B, gen.shape[1] - T), bool)], 1)
    # the oracle grows the mask with ~is_stopping; rebuild it from the trajectory
    for s in range(gen.shape[1] - T):
        stopped = (gen[:, T:T + s + 1, 0] == cfg.im_end_token_id).any(axis=1)
        full_mask[:, T + s] = ~stopped
    n_steps = len(tr.audio_logits)
    for s in range(n_steps):
        if s == 0:
            lg = eng.forward(torch.from_numpy(gen[:, :T]), torch.from_numpy(full_mask[:, :T].astype(np.uint8)), 0)
        else:
            p = T + s - 1
            lg = eng.forward(torch.from_numpy(gen[:, p:p + 1].copy()),
                             torch.from_numpy(full_mask[:, :p + 1].astype(np.uint8)), p)
        parts = [x.float().cpu().numpy() for x in eng.split_logits(lg)]
        got_audio = np.stack(parts[1:], 1)
        want_audio = tr.audio_logits[s]
        fin = np.isfinite(want_audio)
        bad = np.argwhere(np.isfinite(got_audio) != fin)
        assert bad.size == 0, (name, s, bad[:8].tolist(), [float(got_audio[tuple(i)]) for i in bad[:8]])
        scale = np.max(np.abs(np.where(fin, want_audio, 0)), axis=-1, keepdims=True)
        tol = 8 * ulp_bf16(np.broadcast_to(scale, want_audio.shape))
        err = np.abs(got_audio[fin] - want_audio[fin])
        assert (err <= tol[fin]).all(), (s, err.max())
        # argmax agreement on rows with a clear margin
        for b in range(B):
            for j in range(cfg.n_vq):
                w = want_audio[b, j, :1024]
                if margin_top2(w) > 16 * float(ulp_bf16(np.abs(w).max())):
                    assert int(np.argmax(got_audio[b, j, :1024])) == int(np.argmax(w))
    eng.close()


def test_continuation_state_and_shapes(gpu, golden):
    """B=1 continuation prompt: output width, start_length and the audio delay
    structure match the reference's golden trajectory exactly."""
    from moss_tts_amd.engine import sampling_params
    name = "g_nvq4_b1_fp32"
    g, c, cfg, W = case(golden, name)
    ids, mask = g[name + "/input_ids"], g[name + "/mask"]
    eng = make_engine(cfg, W)
    out = eng.generate_ids(torch.from_numpy(ids), torch.from_numpy(mask), c["steps"],
                           sampling_params(text_temperature=0, audio_temperature=0)).cpu().numpy()
    eng.close()
    start = int(O.find_last_equal_C(ids[..., 0], cfg.im_start_token_id)[0]) + 3
    assert ids.shape[1] - start == c["starts"][0]
    got = out[0, start:]
    # the text channel of a continuation is gen/delay/audio_end/text; pads follow the delay rule
    assert got[ids.shape[1] - start, 0] in (cfg.audio_assistant_gen_slot_token_id,
                                            cfg.audio_assistant_delay_slot_token_id)


def test_decode_bitwise_deterministic(gpu, golden):
    """Every reduction of the decode path has a fixed order: two engines fed the same
    teacher-forced sequence produce bit-identical logits (guards against LDS/global races)."""
    name = "g_nvq32_bf16"
    g, c, cfg, W = case(golden, name)
    ids, mask = g[name + "/input_ids"], g[name + "/mask"]
    B, T, C = ids.shape
    rng = np.random.default_rng(3)
    steps = 10
    extra = np.concatenate([rng.integers(0, 1024, (B, steps, 1)) + 151000,
                            rng.integers(0, 1025, (B, steps, cfg.n_vq))], 2).astype(np.int64)
    seq = np.concatenate([ids, extra], 1)
    full = np.concatenate([mask, np.ones((B, steps), bool)], 1).astype(np.uint8)
    outs = []
    for _ in range(2):
        eng = make_engine(cfg, W)
        lg = [eng.forward(torch.from_numpy(seq[:, :T]), torch.from_numpy(full[:, :T]), 0).cpu()]
        for s in range(steps):
            p = T + s
            lg.append(eng.forward(torch.from_numpy(seq[:, p:p + 1].copy()), torch.from_numpy(full[:, :p + 1]), p).cpu())
        eng.close()
        outs.append(torch.stack(lg).view(torch.int16).numpy())
    assert np.array_equal(outs[0], outs[1])


def test_text_head_gating_is_exact(gpu, golden):
    """Decode evaluates the full text head only when some row samples text outside audio
    mode; generate() output must be bit-identical to evaluating it every step
    (MTTS_FULL_TEXT_HEAD is read when an engine is created).  The gated launch walks its tiles
    from a capped grid (gemv.hip gate_grid): MTTS_GATE_GRID=3 makes each block of these small
    configs take several tiles, as the 8B text head does at the default cap."""
    import os
    from moss_tts_amd.engine import sampling_params
    outs = []
    for name in ("g_nvq4_stop_fp32", "g_nvq16_bf16"):
        g, c, cfg, W = case(golden, name)
        ids, mask = g[name + "/input_ids"], g[name + "/mask"]
        res = []
        for flag, grid in (("0", None), ("1", None), ("0", "3")):
            os.environ["MTTS_FULL_TEXT_HEAD"] = flag
            if grid:
                os.environ["MTTS_GATE_GRID"] = grid
            try:
                eng = make_engine(cfg, W)
                res.append(eng.generate_ids(torch.from_numpy(ids), torch.from_numpy(mask), 40,
                                            sampling_params(text_temperature=0, audio_temperature=0)).cpu().numpy())
                eng.close()
            finally:
                os.environ.pop("MTTS_FULL_TEXT_HEAD")
                os.environ.pop("MTTS_GATE_GRID", None)
        for r in res[1:]:
            assert r.shape == res[0].shape and (r == res[0]).all(), name


@pytest.mark.parametrize("unfused_norm", ["0", "1"])
def test_packed_activations_17_32_rows(gpu, golden, unfused_norm):
    """17-32 row decode keeps the GEMV inputs (normed x, attention output, SwiGLU output) in
    the fragment-packed layout (kernels.h xpk_index).  Teacher-forced over a golden case tiled
    to 24 rows: every decode step's logits are bit-identical to the row-major layout
    (MTTS_XPACK=0) and within the bf16 band of the oracle.  MTTS_UNFUSED_NORM=1 routes the
    RMSNorms through the standalone kernel, which then writes the packed layout itself."""
    import os
    name = "g_nvq4_bf16"
    g, c, cfg, W = case(golden, name)
    ids, mask = g[name + "/input_ids"], g[name + "/mask"]
    tr = O.StepTrace()
    ref = O.generate(W, cfg, ids, mask, max_new_tokens=6, text_temperature=0, audio_temperature=0,
                     dtype="bf16", trace=tr)
    B0, T, C = ids.shape
    starts = O.find_last_equal_C(ids[..., 0], cfg.im_start_token_id) + 3
    gen = np.stack([np.concatenate([ids[b, :starts[b]], ref[b][1]], 0) for b in range(B0)])
    full_mask = np.concatenate([mask, np.ones((B0, gen.shape[1] - T), bool)], 1)
    for s in range(gen.shape[1] - T):
        stopped = (gen[:, T:T + s + 1, 0] == cfg.im_end_token_id).any(axis=1)
        full_mask[:, T + s] = ~stopped
    rep = (24 + B0 - 1) // B0
    genr, maskr = np.tile(gen, (rep, 1, 1)), np.tile(full_mask, (rep, 1))
    B = genr.shape[0]
    assert 16 < B <= 32
    n_steps = min(len(tr.audio_logits), 5)
    runs = []
    for flag in ("1", "0"):
        os.environ["MTTS_XPACK"] = flag
        os.environ["MTTS_UNFUSED_NORM"] = unfused_norm
        try:
            eng = make_engine(cfg, W, max_batch=B)
        finally:
            os.environ.pop("MTTS_XPACK")
            os.environ.pop("MTTS_UNFUSED_NORM")
        out = []
        for s in range(n_steps):
            if s == 0:
                lg = eng.forward(torch.from_numpy(genr[:, :T].copy()), torch.from_numpy(maskr[:, :T].astype(np.uint8)), 0)
            else:
                p = T + s - 1
                lg = eng.forward(torch.from_numpy(genr[:, p:p + 1].copy()),
                                 torch.from_numpy(maskr[:, :p + 1].astype(np.uint8)), p)
            out.append(lg.cpu())
        runs.append(out)
        eng.close()
    for s in range(n_steps):
        assert torch.equal(runs[0][s].view(torch.int16), runs[1][s].view(torch.int16)), f"step {s}"
    # the packed run against the oracle (rows repeat the B0 golden rows)
    for s in range(1, n_steps):
        lg = runs[0][s].float().numpy()
        want = np.tile(tr.audio_logits[s], (rep, 1, 1))
        V = cfg.vocab
        got = lg[:, V:].reshape(B, cfg.n_vq, -1)[:, :, :want.shape[-1]]
        fin = np.isfinite(want)
        assert (np.isfinite(got) == fin).all(), s
        scale = np.max(np.abs(np.where(fin, want, 0)), axis=-1, keepdims=True)
        tol = 8 * ulp_bf16(np.broadcast_to(scale, want.shape))
        assert (np.abs(got[fin] - want[fin]) <= tol[fin]).all(), (s, float(np.abs(got[fin] - want[fin]).max()))


@pytest.mark.parametrize("rows", [48, 100, 160, 250, 300, 500, 1024])
def test_packed_activations_long_prefill(gpu, golden, rows):
    """Prefills of >= 33 token rows keep the GEMM inputs fragment-packed (xpkT_index with
    T = M / 16 token tiles; split-K partial launches read them packed): logits bit-identical to
    the row-major layout (MTTS_XPACK=0), and within the oracle's bf16 band (a golden case tiled
    to >= rows prompt rows)."""
    import os
    name = "g_nvq4_bf16"
    g, c, cfg, W = case(golden, name)
    ids, mask = g[name + "/input_ids"], g[name + "/mask"]
    tr = O.StepTrace()
    O.generate(W, cfg, ids, mask, max_new_tokens=1, text_temperature=0, audio_temperature=0, dtype="bf16", trace=tr)
    B0, T, C = ids.shape
    rep = (rows // T + B0) // B0 + 1
    idr, mkr = np.tile(ids, (rep, 1, 1)), np.tile(mask, (rep, 1))
    B = idr.shape[0]
    assert B * T >= rows
    runs = []
    for flag in ("1", "0"):
        os.environ["MTTS_XPACK"] = flag
        try:
            eng = make_engine(cfg, W, max_batch=B, max_prefill_tokens=max(2048, (B * T + 15) // 16 * 16))
        finally:
            os.environ.pop("MTTS_XPACK")
        runs.append(eng.forward(torch.from_numpy(idr), torch.from_numpy(mkr.astype(np.uint8)), 0).cpu())
        eng.close()
    assert torch.equal(runs[0].view(torch.int16), runs[1].view(torch.int16))
    lg = runs[0].float().numpy()
    want = np.tile(tr.audio_logits[0], (rep, 1, 1))
    got = lg[:, cfg.vocab:].reshape(B, cfg.n_vq, -1)[:, :, :want.shape[-1]]
    fin = np.isfinite(want)
    assert (np.isfinite(got) == fin).all()
    scale = np.max(np.abs(np.where(fin, want, 0)), axis=-1, keepdims=True)
    tol = 8 * ulp_bf16(np.broadcast_to(scale, want.shape))
    assert (np.abs(got[fin] - want[fin]) <= tol[fin]).all(), float(np.abs(got[fin] - want[fin]).max())


@pytest.mark.parametrize("T", [1290, 2600])
def test_long_context_16_wave_attention(gpu, golden, T):
    """Batch-1 decode past the engine's long-context threshold (MTTS_ATTN_LONG, lowered to 1,000
    here; TTSD's default 4,096) runs 16-wave (512-key) attention blocks: at 1,290 cached keys 3
    blocks per KV head whose partials o_proj merges, at 2,600 6 that the attention merges itself.
    Teacher-forced logits vs the oracle, a left-padded prompt."""
    import os
    name = "g_nvq4_bf16"
    g, c, cfg, W = case(golden, name)
    rng = np.random.default_rng(T)
    steps = 4
    ids = np.full((1, T + steps, cfg.n_vq + 1), cfg.audio_pad_code, np.int64)
    ids[..., 0] = rng.integers(200, 20000, (1, T + steps))
    ids[:, :, 1:] = rng.integers(0, 1024, (1, T + steps, cfg.n_vq))
    mask = np.ones((1, T + steps), bool)
    mask[0, :29] = False
    ids[0, :29, 0] = cfg.pad_token_id
    os.environ["MTTS_ATTN_LONG"] = "1000"
    try:
        eng = make_engine(cfg, W, max_batch=1, max_ctx=(T + steps + 63) // 64 * 64, max_prefill_tokens=4096)
    finally:
        os.environ.pop("MTTS_ATTN_LONG")
    eng.kv_fill(0x7FC0)  # NaN in every row not yet written: no kernel may read one into a result
    ctx = O._Ctx("bf16")
    cache = O.KVCache(cfg.layers)
    for s in range(steps + 1):
        p0, p1 = (0, T) if s == 0 else (T + s - 1, T + s)
        want = O.forward(ctx, W, cfg, ids[:, p0:p1], mask[:, :p1], cache, last_only=True)
        lg = eng.forward(torch.from_numpy(ids[:, p0:p1].copy()), torch.from_numpy(mask[:, :p1].astype(np.uint8)), p0)
        got = [x.float().cpu().numpy() for x in eng.split_logits(lg)]
        for j in range(1, cfg.n_vq + 1):
            w = want[j][:, -1]
            fin = np.isfinite(w)
            assert (np.isfinite(got[j]) == fin).all()
            scale = np.max(np.abs(np.where(fin, w, 0)), axis=-1, keepdims=True)
            tol = 8 * ulp_bf16(np.broadcast_to(scale, w.shape))
            err = np.abs(got[j][fin] - w[fin])
            assert (err <= tol[fin]).all(), (s, j, float(err.max()))
    eng.close()


def test_long_context_decode_logits(gpu, golden):
    """Decode steps at contexts of 5-6 attention blocks per KV head: past the publish-only
    threshold (attn_publish_max_splits) the attention merges its split partials itself and
    o_proj reads the merged rows.  Teacher-forced logits vs the oracle, ragged batch."""
    name = "g_nvq4_bf16"
    g, c, cfg, W = case(golden, name)
    rng = np.random.default_rng(5)
    B, T, steps = 2, 1290, 6
    ids = np.full((B, T + steps, cfg.n_vq + 1), cfg.audio_pad_code, np.int64)
    ids[..., 0] = rng.integers(200, 20000, (B, T + steps))
    ids[:, :, 1:] = rng.integers(0, 1024, (B, T + steps, cfg.n_vq))
    mask = np.ones((B, T + steps), bool)
    mask[1, :37] = False  # left padding of row 1
    ids[1, :37, 0] = cfg.pad_token_id
    eng = make_engine(cfg, W, max_ctx=1408, max_prefill_tokens=4096)
    eng.kv_fill(0x7FC0)  # NaN in every row not yet written (the prefill flash tiles, the decode splits)
    ctx = O._Ctx("bf16")
    cache = O.KVCache(cfg.layers)
    for s in range(steps + 1):
        p0, p1 = (0, T) if s == 0 else (T + s - 1, T + s)
        want = O.forward(ctx, W, cfg, ids[:, p0:p1], mask[:, :p1], cache, last_only=True)
        lg = eng.forward(torch.from_numpy(ids[:, p0:p1].copy()), torch.from_numpy(mask[:, :p1].astype(np.uint8)), p0)
        got = [x.float().cpu().numpy() for x in eng.split_logits(lg)]
        for j in range(1, cfg.n_vq + 1):
            w = want[j][:, -1]
            fin = np.isfinite(w)
            assert (np.isfinite(got[j]) == fin).all()
            scale = np.max(np.abs(np.where(fin, w, 0)), axis=-1, keepdims=True)
            tol = 8 * ulp_bf16(np.broadcast_to(scale, w.shape))
            err = np.abs(got[j][fin] - w[fin])
            assert (err <= tol[fin]).all(), (s, j, float(err.max()))
    eng.close()
