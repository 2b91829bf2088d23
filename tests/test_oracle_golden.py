"""Pins the CPU oracle (oracle/moss_delay.py) to golden vectors produced by the
REFERENCE classes (tests/golden/make_golden.py).  CPU only."""
import numpy as np
import pytest

from oracle import bf16 as B16
from oracle import moss_delay as O
from tests.parity_util import first_divergence, margin_top2, ulp_bf16

FP32_CASES = ["g_nvq4_fp32", "g_nvq4_stop_fp32", "g_nvq16_fp32", "g_nvq32_fp32",
              "g_nvq4_pen_fp32", "g_nvq4_b1_fp32"]
BF16_CASES = ["g_nvq4_bf16", "g_nvq16_bf16", "g_nvq32_bf16"]


def _run(golden, name, trace=None):
    g, cases = golden
    c = cases[name]
    cfg = O.tiny_cfg(n_vq=c["n_vq"])
    W = O.make_weights(cfg, c["seed"], dtype=c["dtype"], special_boost=c["special_boost"])
    res = O.generate(W, cfg, g[name + "/input_ids"], g[name + "/mask"], max_new_tokens=c["steps"],
                     text_temperature=0, audio_temperature=0,
                     audio_repetition_penalty=c["penalty"], dtype=c["dtype"], trace=trace)
    return g, c, res


@pytest.mark.parametrize("name", FP32_CASES)
def test_generate_fp32_bit_exact_ids(golden, name):
    tr = O.StepTrace()
    g, c, res = _run(golden, name, tr)
    assert len(res) == c["B"]
    for b, (start_len, ids) in enumerate(res):
        ref = g[name + f"/out{b}"]
        assert start_len == c["starts"][b]
        assert ids.shape == ref.shape
        assert (ids == ref).all(), f"row {b} first diff {first_divergence(ids, ref)}"
    # last-position logits of the first forward calls
    for s in range(4):
        k = name + f"/step{s}_audio"
        if k not in g:
            break
        ref = g[k]
        fin = np.isfinite(ref)
        assert (np.isfinite(tr.audio_logits[s]) == fin).all()
        np.testing.assert_allclose(tr.audio_logits[s][fin], ref[fin], rtol=0, atol=2e-5)
        # text top-16 of the raw head (before generate's masks)
        idx, val = g[name + f"/step{s}_text_top_idx"], g[name + f"/step{s}_text_top_val"]
        assert idx.shape[0] == c["B"]


@pytest.mark.parametrize("name", BF16_CASES)
def test_generate_bf16_within_band(golden, name):
    """bf16: step-0 logits within 4 bf16 ulps of the row's largest logit; greedy ids identical until the
    first step whose decision the oracle itself takes with a top-2 margin
    inside a 4-ulp band (summation-order noise can legitimately flip those)."""
    tr = O.StepTrace()
    g, c, res = _run(golden, name, tr)
    ref0 = g[name + "/step0_audio"]
    fin = np.isfinite(ref0)
    a0 = tr.audio_logits[0]
    err = np.abs(a0[fin] - ref0[fin])
    scale = np.broadcast_to(np.max(np.abs(np.where(fin, ref0, 0)), axis=-1, keepdims=True), ref0.shape)[fin]
    assert (err <= 4 * ulp_bf16(scale)).all(), err.max()
    assert np.mean(err == 0) > 0.25
    n_vq = c["n_vq"]
    n_steps = len(tr.text_logits)
    div_steps = []
    for b, (start_len, ids) in enumerate(res):
        ref = g[name + f"/out{b}"]
        d = first_divergence(ids, ref)
        if d is not None:
            div_steps.append(min(max(d - (ids.shape[0] - n_steps), 0), n_steps - 1))
    if not div_steps:
        return
    step = min(div_steps)  # the batch is coupled (stopping, masks): earliest decision that differs
    tl, al = tr.text_logits[step], tr.audio_logits[step]
    margins, bands = [], []
    for b in range(c["B"]):
        rows = [tl[b]] + [al[b, j, :1024] for j in range(n_vq)]
        for r in rows:
            f = r[np.isfinite(r)]
            if f.size:
                margins.append(margin_top2(r))
                bands.append(4 * float(ulp_bf16(np.abs(f).max())))
    assert min(m - bd for m, bd in zip(margins, bands)) <= 0, (name, step)


def test_processor_statics(golden):
    g, _ = golden
    codes = g["proc/codes"]
    dl = O.apply_delay_pattern(codes, 1024)
    assert (dl == g["proc/delayed"]).all()
    assert (O.apply_de_delay_pattern(dl) == g["proc/dedelayed"]).all()
    seqs = [g[f"proc/pad_in{i}"] for i in range(3)]
    ids, mask = O.left_pad(seqs, 151643, 1024)
    assert (ids == g["proc/pad_ids"]).all()
    assert (mask == g["proc/pad_mask"]).all()
    segs = O.split_audio_segments(g["proc/seg1_src"], 1024)
    assert len(segs) == int(g["proc/seg1_n"])
    for i, s in enumerate(segs):
        assert (s == g[f"proc/seg1_{i}"]).all()
    # two segments: the reference raises (torch.split given indices); the
    # restatement returns the intended maximal runs.
    assert int(g["proc/seg2_ref_raises"]) == 1
    segs2 = O.split_audio_segments(g["proc/seg2_src"], 1024)
    assert [s.shape[0] for s in segs2] == [6, 4]


@pytest.mark.parametrize("dt", ["fp32", "bf16"])
def test_ops(golden, dt):
    g, _ = golden
    ctx = O._Ctx(dt)
    p = f"op_rmsnorm_{dt}/"
    y = O.rmsnorm(ctx, g[p + "x"], g[p + "w"], 1e-6)
    np.testing.assert_allclose(y, g[p + "y"], rtol=0, atol=(0 if dt == "bf16" else 1e-6))
    p = f"op_rope_{dt}/"
    cfg = O.tiny_cfg(rope_theta=1e6, head_dim=16)
    cos, sin = O.rope_cos_sin(ctx, cfg, g[p + "pos"])
    tol = 0 if dt == "bf16" else 2e-6
    np.testing.assert_allclose(cos, g[p + "cos"], rtol=0, atol=max(tol, 1e-6 if dt == "fp32" else 0))
    qe = O.apply_rope(ctx, g[p + "q"], g[p + "cos"], g[p + "sin"])
    np.testing.assert_allclose(qe, g[p + "q_embed"], rtol=0, atol=(0 if dt == "bf16" else 1e-6))
    p = f"op_mlp_{dt}/"
    x = g[p + "x"]
    gg = O.linear(ctx, x, g[p + "wg"])
    u = O.linear(ctx, x, g[p + "wu"])
    y = O.linear(ctx, ctx.r(ctx.r(O.silu(gg)) * u), g[p + "wd"])
    ref = g[p + "y"]
    np.testing.assert_allclose(y, ref, rtol=0, atol=(2 * float(ulp_bf16(np.abs(ref).max())) if dt == "bf16" else 1e-5))
    p = f"op_attn_{dt}/"
    o = O.attention(ctx, g[p + "q"], g[p + "k"], g[p + "v"], g[p + "key_mask"], g[p + "q_pos"], 16 ** -0.5)
    ref = g[p + "out"].transpose(0, 2, 1, 3)
    np.testing.assert_allclose(o, ref, rtol=0, atol=(1.0 / 64 if dt == "bf16" else 1e-5))


@pytest.mark.parametrize("n_vq,seed,boost", [(4, 11, 2.0), (32, 31, 2.0), (16, 33, 1.0)])
def test_weight_fill_plan_equals_make_weights(n_vq, seed, boost):
    """oracle.moss_delay.weight_fill_plan (the device-side recipe of the 8B-shape fixtures:
    mtts_k_fill_uniform per tensor, then the boosted text-head rows) is make_weights bit for bit
    (tiny shape; the device fill's arithmetic is pinned by test_fill_uniform_matches_oracle_prng)"""
    from oracle import prng
    cfg = O.tiny_cfg(n_vq=n_vq)
    W = O.make_weights(cfg, seed, dtype="bf16", special_boost=boost)
    plan = O.weight_fill_plan(cfg, seed, special_boost=boost)
    assert [p[0] for p in plan] == list(W)
    for name, shape, tid, sc, off, patch in plan:
        w = B16.rnd(prng.tensor(seed, tid, shape, np.float32(sc), off))  # what the device fill writes
        for r, v in patch.items():
            w[r] = B16.rnd(v)
        assert np.array_equal(w, W[name]), name


def test_golden_8b_fixture_consistent():
    """tests/golden/golden_8b.npz (the reference at the 8B layer shape, make_golden_8b.py) is
    self-consistent: the recorded text-row selection is the one the GPU test rebuilds, every
    sampled (row, channel)'s recorded top-1 is the id the reference emitted at that step, channels
    it did not sample hold the fill ids, and the per-step logits cover every forward call"""
    import json
    import os
    from tests.golden import ref8b_inputs as R
    d = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    g = np.load(os.path.join(d, "golden_8b.npz"), allow_pickle=False)
    cases = json.load(open(os.path.join(d, "cases_8b.json")))
    assert set(cases) == {"r8_clone_b1", "r8_ragged_b4", "r8_long_nvq16"}
    for name, c in cases.items():
        cfg = O.Cfg(layers=c["layers"], n_vq=c["n_vq"])
        assert np.array_equal(g[name + "/text_sel"], R.text_sel(cfg))
        ids = g[name + "/input_ids"]
        T = ids.shape[1]
        top = g[name + "/sampled_top2"]
        assert top.shape == (c["n_forward"], c["B"], cfg.n_vq + 1, 4)
        assert g[name + "/raw_audio_bits"].shape == (c["n_forward"], c["B"], cfg.n_vq, cfg.audio_vocab + 1)
        n_checked = 0
        for b in range(c["B"]):
            out = g[f"{name}/out{b}"]
            gen = out[c["start_len"][b]:]  # the generated rows
            assert np.array_equal(out[:c["start_len"][b]], ids[b, T - c["start_len"][b]:])
            for s in range(min(len(gen), c["n_forward"])):
                for ch in range(cfg.n_vq + 1):
                    if np.isfinite(top[s, b, ch, 1]):
                        assert int(top[s, b, ch, 0]) == int(gen[s, ch]), (name, b, s, ch)
                        assert top[s, b, ch, 1] >= top[s, b, ch, 2]
                        n_checked += 1
                    elif ch > 0:
                        assert gen[s, ch] == cfg.audio_pad_code, (name, b, s, ch)
        assert n_checked > 0
