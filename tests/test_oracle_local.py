"""The MossTTSLocal oracle (oracle/moss_local.py) against golden vectors made by the
reference's own modules (tests/golden/make_golden_local.py)."""
import json
import os

import numpy as np
import pytest

from oracle import moss_local as L
from tests.parity_util import ulp_bf16

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def gl():
    g = np.load(os.path.join(HERE, "golden", "golden_local.npz"))
    cases = json.load(open(os.path.join(HERE, "golden", "cases_local.json")))
    return g, cases


def run(gl, name, steps=None):
    g, cases = gl
    c = cases[name]
    cfg = L.tiny_lcfg(n_vq=c["n_vq"])
    W = L.make_weights(cfg, c["seed"], dtype=c["dtype"], eos_boost=c["eos_boost"])
    trace = []
    mask = g[name + "/attention_mask"] if name + "/attention_mask" in g.files else None
    out = L.generate(W, cfg, g[name + "/input_ids"], attention_mask=mask, max_new_tokens=steps or c["steps"],
                     n_vq_for_inference=c["n_vq_inf"], dtype=c["dtype"], trace=trace)
    return g, c, cfg, out, trace


@pytest.mark.parametrize("name", ["l_nvq4_fp32", "l_nvq4_stop_fp32", "l_nvq4_ragged_fp32"])
def test_local_oracle_fp32_exact_ids(gl, name):
    """fp32: ids bit-exact and logits to 2e-5 against the reference's modules -- including a
    left-padded batch driven with GenerationMixin's position ids (pads excluded)"""
    g, c, cfg, out, trace = run(gl, name)
    ref = g[name + "/out"]
    ids = g[name + "/input_ids"]
    starts = L.find_last_equal_C(ids[..., 0], cfg.audio_start_token_id)
    for b in range(c["B"]):
        start_len, rows = out[b]
        assert start_len == ids.shape[1] - starts[b] - 1
        assert np.array_equal(rows, ref[b, starts[b]:]), b
    for k in range(c["n_logits"]):
        want = g[f"{name}/logit{k}"]
        fin = np.isfinite(want)
        assert (np.isfinite(trace[k]) == fin).all()
        assert np.allclose(trace[k][fin], want[fin], rtol=2e-5, atol=2e-5), k


@pytest.mark.parametrize("name", ["l_nvq4_bf16", "l_nvq8_clone_bf16", "l_nvq8_depth4_bf16", "l_nvq8_ragged_bf16"])
def test_local_oracle_bf16(gl, name):
    """bf16, teacher-forced on the reference's frames: every channel's logits of the first
    two frames within 12 bf16 ulps of the row scale (rounding noise compounds through the
    backbone and the depth transformer; measured max 10.2), argmax equal where the top-2
    margin is clear (free-running greedy ids can part at bf16 near-ties)."""
    g, cases = gl
    c = cases[name]
    cfg = L.tiny_lcfg(n_vq=c["n_vq"])
    W = L.make_weights(cfg, c["seed"], dtype="bf16", eos_boost=c["eos_boost"])
    ids, ref = g[name + "/input_ids"], g[name + "/out"]
    mask = g[name + "/attention_mask"] if name + "/attention_mask" in g.files else None
    T = ids.shape[1]
    trace = []
    L.generate(W, cfg, ids, attention_mask=mask, max_new_tokens=2, n_vq_for_inference=c["n_vq_inf"], dtype="bf16",
               trace=trace, forced=ref[:, T:T + 2])
    for k in range(c["n_logits"]):
        want = g[f"{name}/logit{k}"]
        fin = np.isfinite(want)
        assert (np.isfinite(trace[k]) == fin).all()
        scale = np.max(np.abs(np.where(fin, want, 0)), axis=-1, keepdims=True)
        u = ulp_bf16(np.broadcast_to(scale, want.shape))
        assert (np.abs(trace[k] - np.where(fin, want, 0))[fin] <= 12 * u[fin]).all(), k
        srt = np.sort(np.where(fin, want, -np.inf), axis=-1)
        clear = (srt[:, -1] - srt[:, -2]) > 24 * u[:, 0]
        assert (np.argmax(trace[k], -1) == np.argmax(want, -1))[clear].all(), k


def test_local_oracle_positions_exclude_pads(gl):
    """Which position convention the ragged fixtures pin.  RoPE scores depend on position
    differences only, so shifting a row's positions by its pad count changes its logits only
    through the rounding of cos / sin at other absolute positions (fp32: both forms within 2e-5).
    In bf16 that rounding shows: teacher-forced on the reference's first frame, the padded rows
    of l_nvq8_ragged_bf16 match the reference's logits more closely (more bit-equal logits, no
    larger error) with GenerationMixin's cumsum(mask) - 1 than with the pad-inclusive arange(T)."""
    g, cases = gl
    name = "l_nvq8_ragged_bf16"
    c = cases[name]
    cfg = L.tiny_lcfg(n_vq=c["n_vq"])
    W = L.make_weights(cfg, c["seed"], dtype="bf16")
    ids, mask = g[name + "/input_ids"], g[name + "/attention_mask"]
    n_ch = cfg.n_vq + 1
    forced = g[name + "/out"][:, ids.shape[1], :n_ch]
    padded = ~mask.all(axis=1)
    stats = []
    for pos in (L.hf_position_ids(mask), np.broadcast_to(np.arange(ids.shape[1]), mask.shape)):
        ctx = L._Ctx("bf16")
        gstate = L.backbone(ctx, W, cfg, ids, mask, L.Cache(cfg.layers), n_ch, position_ids=pos)
        trace = []
        L.local_frame(ctx, W, cfg, gstate, n_ch, trace=trace, forced=forced)
        eq, err = [], []
        for k in range(n_ch):
            want = g[f"{name}/logit{k}"]
            fin = np.isfinite(want)
            eq.append(((trace[k] == want) | ~fin).mean(axis=1))
            err.append(np.abs(np.where(fin, trace[k] - np.where(fin, want, 0), 0)).max(axis=1))
        stats.append((np.mean(eq, axis=0)[padded], np.max(err, axis=0)[padded]))
    (eq_hf, err_hf), (eq_inc, err_inc) = stats
    assert (eq_hf >= eq_inc).all() and (err_hf <= err_inc).all(), stats
    assert (eq_hf > eq_inc).any(), stats
