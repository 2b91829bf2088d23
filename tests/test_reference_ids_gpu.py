"""HIP greedy generate() against the REFERENCE's own trajectories, on all 9 golden cases.

`tests/golden/make_golden.py` ran `moss_tts_delay.modeling_moss_tts.MossTTSDelayModel.generate`
(`/root/reference/moss_tts_delay/modeling_moss_tts.py:392-525`, greedy: temperature 0) on tiny
random-weight configs in this container and committed its output ids (`golden.npz` `<case>/out<b>`).
Here the HIP engine runs the same prompts with the same weights (bf16: the engine's dtype) and its
ids are compared with the reference's row by row:
  * equal up to the first divergence (or to the end);
  * at the first divergence, the reference's own top-2 logit margin in the diverging channel must be
    a near-tie for the precision gap -- 8 bf16 ulps of the row scale for the bf16 cases (the
    reference ran bf16 too), 3 % of the row scale for the fp32 cases (the reference ran fp32 weights
    and arithmetic; bf16 vs fp32 logits differ by up to 1.2 % of the row scale on these models,
    measured with the oracle).
The reference's logits at a step come from `oracle.moss_delay` run in the case's dtype along the
reference trajectory: in fp32 it reproduces the reference's ids bit for bit and its logits to 2e-6
(tests/test_oracle_golden.py); in bf16 it follows them to the first 4-ulp near-tie.

Every case prints one `REFIDS {json}` line (case, rows, first divergence step per row, margin and
tolerance there); DESIGN.md section 4 tabulates them."""
import json

import numpy as np
import pytest

from oracle import moss_delay as O
from tests.parity_util import first_divergence, margin_top2, ulp_bf16

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

CASES = ["g_nvq4_fp32", "g_nvq4_bf16", "g_nvq4_stop_fp32", "g_nvq4_pen_fp32", "g_nvq4_b1_fp32",
         "g_nvq16_fp32", "g_nvq16_bf16", "g_nvq32_fp32", "g_nvq32_bf16"]


@pytest.fixture(scope="module")
def gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


@pytest.mark.parametrize("name", CASES)
def test_generate_ids_vs_reference(gpu, golden, name):
    from moss_tts_amd.engine import Engine, EngineConfig, sampling_params
    g, cases = golden
    c = cases[name]
    cfg = O.tiny_cfg(n_vq=c["n_vq"])
    ids, mask = g[name + "/input_ids"], g[name + "/mask"]
    B = c["B"]
    W = O.make_weights(cfg, c["seed"], dtype="bf16", special_boost=c["special_boost"])
    eng = Engine(EngineConfig(hidden=cfg.hidden, layers=cfg.layers, n_heads=cfg.n_heads, n_kv=cfg.n_kv,
                              head_dim=cfg.head_dim, inter=cfg.inter, vocab=cfg.vocab, n_vq=cfg.n_vq,
                              rope_theta=cfg.rope_theta, max_batch=4, max_ctx=256, max_prefill_tokens=512), 0)
    try:
        eng.load_state_dict({k: torch.from_numpy(v) for k, v in W.items()})
        out = eng.generate_ids(torch.from_numpy(ids), torch.from_numpy(mask), c["steps"],
                               sampling_params(text_temperature=0, audio_temperature=0,
                                               audio_repetition_penalty=c["penalty"])).cpu().numpy()
    finally:
        eng.close()
    starts = O.find_last_equal_C(ids[..., 0], cfg.im_start_token_id) + 3
    # the reference's logits along its own trajectory (the oracle in the case's dtype)
    Wr = W if c["dtype"] == "bf16" else O.make_weights(cfg, c["seed"], dtype=c["dtype"],
                                                      special_boost=c["special_boost"])
    tr = O.StepTrace()
    O.generate(Wr, cfg, ids, mask, max_new_tokens=c["steps"], text_temperature=0, audio_temperature=0,
               audio_repetition_penalty=c["penalty"], dtype=c["dtype"], trace=tr)
    rows = []
    for b in range(B):
        want = g[f"{name}/out{b}"]
        got = out[b, starts[b]:]
        n_pre = ids.shape[1] - starts[b]  # prompt rows inside the reference's output slice
        d = first_divergence(got[:len(want)], want)
        if d is None and len(got) >= len(want):
            rows.append(dict(row=b, first_divergence=None))
            continue
        assert d is not None, (name, b, "HIP stopped early with an equal prefix")
        assert d >= n_pre, (name, b, "prompt rows differ")
        step = d - n_pre
        assert step < len(tr.text_logits), (name, b, step)
        chans = np.nonzero(got[d] != want[d])[0]
        tl, al = tr.text_logits[step][b], tr.audio_logits[step][b]
        worst = None
        for j in chans:
            r = tl if j == 0 else al[j - 1, :1024].copy()
            if j > 0 and c["penalty"] != 1.0:
                # the batch-wide penalty set of the reference (inference_utils.py:79-88): every row's
                # history of channel 1 (j == 1) or of channels >= 2, prompt included, up to this step
                hist = np.concatenate([np.concatenate([ids[bb, :starts[bb]], g[f"{name}/out{bb}"][:(ids.shape[1] - starts[bb]) + step]])
                                       for bb in range(B)])
                h = np.unique(hist[:, 1] if j == 1 else hist[:, 2:])
                h = h[h < 1024]
                r[h] = np.where(r[h] > 0, r[h] / c["penalty"], r[h] * c["penalty"])
            f = r[np.isfinite(r)]
            scale = float(np.abs(f).max())
            tol = 8 * float(ulp_bf16(scale)) if c["dtype"] == "bf16" else 0.03 * scale
            m = margin_top2(r)
            if worst is None or m - tol > worst[1] - worst[2]:
                worst = (int(j), m, tol)
        rows.append(dict(row=b, first_divergence=int(step), channel=worst[0], ref_margin=worst[1], tol=worst[2]))
        assert worst[1] <= worst[2], (name, b, step, worst)
    print("REFIDS " + json.dumps(dict(case=name, dtype=c["dtype"], n_vq=c["n_vq"], B=B, steps=c["steps"],
                                      rows=rows)))
