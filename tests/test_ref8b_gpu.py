"""The launches that carry the bench numbers, pinned DIRECTLY to the reference at the 8B layer shape.

`tests/golden/make_golden_8b.py` ran the reference's own `MossTTSDelayModel`
(`/root/reference/moss_tts_delay/modeling_moss_tts.py:159-300`, `generate` `:392-525`) in bf16 at
h 4096, 32 / 8 heads x 128, I 12,288, the full 151,936-row text head, 2 layers, n_vq 32 (16 for the
TTSD case), greedy, and committed its ids, its last-position logits of every forward call (bf16 bits)
and the processed top-2 of every sampled (row, channel).  Here the HIP engine gets the same weights --
rebuilt on the device from the seeds (`oracle.moss_delay.weight_fill_plan` + `mtts_k_fill_uniform`,
bit-identical to the generator's `make_weights`) -- and runs:
  * greedy `generate()` (hipGraph steps): ids equal to the reference's, or the first divergence on a
    reference near-tie: its own processed top-2 margin in the diverging channel <= 8 bf16 ulps of the
    row scale (both sides are bf16 engines; a channel the reference did not sample may never differ);
  * teacher-forced forwards along the reference's trajectory: every call's logits (audio heads whole,
    the text head at 2,400 recorded rows) within the band below of the reference's, argmax equal
    where the reference's top-2 margin is clear.
Paths: B=1 -> the persistent launch (pse.hip) and the per-op launches (MTTS_PSE=0); B=4 -> pse4.hip
and the per-op launches (MTTS_PSE4=0); the 2,117-row TTSD prompt -> one-chunk prefill (attn_prefill32,
gemm5 long forms) then the launch's long-context form at 2.1 K keys, the per-op launches, and a
1,024-token chunked prefill.  Per-op vectors at D = 128 pin RMSNorm (4,096 / 12,288), the RoPE tables
and q/k norm + RoPE up to position 9,599, and SDPA (GQA 4:1, left pads, 2,100 keys; the 32-token
prefill kernel, a decode query through both attention kernels) to the transformers modules.

Band: |HIP - reference| <= TOL_ULPS bf16 ulps of the row's max |logit|.  TOL_ULPS = 4, half the band the
oracle-vs-HIP tests use at this shape: measured against these reference logits the engine sits within
1.0-1.75 ulps on every path, so a divergence of greedy ids can only come from a
reference margin <= 2 x 1.75 ulps, and 4 ulps bounds it."""
import ctypes
import json
import os

import numpy as np
import pytest

from oracle import bf16 as B16
from oracle import moss_delay as O
from tests.golden import ref8b_inputs as R
from tests.parity_util import first_divergence, ulp_bf16

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
HERE = os.path.dirname(os.path.abspath(__file__))
TOL_ULPS = 4


@pytest.fixture(scope="module")
def g8():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    g = np.load(os.path.join(HERE, "golden", "golden_8b.npz"), allow_pickle=False)
    with open(os.path.join(HERE, "golden", "cases_8b.json")) as f:
        cases = json.load(f)
    return g, cases


def P(t):
    return ctypes.c_void_p(t.data_ptr())


def case_cfg(c):
    return O.Cfg(layers=c["layers"], n_vq=c["n_vq"])


_W = {}


def device_weights(c):
    """the generator's make_weights(cfg, seed, "bf16", special_boost) rebuilt on the device"""
    from moss_tts_amd import _native as N
    key = (c["n_vq"], c["seed"], c["special_boost"])
    if key in _W:
        return _W[key]
    _W.clear()
    torch.cuda.empty_cache()
    out = {}
    for name, shape, tid, sc, off, patch in O.weight_fill_plan(case_cfg(c), c["seed"], special_boost=c["special_boost"]):
        t = torch.empty(shape, dtype=torch.bfloat16, device="cuda")
        N.call("mtts_k_fill_uniform", P(t), t.numel(), c["seed"], tid, ctypes.c_float(sc), ctypes.c_float(off), None)
        for r, v in patch.items():
            t[r] = torch.from_numpy(B16.rnd(v)).to(torch.bfloat16).cuda()
        out[name] = t
    torch.cuda.synchronize()
    _W[key] = out
    return out


def make_engine(c, path, T, max_prefill=4096):
    from moss_tts_amd.engine import Engine, EngineConfig
    env = {"per_op": {"MTTS_PSE": "0", "MTTS_PSE4": "0"}}.get(path, {})
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        eng = Engine(EngineConfig(layers=c["layers"], n_vq=c["n_vq"], max_batch=c["B"], max_ctx=T + c["steps"] + 64,
                                  max_prefill_tokens=max_prefill), 0)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k)
            else:
                os.environ[k] = v
    if path == "persistent":
        if c["B"] == 1 and not eng.pse_active():
            eng.close()
            pytest.skip("batch-1 persistent launch unsupported on this device")
        if c["B"] == 4 and not eng.pse4_active():
            eng.close()
            pytest.skip("batch-4 persistent launch unsupported on this device")
    eng.load_state_dict(device_weights(c))
    return eng


def reference_trajectory(g, c, name):
    """the reference's generation_ids [B, T + n, C] and the attention mask its forward calls saw"""
    ids, mask = g[name + "/input_ids"], g[name + "/mask"]
    B, T = ids.shape[:2]
    full = np.stack([np.concatenate([ids[b, :T - c["start_len"][b]], g[f"{name}/out{b}"]]) for b in range(B)])
    cfg = case_cfg(c)
    # generate appends ~is_stopping after each step (`:512`); a row stops on im_end (`:473`)
    stopped = np.cumsum(full[:, T:, 0] == cfg.im_end_token_id, axis=1) > 0
    mfull = np.concatenate([mask.astype(np.uint8), (~stopped).astype(np.uint8)], axis=1)
    return full, mfull


def band(got, want, what):
    fin = np.isfinite(want)
    assert (np.isfinite(got) == fin).all(), what
    scale = np.abs(want[fin]).max()
    u = float(ulp_bf16(scale))
    err = float(np.abs(got[fin] - want[fin]).max())
    assert err <= TOL_ULPS * u, (what, err / u, float(scale))
    srt = np.sort(want[fin])
    if srt[-1] - srt[-2] > 2 * TOL_ULPS * u:
        assert int(np.argmax(np.where(fin, got, -np.inf))) == int(np.argmax(np.where(fin, want, -np.inf))), what
    return err / u


def check_ids(g, c, name, out):
    """HIP ids vs the reference's; the first divergence must sit on a reference near-tie"""
    ids = g[name + "/input_ids"]
    T = ids.shape[1]
    top = g[name + "/sampled_top2"]
    rows = []
    for b in range(c["B"]):
        # generate returns (start_length, generation_ids[start:]) with start = the last im_start + 3
        # (`:518-525`), i.e. the last start_length prompt rows and everything generated
        n_pre = c["start_len"][b]
        want = g[f"{name}/out{b}"]
        got = out[b, T - n_pre:]
        d = first_divergence(got[:len(want)], want)
        if d is None and len(got) >= len(want):
            rows.append(None)
            continue
        assert d is not None, (name, b, "HIP stopped early with an equal prefix")
        assert d >= n_pre, (name, b, "prompt rows differ")
        step = d - n_pre
        margins = []
        for j in np.nonzero(got[d] != want[d])[0]:
            t1idx, t1, t2, scale = top[step, b, j]
            assert np.isfinite(t1), (name, b, step, int(j), "the reference did not sample this channel")
            margins.append((t1 - t2) / float(ulp_bf16(scale)))
            assert margins[-1] <= TOL_ULPS, (name, b, step, int(j), t1 - t2, scale)
        worst = max(margins)
        rows.append((step, round(float(worst), 2)))
    print(f"REF8B ids {name}: first divergence per row (step, reference top-2 margin in ulps) {rows} "
          f"of {c['steps']} steps")
    return rows


CASES = [("r8_clone_b1", "persistent"), ("r8_clone_b1", "per_op"), ("r8_ragged_b4", "persistent"),
         ("r8_ragged_b4", "per_op"), ("r8_long_nvq16", "persistent"), ("r8_long_nvq16", "per_op"),
         ("r8_long_nvq16", "chunked")]


@pytest.mark.parametrize("name,path", CASES)
def test_ref8b_generate_ids(g8, name, path):
    from moss_tts_amd.engine import sampling_params
    g, cases = g8
    c = cases[name]
    ids, mask = g[name + "/input_ids"], g[name + "/mask"]
    eng = make_engine(c, path, ids.shape[1], max_prefill=1024 if path == "chunked" else 4096)
    try:
        out = eng.generate_ids(torch.from_numpy(ids), torch.from_numpy(mask), c["steps"],
                               sampling_params(text_temperature=0, audio_temperature=0)).cpu().numpy()
        if path == "persistent" and c["B"] == 1:
            assert eng.pse_active(), "the launch must not have fallen back"
    finally:
        eng.close()
    check_ids(g, c, name, out)


@pytest.mark.parametrize("name,path", CASES)
def test_ref8b_teacher_forced_logits(g8, name, path):
    g, cases = g8
    c = cases[name]
    cfg = case_cfg(c)
    V, A = cfg.vocab, cfg.audio_vocab + 1
    ids = g[name + "/input_ids"]
    T = ids.shape[1]
    full, mfull = reference_trajectory(g, c, name)
    sel = g[name + "/text_sel"]
    rt = B16.from_bits(g[name + "/raw_text_bits"])
    ra = B16.from_bits(g[name + "/raw_audio_bits"])
    eng = make_engine(c, path, T, max_prefill=1024 if path == "chunked" else 4096)
    worst = 0.0
    try:
        for s in range(c["n_forward"]):
            if s == 0:
                x, past = full[:, :T], 0
            else:
                x, past = full[:, T + s - 1:T + s], T + s - 1
            lg = eng.forward(torch.from_numpy(np.ascontiguousarray(x)), torch.from_numpy(mfull[:, :past + x.shape[1]].copy()),
                             past).float().cpu().numpy()
            for b in range(c["B"]):
                worst = max(worst, band(lg[b][sel], rt[s, b], (name, s, b, "text")))
                for j in range(cfg.n_vq):
                    worst = max(worst, band(lg[b][V + j * A:V + (j + 1) * A], ra[s, b, j], (name, s, b, j)))
        eng.pse_check()
    finally:
        eng.close()
    print(f"REF8B logits {name} [{path}]: {c['n_forward']} forward calls, worst {worst:.2f} bf16 ulps of the row scale")


# ---------------- per-op vectors at D = 128 ----------------
def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a, np.float32)).to(torch.bfloat16).cuda()


@pytest.mark.parametrize("H", [4096, 12288])
def test_ref8b_rmsnorm(g8, H):
    from moss_tts_amd import _native as N
    g, _ = g8
    x, w = R.rmsnorm_inputs(H)
    want = B16.from_bits(g[f"op8_rmsnorm_{H}/y_bits"])
    xd, wd = dev(x), dev(w)
    y = torch.zeros(x.shape, dtype=torch.bfloat16, device="cuda")
    N.call("mtts_k_rmsnorm", P(xd), 0, H, P(wd), P(y), x.shape[0], H, ctypes.c_float(1e-6), None)
    torch.cuda.synchronize()
    got = y.float().cpu().numpy()
    assert (np.abs(got - want) <= ulp_bf16(want) + 1e-30).all()
    assert np.mean(got == want) > 0.99


@pytest.mark.parametrize("past", R.ROPE_PASTS)
def test_ref8b_qk_norm_rope(g8, past):
    """the engine's RoPE table (mtts_rope_table) and the q/k norm + RoPE + cache append kernel
    against Qwen3RotaryEmbedding + Qwen3RMSNorm + apply_rotary_pos_emb at positions up to 9,599"""
    from moss_tts_amd import _native as N
    g, _ = g8
    S, D, Hq, Hkv = R.ROPE_S, 128, 32, 8
    Cmax = (past + S + 63) // 64 * 64
    cs = np.zeros((Cmax, D), np.uint16)
    sn = np.zeros((Cmax, D), np.uint16)
    N.call("mtts_rope_table", ctypes.c_float(1e6), D, Cmax, cs.ctypes.data_as(ctypes.c_void_p),
           sn.ctypes.data_as(ctypes.c_void_p))
    for tab, key in ((cs, "cos"), (sn, "sin")):
        ref = g[f"op8_rope_{past}/{key}_bits"]
        mine = tab[past:past + S]
        assert np.mean(mine == ref) > 0.99, key
        assert np.abs(B16.from_bits(mine) - B16.from_bits(ref)).max() <= 2 ** -8, key
    qkv, qn, kn = R.qk_inputs(past)
    keep = [dev(a) for a in (qkv, qn, kn)]
    ct = torch.from_numpy(cs.view(np.int16)).cuda()
    st = torch.from_numpy(sn.view(np.int16)).cuda()
    kc = torch.zeros(1, Hkv, Cmax, D, dtype=torch.bfloat16, device="cuda")
    vc = torch.zeros(1, Hkv, D, Cmax, dtype=torch.bfloat16, device="cuda")
    qo = torch.zeros(S, Hq * D, dtype=torch.bfloat16, device="cuda")
    pos = torch.tensor([past], dtype=torch.int32, device="cuda")
    N.call("mtts_k_qk_norm_rope", P(keep[0]), P(qo), P(kc), P(vc), P(keep[1]), P(keep[2]), P(ct), P(st), P(pos),
           S, S, Hq, Hkv, D, Cmax, ctypes.c_float(1e-6), None)
    torch.cuda.synchronize()
    q_ref = B16.from_bits(g[f"op8_rope_{past}/q_bits"])  # [Hq, S, D]
    k_ref = B16.from_bits(g[f"op8_rope_{past}/k_bits"])  # [Hkv, S, D]
    q = qo.float().cpu().numpy().reshape(S, Hq, D).transpose(1, 0, 2)
    k = kc.float().cpu().numpy()[0, :, past:past + S]
    for got, want in ((q, q_ref), (k, k_ref)):
        # the rotation is a difference of two products: the band is taken against the head's scale
        scale = np.maximum(np.abs(want), np.abs(want).max(axis=-1, keepdims=True))
        assert (np.abs(got - want) <= ulp_bf16(scale) + 1e-30).all()
        assert np.mean(got == want) > 0.97
    assert (vc.float().cpu().numpy()[0, :, :, past:past + S].transpose(0, 2, 1) ==
            qkv.reshape(S, 48, D)[:, 40:].transpose(1, 0, 2)).all()


@pytest.mark.parametrize("S,kernel", [(64, "prefill"), (1, "prefill"), (1, "decode")])
def test_ref8b_sdpa(g8, S, kernel):
    """sdpa_attention_forward (GQA 4:1, causal, a 45-key left pad on row 1, 2,100 keys) against the
    32-token LDS-staged prefill kernel (S = 64), and a decode query through the prefill kernel and the
    split-K decode attention"""
    from moss_tts_amd import _native as N
    g, _ = g8
    q, k, v, km, qpos = R.sdpa_inputs(S)
    B, Hq, Hkv, D, C = R.SDPA_B, R.SDPA_HQ, R.SDPA_HKV, 128, R.SDPA_C
    Cmax = (C + 63) // 64 * 64
    kc0 = np.full((B, Hkv, Cmax, D), np.nan, np.float32)
    vc0 = np.full((B, Hkv, D, Cmax), np.nan, np.float32)
    kc0[:, :, :C] = k
    vc0[:, :, :, :C] = v.transpose(0, 1, 3, 2)
    mask = np.zeros((B, Cmax), np.uint8)
    mask[:, :C] = km
    qd = dev(q.transpose(0, 2, 1, 3).reshape(B * S, Hq * D))
    kc, vc, md = dev(kc0), dev(vc0), torch.from_numpy(mask).cuda()
    pos = torch.tensor([C - S], dtype=torch.int32, device="cuda")
    out = torch.zeros(B * S, Hq * D, dtype=torch.bfloat16, device="cuda")
    if kernel == "prefill":
        N.call("mtts_k_attention_prefill", P(qd), P(kc), P(vc), P(md), P(pos), P(out), B * S, S, Hq, Hkv, D, Cmax,
               None)
    else:
        n_split = (C + 255) // 256
        ws = torch.zeros(N.load().mtts_k_attention_ws_bytes(B * S, Hq, D, n_split) // 4 + 1, dtype=torch.float32,
                         device="cuda")
        N.call("mtts_k_attention", P(qd), P(kc), P(vc), P(md), P(pos), P(out), P(ws), B * S, S, Hq, Hkv, D, Cmax,
               256, n_split, None)
    torch.cuda.synchronize()
    want = B16.from_bits(g[f"op8_sdpa_{S}/out_bits"])  # [B, S, Hq, D]
    got = out.float().cpu().numpy().reshape(B, S, Hq, D)
    assert np.isfinite(got).all()
    err = np.abs(got - want)
    assert (err <= 4 * 2.0 ** -8 * np.maximum(np.abs(want), 1.0)).all(), float(err.max())
