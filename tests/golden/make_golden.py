#!/usr/bin/env python3
"""Generate golden vectors by running the REFERENCE classes in this container.

Run from the repo root (needs /root/reference, which exists only in the build
container, never on the GPU box):

    python tests/golden/make_golden.py

What it does (SURVEY.md §8c golden-vector plan):
* builds tiny `MossTTSDelayModel`s (`moss_tts_delay/modeling_moss_tts.py:159`)
  whose weights come from the portable splitmix64 PRNG in `oracle/prng.py`
  (so only seeds travel; the GPU box regenerates identical weights);
* runs the reference `generate()` greedy (and with repetition penalty) on
  synthetic prompts (direct / clone / continuation / ragged batch), fp32 and
  bf16, recording the token ids and last-position logits of the first steps;
* records per-op vectors from the transformers Qwen3 modules the backbone
  uses (RMSNorm, RoPE, attention with a padding mask, SwiGLU MLP);
* records the processor statics (delay / de-delay / left pad / segment split).

Outputs: tests/golden/*.npz (allow_pickle=False) + tests/golden/cases.json.
"""
import json
import os
import sys
import types

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, "/root/reference")

import torch  # noqa: E402

torch.manual_seed(0)
torch.set_num_threads(8)

from oracle import moss_delay as O  # noqa: E402
from oracle import bf16 as B16  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden")


def ref_model(cfg, W, dtype):
    from transformers import Qwen3Config
    from moss_tts_delay.configuration_moss_tts import MossTTSDelayConfig
    from moss_tts_delay.modeling_moss_tts import MossTTSDelayModel
    lc = Qwen3Config(vocab_size=cfg.vocab, hidden_size=cfg.hidden, intermediate_size=cfg.inter,
                     num_hidden_layers=cfg.layers, num_attention_heads=cfg.n_heads,
                     num_key_value_heads=cfg.n_kv, head_dim=cfg.head_dim,
                     rope_theta=cfg.rope_theta, rms_norm_eps=cfg.eps,
                     max_position_embeddings=4096)
    mc = MossTTSDelayConfig(language_config=lc, n_vq=cfg.n_vq)
    m = MossTTSDelayModel(mc).eval()
    sd = {k: torch.from_numpy(v.copy()) for k, v in W.items()}
    missing, unexpected = m.load_state_dict(sd, strict=False)
    missing = [k for k in missing if "rotary" not in k]
    assert not missing and not unexpected, (missing, unexpected)
    if dtype == "bf16":
        m = m.to(torch.bfloat16)
        # `.to(bf16)` also rounds the rotary inv_freq buffer; the deployment path
        # (`from_pretrained(..., torch_dtype=bf16)`, clis/moss_tts_app.py:95-107)
        # keeps it fp32 -- restore that so the fixtures match what users run.
        rot = m.language_model.rotary_emb
        inv, _ = rot.compute_default_rope_parameters(m.language_model.config)
        rot.inv_freq = inv.to(torch.float32)
    return m


# --------------------------------------------------------------------------
# synthetic prompts (no tokenizer in the container: raw ids)
# --------------------------------------------------------------------------
def prompt_direct(cfg, rng, n_text):
    t = [cfg.im_start_token_id, 872, 198] + list(rng.integers(200, 20000, n_text)) + \
        [cfg.im_end_token_id, 198, cfg.im_start_token_id, 77091, 198]
    ids = np.full((len(t), cfg.n_vq + 1), cfg.audio_pad_code, np.int64)
    ids[:, 0] = t
    return ids


def prompt_clone(cfg, rng, n_text, n_frames):
    """user turn holding a reference-audio block (`processing_moss_tts.py:453-461`,
    `:539-641` with role=user: slots are audio_user_slot), then the assistant header."""
    codes = rng.integers(0, cfg.audio_vocab, (n_frames, cfg.n_vq)).astype(np.int64)
    dl = O.apply_delay_pattern(codes, cfg.audio_pad_code)
    pre = [cfg.im_start_token_id, 872, 198] + list(rng.integers(200, 20000, 4))
    rows = []
    for t in pre:
        rows.append([t] + [cfg.audio_pad_code] * cfg.n_vq)
    rows.append([cfg.audio_start_token_id] + [cfg.audio_pad_code] * cfg.n_vq)
    for r in dl:
        rows.append([cfg.audio_user_slot_token_id] + list(r))
    rows.append([cfg.audio_end_token_id] + [cfg.audio_pad_code] * cfg.n_vq)
    post = list(rng.integers(200, 20000, n_text)) + [cfg.im_end_token_id, 198,
                                                     cfg.im_start_token_id, 77091, 198]
    for t in post:
        rows.append([t] + [cfg.audio_pad_code] * cfg.n_vq)
    return np.array(rows, np.int64)


def prompt_continuation(cfg, rng, n_text, n_frames):
    """assistant turn already started with audio (mode='continuation',
    truncation drops the last n_vq-1 delayed rows, `processing_moss_tts.py:619-622`)."""
    codes = rng.integers(0, cfg.audio_vocab, (n_frames, cfg.n_vq)).astype(np.int64)
    dl = O.apply_delay_pattern(codes, cfg.audio_pad_code)[: n_frames]
    rows = []
    pre = [cfg.im_start_token_id, 872, 198] + list(rng.integers(200, 20000, n_text)) + \
        [cfg.im_end_token_id, 198, cfg.im_start_token_id, 77091, 198]
    for t in pre:
        rows.append([t] + [cfg.audio_pad_code] * cfg.n_vq)
    rows.append([cfg.audio_start_token_id] + [cfg.audio_pad_code] * cfg.n_vq)
    for r in dl:
        rows.append([cfg.audio_assistant_gen_slot_token_id] + list(r))
    return np.array(rows, np.int64)


# --------------------------------------------------------------------------
def run_generate(m, ids, mask, steps, dtype, penalty=1.0, capture=4):
    """Reference generate(), greedy; captures last-position logits of the first
    `capture` forward calls."""
    logs = []
    orig = m.forward

    def fwd(*a, **k):
        out = orig(*a, **k)
        if len(logs) < capture:
            logs.append([l[:, -1, :].float().numpy().copy() for l in out.logits])
        return out

    m.forward = fwd
    try:
        res = m.generate(torch.from_numpy(ids), torch.from_numpy(mask), max_new_tokens=steps,
                         text_temperature=0, audio_temperature=0,
                         audio_repetition_penalty=penalty)
    finally:
        m.forward = orig
    return res, logs


def main():
    cases = {}
    arrays = {}

    specs = [
        # name, n_vq, seed, dtype, kind, B, steps, penalty, special_boost
        ("g_nvq4_fp32", 4, 11, "fp32", "mixed", 3, 48, 1.0, 2.0),
        ("g_nvq4_bf16", 4, 11, "bf16", "mixed", 3, 48, 1.0, 2.0),
        ("g_nvq4_stop_fp32", 4, 14, "fp32", "mixed", 3, 48, 1.0, 1.6),
        ("g_nvq16_fp32", 16, 12, "fp32", "mixed", 3, 64, 1.0, 2.0),
        ("g_nvq16_bf16", 16, 14, "bf16", "mixed", 3, 64, 1.0, 2.0),
        ("g_nvq32_fp32", 32, 13, "fp32", "mixed", 3, 64, 1.0, 2.0),
        ("g_nvq32_bf16", 32, 13, "bf16", "mixed", 3, 64, 1.0, 2.0),
        ("g_nvq4_pen_fp32", 4, 11, "fp32", "mixed", 3, 48, 1.1, 2.0),
        ("g_nvq4_b1_fp32", 4, 15, "fp32", "continuation", 1, 40, 1.0, 2.0),
    ]
    for name, n_vq, seed, dtype, kind, B, steps, pen, sb in specs:
        cfg = O.tiny_cfg(n_vq=n_vq)
        W = O.make_weights(cfg, seed, dtype=dtype, special_boost=sb)
        rng = np.random.default_rng(seed + 1000)
        if kind == "continuation":
            seqs = [prompt_continuation(cfg, rng, 5, 6)]
        else:
            seqs = [prompt_direct(cfg, rng, 7), prompt_clone(cfg, rng, 5, 6),
                    prompt_continuation(cfg, rng, 3, 5)][:B]
        ids, mask = O.left_pad(seqs, cfg.pad_token_id, cfg.audio_pad_code)
        m = ref_model(cfg, W, dtype)
        res, logs = run_generate(m, ids, mask, steps, dtype, penalty=pen)
        out_ids = [r[1].numpy() for r in res]
        starts = [int(r[0]) for r in res]
        cases[name] = dict(n_vq=n_vq, seed=seed, dtype=dtype, B=B, steps=steps, penalty=pen, special_boost=sb,
                           starts=starts, n_out=[int(x.shape[0]) for x in out_ids])
        arrays[name + "/input_ids"] = ids
        arrays[name + "/mask"] = mask
        for b, o in enumerate(out_ids):
            arrays[name + f"/out{b}"] = o
        for s, lg in enumerate(logs):
            t = lg[0]
            top = np.argsort(-t, axis=1, kind="stable")[:, :16]
            arrays[name + f"/step{s}_text_top_idx"] = top
            arrays[name + f"/step{s}_text_top_val"] = np.take_along_axis(t, top, 1)
            arrays[name + f"/step{s}_audio"] = np.stack(lg[1:], 1)
        print(name, "outputs", [x.shape for x in out_ids], "first text ids",
              [list(x[:, 0][:12]) for x in out_ids][:1])

    # ---------------- per-op vectors ----------------
    from transformers.models.qwen3 import modeling_qwen3 as q3
    rng = np.random.default_rng(7)
    x = rng.standard_normal((3, 5, 64)).astype(np.float32)
    w = (1 + 0.25 * rng.standard_normal(64)).astype(np.float32)
    for dt, tdt in (("fp32", torch.float32), ("bf16", torch.bfloat16)):
        xx = B16.rnd(x) if dt == "bf16" else x
        ww = B16.rnd(w) if dt == "bf16" else w
        n = q3.Qwen3RMSNorm(64, eps=1e-6)
        n.weight.data = torch.from_numpy(ww).to(tdt)
        arrays[f"op_rmsnorm_{dt}/x"] = xx
        arrays[f"op_rmsnorm_{dt}/w"] = ww
        arrays[f"op_rmsnorm_{dt}/y"] = n(torch.from_numpy(xx).to(tdt)).float().detach().numpy()
        # rope
        cfg = O.tiny_cfg(rope_theta=1e6, head_dim=16)
        from transformers import Qwen3Config
        lc = Qwen3Config(hidden_size=64, num_attention_heads=4, num_key_value_heads=2, head_dim=16,
                         rope_theta=1e6)
        rot = q3.Qwen3RotaryEmbedding(lc)
        pos = torch.tensor([[0, 1, 7, 100, 1000, 4095]])
        cos, sin = rot(torch.zeros(1, dtype=tdt), pos)
        qq = rng.standard_normal((1, 4, 6, 16)).astype(np.float32)
        qq = B16.rnd(qq) if dt == "bf16" else qq
        qe, _ = q3.apply_rotary_pos_emb(torch.from_numpy(qq).to(tdt), torch.from_numpy(qq).to(tdt), cos, sin)
        arrays[f"op_rope_{dt}/pos"] = pos.numpy()[0]
        arrays[f"op_rope_{dt}/cos"] = cos.float().numpy()[0]
        arrays[f"op_rope_{dt}/sin"] = sin.float().numpy()[0]
        arrays[f"op_rope_{dt}/q"] = qq
        arrays[f"op_rope_{dt}/q_embed"] = qe.float().numpy()
        # mlp
        mlp_cfg = Qwen3Config(hidden_size=64, intermediate_size=96, hidden_act="silu")
        mlp = q3.Qwen3MLP(mlp_cfg)
        wg = (rng.standard_normal((96, 64)) * 0.125).astype(np.float32)
        wu = (rng.standard_normal((96, 64)) * 0.125).astype(np.float32)
        wd = (rng.standard_normal((64, 96)) * 0.1).astype(np.float32)
        if dt == "bf16":
            wg, wu, wd = B16.rnd(wg), B16.rnd(wu), B16.rnd(wd)
        mlp.gate_proj.weight.data = torch.from_numpy(wg)
        mlp.up_proj.weight.data = torch.from_numpy(wu)
        mlp.down_proj.weight.data = torch.from_numpy(wd)
        mlp = mlp.to(tdt)
        arrays[f"op_mlp_{dt}/x"] = xx
        arrays[f"op_mlp_{dt}/wg"] = wg
        arrays[f"op_mlp_{dt}/wu"] = wu
        arrays[f"op_mlp_{dt}/wd"] = wd
        arrays[f"op_mlp_{dt}/y"] = mlp(torch.from_numpy(xx).to(tdt)).float().detach().numpy()
        # attention with a padding mask, via the sdpa interface the backbone calls
        from transformers.integrations.sdpa_attention import sdpa_attention_forward
        Bq, Hq, Hk, S, C, D = 2, 4, 2, 3, 9, 16
        q = rng.standard_normal((Bq, Hq, S, D)).astype(np.float32)
        k = rng.standard_normal((Bq, Hk, C, D)).astype(np.float32)
        v = rng.standard_normal((Bq, Hk, C, D)).astype(np.float32)
        if dt == "bf16":
            q, k, v = B16.rnd(q), B16.rnd(k), B16.rnd(v)
        km = np.ones((Bq, C), bool)
        km[1, :3] = False  # left pads in row 1
        qpos = np.arange(C - S, C)
        allowed = km[:, None, None, :] & (np.arange(C)[None, None, None, :] <= qpos[None, None, :, None])
        am = torch.from_numpy(allowed)
        mod = types.SimpleNamespace(num_key_value_groups=Hq // Hk, is_causal=True, training=False)
        o, _ = sdpa_attention_forward(mod, torch.from_numpy(q).to(tdt), torch.from_numpy(k).to(tdt),
                                      torch.from_numpy(v).to(tdt), am, scaling=D ** -0.5)
        arrays[f"op_attn_{dt}/q"] = q
        arrays[f"op_attn_{dt}/k"] = k
        arrays[f"op_attn_{dt}/v"] = v
        arrays[f"op_attn_{dt}/key_mask"] = km
        arrays[f"op_attn_{dt}/q_pos"] = qpos
        arrays[f"op_attn_{dt}/out"] = o.float().numpy()  # [B, S, Hq, D]

    # ---------------- processor statics ----------------
    sys.modules.setdefault("torchaudio", types.ModuleType("torchaudio"))
    from moss_tts_delay.processing_moss_tts import MossTTSDelayProcessor as P
    rng = np.random.default_rng(3)
    codes = rng.integers(0, 1024, (7, 4)).astype(np.int64)
    dl = P.apply_delay_pattern(torch.from_numpy(codes), 1024).numpy()
    arrays["proc/codes"] = codes
    arrays["proc/delayed"] = dl
    arrays["proc/dedelayed"] = P.apply_de_delay_pattern(torch.from_numpy(dl)).numpy()
    # _pad is an instance method that only reads model_config
    fake = types.SimpleNamespace(model_config=types.SimpleNamespace(audio_pad_code=1024, pad_token_id=151643))
    seqs = [torch.from_numpy(rng.integers(0, 1000, (n, 5)).astype(np.int64)) for n in (4, 7, 1)]
    padded = P._pad(fake, seqs)
    for i, s in enumerate(seqs):
        arrays[f"proc/pad_in{i}"] = s.numpy()
    arrays["proc/pad_ids"] = padded["input_ids"].numpy()
    arrays["proc/pad_mask"] = padded["attention_mask"].numpy()
    # segment split of _parse_audio_codes (stub the codec decode to identity)
    seg_src = np.full((20, 4), 1024, np.int64)
    body = rng.integers(0, 1024, (6, 4))
    body2 = rng.integers(0, 1024, (4, 4))
    a = np.full((16, 4), 1024, np.int64)
    a[1:7] = body
    a[10:14] = body2
    seg_src = P.apply_delay_pattern(torch.from_numpy(a), 1024).numpy()
    fake2 = types.SimpleNamespace(model_config=fake.model_config, apply_de_delay_pattern=P.apply_de_delay_pattern,
                                  decode_audio_codes=lambda lst: [x.clone() for x in lst])
    # one segment: the reference splits correctly
    one = np.full((12, 4), 1024, np.int64)
    one[2:9] = rng.integers(0, 1024, (7, 4))
    one_src = P.apply_delay_pattern(torch.from_numpy(one), 1024).numpy()
    segs = P._parse_audio_codes(fake2, 0, torch.from_numpy(one_src))
    arrays["proc/seg1_src"] = one_src
    arrays["proc/seg1_n"] = np.array(len(segs))
    for i, s_ in enumerate(segs):
        arrays[f"proc/seg1_{i}"] = s_.numpy()
    # two segments: the reference passes break INDICES to torch.split (which
    # wants SIZES) and raises -- recorded as a quirk (parity notes)
    try:
        P._parse_audio_codes(fake2, 0, torch.from_numpy(seg_src))
        raised = 0
    except RuntimeError:
        raised = 1
    arrays["proc/seg2_src"] = seg_src
    arrays["proc/seg2_ref_raises"] = np.array(raised)

    np.savez_compressed(os.path.join(OUT, "golden.npz"), **arrays)
    with open(os.path.join(OUT, "cases.json"), "w") as f:
        json.dump(cases, f, indent=1, sort_keys=True)
    print("wrote", len(arrays), "arrays")


if __name__ == "__main__":
    main()
