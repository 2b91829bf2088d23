#!/usr/bin/env python3
"""Golden vectors for MossTTSLocal, from the REFERENCE's own modules in this container.

Run from the repo root (needs /root/reference, which exists only in the build container):

    python tests/golden/make_golden_local.py

The reference `generate()` (GenerationMixin + `CustomMixin._sample`,
`moss_tts_local/modeling_moss_tts.py:315-477`) does not run on the installed transformers
5.15, so the greedy loop of `_sample` (:377-456) is restated here around
the reference's modules, called exactly as `_sample` calls them:
  backbone    `model.model(...)` with a DynamicCache, `hidden_states[-1][:, -1]` (:384-390),
              with the `attention_mask` and `position_ids` that the installed GenerationMixin
              hands the forward (the reference forward takes `position_ids`, :536 / :656, so
              `generate` fills them, transformers/generation/utils.py:2564-2567):
              cumsum(mask) - 1 with pads set to 0 (:751-773), then last + 1 per step, the mask
              grown by ones (`_update_model_kwargs_for_generation`, :975-992); for a left-padded
              row the positions EXCLUDE its pads (the Delay path's include them)
  depth loop  `speech_embedding_to_local_mlp` (:395, :423), `local_transformer.layers[l]`
              + `local_transformer.norm` over the channel inputs so far (the body of
              `MossTTSLocalTransformer.forward`, :260-281, whose mask helper call fails on
              5.15), `local_to_speech_embedding_mlps[i]`, `layer_norm_before_lm_heads[i]`,
              `lm_heads[i]` with the pad column -inf for i >= 1 (:402-413), argmax (:419)
  stop        eos on channel 0, finished rows filled with eos / pad (:429-441)
Weights come from the portable PRNG (oracle/prng.py), so only seeds travel.
Outputs: tests/golden/golden_local.npz (allow_pickle=False) + cases_local.json.
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
import transformers  # noqa: E402,F401

sys.modules.setdefault("torchaudio", types.ModuleType("torchaudio"))

from oracle import moss_local as L  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden")


def ref_model(cfg, W, dtype):
    from transformers import Qwen3Config
    from moss_tts_local.configuration_moss_tts import MossTTSDelayConfig
    from moss_tts_local.modeling_moss_tts import MossTTSDelayModel
    lc = Qwen3Config(vocab_size=cfg.vocab, hidden_size=cfg.hidden, intermediate_size=cfg.inter,
                     num_hidden_layers=cfg.layers, num_attention_heads=cfg.n_heads, num_key_value_heads=cfg.n_kv,
                     head_dim=cfg.head_dim, rope_theta=cfg.rope_theta, rms_norm_eps=cfg.eps,
                     max_position_embeddings=4096)
    mc = MossTTSDelayConfig(language_config=lc, n_vq=cfg.n_vq, additional_mlp_ffn_hidden_size=cfg.mlp_ffn,
                            local_ffn_hidden_size=cfg.local_inter, local_hidden_size=cfg.local_hidden,
                            local_num_layers=cfg.local_layers)
    m = MossTTSDelayModel(mc).eval()
    sd = {k: torch.from_numpy(v.copy()) for k, v in W.items()}
    missing, unexpected = m.load_state_dict(sd, strict=False)
    # the backbone's own embed_tokens is never used (inputs_embeds come from embedding_list)
    missing = [k for k in missing if "rotary" not in k and k != "model.language_model.embed_tokens.weight"]
    assert not missing and not unexpected, (missing, unexpected)
    if dtype == "bf16":
        m = m.to(torch.bfloat16)
        rot = m.model.language_model.rotary_emb  # keep fp32 inv_freq like from_pretrained(torch_dtype=bf16)
        inv, _ = rot.compute_default_rope_parameters(m.model.language_model.config)
        rot.inv_freq = inv.to(torch.float32)
    return m


@torch.no_grad()
def ref_generate(m, cfg, ids, max_new, n_vq_inf, dtype, mask0=None):
    from transformers.cache_utils import DynamicCache
    dt = torch.bfloat16 if dtype == "bf16" else torch.float32
    B, T, C = ids.shape
    n_ch = min(C, 1 + n_vq_inf)
    cur = torch.from_numpy(ids)
    mask = torch.ones(B, T, dtype=torch.long) if mask0 is None else torch.from_numpy(mask0.astype(np.int64))
    pos = mask.cumsum(-1) - 1
    pos = pos.masked_fill(mask == 0, 0)
    cache = DynamicCache()
    unfinished = torch.ones(B, dtype=torch.long)
    step_in = cur
    logits_trace = []
    for step in range(max_new):
        out = m.model(input_ids=step_in, attention_mask=mask, position_ids=pos[:, -step_in.shape[1]:],
                      past_key_values=cache, use_cache=True, output_hidden_states=True, return_dict=True,
                      n_vq_for_inference=n_vq_inf)
        g = out.hidden_states[-1][:, -1, :]
        last = out.last_hidden_state[:, -1, :]
        assert torch.equal(g, last), "hidden_states[-1] is the final-normed state"
        local_inputs = torch.zeros(B, 0, cfg.local_hidden, dtype=dt)
        x = m.speech_embedding_to_local_mlp(g)
        toks = []
        for i in range(n_ch):
            local_inputs = torch.cat([local_inputs, x.unsqueeze(1)], dim=1)
            h = local_inputs
            for layer in m.local_transformer.layers:
                h = layer(h, attention_mask=None, position_ids=None, past_key_values=None, use_cache=False,
                          cache_position=None, position_embeddings=None)
                if isinstance(h, tuple):
                    h = h[0]
            h = m.local_transformer.norm(h)
            z = m.layer_norm_before_lm_heads[i](m.local_to_speech_embedding_mlps[i](h))
            lg = m.lm_heads[i](z[:, -1, :])
            if i != 0:
                lg[:, cfg.audio_pad_code] = -torch.inf
            if step < 2:
                logits_trace.append(lg.float().numpy())
            t = torch.argmax(lg, dim=-1)
            toks.append(t)
            x = m.speech_embedding_to_local_mlp(m.model.embedding_list[i](t))
        nxt = torch.zeros(B, C, dtype=torch.long)
        nxt[:, :n_ch] = torch.stack(toks, -1)
        for i in range(C):
            pddp = cfg.eos_token_id if i == 0 else cfg.audio_pad_code
            nxt[:, i] = nxt[:, i] * unfinished + pddp * (1 - unfinished)
        cur = torch.cat([cur, nxt[:, None, :]], 1)
        mask = torch.cat([mask, torch.ones(B, 1, dtype=torch.long)], 1)
        pos = torch.cat([pos, pos[:, -1:] + 1], 1)
        unfinished = unfinished & (nxt[:, 0] != cfg.eos_token_id).long()
        step_in = nxt[:, None, :]
        if unfinished.max() == 0:
            break
    return cur.numpy(), logits_trace


def prompt(cfg, rng, n_text, ref_frames):
    """user turn with an optional reference-audio block (codes aligned, no delay pattern,
    `moss_tts_local/processing_moss_tts.py:597-641`), then the assistant header + audio_start"""
    C = cfg.n_vq + 1
    rows = []

    def text(t):
        r = np.full(C, cfg.audio_pad_code, np.int64)
        r[0] = t
        rows.append(r)

    for t in [151644, 872, 198] + list(rng.integers(200, 20000, n_text)):
        text(t)
    if ref_frames:
        text(cfg.audio_start_token_id)
        for _ in range(ref_frames):
            r = np.empty(C, np.int64)
            r[0] = 151654
            r[1:] = rng.integers(0, 1024, cfg.n_vq)
            rows.append(r)
        text(cfg.audio_start_token_id + 1)
    for t in [151645, 198, 151644, 77091, 198, cfg.audio_start_token_id]:
        text(t)
    return np.stack(rows)


def left_pad(cfg, rows):
    """the processor's batch layout: left pads (channel 0 pad_token_id, codebooks
    audio_pad_code), attention mask False there"""
    T = max(r.shape[0] for r in rows)
    C = rows[0].shape[1]
    ids = np.full((len(rows), T, C), cfg.audio_pad_code, np.int64)
    ids[..., 0] = cfg.pad_token_id
    mask = np.zeros((len(rows), T), bool)
    for b, r in enumerate(rows):
        ids[b, T - r.shape[0]:] = r
        mask[b, T - r.shape[0]:] = True
    return ids, mask


def main():
    cases = {}
    arrays = {}
    specs = [
        # name, n_vq, n_vq_for_inference, B, seed, n_text, ref_frames, steps, eos_boost, dtype
        ("l_nvq4_bf16", 4, 4, 1, 21, 12, 0, 12, 0.0, "bf16"),
        ("l_nvq4_fp32", 4, 4, 1, 21, 12, 0, 12, 0.0, "fp32"),
        ("l_nvq8_clone_bf16", 8, 8, 2, 22, 10, 6, 10, 0.0, "bf16"),
        ("l_nvq8_depth4_bf16", 8, 4, 1, 23, 9, 4, 10, 0.0, "bf16"),
        ("l_nvq4_stop_fp32", 4, 4, 2, 24, 8, 0, 30, 40.0, "fp32"),
        # ragged (left-padded) batches, `MossTTSDelayProcessor._pad` (processing_moss_tts.py:415-436)
        ("l_nvq4_ragged_fp32", 4, 4, 3, 25, [5, 14, 9], [0, 3, 1], 12, 0.0, "fp32"),
        ("l_nvq8_ragged_bf16", 8, 8, 3, 26, [12, 4, 8], [2, 0, 5], 10, 0.0, "bf16"),
    ]
    for name, n_vq, nq_inf, B, seed, n_text, ref_frames, steps, eos_boost, dtype in specs:
        cfg = L.tiny_lcfg(n_vq=n_vq)
        W = L.make_weights(cfg, seed, dtype=dtype, eos_boost=eos_boost)
        rng = np.random.default_rng(seed)
        nt = n_text if isinstance(n_text, list) else [n_text] * B
        rf = ref_frames if isinstance(ref_frames, list) else [ref_frames] * B
        p = [prompt(cfg, rng, nt[b], rf[b]) for b in range(B)]
        ids, mask = left_pad(cfg, p)
        m = ref_model(cfg, W, dtype)
        out, lt = ref_generate(m, cfg, ids, steps, nq_inf, dtype, mask0=mask if not mask.all() else None)
        arrays[name + "/input_ids"] = ids
        if not mask.all():
            arrays[name + "/attention_mask"] = mask
        arrays[name + "/out"] = out
        for k, lg in enumerate(lt):
            arrays[f"{name}/logit{k}"] = lg.astype(np.float32)
        cases[name] = dict(n_vq=n_vq, n_vq_inf=nq_inf, B=B, seed=seed, steps=steps, eos_boost=eos_boost, dtype=dtype,
                           n_logits=len(lt), out_len=int(out.shape[1]), padded=bool(not mask.all()))
        print(name, ids.shape, "->", out.shape, flush=True)
    np.savez_compressed(os.path.join(OUT, "golden_local.npz"), **arrays)
    with open(os.path.join(OUT, "cases_local.json"), "w") as f:
        json.dump(cases, f, indent=1)


if __name__ == "__main__":
    main()
