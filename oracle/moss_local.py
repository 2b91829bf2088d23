"""CPU restatement of the MossTTSLocal decode path -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
module, as the checker.  The product path (moss_tts_amd/) never does.

Restates `moss_tts_local/modeling_moss_tts.py`:
  * backbone: Qwen3 (1.7B shape in production) over the sum of the 1+n_vq channel
    embeddings (`MosiTTSModel._prepare_multi_modal_inputs` :515-530, bf16 adds left to
    right, channels < 1 + n_vq_for_inference);
  * per frame (`CustomMixin._sample` :377-456): the last position's final-normed hidden
    state feeds `speech_embedding_to_local_mlp` (:395); for each channel i the local
    transformer (`MossTTSLocalTransformer` :178-292: Qwen3 decoder layers without RoPE,
    causal, no cache in the reference -- a position's output only depends on earlier
    positions, so recomputing or caching is the same function) runs over the channel
    inputs so far, then `local_to_speech_embedding_mlps[i]` -> `layer_norm_before_lm_heads[i]`
    (MossTTSRMSNorm: NO fp32 upcast, :34-44) -> `lm_heads[i]` (audio pad column -inf for
    i >= 1, :411-413); the chosen token's embedding goes through
    `speech_embedding_to_local_mlp` to become channel i+1's input (:421-423);
  * stop: channel 0 == eos (audio_end, 151653 in the README's GenerationConfig); finished
    rows emit eos / pad (:429-441); output (start_length, ids[last audio_start:]) (:471-477).

Parity pinning: tests/golden/make_golden_local.py runs the REFERENCE's own modules
(backbone `model.model`, the MLP adapters, `local_transformer.layers[i]` + `.norm`, the
norms and heads) in a restated greedy loop, because the reference `generate()` itself does
not run on the installed transformers 5.15.  Batches are unpadded in the
fixtures.  Positions (round 5): the reference forward takes `position_ids`, so the installed
GenerationMixin (transformers 5.15) fills them: cumsum(attention_mask) - 1 with pads set to 0
(`transformers/generation/utils.py:751-773`, called at :2564-2567), then last + 1 per step
(:975-985).  A left-padded row's positions therefore EXCLUDE its pads (the Delay model's
`generate` runs its own loop, whose positions include them).  `generate` below restates that;
the ragged fixtures (`l_*_ragged_*`) pin it to the reference's modules driven with those ids.
"""
from dataclasses import dataclass
from typing import Dict, List

import numpy as np

from . import bf16 as _bf
from . import prng
from .moss_delay import _Ctx, apply_rope, attention, find_last_equal_C, linear, rmsnorm, rope_cos_sin, silu


@dataclass
class LCfg:
    hidden: int = 2048
    layers: int = 28
    n_heads: int = 16
    n_kv: int = 8
    head_dim: int = 128
    inter: int = 6144
    vocab: int = 151936
    n_vq: int = 32
    audio_vocab: int = 1024
    rope_theta: float = 1_000_000.0
    eps: float = 1e-6
    local_hidden: int = 1536
    local_layers: int = 4
    local_inter: int = 8960
    mlp_ffn: int = 2048
    pad_token_id: int = 151643
    audio_start_token_id: int = 151652
    eos_token_id: int = 151653  # audio_end (README GenerationConfig)
    audio_pad_code: int = 1024


def tiny_lcfg(n_vq=4, **kw):
    c = LCfg(hidden=64, layers=2, n_heads=4, n_kv=2, head_dim=16, inter=128, n_vq=n_vq, rope_theta=10000.0,
             local_hidden=64, local_layers=2, local_inter=128, mlp_ffn=96)
    for k, v in kw.items():
        setattr(c, k, v)
    return c


def _layer_specs(prefix, H, cfg, I):
    D = cfg.head_dim
    return [
        (prefix + "self_attn.q_proj.weight", (cfg.n_heads * D, H), "lin"),
        (prefix + "self_attn.k_proj.weight", (cfg.n_kv * D, H), "lin"),
        (prefix + "self_attn.v_proj.weight", (cfg.n_kv * D, H), "lin"),
        (prefix + "self_attn.o_proj.weight", (H, cfg.n_heads * D), "lin"),
        (prefix + "self_attn.q_norm.weight", (D,), "norm"),
        (prefix + "self_attn.k_norm.weight", (D,), "norm"),
        (prefix + "mlp.gate_proj.weight", (I, H), "lin"),
        (prefix + "mlp.up_proj.weight", (I, H), "lin"),
        (prefix + "mlp.down_proj.weight", (H, I), "lin"),
        (prefix + "input_layernorm.weight", (H,), "norm"),
        (prefix + "post_attention_layernorm.weight", (H,), "norm"),
    ]


def weight_specs(cfg: LCfg):
    """Ordered (name, shape, kind) in the reference's state_dict names; tensor id = index."""
    H, LH, F = cfg.hidden, cfg.local_hidden, cfg.mlp_ffn
    C = 1 + cfg.n_vq
    s = [("model.embedding_list.0.weight", (cfg.vocab, H), "emb")]
    s += [(f"model.embedding_list.{i}.weight", (cfg.audio_vocab + 1, H), "emb") for i in range(1, C)]
    for l in range(cfg.layers):
        s += _layer_specs(f"model.language_model.layers.{l}.", H, cfg, cfg.inter)
    s.append(("model.language_model.norm.weight", (H,), "norm"))
    for l in range(cfg.local_layers):
        s += _layer_specs(f"local_transformer.layers.{l}.", LH, cfg, cfg.local_inter)
    s.append(("local_transformer.norm.weight", (LH,), "norm"))
    s += [("speech_embedding_to_local_mlp.gate_proj.weight", (F, H), "lin"),
          ("speech_embedding_to_local_mlp.up_proj.weight", (F, H), "lin"),
          ("speech_embedding_to_local_mlp.down_proj.weight", (LH, F), "lin")]
    for i in range(C):
        s += [(f"local_to_speech_embedding_mlps.{i}.gate_proj.weight", (F, LH), "lin"),
              (f"local_to_speech_embedding_mlps.{i}.up_proj.weight", (F, LH), "lin"),
              (f"local_to_speech_embedding_mlps.{i}.down_proj.weight", (H, F), "lin")]
    s += [(f"layer_norm_before_lm_heads.{i}.weight", (H,), "norm") for i in range(C)]
    s.append(("lm_heads.0.weight", (cfg.vocab, H), "head"))
    s += [(f"lm_heads.{i}.weight", (cfg.audio_vocab + 1, H), "head") for i in range(1, C)]
    return s


def _scale(kind, shape):
    if kind == "emb":
        return 1.0, 0.0
    if kind == "norm":
        return 0.25, 1.0
    return float(np.sqrt(3.0 / shape[-1])), 0.0  # uniform(-1,1) * s: var = 1/K (as oracle.moss_delay)


def make_weights(cfg: LCfg, seed: int, dtype="bf16", eos_boost=0.0) -> Dict[str, np.ndarray]:
    """Deterministic weights from the portable splitmix64 PRNG (twin: csrc/init.hip).
    eos_boost > 0 raises the text head's eos row so that greedy runs stop."""
    out = {}
    for tid, (name, shape, kind) in enumerate(weight_specs(cfg)):
        sc, off = _scale(kind, shape)
        w = prng.tensor(seed, tid, shape, sc, off)
        if name == "lm_heads.0.weight" and eos_boost:
            w[cfg.eos_token_id] *= np.float32(eos_boost)
        if dtype == "bf16":
            w = _bf.rnd(w)
        out[name] = w.astype(np.float32)
    return out


# ----------------------------------------------------------------------------
def moss_rmsnorm_bf16(ctx, x, w, eps):
    """`moss_tts_local/modeling_moss_tts.py:40-44` (MossTTSRMSNorm) in the model dtype,
    no fp32 upcast: norm = mean(x^2) (x^2 rounded, fp32 accumulation, rounded mean),
    rsqrt(norm + eps) rounded, x * r rounded, * weight rounded."""
    x2 = ctx.r(x * x)
    norm = ctx.r(np.mean(x2.astype(np.float32), axis=-1, keepdims=True, dtype=np.float32))
    r = ctx.r(np.float32(1.0) / np.sqrt(ctx.r(norm + np.float32(eps)).astype(np.float32)))
    return ctx.r(ctx.r(x * r) * w)


def swiglu_mlp(ctx, W, prefix, x):
    """MossTTSMLP (:87-95) / Qwen3MLP: down(silu(gate(x)) * up(x)), each op rounded."""
    g = linear(ctx, x, W[prefix + "gate_proj.weight"])
    u = linear(ctx, x, W[prefix + "up_proj.weight"])
    return linear(ctx, ctx.r(ctx.r(silu(g)) * u), W[prefix + "down_proj.weight"])


class Cache:
    def __init__(self, n):
        self.k = [None] * n
        self.v = [None] * n

    def update(self, i, k, v):
        if self.k[i] is None:
            self.k[i], self.v[i] = k, v
        else:
            self.k[i] = np.concatenate([self.k[i], k], axis=2)
            self.v[i] = np.concatenate([self.v[i], v], axis=2)
        return self.k[i], self.v[i]

    def length(self):
        return 0 if self.k[0] is None else self.k[0].shape[2]


def decoder_layer(ctx, W, cfg, prefix, h, cos, sin, cache, li, key_mask, q_pos):
    """Qwen3DecoderLayer (`TF/.../modeling_qwen3.py:294-323`); cos None = the local
    transformer's attention without positional embedding (:126-176)."""
    B, S, H = h.shape
    D = cfg.head_dim
    x = rmsnorm(ctx, h, W[prefix + "input_layernorm.weight"], cfg.eps)
    q = linear(ctx, x, W[prefix + "self_attn.q_proj.weight"]).reshape(B, S, cfg.n_heads, D)
    k = linear(ctx, x, W[prefix + "self_attn.k_proj.weight"]).reshape(B, S, cfg.n_kv, D)
    v = linear(ctx, x, W[prefix + "self_attn.v_proj.weight"]).reshape(B, S, cfg.n_kv, D)
    q = rmsnorm(ctx, q, W[prefix + "self_attn.q_norm.weight"], cfg.eps).transpose(0, 2, 1, 3)
    k = rmsnorm(ctx, k, W[prefix + "self_attn.k_norm.weight"], cfg.eps).transpose(0, 2, 1, 3)
    v = v.transpose(0, 2, 1, 3)
    if cos is not None:
        q = apply_rope(ctx, q, cos, sin)
        k = apply_rope(ctx, k, cos, sin)
    K, V = cache.update(li, k, v)
    a = attention(ctx, q, K, V, key_mask, q_pos, D ** -0.5)
    a = a.transpose(0, 2, 1, 3).reshape(B, S, cfg.n_heads * D)
    h = ctx.r(h + linear(ctx, a, W[prefix + "self_attn.o_proj.weight"]))
    x = rmsnorm(ctx, h, W[prefix + "post_attention_layernorm.weight"], cfg.eps)
    return ctx.r(h + swiglu_mlp(ctx, W, prefix + "mlp.", x))


def embed(ctx, W, cfg, ids, n_ch):
    """:515-530: zeros + embedding_list[i](ids[..., i]) for i < n_ch, each add rounded."""
    e = W["model.embedding_list.0.weight"][ids[..., 0]]
    for i in range(1, n_ch):
        e = ctx.r(e + W[f"model.embedding_list.{i}.weight"][ids[..., i]])
    return e


def hf_position_ids(attention_mask):
    """GenerationMixin._prepare_position_ids_for_generation (transformers 5.15,
    `generation/utils.py:751-773`): cumsum(mask) - 1, pads set to 0.  [B, T] int64."""
    m = np.asarray(attention_mask, bool)
    pos = np.cumsum(m, axis=-1) - 1
    return np.where(m, pos, 0).astype(np.int64)


def backbone(ctx, W, cfg, ids, attention_mask, cache, n_ch, position_ids=None):
    """Qwen3Model over the summed embeddings; returns the final-normed hidden state of the
    last position [B, H].  position_ids [B, S] (RoPE; None: arange(S) + past); the causal mask
    works on cache slots (arange(S) + past) and attention_mask [B, past + S]."""
    B, S, _ = ids.shape
    past = cache.length()
    pos = np.arange(S) + past
    if position_ids is None:
        cos, sin = rope_cos_sin(ctx, cfg, pos)
    else:
        rp = np.asarray(position_ids, np.int64).reshape(B, S)
        cos, sin = rope_cos_sin(ctx, cfg, rp.reshape(-1))
        cos = cos.reshape(B, 1, S, -1)
        sin = sin.reshape(B, 1, S, -1)
    h = embed(ctx, W, cfg, ids, n_ch)
    km = np.asarray(attention_mask, bool)
    for l in range(cfg.layers):
        h = decoder_layer(ctx, W, cfg, f"model.language_model.layers.{l}.", h, cos, sin, cache, l, km, pos)
    h = rmsnorm(ctx, h, W["model.language_model.norm.weight"], cfg.eps)
    return h[:, -1, :]


def local_frame(ctx, W, cfg, g, n_ch, trace=None, forced=None):
    """One frame of the depth loop (:390-423), greedy: g [B, H] backbone state -> tokens
    [B, n_ch].  The local transformer keeps a cache over the channel positions (exact:
    causal, no positional embedding).  forced [B, n_ch]: feed these tokens to the next
    channel instead of the argmax (teacher forcing, for parity checks)."""
    B = g.shape[0]
    cache = Cache(cfg.local_layers)
    x = swiglu_mlp(ctx, W, "speech_embedding_to_local_mlp.", g)  # [B, LH]
    toks = []
    for i in range(n_ch):
        h = x[:, None, :]
        km = np.ones((B, i + 1), bool)
        for l in range(cfg.local_layers):
            h = decoder_layer(ctx, W, cfg, f"local_transformer.layers.{l}.", h, None, None, cache, l, km,
                              np.array([i]))
        y = rmsnorm(ctx, h[:, 0, :], W["local_transformer.norm.weight"], cfg.eps)
        z = swiglu_mlp(ctx, W, f"local_to_speech_embedding_mlps.{i}.", y)
        z = moss_rmsnorm_bf16(ctx, z, W[f"layer_norm_before_lm_heads.{i}.weight"], cfg.eps)
        lg = linear(ctx, z, W[f"lm_heads.{i}.weight"])
        if i != 0:
            lg[:, cfg.audio_pad_code] = -np.inf
        if trace is not None:
            trace.append(lg)
        t = np.argmax(lg, axis=-1).astype(np.int64)
        toks.append(t)
        if forced is not None:
            t = forced[:, i]
        e = W[f"model.embedding_list.{i}.weight"][t]
        x = swiglu_mlp(ctx, W, "speech_embedding_to_local_mlp.", e)
    return np.stack(toks, axis=-1)


def generate(W, cfg: LCfg, input_ids, attention_mask=None, max_new_tokens=100, n_vq_for_inference=None,
             dtype="bf16", trace: List = None, forced=None):
    """Greedy `CustomMixin._sample` (:315-477) with do_samples all False.  Returns
    [(start_length, ids[start_idx:])] like the reference's non-dict output.
    forced [B, steps, 1+n_vq]: teacher forcing (the frames fed back are these rows)."""
    ctx = _Ctx(dtype)
    ids = np.asarray(input_ids, np.int64)
    B, T, C = ids.shape
    nq = cfg.n_vq if n_vq_for_inference is None else n_vq_for_inference
    n_ch = min(C, 1 + nq)
    mask = np.ones((B, T), bool) if attention_mask is None else np.asarray(attention_mask, bool)
    pos = hf_position_ids(mask)  # grows by last + 1 per step (utils.py:975-985)
    cache = Cache(cfg.layers)
    unfinished = np.ones(B, np.int64)
    cur = ids
    step_in = ids
    for _ in range(max_new_tokens):
        g = backbone(ctx, W, cfg, step_in, mask, cache, n_ch, position_ids=pos[:, -step_in.shape[1]:])
        step = cur.shape[1] - T
        fr = local_frame(ctx, W, cfg, g, n_ch, trace=trace,
                         forced=None if forced is None else forced[:, step, :n_ch])
        nxt = np.zeros((B, C), np.int64)
        nxt[:, :n_ch] = fr if forced is None else forced[:, step, :n_ch]
        for i in range(C):
            pddp = cfg.eos_token_id if i == 0 else cfg.audio_pad_code
            nxt[:, i] = nxt[:, i] * unfinished + pddp * (1 - unfinished)
        cur = np.concatenate([cur, nxt[:, None, :]], axis=1)
        mask = np.concatenate([mask, np.ones((B, 1), bool)], axis=1)
        pos = np.concatenate([pos, pos[:, -1:] + 1], axis=1)
        unfinished = unfinished & (nxt[:, 0] != cfg.eos_token_id).astype(np.int64)
        step_in = nxt[:, None, :]
        if unfinished.max() == 0 or (forced is not None and cur.shape[1] - T >= forced.shape[1]):
            break
    starts = find_last_equal_C(ids[..., 0], cfg.audio_start_token_id)
    return [(T - int(starts[b]) - 1, cur[b, int(starts[b]):]) for b in range(B)]


# ----------------------------------------------------------------------------
def hf_pick_distribution(logits, history, ch, temperature, top_k, top_p, penalty):
    """Sampling distribution of one channel's token (`_sample` :356-419 with do_samples[ch]):
    the HF processor chain on the bf16 logits row, then softmax.  Restates
    transformers/generation/logits_process.py (RepetitionPenaltyLogitsProcessor :306,
    TemperatureLogitsWarper :238, TopKLogitsWarper :542, TopPLogitsWarper :473) in bf16:
      penalty (ch != 0): s[h] = bf16(s*p) if s < 0 else bf16(s/p) for h in the history
      temperature: bf16(s / T)
      top-k: drop s < k-th largest (ties kept)
      top-p: ascending sort, bf16 softmax, bf16 cumsum; drop cum <= bf16(1 - top_p); the
             largest is always kept
    Returns probabilities over the row (float64, zeros outside the kept set)."""
    r = _bf.rnd
    s = r(np.asarray(logits, np.float32))
    if ch != 0 and penalty is not None and penalty != 1.0:
        h = np.unique(np.asarray(history, np.int64))
        v = s[h]
        s[h] = np.where(v < 0, r(v * np.float32(penalty)), r(v / np.float32(penalty)))
    s = r(s / np.float32(temperature))
    if top_k is not None and top_k > 0:
        k = min(top_k, s.size)
        kth = np.sort(s)[::-1][k - 1]
        s = np.where(s < kth, -np.inf, s).astype(np.float32)
    if top_p is not None:
        order = np.argsort(s, kind="stable")
        srt = s[order]
        mx = srt[-1]
        e = np.exp((srt - mx).astype(np.float64))
        p = r((e / e.sum()).astype(np.float32))
        cum = r(np.cumsum(p.astype(np.float32), dtype=np.float32))
        rm = cum <= r(np.float32(1.0 - top_p))
        rm[-1] = False
        s = s.copy()
        s[order[rm]] = -np.inf
    fin = np.isfinite(s)
    out = np.zeros(s.size, np.float64)
    e = np.exp((s[fin] - s[fin].max()).astype(np.float64))
    out[fin] = e / e.sum()
    return out
