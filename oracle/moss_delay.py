"""numpy restatement of the MossTTSDelay decode path -- TEST INFRASTRUCTURE ONLY.

Every function cites the reference line it restates.  `/root/reference` is
the upstream checkout (xiami2019/MOSS-TTS); `TF/` is transformers
(`transformers/models/qwen3/modeling_qwen3.py` and friends, 5.15.0 here).

Two arithmetic modes:

* ``dtype="fp32"``: float32 everywhere (the reference model in fp32);
* ``dtype="bf16"``: float32 arithmetic with rounding to bf16 at exactly the
  points the reference rounds: every torch op output on a
  bf16 tensor is rounded; matmuls, RMSNorm statistics, softmax and RoPE
  tables are computed in fp32 first.
"""
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

import numpy as np

from . import bf16 as _bf
from . import prng

INT64_MAX = np.iinfo(np.int64).max


@dataclass
class Cfg:
    """Restates MossTTSDelayConfig defaults (`moss_tts_delay/configuration_moss_tts.py:62-77`)
    plus the Qwen3Config fields the backbone uses."""
    hidden: int = 4096
    layers: int = 36
    n_heads: int = 32
    n_kv: int = 8
    head_dim: int = 128
    inter: int = 12288
    vocab: int = 151936
    n_vq: int = 32
    audio_vocab: int = 1024
    rope_theta: float = 1_000_000.0
    eps: float = 1e-6
    pad_token_id: int = 151643
    im_start_token_id: int = 151644
    im_end_token_id: int = 151645
    audio_start_token_id: int = 151652
    audio_end_token_id: int = 151653
    audio_user_slot_token_id: int = 151654
    audio_assistant_gen_slot_token_id: int = 151656
    audio_assistant_delay_slot_token_id: int = 151662
    audio_pad_code: int = 1024

    @property
    def heads_rows(self):
        return self.vocab + self.n_vq * (self.audio_vocab + 1)


def tiny_cfg(n_vq=4, **kw):
    base = dict(hidden=64, layers=2, n_heads=4, n_kv=2, head_dim=16, inter=128,
                vocab=151936, n_vq=n_vq, rope_theta=10000.0)
    base.update(kw)
    return Cfg(**base)


# ----------------------------------------------------------------------------
# deterministic weights (names follow the reference state_dict,
# `moss_tts_delay/modeling_moss_tts.py:170-191`)
# ----------------------------------------------------------------------------
def weight_specs(cfg: Cfg):
    """Ordered list of (name, shape, kind). tensor_id = index in this list."""
    H, D, I = cfg.hidden, cfg.head_dim, cfg.inter
    specs = [("language_model.embed_tokens.weight", (cfg.vocab, H), "emb")]
    for i in range(cfg.layers):
        p = f"language_model.layers.{i}."
        specs += [
            (p + "self_attn.q_proj.weight", (cfg.n_heads * D, H), "lin"),
            (p + "self_attn.k_proj.weight", (cfg.n_kv * D, H), "lin"),
            (p + "self_attn.v_proj.weight", (cfg.n_kv * D, H), "lin"),
            (p + "self_attn.o_proj.weight", (H, cfg.n_heads * D), "lin"),
            (p + "self_attn.q_norm.weight", (D,), "norm"),
            (p + "self_attn.k_norm.weight", (D,), "norm"),
            (p + "mlp.gate_proj.weight", (I, H), "lin"),
            (p + "mlp.up_proj.weight", (I, H), "lin"),
            (p + "mlp.down_proj.weight", (H, I), "lin"),
            (p + "input_layernorm.weight", (H,), "norm"),
            (p + "post_attention_layernorm.weight", (H,), "norm"),
        ]
    specs.append(("language_model.norm.weight", (H,), "norm"))
    for j in range(cfg.n_vq):
        specs.append((f"emb_ext.{j}.weight", (cfg.audio_vocab + 1, H), "emb"))
    specs.append(("lm_heads.0.weight", (cfg.vocab, H), "head"))
    for j in range(cfg.n_vq):
        specs.append((f"lm_heads.{j + 1}.weight", (cfg.audio_vocab + 1, H), "head"))
    return specs


def scale_for(kind, shape, emb_scale=1.0, head_scale=None):
    """(scale, offset) of the uniform init for one tensor kind."""
    if kind == "lin":
        return float(np.sqrt(3.0 / shape[1])), 0.0
    if kind == "norm":
        return 0.25, 1.0
    if kind == "emb":
        return float(emb_scale), 0.0
    if kind == "head":
        return float(head_scale if head_scale is not None else np.sqrt(3.0 / shape[1])), 0.0
    raise ValueError(kind)


# tokens whose text-head rows are boosted in the tiny golden models, so that a
# random model walks through every state of the delay-pattern machine
BOOST_TOKENS = (151645, 151652) + tuple(range(100, 124))


def make_weights(cfg: Cfg, seed: int, dtype="fp32", emb_scale=1.0, text_boost=4.0,
                 text_damp=0.25, special_boost=1.0) -> Dict[str, np.ndarray]:
    """Deterministic weights for a config.  For bf16 the values are rounded
    to bf16 (what `model.to(torch.bfloat16)` does to fp32 weights)."""
    out = {}
    for tid, (name, shape, kind) in enumerate(weight_specs(cfg)):
        sc, off = scale_for(kind, shape, emb_scale=emb_scale)
        w = prng.tensor(seed, tid, shape, sc, off)
        if name == "lm_heads.0.weight" and text_boost is not None:
            w *= np.float32(text_damp)
            idx = [t for t in BOOST_TOKENS if t < shape[0]]
            # per-token boost in [0.75, 1.25] x text_boost, from the same PRNG
            f = np.float32(0.75) + np.float32(0.5) * prng.uniform(seed, 10_000, len(idx))
            f[:2] *= np.float32(special_boost)  # im_end, audio_start
            w[idx] *= (np.float32(text_boost / text_damp) * f)[:, None]
        if dtype == "bf16":
            w = _bf.rnd(w)
        out[name] = w.astype(np.float32)
    return out


def weight_fill_plan(cfg: Cfg, seed: int, text_boost=4.0, text_damp=0.25, special_boost=1.0):
    """`make_weights(cfg, seed, "bf16", ...)` restated as device fills, for shapes too large to
    build on the host (the 8B-shape reference fixtures, tests/golden/make_golden_8b.py).

    Returns [(name, shape, tensor_id, scale, offset, patch)]: fill the tensor with the portable
    PRNG (`mtts_k_fill_uniform`: bf16(offset + scale * (2u - 1))), then overwrite the rows in
    `patch` ({row: float32 values before bf16 rounding}).  Equal to make_weights bit for bit:
    the text head's damping is a power of two (text_damp 0.25), so folding it into `scale`
    changes no rounding, and the boosted rows are recomputed on the host with make_weights'
    own float32 arithmetic (checked by tests/test_oracle_golden.py at the tiny shape)."""
    plan = []
    for tid, (name, shape, kind) in enumerate(weight_specs(cfg)):
        sc, off = scale_for(kind, shape)
        patch = {}
        if name == "lm_heads.0.weight" and text_boost is not None:
            assert text_damp in (0.5, 0.25, 0.125), "the damping must be a power of two"
            H = shape[1]
            idx = [t for t in BOOST_TOKENS if t < shape[0]]
            f = np.float32(0.75) + np.float32(0.5) * prng.uniform(seed, 10_000, len(idx))
            f[:2] *= np.float32(special_boost)
            fac = np.float32(text_boost / text_damp) * f
            for r, t in enumerate(idx):
                u = prng.uniform(seed, tid, H, start=t * H)
                v = np.float32(off) + np.float32(sc) * (np.float32(2.0) * u - np.float32(1.0))
                v = v.astype(np.float32) * np.float32(text_damp)
                patch[t] = (v * fac[r]).astype(np.float32)
            sc = float(np.float32(sc) * np.float32(text_damp))
        plan.append((name, shape, tid, sc, off, patch))
    return plan


# ----------------------------------------------------------------------------
# backbone ops
# ----------------------------------------------------------------------------
class _Ctx:
    def __init__(self, dtype):
        assert dtype in ("fp32", "bf16")
        self.bf = dtype == "bf16"

    def r(self, x):
        """round an op output to the model dtype"""
        return _bf.rnd(x) if self.bf else np.asarray(x, dtype=np.float32)


def rmsnorm(ctx, x, w, eps):
    """`TF/models/qwen3/modeling_qwen3.py:59-64` (Qwen3RMSNorm.forward):
    fp32 statistics, cast back to the input dtype, then weight * x."""
    x32 = x.astype(np.float32)
    var = np.mean(x32 * x32, axis=-1, keepdims=True, dtype=np.float32)
    y = x32 * (np.float32(1.0) / np.sqrt(var + np.float32(eps))).astype(np.float32)
    return ctx.r(w * ctx.r(y))


def inv_freq(cfg):
    """`TF/.../modeling_qwen3.py:106-122` compute_default_rope_parameters."""
    d = cfg.head_dim
    e = (np.arange(0, d, 2, dtype=np.float32) / np.float32(d)).astype(np.float32)
    # base**e correctly rounded to fp32, then an fp32 division (matches torch's
    # float32 pow to the bit for 63 of the 64 8B-shape frequencies; 1 ulp off on one)
    p = np.power(np.float64(cfg.rope_theta), e.astype(np.float64)).astype(np.float32)
    return (np.float32(1.0) / p).astype(np.float32)


def rope_cos_sin(ctx, cfg, positions):
    """`TF/.../modeling_qwen3.py:126-137`: freqs in fp32, cat(f, f), cos/sin, cast to dtype."""
    f = (inv_freq(cfg)[None, :] * np.asarray(positions, dtype=np.float32)[:, None]).astype(np.float32)
    emb = np.concatenate([f, f], axis=-1)
    return ctx.r(np.cos(emb)), ctx.r(np.sin(emb))


def apply_rope(ctx, x, cos, sin):
    """`TF/.../modeling_qwen3.py:140-170`: x*cos + rotate_half(x)*sin, each op rounded.
    x [..., S, D]; cos/sin [S, D]."""
    h = x.shape[-1] // 2
    rot = np.concatenate([-x[..., h:], x[..., :h]], axis=-1)
    return ctx.r(ctx.r(x * cos) + ctx.r(rot * sin))


def linear(ctx, x, w):
    """nn.Linear without bias: fp32 accumulate, one rounding of the output."""
    return ctx.r(np.asarray(x, np.float32) @ np.asarray(w, np.float32).T)


def silu(x):
    return x / (np.float32(1.0) + np.exp(-x))


class KVCache:
    """Flat per-layer cache [B, n_kv, C, D]; restates DynamicLayer.update
    (`TF/cache_utils.py:127-145`) as an append."""

    def __init__(self, layers):
        self.k = [None] * layers
        self.v = [None] * layers

    def update(self, i, k, v):
        if self.k[i] is None:
            self.k[i], self.v[i] = k, v
        else:
            self.k[i] = np.concatenate([self.k[i], k], axis=2)
            self.v[i] = np.concatenate([self.v[i], v], axis=2)
        return self.k[i], self.v[i]

    def length(self):
        return 0 if self.k[0] is None else self.k[0].shape[2]


def attention(ctx, q, k, v, key_mask, q_pos, scaling):
    """SDPA with a causal+padding mask (`TF/integrations/sdpa_attention.py:79-166`,
    `TF/masking_utils.py`).  q [B,Hq,S,D], k/v [B,Hkv,C,D], key_mask [B,C] bool,
    q_pos [S] absolute positions.  Scores and softmax statistics in fp32; in
    bf16 mode the un-normalised probabilities exp(s - max) are rounded to bf16
    before the P.V product, as torch's flash-attention kernels (CPU and GPU)
    do for bf16 inputs (pinned: 99.3% of outputs bit-equal to the reference's
    CPU SDPA, the rest 1 ulp from summation order); output rounded to dtype."""
    B, Hq, S, D = q.shape
    Hkv, C = k.shape[1], k.shape[2]
    g = Hq // Hkv
    kr = np.repeat(k, g, axis=1)
    vr = np.repeat(v, g, axis=1)
    s = np.einsum("bhsd,bhcd->bhsc", q.astype(np.float32), kr.astype(np.float32)) * np.float32(scaling)
    allowed = key_mask[:, None, None, :] & (np.arange(C)[None, None, None, :] <= np.asarray(q_pos)[None, None, :, None])
    s = np.where(allowed, s, -np.inf).astype(np.float32)
    m = np.max(s, axis=-1, keepdims=True)
    m = np.where(np.isfinite(m), m, 0.0).astype(np.float32)
    p = np.exp(s - m).astype(np.float32)
    l = np.sum(p, axis=-1, keepdims=True, dtype=np.float32)
    pv = ctx.r(p)
    o = np.einsum("bhsc,bhcd->bhsd", pv, vr.astype(np.float32)) / np.where(l > 0, l, 1.0)
    return ctx.r(o.astype(np.float32))


def embed(ctx, W, cfg, ids):
    """`moss_tts_delay/modeling_moss_tts.py:196-213`: text embedding + sum of the
    n_vq audio embeddings, added left to right (each add rounded)."""
    e = W["language_model.embed_tokens.weight"][ids[..., 0]]
    for j in range(cfg.n_vq):
        e = ctx.r(e + W[f"emb_ext.{j}.weight"][ids[..., j + 1]])
    return e


def decoder_layer(ctx, W, cfg, i, h, cos, sin, cache, key_mask, q_pos):
    """`TF/.../modeling_qwen3.py:294-323` + attention `:241-280` + MLP `:81-83`."""
    p = f"language_model.layers.{i}."
    B, S, H = h.shape
    D = cfg.head_dim
    x = rmsnorm(ctx, h, W[p + "input_layernorm.weight"], cfg.eps)
    q = linear(ctx, x, W[p + "self_attn.q_proj.weight"]).reshape(B, S, cfg.n_heads, D)
    k = linear(ctx, x, W[p + "self_attn.k_proj.weight"]).reshape(B, S, cfg.n_kv, D)
    v = linear(ctx, x, W[p + "self_attn.v_proj.weight"]).reshape(B, S, cfg.n_kv, D)
    q = rmsnorm(ctx, q, W[p + "self_attn.q_norm.weight"], cfg.eps).transpose(0, 2, 1, 3)
    k = rmsnorm(ctx, k, W[p + "self_attn.k_norm.weight"], cfg.eps).transpose(0, 2, 1, 3)
    v = v.transpose(0, 2, 1, 3)
    q = apply_rope(ctx, q, cos, sin)
    k = apply_rope(ctx, k, cos, sin)
    K, V = cache.update(i, k, v)
    a = attention(ctx, q, K, V, key_mask, q_pos, D ** -0.5)
    a = a.transpose(0, 2, 1, 3).reshape(B, S, cfg.n_heads * D)
    h = ctx.r(h + linear(ctx, a, W[p + "self_attn.o_proj.weight"]))
    x = rmsnorm(ctx, h, W[p + "post_attention_layernorm.weight"], cfg.eps)
    g = linear(ctx, x, W[p + "mlp.gate_proj.weight"])
    u = linear(ctx, x, W[p + "mlp.up_proj.weight"])
    m = ctx.r(ctx.r(silu(g)) * u)
    h = ctx.r(h + linear(ctx, m, W[p + "mlp.down_proj.weight"]))
    return h


def forward(ctx, W, cfg, ids, attention_mask, cache, last_only=True):
    """`moss_tts_delay/modeling_moss_tts.py:225-300`: embed-sum, Qwen3Model
    (`TF/.../modeling_qwen3.py:367-427`), the 1+n_vq heads with the audio pad
    column forced to -inf (`:298-299`).

    ids [B,S,1+n_vq] int64, attention_mask [B, past+S] bool.  Positions are
    arange(S)+past (`TF/.../modeling_qwen3.py:386-389`) -- left pads included.
    Returns list of logits [B, S', V_i] (S'=1 when last_only)."""
    B, S, _ = ids.shape
    past = cache.length()
    pos = np.arange(S) + past
    cos, sin = rope_cos_sin(ctx, cfg, pos)
    h = embed(ctx, W, cfg, ids)
    for i in range(cfg.layers):
        h = decoder_layer(ctx, W, cfg, i, h, cos, sin, cache, np.asarray(attention_mask, bool), pos)
    h = rmsnorm(ctx, h, W["language_model.norm.weight"], cfg.eps)
    if last_only:
        h = h[:, -1:, :]
    logits = [linear(ctx, h, W["lm_heads.0.weight"])]
    for j in range(cfg.n_vq):
        lg = linear(ctx, h, W[f"lm_heads.{j + 1}.weight"])
        lg[..., -1] = -np.inf
        logits.append(lg)
    return logits


# ----------------------------------------------------------------------------
# sampling (`moss_tts_delay/inference_utils.py`)
# ----------------------------------------------------------------------------
def find_last_equal_C(x, C):
    """`inference_utils.py:148-165`: last index of C per row, -1 if absent."""
    x = np.asarray(x)
    hit = x == C
    T = x.shape[1]
    idx = (T - 1) - np.argmax(hit[:, ::-1], axis=1)
    return np.where(hit.any(axis=1), idx, -1).astype(np.int64)


def repetition_penalty_2d(ctx, logits, prev_tokens, penalty):
    """`inference_utils.py:62-88` (the 2-D branch the generate loop always
    takes, `modeling_moss_tts.py:484-503`): the penalty set is the union of
    prev_tokens over every row and channel."""
    if penalty == 1.0 or prev_tokens is None:
        return logits
    uniq = np.unique(np.asarray(prev_tokens).reshape(-1))
    uniq = uniq[(uniq >= 0) & (uniq < logits.shape[-1])]
    t = logits[:, uniq]
    t = np.where(t > 0, ctx.r(t / np.float32(penalty)), ctx.r(t * np.float32(penalty)))
    logits = logits.copy()
    logits[:, uniq] = t
    return logits


def argmax_first(x):
    """torch.argmax: first index among ties (`inference_utils.py:129-130`)."""
    return np.argmax(x, axis=-1).astype(np.int64)


def topk_filter(logits, k):
    """`inference_utils.py:19-26` apply_top_k (ties: lowest index kept first)."""
    k = min(k, logits.shape[-1])
    out = np.full_like(logits, -np.inf)
    for r in range(logits.shape[0]):
        order = np.lexsort((np.arange(logits.shape[1]), -logits[r]))[:k]
        out[r, order] = logits[r, order]
    return out


def softmax(x):
    x = x.astype(np.float64)
    m = np.max(x, axis=-1, keepdims=True)
    e = np.exp(x - m)
    return e / e.sum(axis=-1, keepdims=True)


def topp_filter(logits, p):
    """`inference_utils.py:44-59` apply_top_p_optimized."""
    out = logits.copy()
    probs = softmax(logits)
    for r in range(logits.shape[0]):
        order = np.lexsort((np.arange(logits.shape[1]), -probs[r]))
        cum = np.cumsum(probs[r, order])
        remove = cum > p
        remove[1:] = remove[:-1].copy()
        remove[0] = False
        out[r, order[remove]] = -np.inf
    return out


def sampling_distribution(logits, top_k=None, top_p=None):
    """The distribution `sample_token` draws from (`inference_utils.py:111-145`)
    with do_sample=True: top-k, then top-p, then softmax."""
    x = np.asarray(logits, dtype=np.float32)
    if top_k is not None and top_k > 0:
        x = topk_filter(x, top_k)
    if top_p is not None and top_p < 1.0:
        x = topp_filter(x, top_p)
    return softmax(x)


class PhiloxDraw:
    """Draw source matching the engine: uniform u = Philox(seed; step, row, channel)
    (`prng.philox_uniform`), channel 0 = text, 1 + j = audio channel j."""

    def __init__(self, seed):
        self.seed = int(seed)

    def u(self, step, row, ch):
        return prng.philox_uniform(self.seed, step, row, ch)


def topk_candidates(x, k):
    """`inference_utils.py:19-26` apply_top_k as the candidate list the draw runs over:
    indices of the min(k, #finite) largest finite scores sorted by (score desc, index asc);
    among scores equal to the k-th, the lowest indices (torch.topk leaves that order
    unspecified; this is the convention the engine fixes).  k None / <= 0: every finite."""
    x = np.asarray(x, np.float32)
    fin = np.nonzero(x > -np.inf)[0]
    order = fin[np.lexsort((fin, -x[fin]))]
    if k is not None and k > 0:
        order = order[:k]
    return order


def torch_keep_probs(vals, top_p, ids=None):
    """`apply_top_p_optimized` (`inference_utils.py:44-59`) + the softmax of `sample_token`
    (:139) on candidates sorted by score (desc; index asc), every torch op on bf16 tensors
    with fp32 internals:
      probs = bf16(e / S), e = exp(s - s_0);
      sort(probs, descending): torch's sort is unstable, so the order inside a run of equal
      bf16 probabilities is implementation-defined (measured: arbitrary on CPU); the score
      order used here is one valid outcome (the kept count never depends on it -- equal
      addends -- only which members of a boundary run survive: the higher scores);
      cum = bf16(fp32 cumsum);  drop where cum > top_p (fp32 compare, torch's CUDA kernels),
      shifted right by one;  q = bf16(e / S2) over the survivors.
    All sums sequential fp32 in score order (the engine's order).  Returns (order, keep, q):
    the survivors are vals[order[:keep]] (order is the identity; kept for callers)."""
    r = _bf.rnd
    f = np.float32
    v = np.asarray(vals, np.float32)
    n = v.size
    ids = np.arange(n) if ids is None else np.asarray(ids)
    ev = np.exp((v - v[0]).astype(np.float32)).astype(np.float32)
    S = f(0)
    for e in ev:
        S = f(S + e)
    order = np.arange(n)
    keep = n
    if top_p is not None and top_p < 1.0:
        pb = r(ev / S)
        cum = f(0)
        for i in range(n):
            cum = f(cum + pb[order[i]])
            if r(cum) > f(top_p):
                keep = i + 1
                break
    S2 = f(0)
    for i in range(keep):
        S2 = f(S2 + ev[order[i]])
    return order, keep, r(np.array([f(ev[order[i]] / S2) for i in range(keep)], np.float32)).reshape(-1)


def torch_draw(vals, top_p, u, ids=None):
    """multinomial(q) of `sample_token` (`inference_utils.py:140`) as the inverse CDF at
    u * sum(q) over `torch_keep_probs` (in its top-p order; ids = the candidates' token ids).
    Returns (position in vals, margin): margin is the distance of the target from the nearest
    CDF step, as a fraction of sum(q)."""
    f = np.float32
    order, keep, q = torch_keep_probs(vals, top_p, ids)
    Q = f(0)
    for x in q:
        Q = f(Q + x)
    target = f(f(u) * Q)
    c, prev = f(0), f(0)
    for i in range(keep):
        prev, c = c, f(c + q[i])
        if c > target:
            return int(order[i]), float(min(target - prev, c - target) / Q)
    return int(order[keep - 1]), 0.0


# ----------------------------------------------------------------------------
# wide candidate sets (text top_k <= 0 or > TOPK_CAP): the key-bin form of the engine
# (`moss_tts_amd/csrc/topk.h` block_wide_draw), restated bit for bit
# ----------------------------------------------------------------------------
TOPK_CAP = 2048
WIDE_BINS, WIDE_NT = 65536, 1024


def okey16(v):
    """order-preserving 16-bit key of bf16-exact floats (+0 / -0 share one)"""
    v = np.where(np.asarray(v, np.float32) == 0, np.float32(0), np.asarray(v, np.float32)).astype(np.float32)
    u = (v.view(np.uint32) >> 16).astype(np.uint32)
    return np.where(u & 0x8000, ~u & 0xFFFF, u | 0x8000).astype(np.int64)


def okey16_val(k):
    k = np.asarray(k, np.uint32)
    u = np.where(k & 0x8000, k & 0x7FFF, ~k & 0xFFFF).astype(np.uint32)
    return (u << 16).view(np.float32)


def _wide_bins(x, K):
    """candidate counts per descending key position (position p = key 65535 - p): every finite
    score, or torch.topk's exactly-K with the lowest indices among the threshold ties"""
    x = np.asarray(x, np.float32)
    fin = x > -np.inf
    cnt = np.bincount(okey16(x[fin]), minlength=WIDE_BINS)[::-1].astype(np.int64).copy()
    n = int(cnt.sum())
    if K is not None and 0 < K < n:
        cum = np.cumsum(cnt)
        p = int(np.searchsorted(cum, K))
        cnt[p] = K - (int(cum[p - 1]) if p else 0)
        cnt[p + 1:] = 0
    return cnt


def _wide_sums(cnt, f):
    """the engine's fixed-order sum of fp32(c * f): per 64-bin chunk sequential, chunk totals
    sequential; returns (total, exclusive chunk prefixes, inclusive in-chunk prefixes)"""
    f32 = np.float32
    m = np.where(cnt > 0, (cnt.astype(f32) * np.nan_to_num(f, nan=0.0, posinf=0.0)).astype(f32), f32(0)).astype(f32)
    incl = np.cumsum(m.reshape(WIDE_NT, 64), axis=1, dtype=f32)
    tot = np.cumsum(incl[:, -1], dtype=f32)
    P = np.concatenate([[f32(0)], tot[:-1]]).astype(f32)
    return f32(tot[-1]), P, incl


def _wide_first(cnt, f, P, incl, passes):
    """first element (position, r) whose cumulative fp32(P_t + fp32(L + fp32(r * f))) passes"""
    f32 = np.float32
    full = (P[:, None] + incl).astype(f32).reshape(-1)
    hit = np.nonzero((cnt > 0) & passes(full))[0]
    if hit.size == 0:
        return -1, 0
    pos = int(hit[0])
    t, j = divmod(pos, 64)
    L = f32(incl[t, j - 1]) if j else f32(0)
    x = f32(f[pos])
    lo, hi = 1, int(cnt[pos])
    while lo < hi:
        mid = (lo + hi) // 2
        if passes(np.array([f32(P[t] + f32(L + f32(f32(mid) * x)))], np.float32))[0]:
            hi = mid
        else:
            lo = mid + 1
    return pos, lo


def wide_keep(x, K, top_p):
    """apply_top_k (:19-26) + apply_top_p_optimized (:44-59) + the softmax (:139) in the key-bin
    form: returns (cnt, q) -- survivors per descending key position and their bf16 probability"""
    f32 = np.float32
    cnt = _wide_bins(x, K)
    if cnt.sum() == 0:
        return cnt, np.zeros(WIDE_BINS, f32)
    keys = WIDE_BINS - 1 - np.arange(WIDE_BINS)
    with np.errstate(invalid="ignore", over="ignore"):
        mx = f32(okey16_val(keys[np.nonzero(cnt)[0][0]]))
        # exp of the fp32 difference in double, rounded once (the engine's correctly rounded form)
        ev = np.exp((okey16_val(keys) - mx).astype(f32).astype(np.float64)).astype(f32)
        if top_p is not None and top_p < 1.0:
            S, _, _ = _wide_sums(cnt, ev)
            pf = _bf.rnd((ev / S).astype(f32))
            _, P, incl = _wide_sums(cnt, pf)
            pos, r = _wide_first(cnt, pf, P, incl, lambda c: _bf.rnd(c) > f32(top_p))
            if pos >= 0:
                cnt = cnt.copy()
                cnt[pos] = r
                cnt[pos + 1:] = 0
        S2, _, _ = _wide_sums(cnt, ev)
        q = _bf.rnd((ev / S2).astype(f32))
    return cnt, np.where(cnt > 0, q, f32(0)).astype(f32)


def wide_draw(x, K, top_p, u):
    """the engine's draw over a wide candidate set at uniform u: the token index (-1: none)"""
    f32 = np.float32
    x = np.asarray(x, np.float32)
    cnt, q = wide_keep(x, K, top_p)
    if cnt.sum() == 0:
        return -1
    Q, P, incl = _wide_sums(cnt, q)
    target = f32(f32(u) * Q)
    pos, r = _wide_first(cnt, q, P, incl, lambda c: c > target)
    if pos < 0:  # rounding: the last survivor
        pos = int(np.nonzero(cnt)[0][-1])
        r = int(cnt[pos])
    key = WIDE_BINS - 1 - pos
    fin = x > -np.inf
    idx = np.nonzero(fin & (okey16(np.where(fin, x, 0)) == key))[0]
    return int(idx[r - 1])


def sample_token(ctx, logits, prev_tokens=None, repetition_penalty=1.0, top_p=None,
                 top_k=None, do_sample=True, rng=None, ctrs=None, wide=False):
    """`inference_utils.py:111-145`.  Greedy is exact.  With do_sample and a `PhiloxDraw`
    rng, row r draws with u = rng.u(*ctrs[r]) through `topk_candidates` + `torch_draw`
    (the engine's stream); another rng draws from `sampling_distribution` (the
    distribution, not torch's RNG stream, is the reference contract)."""
    if prev_tokens is not None and repetition_penalty != 1.0:
        logits = repetition_penalty_2d(ctx, logits, prev_tokens, repetition_penalty)
    if not do_sample:
        return argmax_first(logits)
    if isinstance(rng, PhiloxDraw):
        out = []
        for r_, row in enumerate(np.asarray(logits, np.float32)):
            w = wide if np.isscalar(wide) else wide[r_]
            if w and (top_k is None or top_k <= 0 or top_k > TOPK_CAP):
                # the engine's text sampler without a sortable top-k (sample.hip -> topk.h)
                out.append(wide_draw(row, top_k, top_p, rng.u(*ctrs[r_])))
                continue
            cand = topk_candidates(row, top_k)
            pos, _ = torch_draw(row[cand], top_p, rng.u(*ctrs[r_]), ids=cand)
            out.append(cand[pos])
        return np.array(out, dtype=np.int64)
    probs = sampling_distribution(logits, top_k, top_p)
    rng = rng or np.random.default_rng(0)
    return np.array([rng.choice(probs.shape[1], p=pr) for pr in probs], dtype=np.int64)


# ----------------------------------------------------------------------------
# generate (`moss_tts_delay/modeling_moss_tts.py:392-525`)
# ----------------------------------------------------------------------------
@dataclass
class StepTrace:
    text_logits: list = field(default_factory=list)      # masked text logits per step [B, V]
    audio_logits: list = field(default_factory=list)     # [B, n_vq, 1025] per step (pre-mask)


def init_state(cfg, input_ids):
    """`modeling_moss_tts.py:417-440`: per-row generate() state from the prompt."""
    input_ids = np.asarray(input_ids, dtype=np.int64)
    B, T, _ = input_ids.shape
    last = input_ids[:, -1, 0]
    is_cont = (last == cfg.audio_start_token_id) | (last == cfg.audio_assistant_gen_slot_token_id)
    a_start = find_last_equal_C(input_ids[..., 0], cfg.audio_start_token_id)
    a_mask = is_cont & (a_start != -1)
    audio_lengths = np.zeros(B, np.int64)
    audio_lengths[a_mask] = T - a_start[a_mask]
    return dict(is_stopping=np.zeros(B, bool), audio_lengths=audio_lengths,
                delayed=np.full(B, INT64_MAX, np.int64), is_audio=a_mask.copy())


def decide_step(ctx, cfg, lg, step, st, gen, sp, rng=None, forced_text=None, trace=None):
    """One step of the generate loop after the forward (`modeling_moss_tts.py:451-509`):
    temperature, the text-channel schedule and masks, text / audio sampling, the counter
    updates.  lg: per-head last-position logits [B, V_i]; st: `init_state` dict (updated in
    place); gen: generation_ids so far [B, L, 1+n_vq] (the penalty history); sp: generate()
    sampling kwargs.  Returns (next_text [B], next_audio [B, n_vq])."""
    B = lg[0].shape[0]
    n_vq = len(lg) - 1
    ar = np.arange(n_vq)
    text_do_sample = sp["text_temperature"] > 0
    audio_do_sample = sp["audio_temperature"] > 0
    t_temp = sp["text_temperature"] if text_do_sample else 1
    a_temp = sp["audio_temperature"] if audio_do_sample else 1
    is_stopping, is_audio = st["is_stopping"], st["is_audio"]
    audio_lengths, delayed = st["audio_lengths"], st["delayed"]
    excl0 = [cfg.pad_token_id, cfg.audio_assistant_gen_slot_token_id,
             cfg.audio_assistant_delay_slot_token_id, cfg.audio_end_token_id]
    allow1 = [cfg.audio_assistant_gen_slot_token_id, cfg.audio_assistant_delay_slot_token_id]

    lg = [ctx.r(np.asarray(x, np.float32) / np.float32(t_temp if i == 0 else a_temp)) for i, x in enumerate(lg)]
    nt = np.full(B, cfg.pad_token_id, np.int64)
    nt[~is_stopping & (delayed < n_vq)] = cfg.audio_assistant_delay_slot_token_id
    eos = ~is_stopping & (delayed == n_vq)
    nt[eos] = cfg.audio_end_token_id
    is_audio[eos] = False
    samp_text = ~is_stopping & (delayed > n_vq)
    t = lg[0].copy()
    t[np.ix_(~is_audio, excl0)] = -np.inf
    keep = np.zeros(t.shape[1], bool)
    keep[allow1] = True
    t[np.ix_(is_audio, ~keep)] = -np.inf
    if step == 0:
        t[:, 151662] = -np.inf
    if step <= n_vq:
        t[:, cfg.im_end_token_id] = -np.inf
    if trace is not None:
        trace.text_logits.append(t.copy())
        trace.audio_logits.append(np.stack(lg[1:], axis=1).copy())
    if samp_text.any():
        rows = np.nonzero(samp_text)[0]
        nt[samp_text] = sample_token(ctx, t[samp_text], top_p=sp["text_top_p"], top_k=sp["text_top_k"],
                                     do_sample=text_do_sample, rng=rng, ctrs=[(step, b, 0) for b in rows],
                                     wide=~is_audio[rows])  # audio-mode rows: the 2 allowed ids, sorted form
    if forced_text is not None:
        f = np.asarray(forced_text)
        fs = f[:, step] if f.ndim == 2 else np.full(B, f[step] if step < len(f) else -1)
        sel = (fs >= 0) & ~is_stopping & samp_text
        nt[sel] = fs[sel]
    is_audio[nt == cfg.audio_start_token_id] = True
    is_stopping[nt == cfg.im_end_token_id] = True

    na = np.full((B, n_vq), cfg.audio_pad_code, np.int64)
    pre = audio_lengths[:, None] > ar[None, :]
    post = ar[None, :] > (np.where(delayed == INT64_MAX, 0, delayed) - 1)[:, None]
    post[delayed == INT64_MAX] = True
    sam = pre & post
    if sam.sum() > 0:
        pen = sp["audio_repetition_penalty"]
        ch0 = lg[1][sam[:, 0]].copy()
        rest = np.stack(lg[2:], axis=1)[sam[:, 1:]] if n_vq > 1 else np.zeros((0, lg[1].shape[1]), np.float32)
        ch0[:, cfg.audio_pad_code] = -np.inf
        rest = rest.copy()
        rest[:, cfg.audio_pad_code] = -np.inf
        col0 = na[:, 0]
        col0[sam[:, 0]] = sample_token(ctx, ch0, prev_tokens=gen[:, :, 1], repetition_penalty=pen,
                                       top_p=sp["audio_top_p"], top_k=sp["audio_top_k"],
                                       do_sample=audio_do_sample, rng=rng,
                                       ctrs=[(step, b, 1) for b in np.nonzero(sam[:, 0])[0]])
        na[:, 0] = col0
        if rest.shape[0]:
            bj = np.argwhere(sam[:, 1:])  # row-major (b, j-1), the order of the boolean index
            sub = na[:, 1:]
            sub[sam[:, 1:]] = sample_token(ctx, rest, prev_tokens=gen[:, :, 2:], repetition_penalty=pen,
                                           top_p=sp["audio_top_p"], top_k=sp["audio_top_k"],
                                           do_sample=audio_do_sample, rng=rng,
                                           ctrs=[(step, int(b), 2 + int(j)) for b, j in bj])
            na[:, 1:] = sub
    inc = ((nt == cfg.audio_start_token_id) | (nt == cfg.audio_assistant_gen_slot_token_id)
           | (nt == cfg.audio_assistant_delay_slot_token_id))
    audio_lengths[inc] += 1
    audio_lengths[nt == cfg.audio_end_token_id] = 0
    delayed[(delayed == INT64_MAX) & (nt == cfg.audio_assistant_delay_slot_token_id)] = 0
    delayed[delayed != INT64_MAX] += 1
    delayed[delayed > n_vq] = INT64_MAX
    return nt, na


def generate(W, cfg: Cfg, input_ids, attention_mask=None, max_new_tokens=1000,
             text_temperature=1.5, text_top_p=1.0, text_top_k=50,
             audio_temperature=1.7, audio_top_p=0.8, audio_top_k=25,
             audio_repetition_penalty=1.0, dtype="fp32", rng=None, trace=None,
             forced_text=None):
    """Restates `MossTTSDelayModel.generate` line by line (state machine
    `:417-516`, output slicing `:518-525`).  `forced_text` (optional [steps]
    or [B, steps] int array, -1 = not forced) replaces the text-channel
    decision -- used only to reproduce the benchmark schedule."""
    ctx = _Ctx(dtype)
    input_ids = np.asarray(input_ids, dtype=np.int64)
    B, T, C1 = input_ids.shape
    n_vq = C1 - 1
    assert n_vq == cfg.n_vq
    if attention_mask is None:
        attention_mask = np.ones((B, T), dtype=bool)
    mask = np.asarray(attention_mask, dtype=bool)
    cache = KVCache(cfg.layers)
    cur = input_ids
    gen = input_ids.copy()
    st = init_state(cfg, input_ids)
    sp = dict(text_temperature=text_temperature, text_top_p=text_top_p, text_top_k=text_top_k,
              audio_temperature=audio_temperature, audio_top_p=audio_top_p, audio_top_k=audio_top_k,
              audio_repetition_penalty=audio_repetition_penalty)

    for step in range(max_new_tokens):
        logits = forward(ctx, W, cfg, cur, mask, cache, last_only=True)
        nt, na = decide_step(ctx, cfg, [l[:, -1, :] for l in logits], step, st, gen, sp, rng=rng,
                             forced_text=forced_text, trace=trace)
        cur = np.concatenate([nt[:, None, None], na[:, None, :]], axis=2)
        mask = np.concatenate([mask, (~st["is_stopping"])[:, None]], axis=1)
        gen = np.concatenate([gen, cur], axis=1)
        if st["is_stopping"].sum() == B:
            break

    start = find_last_equal_C(input_ids[..., 0], cfg.im_start_token_id) + 3
    start_len = T - start
    return [(int(sl), gen[b, s:]) for b, (s, sl) in enumerate(zip(start, start_len))]


# ----------------------------------------------------------------------------
# processor statics (`moss_tts_delay/processing_moss_tts.py`)
# ----------------------------------------------------------------------------
def apply_delay_pattern(codes, pad_code):
    """`processing_moss_tts.py:515-525`: out[i+t, i] = codes[t, i]."""
    codes = np.asarray(codes)
    T, n = codes.shape
    out = np.full((T + n - 1, n), pad_code, dtype=codes.dtype)
    for i in range(n):
        out[i:i + T, i] = codes[:, i]
    return out


def apply_de_delay_pattern(delay_codes):
    """`processing_moss_tts.py:527-537`."""
    d = np.asarray(delay_codes)
    n = d.shape[1]
    T = d.shape[0] - n + 1
    out = np.zeros((T, n), dtype=d.dtype)
    for i in range(n):
        out[:, i] = d[i:i + T, i]
    return out


def left_pad(seqs, pad_token_id, audio_pad_code):
    """`processing_moss_tts.py:410-431` (_pad): left pad; channel 0 with the text
    pad id, channels >=1 with the audio pad code; mask False on pads."""
    L = max(s.shape[0] for s in seqs)
    C = seqs[0].shape[1]
    ids = np.full((len(seqs), L, C), audio_pad_code, dtype=np.int64)
    mask = np.zeros((len(seqs), L), dtype=bool)
    for b, s in enumerate(seqs):
        n = s.shape[0]
        ids[b, L - n:] = s
        ids[b, :L - n, 0] = pad_token_id
        mask[b, L - n:] = True
    return ids, mask


def split_audio_segments(audio_codes, pad_code):
    """`processing_moss_tts.py:668-685`: de-delay, drop all-pad rows, split the
    remaining rows into maximal runs of consecutive indices."""
    a = apply_de_delay_pattern(audio_codes)
    non_pad = ~(a == pad_code).all(axis=1)
    if not non_pad.any():
        return []
    idx = np.nonzero(non_pad)[0]
    breaks = np.nonzero(idx[1:] != idx[:-1] + 1)[0] + 1
    return [a[s] for s in np.split(idx, breaks)]
