"""CPU restatement of the codec decoder (test infrastructure: tests/ and bench.py's
cpu_baseline only; the product path never imports this module).

What it restates.  The MOSS-Audio-Tokenizer ("Cat") source and weights are absent from the
reference tree (`moss_audio_tokenizer/` is an empty submodule; `README.md:382-393` describes
a 1.6B CNN-free tokenizer of causal Transformer blocks, RVQ with 32 codebooks at 12.5 Hz,
24 kHz audio).  The decoder restated here is the one include/mtts_codec.h specifies from that
description: residual-vector dequantisation (sum of the first n_q codebook rows, fp32, one
rounding), stages of causal Qwen3-family Transformer blocks (the layer function of
oracle.moss_delay, i.e. `TF/models/qwen3/modeling_qwen3.py:294-323`), a stage RMSNorm and a
linear upsampling projection (reshaped to `upsample` tokens of the next stage), and a final
linear projection to `patch` waveform samples per last-stage token.

Parity status: **parity unpinned** against the real codec (no source, weights or reference
fixtures exist for it); the HIP decoder is pinned to this restatement, and the restatement's
blocks are the oracle functions pinned to the reference's transformers modules."""
from dataclasses import dataclass, field
from typing import Dict, List

import numpy as np

from oracle import moss_delay as O
from oracle import prng


@dataclass
class CodecStage:
    hidden: int
    layers: int
    n_heads: int
    n_kv: int
    head_dim: int
    inter: int
    upsample: int


def default_stages() -> List[CodecStage]:
    """Assumed decode-side shape (not published): 12.5 -> 25 -> 50 -> 100 Hz token rates,
    240-sample patches at 100 Hz = 1920 samples per 12.5 Hz frame = 24 kHz; ~0.63 B params."""
    return [CodecStage(1280, 12, 10, 10, 128, 5120, 2), CodecStage(1024, 12, 8, 8, 128, 4096, 2),
            CodecStage(768, 8, 6, 6, 128, 3072, 2), CodecStage(512, 8, 4, 4, 128, 2048, 1)]


@dataclass
class CodecCfg:
    n_q: int = 32
    codebook_size: int = 1024
    stages: List[CodecStage] = field(default_factory=default_stages)
    patch: int = 240
    rope_theta: float = 10000.0
    eps: float = 1e-6
    sample_rate: int = 24000
    frame_rate: float = 12.5

    @property
    def samples_per_frame(self):
        r = 1
        for s in self.stages:
            r *= s.upsample
        return r * self.patch


def tiny_codec_cfg(**kw):
    base = dict(n_q=4, codebook_size=64, patch=24,
                stages=[CodecStage(128, 2, 2, 1, 64, 256, 2), CodecStage(64, 1, 2, 2, 32, 128, 1)])
    base.update(kw)
    return CodecCfg(**base)


@dataclass
class _StageView:
    """what oracle.moss_delay.decoder_layer / rope_cos_sin read from a config"""
    head_dim: int
    n_heads: int
    n_kv: int
    eps: float
    rope_theta: float


def weight_specs(cfg: CodecCfg):
    out = []
    for q in range(cfg.n_q):
        out.append((f"quantizer.codebooks.{q}.weight", (cfg.codebook_size, cfg.stages[0].hidden), "codebook"))
    for s, g in enumerate(cfg.stages):
        for i in range(g.layers):
            p = f"decoder.stages.{s}.layers.{i}."
            out += [(p + "self_attn.q_proj.weight", (g.n_heads * g.head_dim, g.hidden), "lin"),
                    (p + "self_attn.k_proj.weight", (g.n_kv * g.head_dim, g.hidden), "lin"),
                    (p + "self_attn.v_proj.weight", (g.n_kv * g.head_dim, g.hidden), "lin"),
                    (p + "self_attn.o_proj.weight", (g.hidden, g.n_heads * g.head_dim), "lin"),
                    (p + "self_attn.q_norm.weight", (g.head_dim,), "norm"),
                    (p + "self_attn.k_norm.weight", (g.head_dim,), "norm"),
                    (p + "mlp.gate_proj.weight", (g.inter, g.hidden), "lin"),
                    (p + "mlp.up_proj.weight", (g.inter, g.hidden), "lin"),
                    (p + "mlp.down_proj.weight", (g.hidden, g.inter), "lin"),
                    (p + "input_layernorm.weight", (g.hidden,), "norm"),
                    (p + "post_attention_layernorm.weight", (g.hidden,), "norm")]
        out.append((f"decoder.stages.{s}.norm.weight", (g.hidden,), "norm"))
        if s + 1 < len(cfg.stages):
            out.append((f"decoder.stages.{s}.upsample.weight", (g.upsample * cfg.stages[s + 1].hidden, g.hidden), "lin"))
    out.append(("decoder.out_proj.weight", (cfg.patch, cfg.stages[-1].hidden), "lin"))
    return out


def make_weights(cfg: CodecCfg, seed: int, dtype="bf16") -> Dict[str, np.ndarray]:
    """Deterministic weights (portable splitmix64, oracle/prng.py): matrices +-sqrt(3/K),
    norms 1 +- 0.25, codebooks +-sqrt(3/n_q); the same tensors, in the same order, as the
    device's mtts_codec_init_random."""
    ctx = O._Ctx(dtype)
    W = {}
    for tid, (name, shape, kind) in enumerate(weight_specs(cfg)):
        if kind == "lin":
            v = prng.tensor(seed, tid, shape, np.float32(np.sqrt(3.0 / shape[-1])))
        elif kind == "norm":
            v = prng.tensor(seed, tid, shape, 0.25, 1.0)
        else:
            v = prng.tensor(seed, tid, shape, np.float32(np.sqrt(3.0 / cfg.n_q)))
        W[name] = ctx.r(v)
    return W


class CodecState:
    """Per-stage KV caches of an incremental decode (mtts_codec_reset / _decode)."""

    def __init__(self, cfg: CodecCfg):
        self.caches = [O.KVCache(g.layers) for g in cfg.stages]
        self.pos = 0


def dequant(ctx, W, cfg, codes, n_q):
    """x = sum_{q < n_q} codebook_q[codes[..., q]], fp32 sum in quantizer order, one rounding."""
    acc = np.zeros(codes.shape[:-1] + (cfg.stages[0].hidden,), np.float32)
    for q in range(n_q):
        c = np.clip(codes[..., q], 0, cfg.codebook_size - 1)
        acc += W[f"quantizer.codebooks.{q}.weight"][c].astype(np.float32)
    return ctx.r(acc)


def decode(W, cfg: CodecCfg, codes, n_q=None, state: CodecState = None, dtype="bf16"):
    """codes int [B, T, >= n_q] -> fp32 waveform [B, T * samples_per_frame] of these T frames,
    continuing `state` (frames decoded so far) when given."""
    ctx = O._Ctx(dtype)
    n_q = cfg.n_q if n_q is None else n_q
    state = state or CodecState(cfg)
    B, T = codes.shape[:2]
    h = dequant(ctx, W, cfg, codes, n_q)  # [B, T, D0]
    R = 1
    for s, g in enumerate(cfg.stages):
        view = _StageView(g.head_dim, g.n_heads, g.n_kv, cfg.eps, cfg.rope_theta)
        S = h.shape[1]
        past = state.pos * R
        pos = np.arange(past, past + S)
        cos, sin = O.rope_cos_sin(ctx, view, pos)
        key_mask = np.ones((B, past + S), bool)
        Ws = {f"language_model.layers.{i}.{k.split(f'decoder.stages.{s}.layers.{i}.', 1)[1]}": v
              for i in range(g.layers) for k, v in W.items() if k.startswith(f"decoder.stages.{s}.layers.{i}.")}
        for i in range(g.layers):
            h = O.decoder_layer(ctx, Ws, view, i, h, cos, sin, state.caches[s], key_mask, pos)
        x = O.rmsnorm(ctx, h, W[f"decoder.stages.{s}.norm.weight"], cfg.eps)
        if s + 1 < len(cfg.stages):
            y = O.linear(ctx, x, W[f"decoder.stages.{s}.upsample.weight"])  # [B, S, up * D']
            h = y.reshape(B, S * g.upsample, cfg.stages[s + 1].hidden)
            R *= g.upsample
        else:
            wav = x.astype(np.float32) @ W["decoder.out_proj.weight"].astype(np.float32).T  # [B, S, patch]
    state.pos += T
    return wav.reshape(B, -1).astype(np.float32)
