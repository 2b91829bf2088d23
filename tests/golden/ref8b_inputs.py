"""Seeded inputs of the 8B-shape golden vectors (tests/golden/make_golden_8b.py writes the
reference's outputs for them; tests/test_ref8b_gpu.py regenerates the same inputs here, so only
outputs are committed).  numpy only: no reference import."""
import numpy as np

from oracle import bf16 as B16

ROPE_PASTS = (0, 9590)  # q / k norm + RoPE at positions 0-9 and 9,590-9,599
ROPE_S = 10
SDPA_S = (64, 1)        # a 64-token prefill chunk and one decode query at the end of the keys
SDPA_C = 2100           # keys (the TTSD prompt's order)
SDPA_B, SDPA_HQ, SDPA_HKV, SDPA_PAD = 2, 32, 8, 45


def text_sel(cfg, n_random=2048, seed=5):
    """text-head rows recorded per step: the 16-row tiles from the lowest sampled special id up
    (im_end, audio_start, the slots), the boosted ids 100-123, and n_random others"""
    lo = (min(cfg.im_end_token_id, cfg.audio_assistant_gen_slot_token_id,
              cfg.audio_assistant_delay_slot_token_id) // 16) * 16
    rng = np.random.default_rng(seed)
    return np.unique(np.concatenate([np.arange(lo, cfg.vocab), np.arange(96, 128),
                                     rng.choice(lo, n_random, replace=False)])).astype(np.int64)


def rmsnorm_inputs(H):
    rng = np.random.default_rng(H)
    x = B16.rnd(rng.standard_normal((3, H)).astype(np.float32) * np.float32(3.0))
    w = B16.rnd((1 + 0.25 * rng.standard_normal(H)).astype(np.float32))
    return x, w


def qk_inputs(past):
    """the q|k|v rows of ROPE_S tokens (32 + 8 + 8 heads x 128) and the q / k norm weights"""
    rng = np.random.default_rng(1000 + past)
    qkv = B16.rnd(rng.standard_normal((ROPE_S, 48 * 128)).astype(np.float32) * np.float32(2.0))
    qn = B16.rnd((1 + 0.25 * rng.standard_normal(128)).astype(np.float32))
    kn = B16.rnd((1 + 0.25 * rng.standard_normal(128)).astype(np.float32))
    return qkv, qn, kn


def sdpa_inputs(S):
    """q [B, Hq, S, 128], k / v [B, Hkv, C, 128], key mask [B, C] (row 1 left-padded), query positions"""
    rng = np.random.default_rng(2000 + S)
    q = B16.rnd(rng.standard_normal((SDPA_B, SDPA_HQ, S, 128)).astype(np.float32))
    k = B16.rnd(rng.standard_normal((SDPA_B, SDPA_HKV, SDPA_C, 128)).astype(np.float32))
    v = B16.rnd(rng.standard_normal((SDPA_B, SDPA_HKV, SDPA_C, 128)).astype(np.float32))
    km = np.ones((SDPA_B, SDPA_C), bool)
    km[1, :SDPA_PAD] = False
    return q, k, v, km, np.arange(SDPA_C - S, SDPA_C)
