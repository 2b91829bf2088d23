#!/usr/bin/env python3
"""Golden vectors for the MossTTSDelay sampler arithmetic, from the REFERENCE's own functions
(`moss_tts_delay/inference_utils.py`: apply_top_k :19-26, apply_top_p_optimized :44-59,
apply_repetition_penalty_delay_pattern :62-108, and sample_token's softmax :139) run in this
container on bf16 CPU tensors:

    python tests/golden/make_golden_sampling.py

Per case: a bf16 logits row set (already divided by the temperature, as generate() does at
`modeling_moss_tts.py:451`; stored as bf16 bits), the penalty history, top_k / top_p, and the
reference's outputs: the penalised logits (bits), the ids surviving top-k / top-p (-1 padded)
and the bf16 probabilities multinomial() draws from at those ids (zero elsewhere).  Rows are drawn so that no top-k threshold tie and no
top-p comparison falls in (top_p, bf16(top_p)] -- where torch's CPU kernels (which round the
Python float to bf16 before comparing) and its CUDA kernels (which compare in fp32) differ; the
engine follows CUDA.  Outputs tests/golden/golden_sampling.npz (allow_pickle=False) + .json."""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, "/root/reference")

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from moss_tts_delay import inference_utils as IU  # noqa: E402

CASES = [
    # name, rows, vocab, top_k, top_p, penalty, scale
    ("audio_default", 6, 1025, 25, 0.8, 1.0, 3.0),
    ("audio_pen11", 6, 1025, 25, 0.8, 1.1, 3.0),
    ("audio_k200_p95", 6, 1025, 200, 0.95, 1.3, 2.0),
    ("audio_nok_p50", 4, 1025, 0, 0.5, 0.9, 4.0),
    ("audio_k1", 4, 1025, 1, 0.8, 1.0, 3.0),
    ("text_k50", 3, 151936, 50, 1.0, 1.0, 2.5),
    ("text_k1000_p90", 3, 151936, 1000, 0.9, 1.0, 1.5),
    ("text_k2048_p30", 2, 151936, 2048, 0.3, 1.0, 6.0),
    # wide candidate sets (the engine's key-bin sampler): no top-k filter, top_k above 2,048
    ("text_nok_p100", 2, 151936, 0, 1.0, 1.0, 2.5),
    ("text_nok_p90", 2, 151936, 0, 0.9, 1.0, 1.5),
    ("text_k2500_p95", 2, 151936, 2500, 0.95, 1.0, 1.5),
]


def safe(logits, k, p):
    """no tie at the k-th value; no bf16 cumsum value in (p, bf16(p)]"""
    x = logits.float()
    for r in x:
        f = r[torch.isfinite(r)]
        if k > 0 and f.numel() > k:
            s = torch.sort(f, descending=True).values
            if s[k - 1] == s[k]:
                return False
    if 0 < p < 1:
        t = IU.apply_top_k(logits.clone(), k) if k > 0 else logits.clone()
        probs = F.softmax(t, dim=-1)
        cum = torch.cumsum(torch.sort(probs, descending=True, dim=-1).values, dim=-1).float()
        pb = float(torch.tensor(p, dtype=torch.bfloat16).float())
        lo, hi = min(p, pb), max(p, pb)
        if ((cum > lo) & (cum <= hi)).any():
            return False
    return True


def main():
    rng = np.random.default_rng(2026)
    arrays, meta = {}, {}
    for name, R, V, k, p, pen, scale in CASES:
        for attempt in range(200):
            if V <= 4096:  # distinct bf16 values per row, so ties come only from the penalty
                grid = np.unique(torch.from_numpy(rng.standard_normal(8 * V).astype(np.float32) * scale)
                                 .to(torch.bfloat16).float().numpy())
                x = np.stack([rng.permutation(rng.choice(grid, V, replace=False)) for _ in range(R)])
            else:  # the text vocab exceeds the distinct bf16 values: a distinct-valued head of
                # 3,000 ids over a low, tie-rich floor
                allv = (np.arange(65536, dtype=np.uint32) << 16).view(np.float32)
                grid = allv[np.isfinite(allv) & (np.abs(allv) >= 1e-3) & (allv > -2 * scale) & (allv < 3 * scale)]
                x = rng.standard_normal((R, V)) * 0.5 - 4 * scale
                for r in range(R):
                    x[r, rng.choice(V, 3000, replace=False)] = rng.choice(grid, 3000, replace=False)
            x = torch.from_numpy(x.astype(np.float32)).to(torch.bfloat16)
            if V == 1025:
                x[:, 1024] = float("-inf")  # generate() bans the audio pad code (:486-487)
            hist = torch.from_numpy(rng.integers(0, V, (R, 40))).long()
            xp = IU.apply_repetition_penalty_delay_pattern(x.clone(), hist, pen)
            if safe(xp, k, p):
                break
        else:
            raise RuntimeError(f"{name}: no tie-free draw")
        t = IU.apply_top_k(xp.clone(), k) if k > 0 else xp.clone()
        if p < 1.0:
            t = IU.apply_top_p_optimized(t, p)
        probs = F.softmax(t, dim=-1)
        bits = lambda a: (a.float().numpy().view(np.uint32) >> 16).astype(np.uint16)
        arrays[name + "/logits"] = bits(x)
        arrays[name + "/history"] = hist.numpy().astype(np.int32)
        arrays[name + "/penalized"] = bits(xp)
        # survivors of top-k / top-p (finite filtered logits) and their bf16 probabilities
        kept = [torch.nonzero(torch.isfinite(t[r])).flatten() for r in range(R)]
        n = max(len(k_) for k_ in kept)
        idx = np.full((R, n), -1, np.int32)
        pr = np.zeros((R, n), np.float32)
        for r, k_ in enumerate(kept):
            idx[r, :len(k_)] = k_.numpy()
            pr[r, :len(k_)] = probs[r, k_].float().numpy()
        arrays[name + "/kept"] = idx
        arrays[name + "/probs"] = pr
        assert float(probs.float().sum(-1).min()) > 0.98
        meta[name] = dict(rows=R, vocab=V, top_k=k, top_p=p, penalty=pen)
    np.savez_compressed(os.path.join(HERE, "golden_sampling.npz"), **arrays)
    with open(os.path.join(HERE, "golden_sampling.json"), "w") as f:
        json.dump(meta, f, indent=1)
    print("wrote", len(meta), "cases")


if __name__ == "__main__":
    main()
