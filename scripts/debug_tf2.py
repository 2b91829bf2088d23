#!/usr/bin/env python3
"""Teacher-forced logits: run-to-run determinism and error vs the oracle, fused vs unfused norm."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from oracle import moss_delay as O
from tests.test_engine_gpu import make_engine
from tests.parity_util import ulp_bf16

g = np.load("tests/golden/golden.npz")
cases = json.load(open("tests/golden/cases.json"))
name = sys.argv[1] if len(sys.argv) > 1 else "g_nvq32_bf16"
c = cases[name]
cfg = O.tiny_cfg(n_vq=c["n_vq"])
W = O.make_weights(cfg, c["seed"], dtype="bf16", special_boost=c["special_boost"])
ids, mask = g[name + "/input_ids"], g[name + "/mask"]
tr = O.StepTrace()
ref = O.generate(W, cfg, ids, mask, max_new_tokens=12, text_temperature=0, audio_temperature=0, dtype="bf16", trace=tr)
B, T, C = ids.shape
starts = O.find_last_equal_C(ids[..., 0], cfg.im_start_token_id) + 3
gen = np.stack([np.concatenate([ids[b, :starts[b]], ref[b][1]], 0) for b in range(B)])
full_mask = np.concatenate([mask, np.ones((B, gen.shape[1] - T), bool)], 1)
for s in range(gen.shape[1] - T):
    stopped = (gen[:, T:T + s + 1, 0] == cfg.im_end_token_id).any(axis=1)
    full_mask[:, T + s] = ~stopped


def run():
    eng = make_engine(cfg, W)
    outs = []
    for s in range(len(tr.audio_logits)):
        if s == 0:
            lg = eng.forward(torch.from_numpy(gen[:, :T]), torch.from_numpy(full_mask[:, :T].astype(np.uint8)), 0)
        else:
            p = T + s - 1
            lg = eng.forward(torch.from_numpy(gen[:, p:p + 1].copy()),
                             torch.from_numpy(full_mask[:, :p + 1].astype(np.uint8)), p)
        outs.append(lg.float().cpu().numpy())
    eng.close()
    return outs


V = cfg.vocab
for mode in ["0", "1"]:
    os.environ["MTTS_UNFUSED_NORM"] = mode
    runs = [run() for _ in range(3)]
    for s in range(len(tr.audio_logits)):
        got = runs[0][s][:, V:].reshape(B, cfg.n_vq, 1025)
        want = tr.audio_logits[s]
        fin = np.isfinite(want)
        scale = np.max(np.abs(np.where(fin, want, 0)), axis=-1, keepdims=True)
        err = np.where(fin, np.abs(got - want), 0) / ulp_bf16(np.broadcast_to(scale, want.shape))
        same = all(np.array_equal(runs[0][s], r[s], equal_nan=True) for r in runs[1:])
        if not same:
            for r in runs[1:]:
                d = ~((runs[0][s] == r[s]) | (np.isnan(runs[0][s]) & np.isnan(r[s])))
                print("   differing entries", int(d.sum()), "text part", int(d[:, :V].sum()), "first", np.argwhere(d)[:4].tolist(),
                      "nan", int(np.isnan(runs[0][s]).sum()), int(np.isnan(r[s]).sum()))
        wb = np.unravel_index(np.argmax(err), err.shape)
        print(f"unfused={mode} step {s}: max err {err.max():.1f} ulps at {wb}, deterministic={same}")
