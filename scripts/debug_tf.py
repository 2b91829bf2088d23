#!/usr/bin/env python3
"""Diagnose teacher-forced logits finiteness mismatches (GPU)."""
import json
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from oracle import moss_delay as O
from tests.test_engine_gpu import make_engine

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
eng = make_engine(cfg, W)
full_mask = np.concatenate([mask, np.ones((B, gen.shape[1] - T), bool)], 1)
for s in range(gen.shape[1] - T):
    stopped = (gen[:, T:T + s + 1, 0] == cfg.im_end_token_id).any(axis=1)
    full_mask[:, T + s] = ~stopped
for s in range(len(tr.audio_logits)):
    if s == 0:
        lg = eng.forward(torch.from_numpy(gen[:, :T]), torch.from_numpy(full_mask[:, :T].astype(np.uint8)), 0)
    else:
        p = T + s - 1
        lg = eng.forward(torch.from_numpy(gen[:, p:p + 1].copy()), torch.from_numpy(full_mask[:, :p + 1].astype(np.uint8)), p)
    parts = [x.float().cpu().numpy() for x in eng.split_logits(lg)]
    got = np.stack(parts[1:], 1)
    want = tr.audio_logits[s]
    bad = np.isfinite(got) != np.isfinite(want)
    print("step", s, "finite mismatches", int(bad.sum()), "nan in got", int(np.isnan(got).sum()),
          "text nan", int(np.isnan(parts[0]).sum()))
    if bad.any():
        idx = np.argwhere(bad)[:10]
        for b_, j, v in idx:
            print("  row", b_, "head", j, "col", v, "got", got[b_, j, v], "want", want[b_, j, v])
        print("  mask rows", full_mask[:, :T + s].sum(1), "gen row tokens", gen[:, T + s - 1, 0] if s else None)
        break
