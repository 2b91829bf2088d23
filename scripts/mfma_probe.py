#!/usr/bin/env python3
"""MFMA-busy evidence for the prefill GEMMs (north_star: "MFMA only on the prefill/MLP GEMMs
... evidenced by MFMA-busy counters").  Runs the B=1 clone prefill (181 tokens) and the
32-utterance prefill (ragged 100-130-token prompts, globally padded) at the 8B layer shape for
rocprofv3 counter passes:

    rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d D -o m \\
        --output-format csv -- python3 scripts/mfma_probe.py
    python3 scripts/mfma_probe.py --summarize D > profiles/<round>_pmc_mfma.json

MFMA utilisation of a dispatch = SQ_VALU_MFMA_BUSY_CYCLES / (cycles x 1024 SIMDs), cycles =
GRBM_GUI_ACTIVE / 8 (rocprofv3 sums it over the 8 XCDs; MI355X_MICROARCH.md "DVFS").  Each
dispatch's flops are 2 M N K of its GEMM; TFLOP/s from the kernel-trace duration."""
import argparse
import csv
import glob
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
LAYERS = 4


def run():
    import torch
    from bench import direct_prompt, synthetic_prompt
    from moss_tts_amd.engine import Engine, EngineConfig
    from moss_tts_amd.processing_moss_tts import left_pad
    # MFMA_SHAPES: b1 (the clone prompt), b32 (32 ragged utterances), ttsd (one 2,117-token prompt)
    shapes = os.environ.get("MFMA_SHAPES", "b1,b32").split(",")
    eng = Engine(EngineConfig(layers=LAYERS, max_batch=32, max_ctx=2304, max_prefill_tokens=8192), 0)
    eng.init_random(0)
    rng = np.random.default_rng(1)
    out = {}
    if "b1" in shapes:
        one = torch.from_numpy(synthetic_prompt(dict(n_vq=32), rng)[None]).cuda()
        for _ in range(3):
            eng.forward(one, torch.ones(1, one.shape[1], dtype=torch.uint8, device="cuda"), 0)
        out["B1_tokens"] = int(one.shape[1])
    if "b32" in shapes:
        lens = np.random.default_rng(0).integers(100, 131, 32)
        p = left_pad([torch.from_numpy(direct_prompt(rng, int(T))) for T in lens], 151643, 1024)
        ids32, mask32 = p["input_ids"].cuda(), p["attention_mask"].cuda()
        for _ in range(2):
            eng.forward(ids32, mask32, 0)
        out["B32_tokens"] = int(ids32.shape[0] * ids32.shape[1])
    if "ttsd" in shapes:
        long = torch.from_numpy(direct_prompt(rng, 2117)[None]).cuda()
        for _ in range(2):
            eng.forward(long, torch.ones(1, long.shape[1], dtype=torch.uint8, device="cuda"), 0)
        out["ttsd_tokens"] = int(long.shape[1])
    torch.cuda.synchronize()
    print(json.dumps(out))
    eng.close()


def summarize(d):
    per = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0]
            if "gemm" not in k and "attn_prefill" not in k:
                continue
            key = (k, r.get("Dispatch_Id", r.get("Correlation_Id", "")))
            per.setdefault(key, {})[r["Counter_Name"]] = per.setdefault(key, {}).get(r["Counter_Name"], 0.0) + \
                float(r["Counter_Value"])
    agg = {}
    for (k, _), c in per.items():
        if "SQ_VALU_MFMA_BUSY_CYCLES" not in c or "GRBM_GUI_ACTIVE" not in c:
            continue
        a = agg.setdefault(k, {"dispatches": 0, "mfma_busy": 0.0, "cycles": 0.0, "utils": []})
        cyc = c["GRBM_GUI_ACTIVE"] / 8.0
        a["dispatches"] += 1
        a["mfma_busy"] += c["SQ_VALU_MFMA_BUSY_CYCLES"]
        a["cycles"] += cyc
        a["utils"].append(c["SQ_VALU_MFMA_BUSY_CYCLES"] / max(cyc * 1024.0, 1.0))
    out = {"counters": "SQ_VALU_MFMA_BUSY_CYCLES, GRBM_GUI_ACTIVE (one pass, kernel trace)",
           "util_def": "MFMA_BUSY / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs)", "kernels": {}}
    for k, a in sorted(agg.items(), key=lambda kv: -kv[1]["mfma_busy"]):
        out["kernels"][k] = {"dispatches": a["dispatches"],
                             "mfma_util_weighted": round(a["mfma_busy"] / max(a["cycles"] * 1024.0, 1.0), 4),
                             "mfma_util_median": round(float(np.median(a["utils"])), 4),
                             "mfma_util_max": round(float(np.max(a["utils"])), 4)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--summarize")
    a = ap.parse_args()
    summarize(a.summarize) if a.summarize else run()
