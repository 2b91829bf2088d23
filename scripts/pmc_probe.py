#!/usr/bin/env python3
"""Launch the bench's dominant kernel on its own (the decode step's gate|up GEMV instance, via
mtts_engine_time_gemv: layers rotated, so no launch re-reads a matrix the previous one left in
the 256 MB MALL; --config local: the depth stack's gate|up at B=8, its 4 layers walked as the
frame walks them; --config pse / pse4: the batch-1 / batch-4 persistent streaming decode launch, every
layer) for
rocprofv3 PMC passes:

    rocprofv3 --pmc FETCH_SIZE --kernel-trace -d D -o f --output-format csv -- python3 scripts/pmc_probe.py --config clone
    rocprofv3 --pmc WRITE_SIZE --kernel-trace -d D -o w --output-format csv -- python3 scripts/pmc_probe.py --config clone
    python3 scripts/pmc_probe.py --summarize D --config clone > profiles/<round>_pmc_<config>.json

HBM traffic per launch = 2 x FETCH_SIZE (gfx950 tallies wide coalesced reads at half their
bytes, MI355X_MICROARCH.md 'HBM') + WRITE_SIZE, both in KiB as rocprofv3 reports them."""
import argparse
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(cfg_name, iters):
    import ctypes
    import torch
    from moss_tts_amd.engine import Engine, EngineConfig
    from moss_tts_amd import _native as N
    if cfg_name == "local":
        cfg = EngineConfig(hidden=2048, layers=28, n_heads=16, n_kv=8, head_dim=128, inter=6144, n_vq=32, max_batch=8,
                           max_ctx=512, model_kind=1, local_hidden=1536, local_layers=4, local_inter=8960,
                           local_mlp_ffn=2048)
        B = 8
    else:
        B = 4 if cfg_name == "pse4" else 1
        cfg = EngineConfig(max_batch=B, max_ctx=512)
    eng = Engine(cfg, 0)
    eng.init_random(0)
    which = 6 if cfg_name == "local" else 2  # local: the depth stack's gate|up (the frame's dominant launch)
    if cfg_name in ("pse", "pse4"):  # the decode stack as one persistent launch (pse.hip / pse4.hip)
        if not (eng.pse_active() if cfg_name == "pse" else eng.pse4_active()):
            raise SystemExit("persistent streaming decode inactive")
        which = 5
    ms, nb = ctypes.c_float(), ctypes.c_uint64()
    N.check(N.load().mtts_engine_time_gemv(eng._h, which, 0, B, iters, ctypes.byref(ms), ctypes.byref(nb)), "time_gemv")
    torch.cuda.synchronize()
    print(json.dumps({"avg_launch_us": ms.value * 1e3, "alg_bytes": nb.value, "B": B}))
    eng.close()


def summarize(d, cfg_name):
    vals = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            want = {"pse": "pse_kernel", "pse4": "pse4_kernel"}.get(cfg_name, "gemv_kernel")
            if want not in r["Kernel_Name"]:
                continue
            vals.setdefault(r["Counter_Name"], {}).setdefault(r["Kernel_Name"], []).append(float(r["Counter_Value"]))
    out = {"config": cfg_name, "unit_raw": "KiB (rocprofv3 FETCH_SIZE / WRITE_SIZE)"}
    for name, per_k in vals.items():
        # the dominant (most launched) gemv instance = the probed gate|up kernel
        k, v = max(per_k.items(), key=lambda kv: len(kv[1]))
        v = sorted(v)[1:] if len(v) > 2 else v  # drop the first-touch launch
        out[name] = {"kernel": k, "launches": len(v), "mean_kib": sum(v) / len(v)}
    fetch = out.get("FETCH_SIZE", {}).get("mean_kib")
    write = out.get("WRITE_SIZE", {}).get("mean_kib")
    if fetch is not None and write is not None:
        out["traffic_bytes_per_launch"] = int((2 * fetch + write) * 1024)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", choices=["clone", "local", "pse", "pse4"], default="clone")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--summarize", default=None)
    a = ap.parse_args()
    if a.summarize:
        summarize(a.summarize, a.config)
    else:
        run(a.config, a.iters)
