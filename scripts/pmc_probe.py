#!/usr/bin/env python3
"""Launch the bench's dominant kernel on its own (the decode step's gate|up GEMV instance, via
mtts_engine_time_gemv: layers rotated, so no launch re-reads a matrix the previous one left in
the 256 MB MALL; --config local: the depth stack's gate|up at B=8, its 4 layers walked as the
frame walks them; --config pse / pse4: the batch-1 / batch-4 persistent streaming decode launch, every
layer; --config ttsd: WHOLE decode steps of the TTSD long form at its mean context, i.e. every
kernel of the captured decode graph) for rocprofv3 PMC passes:

    rocprofv3 --pmc FETCH_SIZE --kernel-trace -d D -o f --output-format csv -- python3 scripts/pmc_probe.py --config clone
    rocprofv3 --pmc WRITE_SIZE --kernel-trace -d D -o w --output-format csv -- python3 scripts/pmc_probe.py --config clone
    python3 scripts/pmc_probe.py --summarize D --config clone > profiles/<round>_pmc_<config>.json

HBM traffic per launch = 2 x FETCH_SIZE (gfx950 tallies wide coalesced reads at half their
bytes, MI355X_MICROARCH.md 'HBM') + WRITE_SIZE, both in KiB as rocprofv3 reports them."""
import argparse
import collections
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


TTSD_TEXT, TTSD_A, TTSD_B = 5750, 24, 56  # prompt 5,867 rows = the bench's mean TTSD context (2,117 + 7,519 / 2)
LOCAL_A, LOCAL_B = 2, 6  # MossTTSLocal frames of the two generations (--config local_frame; ~1,050 dispatches a frame:
# rocprofv3 --pmc crashed on the host collecting 2 x 24 frames of graph replays)


def run_local_frame():
    """Two greedy MossTTSLocal generations (the 1.7B shape, B = 8, bench.py's ragged prompts) of
    LOCAL_A and LOCAL_B frames: identical prefills and first LOCAL_A frames, so the counters of the
    second minus the first are LOCAL_B - LOCAL_A whole frames (hipGraph replays: the backbone step,
    33 channels of depth transformer + adapters + norm + head + pick, the frame end)."""
    import numpy as np
    import torch
    from bench import local_prompt
    from moss_tts_amd.engine import Engine, EngineConfig
    os.environ.setdefault("MTTS_LOCAL_NO_GRAPH", "1")  # direct launches (the same kernels) for the profiler
    rng = np.random.default_rng(1)
    B = 8
    prompts = [local_prompt(rng, text_tokens=int(n)) for n in rng.integers(36, 61, B)]
    T = max(p.shape[0] for p in prompts)
    ids = np.full((B, T, 33), 1024, np.int64)
    ids[..., 0] = 151643
    mask = np.zeros((B, T), bool)
    for b, p in enumerate(prompts):
        ids[b, T - p.shape[0]:] = p
        mask[b, T - p.shape[0]:] = True
    eng = Engine(EngineConfig(hidden=2048, layers=28, n_heads=16, n_kv=8, head_dim=128, inter=6144, n_vq=32,
                              max_batch=B, max_ctx=T + LOCAL_B + 16, max_prefill_tokens=256 * B, model_kind=1,
                              local_hidden=1536, local_layers=4, local_inter=8960, local_mlp_ffn=2048), 0)
    eng.init_random(0)
    ids_d, mask_d = torch.from_numpy(ids).cuda(), torch.from_numpy(mask).cuda()
    for n in (LOCAL_A, LOCAL_B):
        eng.local_generate_ids(ids_d, mask_d, n, -1, chunk=32)
        torch.cuda.synchronize()
    kv = 28 * 2 * 8 * 128 * 2 * B * (T + (LOCAL_A + LOCAL_B) / 2)
    print(json.dumps({"T": T, "frames": [LOCAL_A, LOCAL_B], "lpse": eng.lpse_active(),
                      "alg_bytes_per_frame": int(eng.local_frame_bytes(-1) + kv)}))
    eng.close()


def run_ttsd():
    """Two greedy generations from one ~5.9 K-token TTSD-shaped prompt (n_vq 16), the same forced
    schedule, max_new TTSD_A then TTSD_B: identical prefills and first TTSD_A steps, so the
    counters of the second minus the first are TTSD_B - TTSD_A whole decode steps (hipGraph replays:
    the batch-1 persistent launch's long form + embedding, final norm, heads, samplers)."""
    import numpy as np
    import torch
    from bench import synthetic_prompt, forced_schedule
    from moss_tts_amd.engine import Engine, EngineConfig, sampling_params
    n_vq = 16
    ids = synthetic_prompt(dict(n_vq=n_vq), np.random.default_rng(1), text_tokens=TTSD_TEXT)  # [T, 1 + n_vq]
    T = ids.shape[0]
    eng = Engine(EngineConfig(n_vq=n_vq, max_batch=1, max_ctx=T + TTSD_B + 64, max_prefill_tokens=1024), 0)
    eng.init_random(0)
    ids_d = torch.from_numpy(ids[None]).cuda()
    mask_d = torch.ones((1, T), dtype=torch.uint8, device="cuda")
    forced = torch.from_numpy(forced_schedule(TTSD_B, n_vq, TTSD_B - (n_vq + 3))).cuda()
    sp = sampling_params(text_temperature=0, audio_temperature=0)
    for n in (TTSD_A, TTSD_B):
        eng.generate_ids(ids_d, mask_d, n, sp, forced_text=forced, chunk=16)
        torch.cuda.synchronize()
    wl = eng.weight_bytes() - (min(151645, 151656, 151662) // 16) * 16 * 4096 * 2  # text head gated off
    kv = 36 * 2 * 8 * 128 * 2 * (T + (TTSD_A + TTSD_B) / 2 + 1)
    print(json.dumps({"T": T, "steps": [TTSD_A, TTSD_B], "pse_long": eng.pse_long_active(),
                      "alg_bytes_per_step": int(wl + kv)}))
    eng.close()


def summarize_ttsd(d, cfg_name="ttsd"):
    """per-step bytes = (second generation - first) / (TTSD_B - TTSD_A); a generation starts at
    the first prefill GEMM after a decode-step kernel (local_frame: per frame, LOCAL_B - LOCAL_A)"""
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            key = r.get("Dispatch_Id") or r.get("Correlation_Id") or str(len(rows))
            rows.append((int(key), r["Kernel_Name"], r["Counter_Name"], float(r["Counter_Value"])))
    local = cfg_name == "local_frame"
    n_a, n_b = (LOCAL_A, LOCAL_B) if local else (TTSD_A, TTSD_B)
    out = {"config": cfg_name, "unit_raw": "KiB (rocprofv3 FETCH_SIZE / WRITE_SIZE)",
           "what": (f"whole MossTTSLocal frames (B = 8, ragged prompts): generation of {n_b} frames minus one of {n_a}"
                    if local else
                    f"whole decode steps at the mean TTSD context: generation of {n_b} steps minus one of {n_a}")}
    for cname in sorted({r[2] for r in rows}):
        seq = sorted((r for r in rows if r[2] == cname), key=lambda r: r[0])
        seg, dec_seen, tot = -1, True, [0.0, 0.0]
        per_k = [collections.defaultdict(float), collections.defaultdict(float)]
        for _, kname, _, v in seq:
            if "gemm" in kname and dec_seen:
                seg, dec_seen = seg + 1, False
            if "pse_kernel" in kname or "finalize" in kname or "attn_decode" in kname or "lpse" in kname:
                dec_seen = True
            if 0 <= seg < 2:
                tot[seg] += v
                per_k[seg][kname.split("(")[0]] += v
        steps = n_b - n_a
        by_kernel = {k: round((per_k[1][k] - per_k[0].get(k, 0.0)) / steps, 1) for k in per_k[1]}
        by_kernel = dict(sorted(by_kernel.items(), key=lambda kv: -kv[1])[:8])
        out[cname] = {"segments": seg + 1, "gen_kib": tot, "per_step_kib": (tot[1] - tot[0]) / steps,
                      "per_step_kib_by_kernel": by_kernel}
    fetch = out.get("FETCH_SIZE", {}).get("per_step_kib")
    write = out.get("WRITE_SIZE", {}).get("per_step_kib")
    if fetch is not None and write is not None:
        out["traffic_bytes_per_launch"] = int((2 * fetch + write) * 1024)
        out["traffic_unit"] = ("bytes per frame (hipGraph replay, every kernel)" if local else
                               "bytes per decode step (hipGraph replay, every kernel)")
    print(json.dumps(out, indent=1))


def run(cfg_name, iters):
    import ctypes
    import torch
    from moss_tts_amd.engine import Engine, EngineConfig
    from moss_tts_amd import _native as N
    if cfg_name == "ttsd":
        return run_ttsd()
    if cfg_name == "local_frame":
        return run_local_frame()
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
    if cfg_name in ("ttsd", "local_frame"):
        return summarize_ttsd(d, cfg_name)
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
    ap.add_argument("--config", choices=["clone", "local", "local_frame", "pse", "pse4", "ttsd"], default="clone")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--summarize", default=None)
    a = ap.parse_args()
    if a.summarize:
        summarize(a.summarize, a.config)
    else:
        run(a.config, a.iters)
