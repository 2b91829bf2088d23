#!/usr/bin/env python3
"""Benchmark: MossTTSDelay generate() throughput (audio-seconds/sec) on MI355X.

Workload (BASELINE.json configs[1]): MossTTSDelay-8B shape (Qwen3-8B backbone, 36 layers,
h 4096, 32/8 heads, I 12288, V 151936, n_vq 32), bf16, random-init weights (no checkpoint
is available offline), batch 1 per GPU, a synthetic zero-shot-clone prompt (3 s of
reference audio = 38 frames in a user audio block + a 200-character text, T = 180 tokens),
greedy decoding with a forced text schedule of 208 steps (audio_start, 173 gen slots,
the delay tail, audio_end, im_end) so every run does the same work.

One "step" = one complete generate() call (prefill + 208 hipGraph decode steps) for the
batch resident in HBM.  value = audio seconds produced by all ranks / max-over-ranks wall
time.  Run N GPUs with torch.distributed.run (one process per GPU, no collective in the
data path: utterances are independent, weak scaling).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "audio-seconds/sec/GPU (RTF) + p50 first-chunk latency, MossTTSDelay b=1/32"
FRAME_RATE = 12.5
HBM_PEAK_GBS = 8000.0


def synthetic_prompt(cfg, rng, text_tokens=48, ref_frames=38, template_tokens=56):
    """Clone prompt laid out like processing_moss_tts.py:539-641 (user turn with an audio
    block of ref_frames delayed frames, assistant header); random ids stand in for text."""
    n_vq, pad = cfg["n_vq"], 1024
    rows = []

    def text(t):
        rows.append([int(t)] + [pad] * n_vq)

    text(151644)
    for t in rng.integers(200, 20000, template_tokens):
        text(t)
    codes = rng.integers(0, 1024, (ref_frames, n_vq))
    dl = np.full((ref_frames + n_vq - 1, n_vq), pad, np.int64)
    for i in range(n_vq):
        dl[i:i + ref_frames, i] = codes[:, i]
    text(151652)
    for r in dl:
        rows.append([151654] + [int(v) for v in r])
    text(151653)
    for t in rng.integers(200, 20000, text_tokens):
        text(t)
    for t in (151645, 198, 151644, 77091, 198):
        text(t)
    return np.array(rows, np.int64)


def direct_prompt(rng, T, n_vq=32):
    """configs[2]'s direct-generation prompt of T rows (no reference audio; processing_moss_tts.py
    :539-641): <|im_start|>, T - 6 text ids standing in for the templated 200-character request,
    <|im_end|>, then the assistant header"""
    pad = 1024
    rows = [[151644] + [pad] * n_vq]
    rows += [[int(t)] + [pad] * n_vq for t in rng.integers(200, 20000, T - 6)]
    rows += [[t] + [pad] * n_vq for t in (151645, 198, 151644, 77091, 198)]
    return np.array(rows, np.int64)


def dp_global_leg(eng, world, rank, n_steps, forced, sp, per_gpu=4, reps=2):
    """BASELINE configs[2] as written: ONE global batch of per_gpu x world synthetic prompts with
    ragged lengths T in [100, 130] (seed 0), left-padded GLOBALLY (positions include
    the pads, TF/models/qwen3/modeling_qwen3.py:386-389), row-sharded over the ranks by
    moss_tts_amd.dp.generate_dp (each rank's engine generates its contiguous shard; one gather of
    the finished rows at the end, right-padded to the global step count).  At 8 GPUs this is the
    32-utterance batch; per-GPU work is fixed (weak scaling)."""
    import torch
    import torch.distributed as dist
    from moss_tts_amd.dp import generate_dp
    from moss_tts_amd.processing_moss_tts import left_pad
    rng = np.random.default_rng(0)
    B = per_gpu * world
    lens = rng.integers(100, 131, B)
    padded = left_pad([torch.from_numpy(direct_prompt(rng, int(T))) for T in lens], 151643, 1024)
    ids, mask = padded["input_ids"], padded["attention_mask"]

    def gen(ids_s, mask_s, **kw):
        out = eng.generate_ids(ids_s.cuda(), mask_s.cuda(), n_steps, sp, forced_text=forced, chunk=16)
        hit = (ids_s[..., 0] == 151644).int()
        starts = (ids_s.shape[1] - 1 - hit.flip(1).argmax(1) + 3).tolist()  # last <|im_start|> + 3 (:518-525)
        return [(ids_s.shape[1] - s_, out[b, s_:]) for b, s_ in enumerate(starts)]

    def sync():
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    out = generate_dp(gen, ids, mask)  # warm-up (graph capture)
    sync()
    t0 = time.perf_counter()
    for _ in range(reps):
        out = generate_dp(gen, ids, mask)
    sync()
    dt = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device="cuda")
    if world > 1:
        dist.all_reduce(dt, op=dist.ReduceOp.MAX)
    dt = float(dt[0])
    frames = [count_audio_frames(rows.numpy(), int(sl), 32) for sl, rows in out]
    audio_s = sum(frames) / FRAME_RATE * reps
    # first-chunk latency of this rank's shard (its per-GPU batch, global padding): prefill + the
    # decode steps until the first 1 s of audio (13 frames) has all 32 codebooks (frame f is final
    # n_vq - 1 steps after its first code, processing_moss_tts.py:515-525); p50 over 5 runs
    import ctypes
    from moss_tts_amd import _native as Nn
    from moss_tts_amd.dp import shard_bounds
    lo, hi = shard_bounds(B, world, rank)
    ids_d = ids[lo:hi].contiguous().cuda()
    mask_d = mask[lo:hi].to(torch.uint8).contiguous().cuda()
    first_steps = 1 + 13 + 32
    lat = []
    for _ in range(5):
        torch.cuda.synchronize()
        a = time.perf_counter()
        Nn.check(Nn.load().mtts_generate_begin(eng._h, ctypes.c_void_p(ids_d.data_ptr()), ctypes.c_void_p(mask_d.data_ptr()),
                                               hi - lo, int(ids.shape[1]), n_steps, ctypes.byref(sp),
                                               ctypes.c_void_p(forced.data_ptr()), None), "begin")
        Nn.check(Nn.load().mtts_generate_decode(eng._h, first_steps - 1, None), "decode")
        Nn.check(Nn.load().mtts_generate_poll(eng._h, None, None, None), "poll")
        lat.append((time.perf_counter() - a) * 1e3)
    p50 = torch.tensor([float(np.median(lat))], dtype=torch.float64, device="cuda")
    if world > 1:
        dist.all_reduce(p50, op=dist.ReduceOp.MAX)
    return {"workload": f"BASELINE configs[2] form: MossTTSDelay bf16, one global batch of {B} synthetic direct prompts "
                        f"(T {int(lens.min())}-{int(lens.max())}, seed 0), global left padding, row-sharded data "
                        f"parallel over {world} GPU(s) via moss_tts_amd.dp.generate_dp (gather + right-pad)",
            "global_batch": B, "per_gpu": per_gpu, "n_gpus": world, "reps": reps,
            "audio_s_per_s": round(audio_s / dt, 3), "audio_s_per_s_per_gpu": round(audio_s / dt / world, 3),
            "ms_per_global_batch": round(dt / reps * 1e3, 2), "frames_per_utt": int(np.median(frames)),
            "padded_T": int(ids.shape[1]),
            "p50_first_chunk_ms": round(float(p50[0]), 2),
            "first_chunk_def": (f"per-GPU shard of {hi - lo} rows (max over ranks): prefill + {first_steps - 1} decode "
                                "steps (first 1 s of audio codes complete), codec excluded")}


def forced_schedule(n_steps, n_vq, gen_frames):
    """text decisions for rows that sample: audio_start, gen slots, delay slot, ..., im_end"""
    f = np.full(n_steps, -1, np.int32)
    f[0] = 151652
    f[1:1 + gen_frames] = 151656
    f[1 + gen_frames] = 151662
    f[n_steps - 1] = 151645
    return f


def count_audio_frames(gen_row, start, n_vq):
    import torch
    from moss_tts_amd.processing_moss_tts import split_audio_segments
    a = torch.from_numpy(gen_row[start:, 1:])
    segs = split_audio_segments(a, 1024) if a.shape[0] >= n_vq else []
    return sum(int(s.shape[0]) for s in segs)


def _torch_cpu_layer(W, h, cos, sin, kc, vc, pos0, n_heads, n_kv, D, eps=1e-6):
    """One Qwen3 decoder layer in torch-CPU ops (the oracle's decoder_layer restated on
    torch matmuls: `TF/models/qwen3/modeling_qwen3.py:294-323`), appending to the caches."""
    import torch
    import torch.nn.functional as F

    def rms(x, w):
        return w * (x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + eps))

    def rope(x):
        half = x.shape[-1] // 2
        return x * cos + torch.cat([-x[..., half:], x[..., :half]], -1) * sin

    B, S, H = h.shape
    x = rms(h, W["in"])
    q = (x @ W["q"].T).view(B, S, n_heads, D)
    k = (x @ W["k"].T).view(B, S, n_kv, D)
    v = (x @ W["v"].T).view(B, S, n_kv, D)
    q = rope(rms(q, W["qn"]).transpose(1, 2))
    k = rope(rms(k, W["kn"]).transpose(1, 2))
    kc[:, :, pos0:pos0 + S] = k
    vc[:, :, pos0:pos0 + S] = v.transpose(1, 2)
    K, V = kc[:, :, :pos0 + S], vc[:, :, :pos0 + S]
    a = F.scaled_dot_product_attention(q, K, V, is_causal=S > 1, enable_gqa=True)
    h = h + a.transpose(1, 2).reshape(B, S, n_heads * D) @ W["o"].T
    x = rms(h, W["post"])
    return h + (F.silu(x @ W["g"].T) * (x @ W["u"].T)) @ W["d"].T


def cpu_baseline(args, T, n_steps, frames, timed_steps=8):
    """A CPU restatement of the decode path at the full 8B shape in bf16 torch-CPU ops (the
    oracle's layer math on torch matmuls, in the reference deployment's dtype: `torch_dtype=bf16`,
    clis/moss_tts_app.py:95-107) on this host's cores.  Round 5: WHOLE steps timed end to end -- the
    33-channel embedding sum, 36 decoder layers with their own KV caches, the final norm, the 1+32
    heads and the greedy picks -- a full prefill over the T prompt tokens, then `timed_steps` decode
    steps after one untimed warm-up step; the utterance is prefill + n_steps x the mean step.  (One
    layer's weights serve all 36 layers: 385 MB per layer does not stay in the host caches, so every
    layer still streams its bytes from DRAM, and the 14 GB a distinct set would need is not
    generated.)  SURVEY.md §6 measured the reference's own torch-CPU path at 0.44 s per decode step
    (0.18 audio-s/s) on the 8-core build container."""
    import torch
    cores = torch.get_num_threads()
    H, I, D, nh, nkv, L, n_vq, V, A = 4096, 12288, 128, 32, 8, 36, 32, 151936, 1025
    g = torch.Generator().manual_seed(0)
    bf = torch.bfloat16

    base = torch.empty(1 << 20, dtype=bf).uniform_(-1.0, 1.0, generator=g)

    def rnd(*shape):  # uniform(-1, 1) * sqrt(3 / K) (variance 1 / K): a 1 M-value random block tiled, since
        # a generator fills ~0.1 G values/s single-threaded and the values do not change the work
        t = torch.empty(*shape, dtype=bf)
        flat = t.view(-1)
        n = flat.numel()
        full = n // base.numel()
        if full:
            flat[:full * base.numel()].view(full, -1).copy_(base.expand(full, -1))
        flat[full * base.numel():] = base[:n - full * base.numel()]
        return t.mul_((3.0 / shape[-1]) ** 0.5)

    one = lambda n: torch.ones(n, dtype=bf)  # noqa: E731
    W = {"q": rnd(nh * D, H), "k": rnd(nkv * D, H), "v": rnd(nkv * D, H), "o": rnd(H, nh * D), "g": rnd(I, H),
         "u": rnd(I, H), "d": rnd(H, I), "in": one(H), "post": one(H), "qn": one(D), "kn": one(D)}
    heads = rnd(V + n_vq * A, H)
    emb_t = rnd(V, H)
    emb_a = rnd(n_vq, A, H)
    inv = 1.0 / (1e6 ** (torch.arange(0, D, 2, dtype=torch.float32) / D))
    C = T + timed_steps + 2
    f = torch.arange(C, dtype=torch.float32)[:, None] * inv[None]
    cos, sin = torch.cat([f, f], -1).cos().to(bf), torch.cat([f, f], -1).sin().to(bf)
    kcs = [torch.zeros(1, nkv, C, D, dtype=bf) for _ in range(L)]
    vcs = [torch.zeros(1, nkv, C, D, dtype=bf) for _ in range(L)]
    ids = torch.randint(0, 1024, (1, T, n_vq + 1), generator=g)

    def step(ids_s, pos0):
        S = ids_s.shape[1]
        h = emb_t[ids_s[..., 0]]
        for j in range(n_vq):  # the 33-way embedding sum (modeling_moss_tts.py:196-213)
            h = h + emb_a[j][ids_s[..., j + 1]]
        for l in range(L):
            h = _torch_cpu_layer(W, h, cos[pos0:pos0 + S], sin[pos0:pos0 + S], kcs[l], vcs[l], pos0, nh, nkv, D)
        x = h[:, -1]
        x = x * torch.rsqrt(x.float().pow(2).mean(-1, keepdim=True) + 1e-6).to(bf)
        lg = x @ heads.T  # 1 + 32 heads (:279-300)
        nxt = torch.empty(1, 1, n_vq + 1, dtype=torch.long)
        nxt[0, 0, 0] = lg[0, :V].argmax()
        nxt[0, 0, 1:] = lg[0, V:].view(n_vq, A)[:, :A - 1].argmax(-1)
        return nxt

    with torch.inference_mode():
        t0 = time.perf_counter()
        cur = step(ids, 0)
        t_prefill = time.perf_counter() - t0
        cur = step(cur, T)  # warm-up decode step (untimed)
        t0 = time.perf_counter()
        for s in range(timed_steps):
            cur = step(cur, T + 1 + s)
        t_step = (time.perf_counter() - t0) / timed_steps
    del W, heads, emb_t, emb_a, kcs, vcs
    utt = t_prefill + n_steps * t_step
    return {"value": round(frames / FRAME_RATE / utt, 5), "unit": "audio-s/s", "cores": int(cores), "kind": "port",
            "sample": (f"bf16 torch-CPU restatement of the whole decode path at the 8B shape, batch 1: a full prefill "
                       f"(36 layers over T={T} tokens + heads, {t_prefill:.2f}s) and {timed_steps} whole decode steps "
                       f"(embedding sum, 36 layers, norm, 1+32 heads, greedy picks; {t_step * 1e3:.0f}ms each) timed end "
                       f"to end; one utterance = prefill + {n_steps} steps = {utt:.1f}s"),
            "reference_measured_in_build_container": "SURVEY.md §6: the reference's torch-CPU decode step 0.44 s "
                                                      "(0.18 audio-s/s), 8 cores"}


def pmc_traffic(config):
    """HBM bytes per launch of the roofline kernel from the newest committed rocprofv3 PMC
    summary (profiles/r*_pmc_<config>.json, made by scripts/pmc_round.sh: separate FETCH_SIZE /
    WRITE_SIZE passes over the same kernel instance, 2 x FETCH_SIZE + WRITE_SIZE per the gfx950
    correction); None when absent."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"r*_pmc_{config}.json")))
    if not files:
        return None, None
    try:
        d = json.load(open(files[-1]))
        return int(d["traffic_bytes_per_launch"]), os.path.relpath(files[-1], ROOT)
    except Exception:
        return None, None


def local_prompt(rng, n_vq=32, text_tokens=48, ref_frames=38, template_tokens=56):
    """MossTTSLocal clone prompt (moss_tts_local/processing_moss_tts.py:597-641): user turn with
    an aligned (undelayed) reference-audio block, then the assistant header + audio_start"""
    pad = 1024
    rows = []

    def text(t):
        rows.append([int(t)] + [pad] * n_vq)

    text(151644)
    for t in rng.integers(200, 20000, template_tokens):
        text(t)
    text(151652)
    for r in rng.integers(0, 1024, (ref_frames, n_vq)):
        rows.append([151654] + [int(v) for v in r])
    text(151653)
    for t in rng.integers(200, 20000, text_tokens):
        text(t)
    for t in (151645, 198, 151644, 77091, 198, 151652):
        text(t)
    return np.array(rows, np.int64)


def cpu_baseline_local(T, frames):
    """oracle.moss_local (numpy fp32) at the MossTTSLocal-1.7B shape on this host's cores, on a
    bounded sample: 1 backbone prefill layer (T tokens), 2 backbone decode layer-steps, 2
    depth-transformer layer-steps (at channel position 16), one adapter pair and the text and
    one audio head; composed into one utterance of `frames` frames (28 backbone layers +
    33 channels x (4 depth layers + adapters + head) per frame)."""
    from oracle import moss_delay as O
    from oracle import moss_local as L
    try:
        from threadpoolctl import threadpool_info
        cores = max([p.get("num_threads", 1) for p in threadpool_info()] or [os.cpu_count() or 1])
    except Exception:
        cores = os.cpu_count() or 1
    cfg = L.LCfg()
    ctx = O._Ctx("fp32")
    rng = np.random.default_rng(0)
    D = cfg.head_dim

    def rnd(shape, s=None):
        return rng.standard_normal(shape, dtype=np.float32) * np.float32(s if s else shape[-1] ** -0.5)

    def layer_w(pf, H, I):
        return {pf + "self_attn.q_proj.weight": rnd((cfg.n_heads * D, H)), pf + "self_attn.k_proj.weight": rnd((cfg.n_kv * D, H)),
                pf + "self_attn.v_proj.weight": rnd((cfg.n_kv * D, H)), pf + "self_attn.o_proj.weight": rnd((H, cfg.n_heads * D)),
                pf + "self_attn.q_norm.weight": np.ones(D, np.float32), pf + "self_attn.k_norm.weight": np.ones(D, np.float32),
                pf + "mlp.gate_proj.weight": rnd((I, H)), pf + "mlp.up_proj.weight": rnd((I, H)),
                pf + "mlp.down_proj.weight": rnd((H, I)), pf + "input_layernorm.weight": np.ones(H, np.float32),
                pf + "post_attention_layernorm.weight": np.ones(H, np.float32)}

    H, LH = cfg.hidden, cfg.local_hidden
    bp, lp = "b.", "l."
    W = {**layer_w(bp, H, cfg.inter), **layer_w(lp, LH, cfg.local_inter)}
    cos, sin = O.rope_cos_sin(ctx, cfg, np.arange(T + 4))
    cache = L.Cache(1)
    t0 = time.perf_counter()
    L.decoder_layer(ctx, W, cfg, bp, rnd((1, T, H), 1.0), cos[:T], sin[:T], cache, 0, np.ones((1, T), bool), np.arange(T))
    t_pf = time.perf_counter() - t0
    t0 = time.perf_counter()
    for s in range(2):
        L.decoder_layer(ctx, W, cfg, bp, rnd((1, 1, H), 1.0), cos[T + s:T + s + 1], sin[T + s:T + s + 1], cache, 0,
                        np.ones((1, T + s + 1), bool), np.array([T + s]))
    t_bl = (time.perf_counter() - t0) / 2
    lc = L.Cache(1)
    for s in range(16):
        L.decoder_layer(ctx, W, cfg, lp, rnd((1, 1, LH), 1.0), None, None, lc, 0, np.ones((1, s + 1), bool), np.array([s]))
    t0 = time.perf_counter()
    for s in range(2):
        L.decoder_layer(ctx, W, cfg, lp, rnd((1, 1, LH), 1.0), None, None, lc, 0, np.ones((1, 17 + s), bool),
                        np.array([16 + s]))
    t_ll = (time.perf_counter() - t0) / 2
    F = cfg.mlp_ffn
    A = {"i.gate_proj.weight": rnd((F, H)), "i.up_proj.weight": rnd((F, H)), "i.down_proj.weight": rnd((LH, F)),
         "o.gate_proj.weight": rnd((F, LH)), "o.up_proj.weight": rnd((F, LH)), "o.down_proj.weight": rnd((H, F))}
    t0 = time.perf_counter()
    L.swiglu_mlp(ctx, A, "i.", rnd((1, H), 1.0))
    L.swiglu_mlp(ctx, A, "o.", rnd((1, LH), 1.0))
    t_ad = time.perf_counter() - t0
    del W, A
    x = rnd((1, H), 1.0)
    th = rnd((cfg.vocab, H))
    t0 = time.perf_counter()
    _ = x @ th.T
    t_th = time.perf_counter() - t0
    del th
    ah = rnd((cfg.audio_vocab + 1, H))
    t0 = time.perf_counter()
    _ = x @ ah.T
    t_ah = time.perf_counter() - t0
    C = cfg.n_vq + 1
    frame = cfg.layers * t_bl + C * (cfg.local_layers * t_ll + t_ad) + t_th + cfg.n_vq * t_ah
    utt = cfg.layers * t_pf + frames * frame
    return {"value": round(frames / FRAME_RATE / utt, 5), "unit": "audio-s/s", "cores": int(cores), "kind": "port",
            "sample": (f"oracle.moss_local fp32 at the 1.7B shape, batch 1: 1 prefill layer (T={T}, {t_pf:.2f}s), "
                       f"backbone layer-step {t_bl * 1e3:.1f}ms, depth layer-step {t_ll * 1e3:.1f}ms, adapters "
                       f"{t_ad * 1e3:.1f}ms, text head {t_th * 1e3:.0f}ms, audio head {t_ah * 1e3:.1f}ms; composed to "
                       f"one utterance of {frames} frames = {utt:.1f}s")}


def main_local(args, world, rank, local):
    """BASELINE configs[3]: MossTTSLocal-1.7B shape, bf16, batch 8 per GPU, greedy depth loop
    over 1 + 32 channels per frame, 173 frames (13.84 s of audio) per utterance."""
    import ctypes
    import torch
    import torch.distributed as dist
    from moss_tts_amd.engine import Engine, EngineConfig
    from moss_tts_amd import _native as Nn
    B = args.batch if args.batch > 1 else 8
    frames = args.decode_steps if args.decode_steps != 208 else 173
    rng = np.random.default_rng(1 + rank)
    # ragged, as configs[3]'s 8 different 200-char prompts are: 36-60 text tokens per row, left-padded
    # the processor's way (`_pad`, moss_tts_local/processing_moss_tts.py:415-436; the backbone's
    # positions then exclude each row's pads, as GenerationMixin's do)
    prompts = [local_prompt(rng, text_tokens=int(n)) for n in rng.integers(36, 61, B)]
    T = max(p.shape[0] for p in prompts)
    ids = np.full((B, T, 33), 1024, np.int64)
    ids[..., 0] = 151643
    mask = np.zeros((B, T), bool)
    for b, p in enumerate(prompts):
        ids[b, T - p.shape[0]:] = p
        mask[b, T - p.shape[0]:] = True
    ecfg = EngineConfig(hidden=2048, layers=args.layers if args.layers != 36 else 28, n_heads=16, n_kv=8, head_dim=128,
                        inter=6144, n_vq=32, max_batch=B, max_ctx=T + frames + 16, max_prefill_tokens=max(256 * B, 256),
                        model_kind=1, local_hidden=1536, local_layers=4, local_inter=8960, local_mlp_ffn=2048)
    eng = Engine(ecfg, local)
    eng.init_random(seed=0)
    ids_d = torch.from_numpy(ids).cuda()
    mask_d = torch.from_numpy(mask).cuda()
    mask_u8 = mask_d.to(torch.uint8).contiguous()

    def one():
        return eng.local_generate_ids(ids_d, mask_d, frames, -1, chunk=32)

    for _ in range(args.warmup):
        out = one()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out = one()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    g = out.cpu().numpy()
    # frames until (and excluding) the eos frame of each row
    made = []
    for b in range(B):
        ch0 = g[b, T:, 0]
        e = np.nonzero(ch0 == 151653)[0]
        made.append(int(e[0]) if e.size else int(ch0.shape[0]))
    audio_s = sum(made) / FRAME_RATE * args.steps
    t = torch.tensor([dt, audio_s], dtype=torch.float64, device="cuda")
    if world > 1:
        tmax = t.clone()
        dist.all_reduce(tmax[0:1], op=dist.ReduceOp.MAX)
        dist.all_reduce(t[1:2], op=dist.ReduceOp.SUM)
        t[0] = tmax[0]
    dt_max, audio_total = float(t[0]), float(t[1])
    # prefill + frame 0 alone, and first chunk (1 s of audio = 13 frames)
    sp = None
    tb, lat = [], []
    for k in range(8):
        torch.cuda.synchronize()
        a = time.perf_counter()
        Nn.check(Nn.load().mtts_local_generate_begin(eng._h, ctypes.c_void_p(ids_d.data_ptr()),
                                                     ctypes.c_void_p(mask_u8.data_ptr()), B, T, frames, -1, sp, None),
                 "begin")
        if k >= 3:
            Nn.check(Nn.load().mtts_local_generate_decode(eng._h, 12, None), "decode")
        Nn.check(Nn.load().mtts_generate_poll(eng._h, None, None, None), "poll")
        (tb if k < 3 else lat).append((time.perf_counter() - a) * 1e3)
    res = None
    if rank == 0:
        fb = eng.local_frame_bytes(-1)
        per_utt_ms = dt_max / args.steps * 1e3
        t_begin = float(np.median(tb))
        frame_ms = (per_utt_ms - t_begin) / (frames - 1)
        kv_pos = 28 * 2 * 8 * 128 * 2
        frame_bytes = fb + kv_pos * B * (T + frames / 2)
        ms = ctypes.c_float()
        nb = ctypes.c_uint64()
        # the frame's dominant launch: the depth stack's gate|up (4 layers x 33 channels per frame;
        # r02_h_local_kernel_stats.csv: 21 % of GPU time, then the depth down at 17 %)
        Nn.check(Nn.load().mtts_engine_time_gemv(eng._h, 6, 0, B, 200, ctypes.byref(ms), ctypes.byref(nb)), "time_gemv")
        ach = nb.value / (ms.value * 1e-3) / 1e9
        ms_dn = ctypes.c_float()
        nb_dn = ctypes.c_uint64()
        Nn.check(Nn.load().mtts_engine_time_gemv(eng._h, 7, 0, B, 200, ctypes.byref(ms_dn), ctypes.byref(nb_dn)),
                 "time_gemv")
        ach_dn = nb_dn.value / (ms_dn.value * 1e-3) / 1e9
        traffic, traffic_src = pmc_traffic("local_frame")
        frame_ach = frame_bytes / (frame_ms * 1e-3) / 1e9
        res = {
            "metric": METRIC, "value": round(audio_total / dt_max, 4), "unit": "audio-s/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(per_utt_ms, 3),
            "step_def": f"one bench step = one generate() call over the batch ({frames} frames); the per-frame "
                        "time is ms_per_frame",
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "bf16",
            "data": "synthetic (random-init bf16 weights at the MossTTSLocal-1.7B shape; synthetic clone prompts)",
            "config": {"workload": f"MossTTSLocal bf16 batch={B} on 1xMI355X (depth transformer, 1+32 channels/frame)",
                       "n_vq": 32, "batch_per_gpu": B, "prompt_tokens": int(T),
                       "prompt_rows_unpadded": [int(m) for m in mask.sum(1)], "frames": frames,
                       "parallelism": f"dp{world}", "sampling": "greedy"},
            "audio_s_per_s_per_gpu": round(audio_total / dt_max / world, 4),
            "audio_frames_per_utt": made[0],
            "prefill_ms": round(t_begin, 3),
            "p50_first_chunk_ms": round(float(np.median(lat)), 2),
            "first_chunk_def": "prefill + 13 frames (first 1 s of audio codes complete), codec excluded",
            "ms_per_frame": round(frame_ms, 4),
            "frame_alg_bytes": int(frame_bytes),
            "frame_hbm_frac": round(frame_bytes / (frame_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            # round 5: the WHOLE frame against its algorithmic bytes (every weight byte the
            # frame streams + the backbone KV at the mean context), traffic = PMC bytes of whole frames
            # (scripts/pmc_probe.py --config local_frame); the frame's most-time GEMVs ride along
            "roofline": {"bound": "hbm", "achieved": round(frame_ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(frame_ach / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_src": traffic_src,
                         "kernel": "whole frame (hipGraph replay: backbone step, 33 channels of depth transformer + "
                                   "adapters + norm + head + pick, frame end)",
                         "alg_bytes_per_launch": int(frame_bytes), "avg_launch_us": round(frame_ms * 1e3, 2),
                         "depth_gate_up": {"achieved": round(ach, 1), "frac": round(ach / HBM_PEAK_GBS, 4),
                                           "alg_bytes_per_launch": int(nb.value),
                                           "avg_launch_us": round(ms.value * 1e3, 2)},
                         "depth_down": {"achieved": round(ach_dn, 1), "frac": round(ach_dn / HBM_PEAK_GBS, 4),
                                        "alg_bytes_per_launch": int(nb_dn.value),
                                        "avg_launch_us": round(ms_dn.value * 1e3, 2)}},
        }
        if not args.no_cpu_baseline and world == 1:
            res["cpu_baseline"] = cpu_baseline_local(int(T), frames)
    eng.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps(res), flush=True)


def codec_leg(frames: int, n_vq: int) -> dict:
    """Codec decoder (csrc/codec.cpp, the assumed MOSS-Audio-Tokenizer decode shape with random
    weights): one utterance's frames decoded at once, and the first 1 s chunk (13 frames) as a
    streaming decode would emit it.  Codes are synthetic (the decoder's cost does not depend on
    their values)."""
    import torch
    from moss_tts_amd.codec import AudioTokenizerDecoder, CodecConfig
    dec = AudioTokenizerDecoder(CodecConfig(max_batch=1, max_frames=max(256, frames + 16), max_chunk_frames=256), 0)
    dec.init_random(0)
    codes = torch.randint(0, 1024, (1, frames, n_vq), dtype=torch.int64, device="cuda")
    first = codes[:, :13]

    def timed(fn, reps):
        ts = []
        for _ in range(reps):
            dec.reset()
            torch.cuda.synchronize()
            a = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - a) * 1e3)
        return float(np.median(ts))

    timed(lambda: dec.decode_frames(codes), 2)  # warm-up
    whole = timed(lambda: dec.decode_frames(codes), 5)
    chunk = timed(lambda: dec.decode_frames(first), 5)
    out = {"frames": frames, "ms": round(whole, 3), "audio_s_per_s": round(frames / FRAME_RATE / (whole * 1e-3), 2),
           "first_chunk_frames": 13, "first_chunk_ms": round(chunk, 3), "weight_bytes": dec.weight_bytes(),
           "samples_per_frame": dec.samples_per_frame,
           "shape": "assumed decoder (RVQ 32x1024, 4 causal Transformer stages 12.5->100 Hz, 240-sample patches); "
                    "parity unpinned vs the real codec (absent from the reference)"}
    dec.close()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--batch", type=int, default=1, help="utterances per GPU")
    ap.add_argument("--layers", type=int, default=36)
    ap.add_argument("--decode-steps", type=int, default=208)
    ap.add_argument("--text-tokens", type=int, default=0,
                    help="override the synthetic prompt's text length (profiling long contexts)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--no-codec", action="store_true", help="skip the codec-decoder leg")
    ap.add_argument("--no-dp-leg", action="store_true", help="skip the configs[2] global-batch data-parallel leg")
    ap.add_argument("--extra-batches", default="4,32", help="extra per-GPU batch sizes reported in batch_sweep")
    ap.add_argument("--config", choices=["clone", "ttsd", "local"], default="clone",
                    help="clone: configs[1] (default); ttsd: configs[4], MOSS-TTSD long form (n_vq 16, a "
                         "2,000-token script, 10 min = 7,500 frames of audio, position-chunked prefill); "
                         "local: configs[3], MossTTSLocal-1.7B batch 8, 173 frames")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    if args.config == "local":
        return main_local(args, world, rank, local)

    from moss_tts_amd.engine import Engine, EngineConfig, sampling_params
    from moss_tts_amd import _native as Nn
    import ctypes
    n_vq = 32
    text_tokens = 48
    if args.config == "ttsd":
        n_vq, text_tokens = 16, 2000
        if args.decode_steps == 208:
            args.decode_steps = 7500 + n_vq + 3
        args.extra_batches = ""
    if args.text_tokens > 0:
        text_tokens = args.text_tokens
    n_steps = args.decode_steps
    gen_frames = n_steps - (n_vq + 3)
    extra = [int(x) for x in args.extra_batches.split(",") if x] if args.extra_batches else []
    max_b = max([args.batch] + extra)
    prompt_cap = 64 + text_tokens + 2 * n_vq + 64
    ecfg = EngineConfig(layers=args.layers, n_vq=n_vq, max_batch=max_b, max_ctx=prompt_cap + n_steps + 16,
                        # TTSD: the whole ~2,100-token script in one prefill chunk, so every weight byte
                        # streams once (1,024-token chunks streamed the 13.9 GB three times)
                        max_prefill_tokens=max(256 * max_b, 256) if args.config == "clone" else 4096)
    eng = Engine(ecfg, local)
    eng.init_random(seed=0)
    forced = torch.from_numpy(forced_schedule(n_steps, n_vq, gen_frames)).cuda()
    sp = sampling_params(text_temperature=0, audio_temperature=0)

    def run_batch(B, steps, warmup, latency=False):
        """steps x generate() of B utterances; returns (wall s max over ranks, audio s summed
        over ranks, T, frames of row 0, text-head steps, prefill ms, p50 first-chunk ms)"""
        rng = np.random.default_rng(1 + rank)
        prompts = [synthetic_prompt(cfgd, rng, text_tokens=text_tokens) for _ in range(B)]
        from moss_tts_amd.processing_moss_tts import left_pad
        padded = left_pad([torch.from_numpy(p) for p in prompts], 151643, 1024)
        ids, mask = padded["input_ids"].numpy(), padded["attention_mask"].numpy()
        T = ids.shape[1]
        ids_d = torch.from_numpy(ids).cuda()
        mask_d = torch.from_numpy(mask.astype(np.uint8)).cuda()

        def one():
            return eng.generate_ids(ids_d, mask_d, n_steps, sp, forced_text=forced, chunk=16)

        for _ in range(warmup):
            out = one()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            out = one()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        th = ctypes.c_int()
        Nn.check(Nn.load().mtts_generate_stats(eng._h, ctypes.byref(th)), "stats")
        # frames actually produced (de-delayed, non-pad rows after the assistant start)
        g = out.cpu().numpy()
        frames = [count_audio_frames(g[b], T, n_vq) for b in range(B)]
        audio_s = sum(frames) / FRAME_RATE * steps
        t = torch.tensor([dt, audio_s], dtype=torch.float64, device="cuda")
        if world > 1:
            tmax = t.clone()
            dist.all_reduce(tmax[0:1], op=dist.ReduceOp.MAX)
            dist.all_reduce(t[1:2], op=dist.ReduceOp.SUM)
            t[0] = tmax[0]
        t_begin, p50 = None, None
        if latency:
            # first-chunk latency: prefill + decode until the first 1 s of audio (13 frames) has
            # all n_vq codebooks (frame f is complete n_vq steps after its first codebook)
            first_steps = 1 + 13 + n_vq
            begin = lambda: Nn.check(Nn.load().mtts_generate_begin(
                eng._h, ctypes.c_void_p(ids_d.data_ptr()), ctypes.c_void_p(mask_d.data_ptr()), B, T, n_steps,
                ctypes.byref(sp), ctypes.c_void_p(forced.data_ptr()), None), "begin")
            tb, lat = [], []
            for _ in range(3):  # prefill + step 0 alone
                torch.cuda.synchronize()
                a = time.perf_counter()
                begin()
                Nn.check(Nn.load().mtts_generate_poll(eng._h, None, None, None), "poll")
                tb.append((time.perf_counter() - a) * 1e3)
            for _ in range(5):
                torch.cuda.synchronize()
                a = time.perf_counter()
                begin()
                Nn.check(Nn.load().mtts_generate_decode(eng._h, first_steps - 1, None), "decode")
                Nn.check(Nn.load().mtts_generate_poll(eng._h, None, None, None), "poll")
                lat.append((time.perf_counter() - a) * 1e3)
            t_begin, p50 = float(np.median(tb)), float(np.median(lat))
        return float(t[0]), float(t[1]), T, frames[0], th.value, t_begin, p50

    cfgd = dict(n_vq=n_vq)
    dt_max, audio_total, T, frames0, text_steps, t_begin, p50 = run_batch(args.batch, args.steps, args.warmup, True)
    sweep = {}
    for B in extra:
        d, a_s, _, _, _, _, _ = run_batch(B, 1, 1)
        sweep[str(B)] = {"audio_s_per_s_per_gpu": round(a_s / d / world, 3), "ms_per_utt_batch": round(d * 1e3, 2)}
    dp_leg = None
    if args.config == "clone" and not args.no_dp_leg:
        if eng.cfg.max_batch < 4 or eng.cfg.max_ctx < 130 + n_steps:
            eng.reserve(max(4, eng.cfg.max_batch), max(eng.cfg.max_ctx, 130 + n_steps + 16))
        dp_leg = dp_global_leg(eng, world, rank, n_steps, forced, sp)

    res = None
    if rank == 0:
        wb = eng.weight_bytes()
        step_ms = None
        roof = None
        if not args.no_roofline:
            def time_kernel(which, iters):
                ms, nb = ctypes.c_float(), ctypes.c_uint64()
                Nn.check(Nn.load().mtts_engine_time_gemv(eng._h, which, 0, args.batch, iters, ctypes.byref(ms),
                                                         ctypes.byref(nb)), "time_gemv")
                return ms.value, nb.value
            # the gate|up GEMV with the fused SwiGLU (201 MB of weights per launch), layers rotated
            g_ms, g_nb = time_kernel(2, 50)
            g_ach = g_nb / (g_ms * 1e-3) / 1e9
            gemv_roof = {"bound": "hbm", "achieved": round(g_ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(g_ach / HBM_PEAK_GBS, 4),
                         "kernel": "gemv_kernel gate|up (fused RMSNorm prologue, SwiGLU epilogue), layers rotated",
                         "alg_bytes_per_launch": int(g_nb), "avg_launch_us": round(g_ms * 1e3, 2)}
            if args.config == "clone" and ((eng.pse_active() and args.batch == 1) or
                                           (eng.pse4_active() and args.batch == 4)):
                # batch-1 / batch-4 decode runs the whole layer stack as ONE persistent launch
                # (pse.hip / pse4.hip): that launch is the dominant kernel (every layer's weights +
                # the K/V rows read)
                ms, nb = time_kernel(5, 20)
                kname = ("pse_kernel (persistent streaming decode: every backbone layer in one launch, batch 1)"
                         if args.batch == 1 else
                         "pse4_kernel (persistent streaming decode: every backbone layer in one launch, batch 4)")
                traffic, traffic_src = pmc_traffic("pse" if args.batch == 1 else "pse4")
            else:
                ms, nb = g_ms, g_nb
                kname = gemv_roof["kernel"]
                traffic, traffic_src = pmc_traffic("clone") if args.config == "clone" and args.batch == 1 else (None, None)
            ach = nb / (ms * 1e-3) / 1e9
            roof = {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_src": traffic_src,
                    "kernel": kname, "alg_bytes_per_launch": int(nb), "avg_launch_us": round(ms * 1e3, 2)}
            if kname != gemv_roof["kernel"]:
                roof["gemv_gate_up"] = gemv_roof
            if args.config == "ttsd" and eng.pse_long_active():
                # the TTSD step's dominant launch: the persistent launch's long-context form at the
                # end-of-generation context (the line's roofline itself is the whole step, below)
                ms, nb = time_kernel(5, 10)
                ach = nb / (ms * 1e-3) / 1e9
                roof["pse_long_launch"] = {"kernel": "pse_kernel_t<true> (batch 1, long-context attention form)",
                                           "achieved": round(ach, 1), "frac": round(ach / HBM_PEAK_GBS, 4),
                                           "alg_bytes_per_launch": int(nb), "avg_launch_us": round(ms * 1e3, 2)}
        # whole decode step against the weight-stream roofline
        per_utt_ms = dt_max / args.steps * 1e3
        res = {
            "metric": METRIC, "value": round(audio_total / dt_max, 4), "unit": "audio-s/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(per_utt_ms, 3), "step_def": (
                f"one bench step = one generate() call over the batch (prefill + {n_steps} decode steps); "
                "the per-decode-step time is ms_per_decode_step"),
            "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "bf16",
            "data": "synthetic (random-init bf16 weights at the MossTTSDelay-8B shape; synthetic clone prompts)",
            "config": {"workload": (("MOSS-TTSD long form (n_vq 16, 2000-token script, 7500 frames) bf16 batch="
                                    f"{args.batch}/GPU, chunked prefill, hipGraph decode") if args.config == "ttsd" else
                                   "MossTTSDelay bf16 batch=1 zero-shot clone (3s prompt audio) on 1xMI355X, hipGraph "
                                   "decode" if args.batch == 1 else f"MossTTSDelay bf16 batch={args.batch}/GPU"),
                       "n_vq": n_vq,
                       "batch_per_gpu": args.batch, "prompt_tokens": int(T), "decode_steps": n_steps,
                       "layers": args.layers, "parallelism": f"dp{world}", "sampling": "greedy, forced text schedule"},
            "audio_s_per_s_per_gpu": round(audio_total / dt_max / world, 4),
            "audio_frames_per_utt": frames0,
            "decode_path": (f"batch {args.batch}: the 36-layer stack as one persistent streaming launch (csrc/"
                            f"{'pse.hip' if args.batch == 1 else 'pse4.hip'}) for steps with context <= "
                            f"{eng.pse_ctx_max()}, "
                            + ("its long-context (all-CU attention) form beyond"
                               if args.batch == 1 and eng.pse_long_active() else "per-op hipGraph launches beyond")
                            if (eng.pse_active() and args.batch == 1) or (eng.pse4_active() and args.batch == 4)
                            else "per-op hipGraph launches"),
            "p50_first_chunk_ms": round(p50, 2),
            "first_chunk_def": f"prefill + {13 + n_vq + 1} decode steps (first 1 s of audio codes complete), codec excluded",
            "decode_weight_bytes": wb,
            "roofline": roof,
        }
        step_ms = (per_utt_ms - t_begin) / (n_steps - 1)
        res["prefill_ms"] = round(t_begin, 3)
        res["ms_per_decode_step"] = round(step_ms, 4)
        # algorithmic HBM bytes of an average decode step: every weight that step's logits need
        # (the text head rows below the special ids only on steps that sample text freely:
        # text_head_steps of n_steps), plus the KV cache read (36 x 2 x 8 x 128 x 2 B per
        # cached position and row) and the KV append
        text_skip = (min(151645, 151656, 151662) // 16) * 16 * 4096 * 2
        kv_pos = 36 * 2 * 8 * 128 * 2
        mean_ctx = T + n_steps / 2
        step_bytes = (wb - text_skip * (1 - text_steps / n_steps)) + kv_pos * args.batch * (mean_ctx + 1)
        res["text_head_steps"] = text_steps
        res["decode_alg_bytes_per_step"] = int(step_bytes)
        res["decode_step_hbm_frac"] = round(step_bytes / (step_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
        if args.config == "ttsd" and roof is not None:
            # TTSD: the roofline is the WHOLE decode step (every kernel of the captured step), its
            # algorithmic bytes averaged over the generation's contexts, against the PMC bytes of
            # whole steps at the mean context (scripts/pmc_probe.py --config ttsd)
            traffic, traffic_src = pmc_traffic("ttsd")
            ach = step_bytes / (step_ms * 1e-3) / 1e9
            parts = {k: roof[k] for k in ("pse_long_launch", "gemv_gate_up") if k in roof}
            if "gemv_gate_up" not in parts and roof["kernel"].startswith("gemv_kernel"):
                parts["gemv_gate_up"] = {k: roof[k] for k in ("kernel", "achieved", "frac", "alg_bytes_per_launch",
                                                              "avg_launch_us")}
            roof = {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_src": traffic_src,
                    "kernel": "whole decode step (hipGraph replay: embedding, the 36-layer stack, final norm, heads, "
                              "samplers)", "alg_bytes_per_launch": int(step_bytes),
                    "avg_launch_us": round(step_ms * 1e3, 2), **parts}
            res["roofline"] = roof
        if sweep:
            res["batch_sweep"] = sweep
        if dp_leg:
            res["dp_global"] = dp_leg
        if not args.no_codec and args.config == "clone":
            res["codec"] = codec_leg(frames0, n_vq)
            res["p50_first_chunk_ms_incl_codec"] = round(p50 + res["codec"]["first_chunk_ms"], 2)
        if not args.no_cpu_baseline and world == 1:
            res["cpu_baseline"] = cpu_baseline(args, int(T), n_steps, frames0)
        elif not args.no_cpu_baseline:
            res["cpu_baseline"] = None
    eng.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
