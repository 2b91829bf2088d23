"""Data-parallel generate over the HIP engine (moss_tts_amd.dp.generate_dp): two gloo ranks,
each with its own engine (here both on the one GPU of the box; on a node, one per GPU), each
generating its contiguous row shard of the GLOBALLY left-padded batch, then one all_gather of
the finished rows and the right-pad to the global step count
(`moss_tts_delay/modeling_moss_tts.py:453,475,513`).  The gathered result must equal a
single-process generate() of the whole batch (greedy; in the early-stop case the shards stop at
different steps, so the gather's right-pad is what makes them equal)."""
import json
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _engine_generate(case):
    """generate_fn for generate_dp: the engine's device loop, sliced like generate() (:518-525)"""
    from oracle import moss_delay as O
    from moss_tts_amd.engine import Engine, EngineConfig, sampling_params
    g = np.load(os.path.join(HERE, "golden", "golden.npz"))
    c = json.load(open(os.path.join(HERE, "golden", "cases.json")))[case]
    cfg = O.tiny_cfg(n_vq=c["n_vq"])
    W = O.make_weights(cfg, c["seed"], dtype="bf16", special_boost=c["special_boost"])
    eng = Engine(EngineConfig(hidden=cfg.hidden, layers=cfg.layers, n_heads=cfg.n_heads, n_kv=cfg.n_kv,
                              head_dim=cfg.head_dim, inter=cfg.inter, vocab=cfg.vocab, n_vq=cfg.n_vq,
                              rope_theta=cfg.rope_theta, max_batch=4, max_ctx=256, max_prefill_tokens=512), 0)
    eng.load_state_dict({k: torch.from_numpy(v) for k, v in W.items()})

    def gen(ids, mask, **kw):
        out = eng.generate_ids(ids, mask, c["steps"], sampling_params(text_temperature=0, audio_temperature=0)).cpu()
        starts = O.find_last_equal_C(ids[..., 0].numpy(), cfg.im_start_token_id) + 3
        return [(ids.shape[1] - int(s), out[b, int(s):]) for b, s in enumerate(starts)]

    return g, c, eng, gen


def _worker(rank, world, port, case, q):
    import torch.distributed as dist
    from moss_tts_amd.dp import generate_dp
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        g, c, eng, gen = _engine_generate(case)
        out = generate_dp(gen, torch.from_numpy(g[case + "/input_ids"]), torch.from_numpy(g[case + "/mask"]))
        if rank == 0:
            q.put([(int(sl), ids.numpy()) for sl, ids in out])
        eng.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("case", ["g_nvq4_fp32", "g_nvq4_stop_fp32"])
def test_generate_dp_hip_world2(case):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, case, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=240)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    g, c, eng, gen = _engine_generate(case)
    whole = gen(torch.from_numpy(g[case + "/input_ids"]), torch.from_numpy(g[case + "/mask"]))
    eng.close()
    assert len(got) == len(whole) == c["B"]
    for b, ((sl, ids), (wsl, wids)) in enumerate(zip(got, whole)):
        assert sl == int(wsl) == c["starts"][b]
        assert ids.shape == tuple(wids.shape) and (ids == wids.numpy()).all(), b
