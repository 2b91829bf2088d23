"""Multi-process data-parallel path (world_size 2, gloo, CPU): sharded generate + gather
+ right-padding reproduces the single-process result of the whole batch.  The per-shard
generate is the CPU oracle (the GPU engine is exercised by the -m gpu tests)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from moss_tts_amd.dp import generate_dp, shard_bounds


def test_shard_bounds_cover_rows():
    for B in range(0, 12):
        for W in range(1, 6):
            spans = [shard_bounds(B, W, r) for r in range(W)]
            assert spans[0][0] == 0 and spans[-1][1] == B
            assert all(spans[i][1] == spans[i + 1][0] for i in range(W - 1))
            sizes = [e - s for s, e in spans]
            assert max(sizes) - min(sizes) <= 1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, case, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import moss_delay as O
        g = np.load(os.path.join(os.path.dirname(__file__), "golden", "golden.npz"))
        import json
        cases = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "cases.json")))
        c = cases[case]
        cfg = O.tiny_cfg(n_vq=c["n_vq"])
        W = O.make_weights(cfg, c["seed"], dtype="fp32", special_boost=c["special_boost"])

        def gen(ids, mask, **kw):
            res = O.generate(W, cfg, ids.numpy(), mask.numpy(), max_new_tokens=c["steps"], text_temperature=0,
                             audio_temperature=0, dtype="fp32")
            return [(sl, torch.from_numpy(x)) for sl, x in res]

        out = generate_dp(gen, torch.from_numpy(g[case + "/input_ids"]), torch.from_numpy(g[case + "/mask"]))
        if rank == 0:
            q.put([(int(sl), ids.numpy()) for sl, ids in out])
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("case", ["g_nvq4_fp32", "g_nvq4_stop_fp32"])
def test_generate_dp_world2_matches_single_process(golden, case):
    g, cases = golden
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, case, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    c = cases[case]
    assert len(got) == c["B"]
    for b, (sl, ids) in enumerate(got):
        ref = g[case + f"/out{b}"]  # the reference's own single-process batch result
        assert sl == c["starts"][b]
        assert ids.shape == ref.shape, (b, ids.shape, ref.shape)
        assert (ids == ref).all()
