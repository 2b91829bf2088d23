"""Per-stage timeline of the persistent decode launch (csrc/mega.hip) at the 8B shape, B = 1.

Builds a random-weight engine with MTTS_MEGA_TRACE=1, prefills a synthetic prompt, runs a few
teacher-forced decode forwards, then prints, for a few layers, when the workgroups of every
stage started waiting, saw their input ready, had their activations staged, and finished
(microseconds from the launch's first stamp; median / max over workgroups).  Also times the
same decode forward with the per-stage launches (MTTS_MEGA=0)."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def build(mega, layers, T):
    from moss_tts_amd.engine import Engine, EngineConfig
    os.environ["MTTS_MEGA"] = "1" if mega else "0"
    os.environ["MTTS_MEGA_TRACE"] = "1"
    e = Engine(EngineConfig(layers=layers, max_batch=2, max_ctx=512, max_prefill_tokens=512), 0)
    e.init_random(seed=0)
    return e


def run(e, T, steps, B=1):
    rng = np.random.default_rng(0)
    C = e.cfg.n_vq + 1
    ids = torch.from_numpy(rng.integers(0, 1024, (B, T + steps, C))).cuda()
    mask = torch.ones(B, T + steps, dtype=torch.uint8, device="cuda")
    e.forward(ids[:, :T], mask[:, :T], 0)
    torch.cuda.synchronize()
    ts = []
    for s in range(steps):
        p = T + s
        t0 = time.perf_counter()
        e.forward(ids[:, p:p + 1], mask[:, :p + 1], p)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return ts


def main():
    layers, T = 36, 180
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    em = build(True, layers, T)
    P = em.mega_workgroups()
    ts = run(em, T, 6, B)
    print(f"mega: workgroups {P}, forward ms {[round(t * 1e3, 3) for t in ts]}")
    import ctypes
    from moss_tts_amd import _native as N
    n = layers * 5 * P * 4
    buf = (ctypes.c_uint64 * n)()
    N.check(N.load().mtts_mega_trace(em._h, buf, n), "trace")
    tr = np.frombuffer(buf, dtype=np.uint64).reshape(layers, 5, P, 4).astype(np.int64)
    t0 = tr[tr > 0].min()
    us = np.where(tr > 0, (tr - t0) / 100.0, np.nan)  # 100 MHz
    names = ["qkv", "att", "o", "gu", "down"]
    end = np.nanmax(us[:, 4, :, 3], axis=1)
    print(f"launch span {np.nanmax(us):.1f} us; per-layer (down done) deltas: "
          f"median {np.median(np.diff(end)):.2f} us, first {end[0]:.1f}")
    for l in [0, 1, 17, 35]:
        print(f"layer {l}")
        for s in range(5):
            v = us[l, s]
            ok = ~np.isnan(v[:, 3])
            if not ok.any():
                continue
            v = v[ok]
            q = lambda k: f"{np.median(v[:, k]):7.2f}/{np.max(v[:, k]):7.2f}"  # noqa: E731
            print(f"  {names[s]:5s} n={ok.sum():3d} wait {q(0)} ready {q(1)} staged {q(2)} done {q(3)}")
    em.close()
    eu = build(False, layers, T)
    ts = run(eu, T, 6, B)
    print(f"per-stage launches: forward ms {[round(t * 1e3, 3) for t in ts]}")
    eu.close()


if __name__ == "__main__":
    main()
