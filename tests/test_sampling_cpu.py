"""The oracle's MossTTSDelay sampler arithmetic (`oracle.moss_delay`: repetition_penalty_2d,
topk_candidates, torch_keep_probs -- what the engine's sample.hip restates) pinned to the
REFERENCE's own functions: tests/golden/golden_sampling.npz holds the outputs of
`inference_utils.py` apply_repetition_penalty_delay_pattern / apply_top_k /
apply_top_p_optimized / softmax on bf16 tensors (tests/golden/make_golden_sampling.py)."""
import json
import os

import numpy as np
import pytest

from oracle import bf16 as B16
from oracle import moss_delay as O
from oracle import prng

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def gs():
    path = os.path.join(HERE, "golden_sampling.npz")
    if not os.path.exists(path):
        pytest.skip("golden_sampling.npz not shipped to this box")
    with open(os.path.join(HERE, "golden_sampling.json")) as f:
        meta = json.load(f)
    return np.load(path, allow_pickle=False), meta


def test_sampler_matches_reference_functions(gs):
    g, meta = gs
    ctx = O._Ctx("bf16")
    n_exact = n_total = 0
    n_tie_swaps = [0]
    for name, m in meta.items():
        x = B16.from_bits(g[name + "/logits"])
        pen = O.repetition_penalty_2d(ctx, x, g[name + "/history"], m["penalty"])
        want_pen = B16.from_bits(g[name + "/penalized"])
        assert np.array_equal(pen, want_pen), name
        kept, probs = g[name + "/kept"], g[name + "/probs"]
        wide = m["vocab"] > 4096 and (m["top_k"] <= 0 or m["top_k"] > O.TOPK_CAP)
        for r in range(m["rows"]):
            if wide:
                check_wide(pen[r], m, kept[r][kept[r] >= 0], probs[r], name, r)
                continue
            cand = O.topk_candidates(pen[r], m["top_k"])
            order, keep, q = O.torch_keep_probs(pen[r][cand], m["top_p"], ids=cand)
            ids = cand[order[:keep]]
            want_ids = kept[r][kept[r] >= 0]
            assert ids.size == want_ids.size, (name, r, keep, want_ids.size)
            # torch.sort is unstable: members of the run of equal bf16 probabilities that the
            # top-p cut splits may differ -- nothing else may
            e = np.exp(pen[r][cand] - pen[r][cand[0]]).astype(np.float32)
            pb = dict(zip(cand.tolist(), B16.rnd(e / e.sum(dtype=np.float32)).tolist()))
            diff = set(ids.tolist()) ^ set(want_ids.tolist())
            assert all(pb[i] == pb[int(ids[-1])] for i in diff), (name, r, sorted(diff))
            n_tie_swaps[0] += len(diff) // 2
            want_q = dict(zip(want_ids.tolist(), probs[r][:want_ids.size].tolist()))
            same = np.array([i in want_q for i in ids])
            ids, q = ids[same], q[same]
            wq = np.array([want_q[i] for i in ids], np.float32)
            # same formula, fp32 sums in another order: within one bf16 ulp, mostly equal
            ulp = np.maximum(np.abs(wq), 1e-30) * 2.0 ** -7
            assert (np.abs(q - wq) <= ulp).all(), name
            n_exact += int((q == wq).sum())
            n_total += q.size
    assert n_exact >= 0.95 * n_total, (n_exact, n_total)


def check_wide(x, m, want_ids, want_p, name, r):
    """the key-bin sampler (text top_k <= 0 or > 2,048; oracle.wide_keep, the engine's
    topk.h block_wide_draw) against the reference's apply_top_k / apply_top_p_optimized /
    softmax: the same survivors except inside the run of equal probabilities the top-p cut
    splits (one key bin), and the same bf16 probabilities within one ulp"""
    cnt, q = O.wide_keep(x, m["top_k"], m["top_p"])
    fin = x > -np.inf
    keys = O.okey16(np.where(fin, x, 0))
    pos = O.WIDE_BINS - 1 - keys
    # rank of each index inside its key bin (index order): survivors are the first cnt[pos]
    order = np.lexsort((np.arange(x.size), pos))
    rank = np.empty(x.size, np.int64)
    sp = pos[order]
    starts = np.r_[0, np.nonzero(np.diff(sp))[0] + 1]
    run = np.zeros(x.size, np.int64)
    run[starts] = starts
    rank[order] = np.arange(x.size) - np.maximum.accumulate(run)
    surv = fin & (rank < cnt[pos])
    ids = np.nonzero(surv)[0]
    # the top-p cut compares bf16(cumsum) with top_p: torch's CPU cumsum and the engine's fixed
    # chunked order may round a cumulative value sitting on a bf16 boundary to either side, so
    # the kept count may differ by one element (of the boundary probability, checked below)
    assert abs(ids.size - want_ids.size) <= 1, (name, r, ids.size, want_ids.size)
    diff = set(ids.tolist()) ^ set(want_ids.tolist())
    # torch.sort orders equal bf16 probabilities arbitrarily (also across different scores):
    # differences may only be ids whose probability equals the last survivor's
    cut = int(np.nonzero(cnt)[0][-1])
    c0 = O._wide_bins(x, m["top_k"])
    keysd = O.WIDE_BINS - 1 - np.arange(O.WIDE_BINS)
    with np.errstate(invalid="ignore", over="ignore"):
        ev = np.exp((O.okey16_val(keysd) - O.okey16_val(keysd[np.nonzero(c0)[0][0]])).astype(np.float32))
        S, _, _ = O._wide_sums(c0, ev)
        pf = B16.rnd((ev / S).astype(np.float32))
    assert all(pf[pos[i]] == pf[cut] for i in diff), (name, r, len(diff))
    want_q = dict(zip(want_ids.tolist(), want_p[:want_ids.size].tolist()))
    common = np.array([i for i in ids if i in want_q])
    got = q[pos[common]]
    wq = np.array([want_q[i] for i in common], np.float32)
    assert (np.abs(got - wq) <= np.maximum(np.abs(wq), 1e-30) * 2.0 ** -7).all(), name


def test_wide_draw_follows_probabilities():
    """the key-bin draw hits each survivor in proportion to its probability (u sweep), and
    with top_p = 1 and no top-k every finite id can be drawn"""
    rng = np.random.default_rng(4)
    x = B16.rnd((rng.standard_normal(3000) * 0.7).astype(np.float32))
    x[rng.choice(3000, 40, replace=False)] = -np.inf
    cnt, q = O.wide_keep(x, 0, 0.8)
    us = (np.arange(1000) + 0.5) / 1000
    picks = np.array([O.wide_draw(x, 0, 0.8, np.float32(u)) for u in us])
    fin = x > -np.inf
    pos = O.WIDE_BINS - 1 - O.okey16(np.where(fin, x, 0))
    assert fin[picks].all()
    freq_bins = np.bincount(pos[picks], minlength=O.WIDE_BINS)
    want = cnt * q.astype(np.float64)
    want /= want.sum()
    assert np.abs(freq_bins / len(us) - want).max() < 1e-2
    assert O.wide_draw(x, 0, 1.0, np.float32(0.999999)) >= 0


def test_philox_known_answers():
    """the draw stream is a pure function of (seed; step, row, channel): fixed values, in [0, 1)
    with 24-bit resolution, independent across counters"""
    u = [prng.philox_uniform(0, 0, 0, 0), prng.philox_uniform(0, 1, 0, 0), prng.philox_uniform(7, 3, 2, 1)]
    assert all(0.0 <= v < 1.0 for v in u) and len(set(u)) == 3
    assert all(float(v) * 2 ** 24 == int(float(v) * 2 ** 24) for v in u)
    vals = np.array([prng.philox_uniform(5, s, b, c) for s in range(16) for b in range(4) for c in range(8)])
    assert abs(vals.mean() - 0.5) < 0.05 and vals.std() > 0.25


def test_torch_draw_follows_probabilities():
    """inverse CDF over q: u sweeps hit each survivor in proportion to q"""
    vals = B16.rnd(np.array([2.0, 1.5, 1.0, 0.25, -1.0], np.float32))
    order, keep, q = O.torch_keep_probs(vals, 0.8)
    assert 1 <= keep < 5
    us = (np.arange(20000) + 0.5) / 20000
    picks = np.array([O.torch_draw(vals, 0.8, np.float32(u))[0] for u in us])
    freq = np.bincount(picks, minlength=5)[order[:keep]] / len(us)
    assert np.allclose(freq, q / q.sum(), atol=2e-3)
