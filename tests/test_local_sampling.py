"""MossTTSLocal sampling: the oracle's restatement of the HF processor chain
(oracle.moss_local.hf_pick_distribution) pinned to transformers' own processors on CPU,
and the device pick (mtts_k_local_pick) checked against it on the GPU: every draw inside the
kept set, and the empirical distribution of 8192 Philox draws consistent with the oracle's
(chi-square at fixed seeds).  Torch's RNG stream is not reproduced: parity is distributional."""
import numpy as np
import pytest

from oracle import moss_local as L

torch = pytest.importorskip("torch")

CASES = [
    # ch, V, temperature, top_k, top_p, penalty  (README defaults: text 1.5/50/1.0, audio 1.0/50/0.95/1.1)
    (0, 151936, 1.5, 50, 1.0, None),
    (3, 1025, 1.0, 50, 0.95, 1.1),
    (1, 1025, 0.7, 25, 0.8, 1.3),
    (2, 1025, 1.2, 1024, 0.9, 1.1),
    # past the sorted candidate list (round 4): the key-bin walk (topk.h block_wide_draw_hf) on the
    # text row, any top_k on the audio rows (top_k <= 0: no TopKLogitsWarper)
    (0, 151936, 1.5, 0, 0.9, None),
    (0, 151936, 1.0, 5000, 0.95, None),
    (0, 151936, 0.8, 0, 1.0, None),
    (2, 1025, 1.2, 0, 0.9, 1.1),
    (1, 1025, 1.0, 2000, 1.0, 1.3),
]


def make_row(V, ch, seed):
    rng = np.random.default_rng(seed)
    x = (rng.standard_normal(V) * 2.5).astype(np.float32)
    x[rng.integers(0, V, 6)] += 6.0  # a few strong candidates
    if ch > 0:
        x[V - 1] = -np.inf  # audio pad column
    x = torch.from_numpy(x).to(torch.bfloat16).float().numpy()
    hist = rng.integers(0, V - 1, 40) if ch > 0 else np.zeros(0, np.int64)
    return x, hist


def hf_reference(x, hist, ch, temperature, top_k, top_p, penalty):
    from transformers.generation.logits_process import (LogitsProcessorList, RepetitionPenaltyLogitsProcessor,
                                                        TemperatureLogitsWarper, TopKLogitsWarper, TopPLogitsWarper)
    procs = LogitsProcessorList()
    if penalty is not None and ch != 0:
        procs.append(RepetitionPenaltyLogitsProcessor(penalty=penalty))
    procs.append(TemperatureLogitsWarper(temperature=temperature))
    if top_k > 0:  # the reference attaches no TopKLogitsWarper without a top_k (:365-370)
        procs.append(TopKLogitsWarper(top_k=top_k))
    if top_p < 1.0:
        procs.append(TopPLogitsWarper(top_p=top_p))
    ids = torch.from_numpy(np.asarray(hist if len(hist) else [0], np.int64))[None]
    s = procs(ids, torch.from_numpy(x)[None].to(torch.bfloat16))
    return torch.softmax(s.float(), -1)[0].double().numpy()


@pytest.mark.parametrize("case", CASES)
def test_oracle_pick_matches_hf_processors(case):
    ch, V, temperature, top_k, top_p, penalty = case
    x, hist = make_row(V, ch, 7 + ch)
    want = hf_reference(x, hist, ch, temperature, top_k, top_p, penalty)
    got = L.hf_pick_distribution(x, hist, ch, temperature, top_k, top_p, penalty)
    # the same number kept; the sets may differ only inside the run of equal scores the top-p cut
    # splits (torch.sort is not stable on the 151,936-entry row: which tied entries HF drops there
    # is arbitrary -- the oracle drops the lowest indices, as torch does on the short rows)
    assert (want > 0).sum() == (got > 0).sum()
    diff = np.nonzero((want > 0) != (got > 0))[0]
    proc = (torch.from_numpy(x).to(torch.bfloat16) / temperature).to(torch.bfloat16).float().numpy()
    assert np.unique(proc[diff]).size <= 1, "kept sets differ outside one tie run"
    assert np.allclose(got, want, atol=2e-3)


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES)
def test_device_pick_distribution(case):
    import ctypes
    from scipy.stats import chisquare
    from moss_tts_amd import _native as N
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ch, V, temperature, top_k, top_p, penalty = case
    x, hist = make_row(V, ch, 7 + ch)
    probs = L.hf_pick_distribution(x, hist, ch, temperature, top_k, top_p, penalty)
    R, C, A = 8192, 4, 1025
    logits = torch.from_numpy(x).to(torch.bfloat16)[None].expand(R, V).contiguous().cuda()
    seen = torch.zeros(R, C, A, dtype=torch.uint8)
    if ch > 0:
        seen[:, ch, torch.from_numpy(np.unique(hist))] = 1
    seen = seen.cuda()
    out = torch.full((R, C), -1, dtype=torch.int64, device="cuda")
    P = lambda t: ctypes.c_void_p(t.data_ptr())
    N.check(N.load().mtts_k_local_pick(P(logits), V, V, ch, P(seen), P(out), C, R, A, temperature, top_k, top_p,
                                       penalty if penalty else 1.0, 1234, 5, None), "local_pick")
    draws = out[:, ch].cpu().numpy()
    kept = np.nonzero(probs > 0)[0]
    # (the top-p cut may fall one element apart in a long tie run: its scores are equal)
    proc = (torch.from_numpy(x).to(torch.bfloat16) / temperature).to(torch.bfloat16).float().numpy()
    edge = np.nonzero(proc == proc[kept].min())[0] if kept.size < V else kept
    assert np.isin(draws, np.union1d(kept, edge)).all(), "draw outside the kept set"
    draws = draws[np.isin(draws, kept)]
    cnt = np.bincount(draws, minlength=V)[kept].astype(np.float64)
    exp = probs[kept] * draws.size
    big = exp >= 5  # chi-square on the well-populated cells, the rest pooled
    f_obs = np.append(cnt[big], cnt[~big].sum())
    f_exp = np.append(exp[big], exp[~big].sum())
    if f_exp[-1] == 0:
        f_obs, f_exp = f_obs[:-1], f_exp[:-1]
    f_exp *= f_obs.sum() / f_exp.sum()
    assert chisquare(f_obs, f_exp).pvalue > 1e-3


@pytest.mark.gpu
def test_device_pick_threshold_ties_past_the_list():
    """top_k = 50 on a text row whose 50th score is shared by 3,000 entries: HF keeps every tie,
    more than the sorted list holds, so the pick takes the key-bin walk -- draws stay inside the
    kept set and follow its distribution (round 3 reported MTTS_E_UNSUPPORTED here)"""
    import ctypes
    from scipy.stats import chisquare
    from moss_tts_amd import _native as N
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    V, ch = 151936, 0
    x, hist = make_row(V, ch, 31)
    srt = np.sort(x)[::-1]
    tie = srt[40]
    rng = np.random.default_rng(5)
    x[rng.choice(np.nonzero(x < tie)[0], 3000, replace=False)] = tie
    probs = L.hf_pick_distribution(x, hist, ch, 1.0, 50, 1.0, None)
    kept = np.nonzero(probs > 0)[0]
    assert kept.size > 2048
    R, C, A = 8192, 4, 1025
    logits = torch.from_numpy(x).to(torch.bfloat16)[None].expand(R, V).contiguous().cuda()
    seen = torch.zeros(R, C, A, dtype=torch.uint8, device="cuda")
    out = torch.full((R, C), -1, dtype=torch.int64, device="cuda")
    P = lambda t: ctypes.c_void_p(t.data_ptr())
    N.check(N.load().mtts_k_local_pick(P(logits), V, V, ch, P(seen), P(out), C, R, A, 1.0, 50, 1.0, 1.0, 99, 3, None),
            "local_pick")
    draws = out[:, ch].cpu().numpy()
    assert np.isin(draws, kept).all()
    top = probs[kept] >= 5.0 / R  # the strong candidates one by one, the tie run pooled
    cnt = np.bincount(draws, minlength=V)[kept].astype(np.float64)
    f_obs = np.append(cnt[top], cnt[~top].sum())
    f_exp = np.append(probs[kept][top], probs[kept][~top].sum()) * R
    assert chisquare(f_obs, f_exp * f_obs.sum() / f_exp.sum()).pvalue > 1e-3


@pytest.mark.gpu
def test_device_pick_greedy_and_top1():
    """temperature <= 0: torch.argmax (first index); top_k = 1: the tied maxima only"""
    import ctypes
    from moss_tts_amd import _native as N
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    x, hist = make_row(1025, 2, 3)
    x[100] = x[200] = np.float32(x.max() + 1)  # a tie: first index wins
    R, C, A = 4, 4, 1025
    logits = torch.from_numpy(x).to(torch.bfloat16)[None].expand(R, 1025).contiguous().cuda()
    seen = torch.zeros(R, C, A, dtype=torch.uint8, device="cuda")
    out = torch.full((R, C), -1, dtype=torch.int64, device="cuda")
    P = lambda t: ctypes.c_void_p(t.data_ptr())
    N.check(N.load().mtts_k_local_pick(P(logits), 1025, 1025, 2, P(seen), P(out), C, R, A, 0.0, 50, 1.0, 1.0, 1, 0,
                                       None), "pick")
    assert (out[:, 2].cpu() == 100).all()
    N.check(N.load().mtts_k_local_pick(P(logits), 1025, 1025, 2, P(seen), P(out), C, R, A, 1.0, 1, 1.0, 1.0, 1, 0,
                                       None), "pick")
    assert np.isin(out[:, 2].cpu().numpy(), [100, 200]).all()  # TopKLogitsWarper keeps ties
    # top_p 0.3 over the tie (p = 0.5 each): the ascending walk drops the lower index (cum 0.5 <= 0.7)
    # and keeps the higher -- the oracle's stable-argsort order, torch.sort's on these rows
    want = L.hf_pick_distribution(x, hist, 2, 1.0, 1, 0.3, 1.0)
    assert np.nonzero(want)[0].tolist() == [200]
    N.check(N.load().mtts_k_local_pick(P(logits), 1025, 1025, 2, P(seen), P(out), C, R, A, 1.0, 1, 0.3, 1.0, 1, 0,
                                       None), "pick")
    assert (out[:, 2].cpu() == 200).all()


@pytest.mark.gpu
@pytest.mark.parametrize("V,ld", [(1025, 1032), (151936, 151936), (1025, 1025)])
def test_device_pick_greedy_vector_rows(V, ld):
    """greedy pick over 16-byte row loads (ld % 8 == 0) and the scalar form: torch.argmax's
    first index, with the maximum tied across two loads and, in row 1, alone in the V % 8 tail"""
    import ctypes
    from moss_tts_amd import _native as N
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    R, C, A = 3, 4, 1025
    g = torch.Generator().manual_seed(V)
    x = torch.randn(R, ld, generator=g).to(torch.bfloat16)
    x[:, V:] = 100.0  # padding columns beyond V never win
    top = x[:, :V].float().max() + 4
    x[0, 13] = x[0, V - 9] = top  # a tie in two different 8-column loads: first index wins
    x[1, V - 1] = top            # the tail element past the last full load
    logits = x.contiguous().cuda()
    seen = torch.zeros(R, C, A, dtype=torch.uint8, device="cuda")
    out = torch.full((R, C), -1, dtype=torch.int64, device="cuda")
    P = lambda t: ctypes.c_void_p(t.data_ptr())
    ch = 0 if V > A else 1
    N.check(N.load().mtts_k_local_pick(P(logits), ld, V, ch, P(seen), P(out), C, R, A, 0.0, 50, 1.0, 1.0, 1, 0,
                                       None), "pick")
    want = torch.argmax(x[:, :V].float(), dim=1)
    assert out[:, ch].cpu().tolist() == want.tolist()
    assert want[0].item() == 13 and want[1].item() == V - 1
