"""Persistent streaming engine (csrc/pse.hip, MTTS_PSE=1): the batch-1 decode stack as one launch
with run-ahead weight streaming must give the same decode logits as the per-op launches (which
the oracle tests pin), within the bf16 band, at the MossTTSDelay-8B layer shape (random weights,
3 layers), over short and multi-chunk contexts; it must be deterministic, and generate() through
it must match the per-op launches."""
import os

import numpy as np
import pytest

from tests.parity_util import ulp_bf16

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

LAYERS = 3


def make(pse, max_ctx=1024, max_prefill=1024, ctx_limit=1 << 20, long_form=None):
    """ctx_limit: the PSE context range (MTTS_PSE_CTX; unlimited here to test the kernel itself);
    long_form: MTTS_PSE_LONG (None: the default, on)"""
    from moss_tts_amd.engine import Engine, EngineConfig
    os.environ["MTTS_PSE"] = "1" if pse else "0"
    if ctx_limit is not None:
        os.environ["MTTS_PSE_CTX"] = str(ctx_limit)
    if long_form is not None:
        os.environ["MTTS_PSE_LONG"] = "1" if long_form else "0"
    try:
        e = Engine(EngineConfig(layers=LAYERS, max_batch=1, max_ctx=max_ctx, max_prefill_tokens=max_prefill), 0)
    finally:
        os.environ.pop("MTTS_PSE")
        os.environ.pop("MTTS_PSE_CTX", None)
        os.environ.pop("MTTS_PSE_LONG", None)
    e.init_random(seed=3)
    return e


@pytest.fixture(scope="module")
def engines():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ref, pse = make(False), make(True)
    if not pse.pse_active():
        ref.close()
        pse.close()
        pytest.skip("persistent streaming decode unsupported on this device")
    yield ref, pse
    ref.close()
    pse.close()


def prompt(T, steps, seed):
    rng = np.random.default_rng(seed)
    ids = np.full((1, T + steps, 33), 1024, np.int64)
    ids[0, :, 0] = rng.integers(200, 20000, T + steps)
    ids[0, :, 1:] = rng.integers(0, 1024, (T + steps, 32))
    return ids, np.ones((1, T + steps), np.uint8)


def decode_logits(eng, ids, mask, T, steps):
    out = []
    lg = eng.forward(torch.from_numpy(ids[:, :T].copy()), torch.from_numpy(mask[:, :T]), 0)
    for s in range(steps):
        lg = eng.forward(torch.from_numpy(ids[:, T + s:T + s + 1].copy()), torch.from_numpy(mask[:, :T + s + 1]), T + s)
        out.append(lg.float().cpu().numpy()[0])
    return out


def check_logits(ref, want, got):
    V, A = ref.cfg.vocab, 1025
    for s, (w, g) in enumerate(zip(want, got)):
        for j in range(33):
            sl = slice(0, V) if j == 0 else slice(V + (j - 1) * A, V + j * A)
            wr, gr = w[sl], g[sl]
            fin = np.isfinite(wr)
            assert (np.isfinite(gr) == fin).all(), (s, j)
            scale = np.abs(wr[fin]).max()
            err = np.abs(gr[fin] - wr[fin]).max()
            assert err <= 8 * ulp_bf16(scale), (s, j, float(err), float(scale))


@pytest.mark.parametrize("T,steps,pad", [(150, 12, 0), (611, 20, 0), (300, 8, 37)])
def test_pse_decode_logits_match_launches(engines, T, steps, pad):
    """pad: left-padded prompt (mask 0 on the first pad positions; the keys must be masked out)"""
    ref, pse = engines
    ids, mask = prompt(T, steps, T)
    mask[0, :pad] = 0
    check_logits(ref, decode_logits(ref, ids, mask, T, steps), decode_logits(pse, ids, mask, T, steps))


def test_pse_long_context():
    """Thousands of cached keys: every attention wave runs several 32-key chunks"""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ref, pse = make(False, 4096, 4096), make(True, 4096, 4096)
    try:
        if not pse.pse_active():
            pytest.skip("persistent streaming decode unsupported on this device")
        ids, mask = prompt(3500, 3, 5)
        check_logits(ref, decode_logits(ref, ids, mask, 3500, 3), decode_logits(pse, ids, mask, 3500, 3))
    finally:
        ref.close()
        pse.close()


def test_pse_deterministic(engines):
    _, pse = engines
    ids, mask = prompt(90, 6, 7)
    a = decode_logits(pse, ids, mask, 90, 6)
    b = decode_logits(pse, ids, mask, 90, 6)
    assert all(np.array_equal(x, y) for x, y in zip(a, b))


def test_pse_generate_matches_launches(engines):
    from moss_tts_amd.engine import sampling_params
    ref, pse = engines
    ids, mask = prompt(120, 0, 11)
    ids[0, -1, 0] = 151652  # audio_start: the model decodes audio frames
    sp = sampling_params(text_temperature=0, audio_temperature=0)
    forced = torch.full((40,), 151656, dtype=torch.int32)  # gen_slot every step
    outs = [e.generate_ids(torch.from_numpy(ids), torch.from_numpy(mask.astype(bool)), 40, sp,
                           forced_text=forced).cpu().numpy() for e in (ref, pse)]
    assert outs[0].shape == outs[1].shape
    diff = np.nonzero((outs[0] != outs[1]).any(-1)[0])[0]
    if diff.size == 0:
        return
    # random weights give bf16 near-ties in the 1024-way audio argmax: the first divergence must
    # sit at one (the per-op launches' own logits for that row, teacher-forced along the shared
    # prefix, have a top-2 margin within the band of the logit scale)
    r = int(diff[0])
    T = ids.shape[1]
    assert r > T, "the prompt rows must be identical"
    traj = outs[0]
    lg = ref.forward(torch.from_numpy(traj[:, :T].copy()), torch.ones(1, T, dtype=torch.uint8), 0)
    for p in range(T, r):
        lg = ref.forward(torch.from_numpy(traj[:, p:p + 1].copy()), torch.ones(1, p + 1, dtype=torch.uint8), p)
    lg = lg.float().cpu().numpy()[0]
    V, A = ref.cfg.vocab, 1025
    ch = np.nonzero(outs[0][0, r] != outs[1][0, r])[0]
    for j in ch:
        row = lg[:V] if j == 0 else lg[V + (j - 1) * A: V + j * A - 1]
        top = np.sort(row[np.isfinite(row)])[-2:]
        assert top[1] - top[0] <= 8 * ulp_bf16(np.abs(top[1])), (r, int(j), top)


def test_pse_context_gate(engines):
    """The short form runs only within its context range.  Beyond it an engine without the
    long-context form (MTTS_PSE_LONG=0) decodes through the per-op launches (bit-identical), the
    default engine through the long-context form (within the band); within it both take the
    short form (within the band)"""
    ref, _ = engines
    short = make(True, ctx_limit=None, long_form=False)
    dflt = make(True, ctx_limit=None)
    try:
        lim = short.pse_ctx_max()
        assert 0 < lim <= 1000  # lim + 20 cached keys must fit max_ctx
        assert dflt.pse_long_active() and not short.pse_long_active()
        ids, mask = prompt(lim + 20, 2, 9)
        want = decode_logits(ref, ids, mask, lim + 20, 2)
        assert all(np.array_equal(w, g) for w, g in zip(want, decode_logits(short, ids, mask, lim + 20, 2)))
        check_logits(ref, want, decode_logits(dflt, ids, mask, lim + 20, 2))
        ids, mask = prompt(lim - 40, 2, 9)
        want = decode_logits(ref, ids, mask, lim - 40, 2)
        check_logits(ref, want, decode_logits(short, ids, mask, lim - 40, 2))
        check_logits(ref, want, decode_logits(dflt, ids, mask, lim - 40, 2))
    finally:
        short.close()
        dflt.close()


def test_pse_generation_crosses_the_context_range(engines):
    """A generation longer than the PSE range switches to the per-op launches mid-way (per
    decode step); its ids must match the per-op engine's (or diverge first at a bf16 near-tie)"""
    from moss_tts_amd.engine import sampling_params
    ref, _ = engines
    part = make(True, ctx_limit=150)
    try:
        assert part.pse_ctx_max() == 150
        ids, mask = prompt(120, 0, 13)
        ids[0, -1, 0] = 151652
        sp = sampling_params(text_temperature=0, audio_temperature=0)
        forced = torch.full((60,), 151656, dtype=torch.int32)
        outs = [e.generate_ids(torch.from_numpy(ids), torch.from_numpy(mask.astype(bool)), 60, sp,
                               forced_text=forced).cpu().numpy() for e in (ref, part)]
    finally:
        part.close()
    assert outs[0].shape == outs[1].shape
    diff = np.nonzero((outs[0] != outs[1]).any(-1)[0])[0]
    if diff.size == 0:
        return
    r = int(diff[0])
    T = ids.shape[1]
    assert r > T
    traj = outs[0]
    lg = ref.forward(torch.from_numpy(traj[:, :T].copy()), torch.ones(1, T, dtype=torch.uint8), 0)
    for p in range(T, r):
        lg = ref.forward(torch.from_numpy(traj[:, p:p + 1].copy()), torch.ones(1, p + 1, dtype=torch.uint8), p)
    lg = lg.float().cpu().numpy()[0]
    V, A = ref.cfg.vocab, 1025
    for j in np.nonzero(outs[0][0, r] != outs[1][0, r])[0]:
        row = lg[:V] if j == 0 else lg[V + (j - 1) * A: V + j * A - 1]
        top = np.sort(row[np.isfinite(row)])[-2:]
        assert top[1] - top[0] <= 8 * ulp_bf16(np.abs(top[1])), (r, int(j), top)


def test_pse_timeout_falls_back_to_launches(engines):
    """A persistent launch that gives up waiting (its workgroups not all resident: other work on
    the device) never hands the caller invalid logits unannounced.  Default: the forward checks
    its own launch and recomputes the step on the per-op launches before returning (ADVICE r4:
    the HF-style `forward` path has no `pse_check` of its own).  Opt-in lazy form
    (`set_pse_lazy`, no host sync per forward): `pse_check` -- or the next forward once the async
    copy of the error word has landed -- raises PseTimeout once; a generation started in between
    is valid and leaves the timeout owed to the next check.  Either way the engine switches to the
    per-op launches and the recomputed steps are bit-identical to them; generate() restarts there
    by itself.  The timeout is injected through the error word (mtts_pse_inject_timeout)."""
    from moss_tts_amd.engine import sampling_params
    from moss_tts_amd._native import PseTimeout
    ref, _ = engines
    ids, mask = prompt(120, 3, 17)
    want = decode_logits(ref, ids, mask, 120, 3)
    sp = sampling_params(text_temperature=0, audio_temperature=0)
    for how in ("sync", "pse_check", "next_forward", "generate_then_check"):
        e = make(True)
        try:
            e.set_pse_lazy(how != "sync")
            e.forward(torch.from_numpy(ids[:, :120].copy()), torch.from_numpy(mask[:, :120]), 0)
            e.pse_check()  # the prefill (GEMM path) is clean
            assert e.pse_active()
            e.inject_pse_timeout()  # the first decode step's launch sees the word set
            lg = e.forward(torch.from_numpy(ids[:, 120:121].copy()), torch.from_numpy(mask[:, :121]), 120)
            if how == "sync":
                # recomputed inside the call: valid logits, nothing owed
                assert np.array_equal(lg.float().cpu().numpy()[0], want[0])
                assert not e.pse_active()
                e.pse_check()
                continue
            if how == "pse_check":
                with pytest.raises(PseTimeout):
                    e.pse_check()
            elif how == "next_forward":
                torch.cuda.synchronize()  # the async copy has landed: the next forward reports it
                with pytest.raises(PseTimeout):
                    e.forward(torch.from_numpy(ids[:, 121:122].copy()), torch.from_numpy(mask[:, :122]), 121)
            else:
                g = torch.from_numpy(ids[:, :120].copy())
                g[0, -1, 0] = 151652
                e.generate_ids(g, torch.from_numpy(mask[:, :120].astype(bool)), 8, sp)  # valid: runs per-op
                with pytest.raises(PseTimeout):
                    e.pse_check()  # the swallowed timeout is still reported
            assert not e.pse_active()
            e.pse_check()  # reported once
            if how == "generate_then_check":  # the generation rewrote the cache: prefill again
                e.forward(torch.from_numpy(ids[:, :120].copy()), torch.from_numpy(mask[:, :120]), 0)
            got = []
            for s in range(3):  # the invalid step recomputed, then on
                p = 120 + s
                lg = e.forward(torch.from_numpy(ids[:, p:p + 1].copy()), torch.from_numpy(mask[:, :p + 1]), p)
                got.append(lg.float().cpu().numpy()[0])
            assert all(np.array_equal(w, g) for w, g in zip(want, got))
        finally:
            e.close()
    e = make(True)
    try:
        ids, mask = prompt(100, 0, 19)
        ids[0, -1, 0] = 151652
        sp = sampling_params(text_temperature=0, audio_temperature=0)
        forced = torch.full((24,), 151656, dtype=torch.int32)
        want = ref.generate_ids(torch.from_numpy(ids), torch.from_numpy(mask.astype(bool)), 24, sp,
                                forced_text=forced).cpu().numpy()
        e.inject_pse_timeout()
        got = e.generate_ids(torch.from_numpy(ids), torch.from_numpy(mask.astype(bool)), 24, sp,
                             forced_text=forced).cpu().numpy()
        assert not e.pse_active()
        assert np.array_equal(want, got)
    finally:
        e.close()
