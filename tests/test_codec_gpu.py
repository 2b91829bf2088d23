"""HIP codec decoder (csrc/codec.cpp + codec.hip) against the oracle restatement
(oracle/codec.py) on a tiny config: whole and chunked decodes, fewer codebooks, ragged
batches through the processor seam, and the device weight init.  Parity against the real
MOSS-Audio-Tokenizer is unpinned (its source and weights are not in the reference tree)."""
import numpy as np
import pytest
import torch

from oracle import codec as K

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _dec(cfg, W=None, max_chunk=6, max_frames=64, max_batch=3, seed=None):
    from moss_tts_amd.codec import AudioTokenizerDecoder, CodecConfig, CodecStageConfig
    cc = CodecConfig(n_q=cfg.n_q, codebook_size=cfg.codebook_size, patch=cfg.patch, rope_theta=cfg.rope_theta,
                     rms_eps=cfg.eps, stages=[CodecStageConfig(**vars(s)) for s in cfg.stages],
                     max_batch=max_batch, max_frames=max_frames, max_chunk_frames=max_chunk)
    d = AudioTokenizerDecoder(cc, 0)
    if W is not None:
        d.load_state_dict({k: torch.from_numpy(v) for k, v in W.items()})
    else:
        d.init_random(seed)
    return d


def _close(got, want, what):
    """bf16 network, fp32 samples: accumulation-order differences stay within a few bf16
    ulps of the signal scale"""
    scale = float(np.abs(want).max())
    err = np.abs(got - want)
    assert err.max() <= 0.03 * scale and np.sqrt(np.mean(err ** 2)) <= 0.005 * scale, (what, err.max(), scale)


def _codes(cfg, B, T, seed):
    return np.random.default_rng(seed).integers(0, cfg.codebook_size, (B, T, cfg.n_q))


@pytest.mark.parametrize("B,T,chunk", [(1, 5, 6), (2, 13, 6), (3, 7, 1)])
def test_codec_matches_oracle(gpu, B, T, chunk):
    cfg = K.tiny_codec_cfg()
    W = K.make_weights(cfg, 4)
    codes = _codes(cfg, B, T, B * 10 + T)
    want = K.decode(W, cfg, codes)
    d = _dec(cfg, W, max_chunk=chunk)
    got = d.decode_frames(torch.from_numpy(codes)).cpu().numpy()
    d.close()
    _close(got, want, (B, T, chunk))


def test_codec_streaming_equals_whole(gpu):
    """decode calls inside streaming() continue the stream: chunk by chunk == at once"""
    cfg = K.tiny_codec_cfg()
    W = K.make_weights(cfg, 5)
    codes = torch.from_numpy(_codes(cfg, 2, 11, 3))
    d = _dec(cfg, W, max_chunk=4)
    whole = d.decode(codes.permute(2, 0, 1)).audio[:, 0].cpu().numpy()
    with d.streaming(batch_size=2):
        parts = [d.decode(codes[:, a:b].permute(2, 0, 1)).audio[:, 0] for a, b in [(0, 3), (3, 4), (4, 11)]]
    got = torch.cat(parts, 1).cpu().numpy()
    d.close()
    assert got.shape == whole.shape
    _close(got, whole, "streaming")


def test_codec_fewer_codebooks(gpu):
    cfg = K.tiny_codec_cfg()
    W = K.make_weights(cfg, 6)
    codes = _codes(cfg, 1, 6, 4)
    d = _dec(cfg, W)
    got = d.decode_frames(torch.from_numpy(codes), n_q=2).cpu().numpy()
    d.close()
    _close(got, K.decode(W, cfg, codes, n_q=2), "n_q=2")


def test_codec_init_random_is_oracle_weights(gpu):
    cfg = K.tiny_codec_cfg()
    codes = _codes(cfg, 1, 4, 5)
    d = _dec(cfg, None, seed=9)
    got = d.decode_frames(torch.from_numpy(codes)).cpu().numpy()
    d.close()
    _close(got, K.decode(K.make_weights(cfg, 9), cfg, codes), "init_random")


def test_processor_decode_seam(gpu):
    """processor.decode_audio_codes -> audio_tokenizer.decode(codes[NQ,B,T], padding_mask,
    chunk_duration=8): ragged rows come back trimmed to their own lengths."""
    from moss_tts_amd.processing_moss_tts import MossTTSDelayProcessor
    cfg = K.tiny_codec_cfg()
    W = K.make_weights(cfg, 7)
    d = _dec(cfg, W, max_chunk=8)
    proc = MossTTSDelayProcessor.__new__(MossTTSDelayProcessor)
    proc.audio_tokenizer = d
    lens = [9, 4]
    rows = [torch.from_numpy(_codes(cfg, 1, n, 20 + n)[0]) for n in lens]
    wavs = proc.decode_audio_codes(rows)
    d.close()
    spf = cfg.samples_per_frame
    for r, w, n in zip(rows, wavs, lens):
        assert w.shape == (n * spf,) and w.dtype == torch.float32
        _close(w.numpy(), K.decode(W, cfg, r.numpy()[None])[0], ("seam", n))
