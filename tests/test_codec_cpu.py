"""Codec-decoder oracle (oracle/codec.py) properties on the CPU: causal incremental decoding
(chunked == whole), prefix stability, fewer codebooks, and the device-twin weight init.
The real MOSS-Audio-Tokenizer is absent from the reference tree: parity unpinned against it."""
import numpy as np

from oracle import codec as K


def _codes(cfg, B, T, seed=0):
    return np.random.default_rng(seed).integers(0, cfg.codebook_size, (B, T, cfg.n_q))


def test_shapes_and_samples_per_frame():
    cfg = K.tiny_codec_cfg()
    W = K.make_weights(cfg, 1)
    wav = K.decode(W, cfg, _codes(cfg, 2, 5))
    assert wav.shape == (2, 5 * cfg.samples_per_frame) and wav.dtype == np.float32
    assert np.isfinite(wav).all() and np.abs(wav).max() > 0
    assert K.CodecCfg().samples_per_frame == 1920  # 24 kHz at 12.5 Hz


def test_chunked_equals_whole_and_prefix_is_stable():
    cfg = K.tiny_codec_cfg()
    W = K.make_weights(cfg, 2)
    codes = _codes(cfg, 2, 9, 1)
    whole = K.decode(W, cfg, codes)
    st = K.CodecState(cfg)
    parts = [K.decode(W, cfg, codes[:, a:b], state=st) for a, b in [(0, 1), (1, 4), (4, 9)]]
    assert np.array_equal(np.concatenate(parts, 1), whole)
    # causal: the first frames' samples do not depend on later codes
    other = codes.copy()
    other[:, 6:] = (other[:, 6:] + 1) % cfg.codebook_size
    alt = K.decode(W, cfg, other)
    spf = cfg.samples_per_frame
    assert np.array_equal(alt[:, :6 * spf], whole[:, :6 * spf])
    assert not np.array_equal(alt[:, 6 * spf:], whole[:, 6 * spf:])


def test_fewer_codebooks_is_lower_bitrate():
    cfg = K.tiny_codec_cfg()
    W = K.make_weights(cfg, 3)
    codes = _codes(cfg, 1, 4, 2)
    a = K.decode(W, cfg, codes, n_q=2)
    b = K.decode(W, cfg, codes[..., :2], n_q=2)
    assert np.array_equal(a, b)
    assert not np.array_equal(a, K.decode(W, cfg, codes))


def test_weight_specs_match_device_init_order():
    """mtts_codec_init_random fills the same (name, shape, scale) list in the same order."""
    cfg = K.tiny_codec_cfg()
    names = [n for n, _, _ in K.weight_specs(cfg)]
    assert names[0] == "quantizer.codebooks.0.weight" and names[-1] == "decoder.out_proj.weight"
    assert names.index("decoder.stages.0.norm.weight") < names.index("decoder.stages.0.upsample.weight") < \
        names.index("decoder.stages.1.layers.0.self_attn.q_proj.weight")
