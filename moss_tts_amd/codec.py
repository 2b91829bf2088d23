"""Codec decoder on the GPU: the `processor.audio_tokenizer` seam of the reference processors.

The reference processor calls (moss_tts_delay/processing_moss_tts.py:880-930; the Local
processor :913-923; moss_tts_realtime's AudioStreamDecoder, streaming_mossttsrealtime.py:
679-804, and `codec.streaming(batch_size=1)`, :881-884):

    dec = audio_tokenizer.decode(codes[NQ, B, T] long, padding_mask[B, T] bool,
                                 return_dict=True, chunk_duration=8)
    dec.audio [B, 1, S] float, dec.audio_lengths [B] long

`AudioTokenizerDecoder` keeps that surface over the HIP codec decoder of libmtts.so
(include/mtts_codec.h): all arithmetic runs in the library, torch only holds device buffers.
The codec's architecture and weights are not published in the reference tree (see
oracle/codec.py: parity unpinned against the real MOSS-Audio-Tokenizer); `CodecConfig`
describes the decoder the library implements and `load_state_dict` takes its weights by name.
Encoding (reference-audio prompts) is out of scope: `encode` / `batch_encode` raise.
"""
import contextlib
import ctypes
from dataclasses import dataclass, field
from types import SimpleNamespace
from typing import List, Optional

import torch

from . import _native as N


@dataclass
class CodecStageConfig:
    hidden: int
    layers: int
    n_heads: int
    n_kv: int
    head_dim: int
    inter: int
    upsample: int


def _default_stages():
    return [CodecStageConfig(1280, 12, 10, 10, 128, 5120, 2), CodecStageConfig(1024, 12, 8, 8, 128, 4096, 2),
            CodecStageConfig(768, 8, 6, 6, 128, 3072, 2), CodecStageConfig(512, 8, 4, 4, 128, 2048, 1)]


@dataclass
class CodecConfig:
    """Decoder shape (the assumed "Cat" decode side: 12.5 -> 100 Hz, 240-sample patches at 24 kHz)
    and capacity."""
    n_q: int = 32
    codebook_size: int = 1024
    stages: List[CodecStageConfig] = field(default_factory=_default_stages)
    patch: int = 240
    rope_theta: float = 10000.0
    rms_eps: float = 1e-6
    sample_rate: int = 24000
    frame_rate: float = 12.5
    max_batch: int = 8
    max_frames: int = 1024
    max_chunk_frames: int = 100

    def to_c(self) -> N.MttsCodecConfig:
        c = N.MttsCodecConfig()
        c.n_q, c.codebook_size, c.n_stages, c.patch = self.n_q, self.codebook_size, len(self.stages), self.patch
        if not 0 < c.n_stages <= N.MTTS_CODEC_MAX_STAGES:
            raise ValueError("codec: 1..8 stages")
        for i, s in enumerate(self.stages):
            for k in ("hidden", "layers", "n_heads", "n_kv", "head_dim", "inter", "upsample"):
                setattr(c.stages[i], k, int(getattr(s, k)))
        c.rope_theta, c.rms_eps = self.rope_theta, self.rms_eps
        c.max_batch, c.max_frames, c.max_chunk_frames = self.max_batch, self.max_frames, self.max_chunk_frames
        return c


class AudioTokenizerDecoder:
    """GPU codec decoder with the reference `audio_tokenizer` decode surface."""

    def __init__(self, config: Optional[CodecConfig] = None, device: int = 0):
        self.config = config or CodecConfig()
        self.device = torch.device("cuda", device)
        self._dev = device
        self._c = self.config.to_c()
        h = N.P()
        N.check(N.load().mtts_codec_create(ctypes.byref(self._c), device, ctypes.byref(h)), "codec create")
        self._h = h
        self.samples_per_frame = int(N.load().mtts_codec_samples_per_frame(h))
        self._streaming = False

    # ---- lifecycle -------------------------------------------------------------
    def close(self):
        if getattr(self, "_h", None):
            N.load().mtts_codec_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def to(self, device=None, *a, **k):  # the library owns its device placement
        return self

    def eval(self):
        return self

    def parameters(self):
        """`next(audio_tokenizer.parameters()).device` is how the processor finds the device
        (processing_moss_tts.py:770)."""
        yield torch.empty(0, device=self.device)

    def init_random(self, seed: int = 0):
        N.check(N.load().mtts_codec_init_random(self._h, seed), "codec init_random")

    def load_weight(self, name: str, tensor: torch.Tensor):
        t = tensor.detach().to(torch.bfloat16).contiguous()
        on_dev = 1 if t.is_cuda else 0
        if not on_dev:
            t = t.cpu()
        N.check(N.load().mtts_codec_load_weight(self._h, name.encode(), ctypes.c_void_p(t.data_ptr()),
                                                t.numel() * 2, on_dev), f"codec load {name}")
        torch.cuda.synchronize(self.device)

    def load_state_dict(self, sd):
        for k, v in sd.items():
            self.load_weight(k, v if isinstance(v, torch.Tensor) else torch.as_tensor(v))

    def weight_bytes(self) -> int:
        v = ctypes.c_uint64()
        N.check(N.load().mtts_codec_weight_bytes(self._h, ctypes.byref(v)), "codec weight_bytes")
        return int(v.value)

    @property
    def position(self) -> int:
        """frames decoded since the last reset"""
        return int(N.load().mtts_codec_position(self._h))

    def reset(self):
        N.check(N.load().mtts_codec_reset(self._h), "codec reset")

    # ---- decode ----------------------------------------------------------------
    def decode_frames(self, codes_btq: torch.Tensor, n_q: Optional[int] = None) -> torch.Tensor:
        """codes [B, T, NQ] (frame-major) -> fp32 [B, T * samples_per_frame], continuing the
        current stream position (causal: chunked decoding equals decoding at once)."""
        B, T, Q = codes_btq.shape
        n_q = Q if n_q is None else n_q
        codes = codes_btq.to(self.device, torch.int64).contiguous()
        wav = torch.empty(B, T * self.samples_per_frame, dtype=torch.float32, device=self.device)
        stream = ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)
        N.check(N.load().mtts_codec_decode(self._h, ctypes.c_void_p(codes.data_ptr()), B, T, Q, n_q,
                                           ctypes.c_void_p(wav.data_ptr()), wav.shape[1], stream), "codec decode")
        return wav

    def decode(self, audio_codes: torch.Tensor, padding_mask: Optional[torch.Tensor] = None, return_dict: bool = True,
               chunk_duration: Optional[float] = None, num_quantizers: Optional[int] = None):
        """audio_codes [NQ, B, T] (or [NQ, T]) -> .audio [B, 1, T * spf] fp32, .audio_lengths [B].

        chunk_duration (seconds) bounds the frames per forward, as the reference's internal
        streaming does; the decoder is causal, so it does not change the waveform.  Outside a
        `streaming()` context every call starts new streams."""
        codes = audio_codes
        if codes.dim() == 2:
            codes = codes[:, None, :]
        if codes.dim() != 3:
            raise ValueError(f"audio_codes must be [NQ, B, T], got {tuple(audio_codes.shape)}")
        NQ, B, T = codes.shape
        if NQ > self.config.n_q:
            raise ValueError(f"{NQ} codebooks > codec n_q {self.config.n_q}")
        if padding_mask is None:
            lengths = torch.full((B,), T, dtype=torch.long)
        else:
            lengths = padding_mask.to(torch.bool).sum(-1).to(torch.long).cpu()
        if not self._streaming:
            self.reset()
        frames = codes.permute(1, 2, 0).contiguous()  # [B, T, NQ]
        step = T
        if chunk_duration is not None and chunk_duration > 0:
            step = max(1, int(round(chunk_duration * self.config.frame_rate)))
        outs = [self.decode_frames(frames[:, t:t + step], num_quantizers or NQ) for t in range(0, T, step)]
        audio = torch.cat(outs, dim=1)[:, None, :] if outs else torch.zeros(B, 1, 0, device=self.device)
        out = SimpleNamespace(audio=audio, audio_lengths=lengths * self.samples_per_frame)
        if return_dict:
            return out
        return out.audio, out.audio_lengths

    @contextlib.contextmanager
    def streaming(self, batch_size: int = 1):
        """Streaming context (moss_tts_realtime: `with codec.streaming(batch_size=1)`): decode
        calls inside continue the same streams instead of starting new ones."""
        if batch_size > self.config.max_batch:
            raise ValueError("batch_size exceeds the codec capacity")
        self.reset()
        self._streaming = True
        try:
            yield self
        finally:
            self._streaming = False

    # ---- encoder: out of scope ---------------------------------------------------
    def encode(self, *a, **k):
        raise NotImplementedError("codec encoder (reference-audio prompts) is not part of this engine")

    def batch_encode(self, *a, **k):
        raise NotImplementedError("codec encoder (reference-audio prompts) is not part of this engine")
