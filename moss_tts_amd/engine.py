"""Python host side of the engine: owns an `mtts_engine` (libmtts.so) and moves
torch device tensors across the C ABI as raw pointers.

PyTorch is plumbing here (device memory, streams); every arithmetic op of the
decode path runs in the HIP kernels of `csrc/`.
"""
import ctypes
from dataclasses import dataclass
from typing import Dict, Optional

import torch

from . import _native as N


@dataclass
class EngineConfig:
    """Model shape (MossTTSDelayConfig + nested Qwen3Config) and engine capacity."""
    hidden: int = 4096
    layers: int = 36
    n_heads: int = 32
    n_kv: int = 8
    head_dim: int = 128
    inter: int = 12288
    vocab: int = 151936
    n_vq: int = 32
    audio_vocab: int = 1024
    rope_theta: float = 1_000_000.0
    rms_eps: float = 1e-6
    pad_token_id: int = 151643
    im_start_token_id: int = 151644
    im_end_token_id: int = 151645
    audio_start_token_id: int = 151652
    audio_end_token_id: int = 151653
    audio_user_slot_token_id: int = 151654
    audio_assistant_gen_slot_token_id: int = 151656
    audio_assistant_delay_slot_token_id: int = 151662
    audio_pad_code: int = 1024
    max_batch: int = 32
    max_ctx: int = 2048
    max_prefill_tokens: int = 8192
    # MossTTSLocal (model_kind 1): depth transformer + adapters (moss_tts_local/configuration_moss_tts.py)
    model_kind: int = 0
    local_hidden: int = 0
    local_layers: int = 0
    local_inter: int = 0
    local_mlp_ffn: int = 0
    eos_token_id: int = 151653

    def to_c(self):
        c = N.MttsConfig()
        for name, _ in N.MttsConfig._fields_:
            setattr(c, name, getattr(self, name))
        return c

    @classmethod
    def from_hf(cls, config, **cap):
        """From a MossTTSDelayConfig-like object (reference `configuration_moss_tts.py:62-103`)."""
        lc = config.language_config
        rope = getattr(lc, "rope_parameters", None) or {}
        theta = rope.get("rope_theta", getattr(lc, "rope_theta", 10000.0))
        kw = dict(hidden=lc.hidden_size, layers=lc.num_hidden_layers, n_heads=lc.num_attention_heads,
                  n_kv=lc.num_key_value_heads,
                  head_dim=getattr(lc, "head_dim", None) or lc.hidden_size // lc.num_attention_heads,
                  inter=lc.intermediate_size, vocab=lc.vocab_size, n_vq=config.n_vq,
                  audio_vocab=config.audio_vocab_size, rope_theta=float(theta), rms_eps=float(lc.rms_norm_eps),
                  pad_token_id=config.pad_token_id, im_start_token_id=config.im_start_token_id,
                  im_end_token_id=config.im_end_token_id, audio_start_token_id=config.audio_start_token_id,
                  audio_end_token_id=config.audio_end_token_id,
                  audio_user_slot_token_id=config.audio_user_slot_token_id,
                  audio_assistant_gen_slot_token_id=config.audio_assistant_gen_slot_token_id,
                  audio_assistant_delay_slot_token_id=config.audio_assistant_delay_slot_token_id,
                  audio_pad_code=config.audio_pad_code)
        kw.update(cap)
        return cls(**kw)


def _ptr(t: Optional[torch.Tensor]):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _stream_ptr(device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


class Engine:
    """One engine = one GPU.  Not re-entrant (the reference's model object is not either)."""

    def __init__(self, cfg: EngineConfig, device: int = 0):
        if not torch.cuda.is_available():
            raise RuntimeError("moss_tts_amd needs a ROCm GPU (MI355X); no CPU fallback exists")
        self.cfg = cfg
        self.device = torch.device("cuda", device)
        h = ctypes.c_void_p()
        N.check(N.load().mtts_engine_create(ctypes.byref(cfg.to_c()), device, ctypes.byref(h)), "mtts_engine_create")
        self._h = h
        self.heads_ld = N.load().mtts_heads_ld(h)

    def close(self):
        if getattr(self, "_h", None):
            N.load().mtts_engine_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- weights ---------------------------------------------------------------
    def load_weight(self, name: str, tensor: torch.Tensor):
        t = tensor.detach().to(torch.bfloat16).contiguous()
        on_dev = 1 if t.is_cuda else 0
        if t.is_cuda and t.device != self.device:
            t = t.to(self.device)
        # ordered after torch's current stream (where a device source was produced): no device sync
        N.check(N.load().mtts_engine_load_weight_stream(self._h, name.encode(), _ptr(t), t.numel() * 2, on_dev,
                                                        _stream_ptr(self.device)), name)

    def load_state_dict(self, sd: Dict[str, torch.Tensor]):
        for k, v in sd.items():
            if "rotary_emb" in k:
                continue
            self.load_weight(k, v)

    def reserve(self, max_batch: int, max_ctx: int, max_prefill_tokens: int = 0):
        """Grow batch / context capacity (KV cache, activations) without reloading weights."""
        c = self.cfg
        max_prefill_tokens = max(max_prefill_tokens, c.max_prefill_tokens)
        N.check(N.load().mtts_engine_reserve(self._h, max_batch, max_ctx, max_prefill_tokens), "reserve")
        c.max_batch, c.max_ctx, c.max_prefill_tokens = max_batch, max_ctx, max_prefill_tokens

    def init_random(self, seed: int = 0):
        N.check(N.load().mtts_engine_init_random(self._h, seed), "init_random")

    def pse_active(self) -> bool:
        """Whether batch-1 decode steps run the decoder stack as one persistent launch (pse.hip)."""
        return bool(N.load().mtts_pse_active(self._h))

    def pse4_active(self) -> bool:
        """Whether batch-4 decode steps run the decoder stack as one persistent launch (pse4.hip)."""
        return bool(N.load().mtts_pse4_active(self._h))

    def pse_long_active(self) -> bool:
        """Whether batch-1 steps past pse_ctx_max() run the launch's long-context (all-CU attention) form."""
        return bool(N.load().mtts_pse_long_active(self._h))

    def lpse_active(self) -> bool:
        """MossTTSLocal: each channel's depth stage runs as one persistent launch (lpse.hip)"""
        return bool(N.load().mtts_local_lpse_active(self._h))

    def pse_ctx_max(self) -> int:
        """Longest context (prompt + new tokens) a batch-1 decode runs through pse.hip; 0 if inactive."""
        return int(N.load().mtts_pse_ctx_max(self._h))

    def set_pse_lazy(self, lazy: bool = True):
        """Opt into lazily checked teacher-forced forwards through the persistent launch (no host
        sync per `forward`; a timed-out launch surfaces as `PseTimeout` from `pse_check` or a later
        `forward`).  Default: each `forward` checks its launch and recomputes a timed-out step on
        the per-op launches before returning."""
        N.check(N.load().mtts_engine_set_pse_lazy(self._h, 1 if lazy else 0), "set_pse_lazy")

    def pse_check(self):
        """Blocking check of the persistent launch's error word for the teacher-forced forwards so
        far.  Raises `PseTimeout` once when a lazily checked launch (`set_pse_lazy`) timed out:
        those forwards' logits are invalid, the engine now runs the per-op launches."""
        N.check(N.load().mtts_pse_check(self._h), "pse_check")

    def kv_write(self, layer: int, row: int, pos0: int, k, v):
        """test hook: K / V rows (bf16 [n_kv, n, head_dim], host) at positions pos0.. of one row"""
        k = k.detach().to("cpu", torch.bfloat16).contiguous()
        v = v.detach().to("cpu", torch.bfloat16).contiguous()
        assert k.shape == v.shape and k.dim() == 3
        N.check(N.load().mtts_engine_kv_write(self._h, layer, row, pos0, k.shape[1], ctypes.c_void_p(k.data_ptr()),
                                              ctypes.c_void_p(v.data_ptr())), "kv_write")

    def kv_fill(self, bits: int):
        """test hook: the whole KV cache set to one bf16 bit pattern"""
        N.check(N.load().mtts_engine_kv_fill(self._h, bits), "kv_fill")

    def inject_pse_timeout(self):
        """fault injection (tests): the persistent launch's next check sees a timed-out wait"""
        N.check(N.load().mtts_pse_inject_timeout(self._h), "pse_inject_timeout")

    def weight_bytes(self):
        v = ctypes.c_uint64()
        N.check(N.load().mtts_engine_weight_bytes(self._h, ctypes.byref(v)), "weight_bytes")
        return int(v.value)

    # ---- forward / generate ----------------------------------------------------
    def forward(self, ids: torch.Tensor, mask: torch.Tensor, past: int) -> torch.Tensor:
        """Teacher-forced forward: returns bf16 logits [B, heads_ld] of the last position."""
        B, S, _ = ids.shape
        _check_mask(mask, B, past + S)
        ids = ids.to(self.device, torch.int64).contiguous()
        mask = mask.to(self.device, torch.uint8).contiguous()
        out = torch.empty(B, self.heads_ld, dtype=torch.bfloat16, device=self.device)
        N.check(N.load().mtts_forward(self._h, _ptr(ids), _ptr(mask), B, S, past, _ptr(out),
                                      _stream_ptr(self.device)), "forward")
        return out

    def split_logits(self, logits: torch.Tensor):
        V, A = self.cfg.vocab, self.cfg.audio_vocab + 1
        return [logits[:, :V]] + [logits[:, V + j * A: V + (j + 1) * A] for j in range(self.cfg.n_vq)]

    def session(self, input_ids: torch.Tensor, attention_mask: Optional[torch.Tensor], max_new_tokens: int,
                sampling: N.MttsSampling, forced_text: Optional[torch.Tensor] = None) -> "GenerateSession":
        return GenerateSession(self, input_ids, attention_mask, max_new_tokens, sampling, forced_text)

    def generate_ids(self, input_ids: torch.Tensor, attention_mask: Optional[torch.Tensor], max_new_tokens: int,
                     sampling: N.MttsSampling, forced_text: Optional[torch.Tensor] = None, chunk: int = 16):
        """Runs the whole device loop; returns generation_ids [B, T + n, 1+n_vq] (prompt included)."""
        B, T, C = input_ids.shape
        _check_mask(attention_mask, B, T)
        ids = input_ids.to(self.device, torch.int64).contiguous()
        mask = None if attention_mask is None else attention_mask.to(self.device, torch.uint8).contiguous()
        forced = None
        if forced_text is not None:
            forced = forced_text.to(self.device, torch.int32).contiguous()
            assert forced.numel() >= max_new_tokens
        n = ctypes.c_int()
        N.check(N.load().mtts_generate(self._h, _ptr(ids), _ptr(mask), B, T, max_new_tokens, ctypes.byref(sampling),
                                       _ptr(forced), chunk, ctypes.byref(n), _stream_ptr(self.device)), "generate")
        out = torch.empty(B, T + n.value, C, dtype=torch.int64, device=self.device)
        N.check(N.load().mtts_generate_fetch(self._h, _ptr(out), n.value, _stream_ptr(self.device)), "fetch")
        return out


    # ---- MossTTSLocal ------------------------------------------------------------
    def local_forward(self, ids: torch.Tensor, mask: torch.Tensor, past: int, forced: torch.Tensor,
                      n_vq_for_inference: int = -1):
        """Teacher-forced frame (backbone over `ids` at `past`, then the depth loop fed `forced`
        [B, 1+n_vq]); returns bf16 logits per channel [n_ch][B, V_i] (pad column -inf, i >= 1)."""
        B, S, C = ids.shape
        c = self.cfg
        n_ch = C if n_vq_for_inference < 0 else min(C, 1 + n_vq_for_inference)
        ld = (c.vocab + 7) // 8 * 8
        _check_mask(mask, B, past + S)
        ids = ids.to(self.device, torch.int64).contiguous()
        mask = mask.to(self.device, torch.uint8).contiguous()
        forced = forced.to(self.device, torch.int64).contiguous()
        assert tuple(forced.shape) == (B, C)
        out = torch.empty(n_ch, B, ld, dtype=torch.bfloat16, device=self.device)
        N.check(N.load().mtts_local_forward(self._h, _ptr(ids), _ptr(mask), B, S, past, n_vq_for_inference, _ptr(forced),
                                            _ptr(out), ld, _stream_ptr(self.device)), "local_forward")
        A = c.audio_vocab + 1
        return [out[0, :, :c.vocab]] + [out[i, :, :A] for i in range(1, n_ch)]

    def local_generate_ids(self, input_ids: torch.Tensor, attention_mask: Optional[torch.Tensor], max_new_tokens: int,
                           n_vq_for_inference: int = -1, chunk: int = 16, sampling: Optional[N.MttsSampling] = None):
        """MossTTSLocal loop on the device (greedy unless `sampling` has a positive temperature:
        text_* drive channel 0, audio_* the codebook channels); returns generation_ids
        [B, T + n, 1+n_vq]."""
        B, T, C = input_ids.shape
        _check_mask(attention_mask, B, T)
        ids = input_ids.to(self.device, torch.int64).contiguous()
        mask = None if attention_mask is None else attention_mask.to(self.device, torch.uint8).contiguous()
        n = ctypes.c_int()
        sp = None if sampling is None else ctypes.byref(sampling)
        N.check(N.load().mtts_local_generate(self._h, _ptr(ids), _ptr(mask), B, T, max_new_tokens, n_vq_for_inference,
                                             sp, chunk, ctypes.byref(n), _stream_ptr(self.device)), "local_generate")
        out = torch.empty(B, T + n.value, C, dtype=torch.int64, device=self.device)
        N.check(N.load().mtts_generate_fetch(self._h, _ptr(out), n.value, _stream_ptr(self.device)), "fetch")
        return out

    def local_set_sampling(self, channels):
        """MossTTSLocal per-channel processors for the following generations: a list of
        (do_sample, temperature, top_k, top_p, repetition_penalty) per channel (top_k <= 0 /
        top_p 1 / penalty 1 = that processor absent); [] reverts to the sampling struct's split"""
        arr = (N.MttsChannelSampling * max(1, len(channels)))()
        for i, (d, t, k, p, r) in enumerate(channels):
            arr[i] = N.MttsChannelSampling(int(bool(d)), float(t), int(k), float(p), float(r))
        N.check(N.load().mtts_local_set_sampling(self._h, arr, len(channels)), "local_set_sampling")

    def local_frame_bytes(self, n_vq_for_inference: int = -1) -> int:
        v = ctypes.c_uint64()
        N.check(N.load().mtts_local_frame_bytes(self._h, n_vq_for_inference, ctypes.byref(v)), "local_frame_bytes")
        return int(v.value)


class GenerateSession:
    """Step-wise form of Engine.generate_ids for streaming: begin (prefill + step 0), then
    decode chunks of hipGraph steps, polling and fetching the generation rows in between."""

    def __init__(self, eng: "Engine", input_ids: torch.Tensor, attention_mask: Optional[torch.Tensor],
                 max_new_tokens: int, sampling: N.MttsSampling, forced_text: Optional[torch.Tensor] = None):
        self.eng = eng
        self.B, self.T, self.C = input_ids.shape
        _check_mask(attention_mask, self.B, self.T)
        self.max_new = max_new_tokens
        self._ids = input_ids.to(eng.device, torch.int64).contiguous()
        self._mask = None if attention_mask is None else attention_mask.to(eng.device, torch.uint8).contiguous()
        self._forced = None if forced_text is None else forced_text.to(eng.device, torch.int32).contiguous()
        self._sp = sampling
        N.check(N.load().mtts_generate_begin(eng._h, _ptr(self._ids), _ptr(self._mask), self.B, self.T,
                                             max_new_tokens, ctypes.byref(self._sp), _ptr(self._forced),
                                             _stream_ptr(eng.device)), "generate_begin")
        self.steps, self.done_step = 1, -1

    def poll(self):
        st, dn = ctypes.c_int(), ctypes.c_int()
        N.check(N.load().mtts_generate_poll(self.eng._h, ctypes.byref(st), ctypes.byref(dn), None), "poll")
        self.steps, self.done_step = st.value, dn.value
        return self.steps, self.done_step

    @property
    def finished(self) -> bool:
        return self.done_step >= 0 or self.steps >= self.max_new

    @property
    def n_rows(self) -> int:
        """generated rows the reference's generation_ids would hold so far"""
        return self.done_step + 1 if self.done_step >= 0 else self.steps

    def decode(self, n_steps: int):
        n = min(n_steps, self.max_new - self.steps)
        if n > 0 and self.done_step < 0:
            N.check(N.load().mtts_generate_decode(self.eng._h, n, _stream_ptr(self.eng.device)), "generate_decode")
        return self.poll()

    def logits(self) -> torch.Tensor:
        """bf16 [B, heads_ld]: the logits the last sampled step drew from (parity hook)"""
        out = torch.empty(self.B, self.eng.heads_ld, dtype=torch.bfloat16, device=self.eng.device)
        N.check(N.load().mtts_generate_logits(self.eng._h, _ptr(out), _stream_ptr(self.eng.device)), "generate_logits")
        return out

    def fetch(self) -> torch.Tensor:
        """generation_ids [B, T + n_rows, 1 + n_vq] (prompt included) so far"""
        out = torch.empty(self.B, self.T + self.n_rows, self.C, dtype=torch.int64, device=self.eng.device)
        N.check(N.load().mtts_generate_fetch(self.eng._h, _ptr(out), self.n_rows, _stream_ptr(self.eng.device)),
                "fetch")
        return out


def _check_mask(mask, B, L):
    """the C ABI reads B x L mask bytes ([B, past + S] for a forward, [B, T] for generate):
    a shorter mask would be read past its end (the reference forwards any mask to Qwen3)"""
    if mask is not None and tuple(mask.shape) != (B, L):
        raise ValueError(f"attention_mask must be [batch, past + seq] = [{B}, {L}], got {tuple(mask.shape)}")


def sampling_params(text_temperature=1.5, text_top_p=1.0, text_top_k=50, audio_temperature=1.7, audio_top_p=0.8,
                    audio_top_k=25, audio_repetition_penalty=1.0, seed=0):
    s = N.MttsSampling()
    s.text_temperature = text_temperature
    s.text_top_p = text_top_p
    s.text_top_k = text_top_k
    s.audio_temperature = audio_temperature
    s.audio_top_p = audio_top_p
    s.audio_top_k = audio_top_k
    s.audio_repetition_penalty = audio_repetition_penalty
    s.seed = seed
    return s
