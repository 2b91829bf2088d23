"""MossTTSLocal drop-in model: the reference class `MossTTSDelayModel` of
`moss_tts_local/modeling_moss_tts.py:568-743` with the same parameter names (model.embedding_list,
model.language_model, local_transformer, speech_embedding_to_local_mlp,
local_to_speech_embedding_mlps, layer_norm_before_lm_heads, lm_heads) and the
`generate(input_ids, attention_mask, generation_config)` contract of `CustomMixin._sample`
(:315-477), every arithmetic op of the frame loop running in the HIP engine.

generation_config (README `moss_tts_local/README.md:203-220`): `n_vq_for_inference`,
`do_samples` (per channel), `layers` (per channel dict of repetition_penalty / temperature /
top_k / top_p), `max_new_tokens` or `max_length`, `eos_token_id`.  Every channel takes its own
processor set (mtts_local_set_sampling); any top_k (none, or past the sorted candidate list) is served.
"""
import copy
import os
from typing import List, Optional

import torch
import torch.nn as nn
from transformers.modeling_utils import PreTrainedModel
from transformers.models.qwen3 import Qwen3Model
from transformers.models.qwen3.modeling_qwen3 import Qwen3DecoderLayer, Qwen3RMSNorm

from ..engine import Engine, EngineConfig, sampling_params
from ..modeling_moss_tts import find_last_equal_C
from .configuration_moss_tts import MossTTSDelayConfig


class MossTTSMLP(nn.Module):
    """`:47-95` (no pre-norm, no bias): down(silu(gate(x)) * up(x))"""

    def __init__(self, input_size: int, ffn_hidden_size: int, output_size: int):
        super().__init__()
        self.gate_proj = nn.Linear(input_size, ffn_hidden_size, bias=False)
        self.up_proj = nn.Linear(input_size, ffn_hidden_size, bias=False)
        self.down_proj = nn.Linear(ffn_hidden_size, output_size, bias=False)


class MossTTSRMSNorm(nn.Module):
    """`:34-44` (weight only; the bf16 arithmetic runs in the engine)"""

    def __init__(self, dim: int, eps: float = 1e-6):
        super().__init__()
        self.eps = eps
        self.weight = nn.Parameter(torch.ones(dim))


class MossTTSLocalTransformer(nn.Module):
    """`:178-292`: Qwen3 decoder layers (attention without positional embedding) + final norm.
    The reference subclasses Qwen3Model, so its state_dict also holds an unused embed_tokens."""

    def __init__(self, config):
        super().__init__()
        self.embed_tokens = nn.Embedding(config.vocab_size, config.hidden_size)
        self.layers = nn.ModuleList([Qwen3DecoderLayer(config, i) for i in range(config.num_hidden_layers)])
        self.norm = Qwen3RMSNorm(config.hidden_size, eps=config.rms_norm_eps)


class MosiTTSModel(nn.Module):
    """`:495-560`: channel embeddings + the Qwen3 backbone"""

    def __init__(self, config: MossTTSDelayConfig):
        super().__init__()
        H = config.hidden_size
        self.embedding_list = nn.ModuleList([nn.Embedding(config.vocab_size, H)] +
                                            [nn.Embedding(config.audio_vocab_size + 1, H) for _ in range(config.n_vq)])
        self.language_model = Qwen3Model(config.language_config)


class MossTTSDelayModel(PreTrainedModel):
    config_class = MossTTSDelayConfig
    base_model_prefix = "model"
    _no_split_modules = ["Qwen3DecoderLayer"]

    def __init__(self, config: MossTTSDelayConfig):
        super().__init__(config)
        self.config = config
        self.model = MosiTTSModel(config)
        self.channels = 1 + config.n_vq
        lc = copy.deepcopy(config.language_config)
        lc.num_hidden_layers = config.local_num_layers
        lc.hidden_size = config.local_hidden_size
        lc.intermediate_size = config.local_ffn_hidden_size
        self.local_transformer_config = lc
        self.local_transformer = MossTTSLocalTransformer(lc)
        H, LH, F = config.hidden_size, config.local_hidden_size, config.additional_mlp_ffn_hidden_size
        self.speech_embedding_to_local_mlp = MossTTSMLP(H, F, LH)
        self.local_to_speech_embedding_mlps = nn.ModuleList([MossTTSMLP(LH, F, H) for _ in range(self.channels)])
        self.layer_norm_before_lm_heads = nn.ModuleList([MossTTSRMSNorm(H) for _ in range(self.channels)])
        self.lm_heads = nn.ModuleList([nn.Linear(H, config.vocab_size, bias=False)] +
                                      [nn.Linear(H, config.audio_vocab_size + 1, bias=False)
                                       for _ in range(1, self.channels)])
        self._engine: Optional[Engine] = None
        self.post_init()

    def get_input_embeddings(self):
        return self.model.embedding_list[0]

    def get_output_embeddings(self):
        return self.lm_heads[0]

    def can_generate(self):
        return True

    # ---- engine --------------------------------------------------------------
    def _device_index(self) -> int:
        for p in self.parameters():
            if p.is_cuda:
                return p.device.index or 0
        return torch.cuda.current_device()

    def engine(self, batch: int = 1, ctx: int = 2048, eos_token_id: int = 151653) -> Engine:
        want_b = max(batch, int(os.environ.get("MTTS_MAX_BATCH", "8")))
        want_c = max(ctx, int(os.environ.get("MTTS_MAX_CTX", "4096")))
        if self._engine is None:
            c = self.config
            ecfg = EngineConfig.from_hf(c, max_batch=want_b, max_ctx=want_c,
                                        max_prefill_tokens=int(os.environ.get("MTTS_MAX_PREFILL", max(8192, want_c))),
                                        model_kind=1, local_hidden=c.local_hidden_size, local_layers=c.local_num_layers,
                                        local_inter=c.local_ffn_hidden_size,
                                        local_mlp_ffn=c.additional_mlp_ffn_hidden_size, eos_token_id=eos_token_id)
            eng = Engine(ecfg, self._device_index())
            for name, p in self.state_dict().items():
                if "rotary_emb" in name or name == "local_transformer.embed_tokens.weight":
                    continue
                eng.load_weight(name, p)
            for p in self.parameters():  # the engine owns the weights now
                p.data = torch.empty(0, dtype=p.dtype, device=p.device)
            self._engine = eng
        else:
            c = self._engine.cfg
            if eos_token_id != c.eos_token_id:
                raise NotImplementedError("eos_token_id differs from the one the engine was built with")
            if batch > c.max_batch or ctx > c.max_ctx:
                self._engine.reserve(max(batch, c.max_batch), max(ctx, c.max_ctx))
        return self._engine

    # ---- generate -----------------------------------------------------------------
    def _sampling(self, gc, n_ch: int):
        """generation_config.do_samples / layers -> the engine's per-channel processor table
        (`:356-368`: RepetitionPenalty (never on channel 0) -> Temperature -> TopK -> TopP, each
        only when its key is set; channels with do_samples[i] False take the argmax)"""
        do = list(getattr(gc, "do_samples", None) or [bool(getattr(gc, "do_sample", False))] * self.channels)
        layers = list(getattr(gc, "layers", None) or [{}] * self.channels)
        if len(do) < n_ch or len(layers) < n_ch:
            raise ValueError("generation_config.do_samples / layers must cover every generated channel")
        table = []
        for i in range(n_ch):
            lc = layers[i] or {}
            t, k, p, r = (lc.get(x) for x in ("temperature", "top_k", "top_p", "repetition_penalty"))
            table.append((bool(do[i]), 1.0 if t is None else float(t), 0 if k is None else int(k),
                          1.0 if p is None else float(p), 1.0 if (r is None or i == 0) else float(r)))
        seed = int(torch.randint(0, 2 ** 62, (1,)).item())
        return table, sampling_params(text_temperature=0.0, audio_temperature=0.0, seed=seed)

    @torch.inference_mode()
    def generate(self, input_ids: torch.LongTensor, attention_mask: Optional[torch.Tensor] = None,
                 generation_config=None, **kwargs):
        """Returns [(start_length, generation_ids[b, start_idx:])], start_idx = last
        audio_start of channel 0, start_length = T - start_idx - 1 (`:466-477`)."""
        if input_ids.dim() != 3 or input_ids.shape[-1] != self.channels:
            raise ValueError(f"Expected input_ids of shape (batch, seq, {self.channels})")
        gc = copy.deepcopy(generation_config) if generation_config is not None else None
        if gc is None:
            from transformers import GenerationConfig
            gc = GenerationConfig()
        for k, v in kwargs.items():
            setattr(gc, k, v)
        B, T, C = input_ids.shape
        max_new = gc.max_new_tokens if getattr(gc, "max_new_tokens", None) else (gc.max_length or T + 1) - T
        nq = getattr(gc, "n_vq_for_inference", None)
        nq = self.config.n_vq if nq is None else int(nq)
        n_ch = min(C, 1 + nq)
        eos = gc.eos_token_id if gc.eos_token_id is not None else self.config.audio_end_token_id
        if isinstance(eos, (list, tuple)):
            if len(eos) != 1:
                raise NotImplementedError("one eos_token_id")
            eos = eos[0]
        eng = self.engine(B, T + max_new, int(eos))
        table, sp = self._sampling(gc, n_ch)
        eng.local_set_sampling(table)
        try:
            gen = eng.local_generate_ids(input_ids, attention_mask, max_new, nq, sampling=sp).to(input_ids.device)
        finally:
            eng.local_set_sampling([])
        starts = find_last_equal_C(input_ids[..., 0], self.config.audio_start_token_id)
        lengths = T - starts - 1
        return [(lengths[b], gen[b, int(starts[b]):]) for b in range(B)]
