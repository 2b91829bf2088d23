"""MossTTSDelayModel drop-in: same class name, state_dict names, `generate()` signature
and output contract as the reference `moss_tts_delay/modeling_moss_tts.py`, with every
arithmetic op of the decode path running in the HIP engine (libmtts.so).

Loading seam (clis/moss_tts_app.py:95-108): `AutoModel.from_pretrained(path,
trust_remote_code=True, torch_dtype=bf16)` builds this class (a checkpoint's
config.json `auto_map` points at this module -- INTEGRATION.md), torch holds the
checkpoint tensors until the first call, then they are repacked into the engine's
MFMA-tile layout in HBM and the torch copies are released.
"""
import os
from dataclasses import dataclass
from typing import List, Optional, Tuple

import torch
import torch.nn as nn

from transformers.modeling_outputs import ModelOutput
from transformers.modeling_utils import PreTrainedModel
from transformers.models.qwen3 import Qwen3Model

from .configuration_moss_tts import MossTTSDelayConfig
from .engine import Engine, EngineConfig, sampling_params

try:
    from .processing_moss_tts import AssistantMessage, MossTTSDelayProcessor, UserMessage
except Exception:  # pragma: no cover
    UserMessage = AssistantMessage = MossTTSDelayProcessor = None


@dataclass
class MossTTSDelayOutputWithPast(ModelOutput):
    loss: Optional[torch.FloatTensor] = None
    logits: Optional[List[torch.FloatTensor]] = None
    past_key_values: Optional[object] = None
    hidden_states: Optional[Tuple[torch.FloatTensor]] = None
    attentions: Optional[Tuple[torch.FloatTensor]] = None


class EngineCache:
    """Stands in for the reference's DynamicCache: the KV cache lives in the engine; this
    records how many positions it holds (the `past` of the next forward)."""

    def __init__(self, length: int = 0):
        self.length = length

    def get_seq_length(self, layer_idx: int = 0) -> int:
        return self.length


def find_last_equal_C(tensor: torch.Tensor, C: int) -> torch.Tensor:
    """`inference_utils.py:148-165`: last index of C per row, -1 when absent."""
    hit = tensor == C
    T = tensor.shape[1]
    idx = (T - 1) - hit.flip(dims=[1]).int().argmax(dim=1)
    return torch.where(hit.any(dim=1), idx, torch.full_like(idx, -1))


class MossTTSDelayPreTrainedModel(PreTrainedModel):
    config_class = MossTTSDelayConfig
    base_model_prefix = "model"
    _no_split_modules = ["Qwen3DecoderLayer"]
    _skip_keys_device_placement = "past_key_values"
    _supports_sdpa = True

    def _init_weights(self, module):
        super()._init_weights(module)
        if isinstance(module, nn.Embedding) and getattr(module, "num_embeddings", None) == self.config.audio_vocab_size + 1:
            std = getattr(self.config, "initializer_range", 0.02)
            with torch.no_grad():
                module.weight.normal_(0.0, std)


class MossTTSDelayModel(MossTTSDelayPreTrainedModel):
    """Parameters mirror `modeling_moss_tts.py:164-194` (language_model, emb_ext, lm_heads)."""
    UserMessage = UserMessage
    AssistantMessage = AssistantMessage
    Processor = MossTTSDelayProcessor

    def __init__(self, config: MossTTSDelayConfig):
        super().__init__(config)
        self.config = config
        self.language_model = Qwen3Model(config.language_config)
        H = config.language_config.hidden_size
        self.emb_ext = nn.ModuleList([nn.Embedding(config.audio_vocab_size + 1, H) for _ in range(config.n_vq)])
        self.lm_heads = nn.ModuleList([nn.Linear(H, config.language_config.vocab_size, bias=False)] +
                                      [nn.Linear(H, config.audio_vocab_size + 1, bias=False)
                                       for _ in range(config.n_vq)])
        self._engine: Optional[Engine] = None
        self.post_init()

    # ---- engine --------------------------------------------------------------
    def _device_index(self) -> int:
        for p in self.parameters():
            if p.is_cuda:
                return p.device.index or 0
        return torch.cuda.current_device()

    def engine(self, batch: int = 1, ctx: int = 2048) -> Engine:
        """Build the engine on first use (weights -> HBM tiles) and grow its capacity."""
        want_b = max(batch, int(os.environ.get("MTTS_MAX_BATCH", "8")))
        want_c = max(ctx, int(os.environ.get("MTTS_MAX_CTX", "4096")))
        if self._engine is None:
            ecfg = EngineConfig.from_hf(self.config, max_batch=want_b, max_ctx=want_c,
                                        max_prefill_tokens=int(os.environ.get("MTTS_MAX_PREFILL", max(8192, want_c))))
            eng = Engine(ecfg, self._device_index())
            for name, p in self.state_dict().items():
                if "rotary_emb" in name:
                    continue
                eng.load_weight(name, p)
            # the engine owns the weights now; release the torch copies (keep the Parameters so
            # `.parameters()` still reports the device, clis/moss_tts_app.py:108)
            for p in self.parameters():
                p.data = torch.empty(0, dtype=p.dtype, device=p.device)
            self._engine = eng
        else:
            c = self._engine.cfg
            if batch > c.max_batch or ctx > c.max_ctx:
                self._engine.reserve(max(batch, c.max_batch), max(ctx, c.max_ctx))
        return self._engine

    # ---- forward (teacher forcing) ------------------------------------------------
    def get_input_embeddings(self):
        return self.language_model.embed_tokens

    def get_output_embeddings(self):
        return self.lm_heads

    def forward(self, input_ids: Optional[torch.LongTensor] = None, attention_mask: Optional[torch.Tensor] = None,
                past_key_values: Optional[EngineCache] = None, labels=None, use_cache: Optional[bool] = None,
                **kwargs) -> MossTTSDelayOutputWithPast:
        """`modeling_moss_tts.py:225-300`, inference only: appends the S tokens to the engine's
        KV cache and returns the LAST position's logits of the 1+n_vq heads as [B, 1, V_i]
        (generate uses only `logits[:, -1]`, `:451`; the training loss `:309-378` is out of scope)."""
        if input_ids is None or len(input_ids.shape) != 3 or input_ids.shape[-1] != self.config.n_vq + 1:
            raise ValueError("`Input_ids`'s shape should be exactly (batch_size, sequence_length, 1 + n_vq).")
        if labels is not None:
            raise NotImplementedError("training loss is out of scope for the MI355X inference engine")
        B, S, _ = input_ids.shape
        past = past_key_values.get_seq_length() if past_key_values is not None else 0
        eng = self.engine(B, past + S + 1)
        if attention_mask is None:
            attention_mask = torch.ones(B, past + S, dtype=torch.bool, device=input_ids.device)
        logits = eng.forward(input_ids, attention_mask, past)
        parts = [x[:, None, :] for x in eng.split_logits(logits)]
        return MossTTSDelayOutputWithPast(logits=parts, past_key_values=EngineCache(past + S))

    # ---- generate -----------------------------------------------------------------
    @torch.inference_mode()
    def generate(self, input_ids: torch.LongTensor, attention_mask: Optional[torch.Tensor] = None,
                 max_new_tokens: int = 1000, text_temperature: float = 1.5, text_top_p: float = 1.0,
                 text_top_k: int = 50, audio_temperature: float = 1.7, audio_top_p: float = 0.8,
                 audio_top_k: int = 25, audio_repetition_penalty: float = 1.0, forced_text: Optional[torch.Tensor] = None):
        """`modeling_moss_tts.py:392-525`.  Returns [(start_length, generation_ids[b, start:])]
        with start = last <|im_start|> + 3, generation_ids = prompt + one row per step, all
        rows running until every row emitted <|im_end|> (or max_new_tokens).  Temperature
        <= 0 means greedy.  The draws use a Philox stream seeded from torch's default
        generator (so torch.manual_seed makes runs reproducible); `forced_text` is an
        engine extension used only by the benchmark."""
        if input_ids.dim() != 3 or input_ids.shape[-1] != self.config.n_vq + 1:
            raise ValueError("`Input_ids`'s shape should be exactly (batch_size, sequence_length, 1 + n_vq).")
        B, T, _ = input_ids.shape
        eng = self.engine(B, T + max_new_tokens)
        seed = int(torch.randint(0, 2 ** 62, (1,)).item())
        sp = sampling_params(text_temperature=text_temperature, text_top_p=text_top_p, text_top_k=text_top_k,
                             audio_temperature=audio_temperature, audio_top_p=audio_top_p, audio_top_k=audio_top_k,
                             audio_repetition_penalty=audio_repetition_penalty, seed=seed)
        gen = eng.generate_ids(input_ids, attention_mask, max_new_tokens, sp, forced_text=forced_text)
        gen = gen.to(input_ids.device)
        starts = find_last_equal_C(input_ids[..., 0], self.config.im_start_token_id) + 3
        lengths = T - starts
        return [(lengths[b], gen[b, int(starts[b]):]) for b in range(B)]

    @torch.inference_mode()
    def generate_stream(self, input_ids: torch.LongTensor, attention_mask: Optional[torch.Tensor] = None,
                        max_new_tokens: int = 1000, chunk_steps: int = 16, text_temperature: float = 1.5,
                        text_top_p: float = 1.0, text_top_k: int = 50, audio_temperature: float = 1.7,
                        audio_top_p: float = 0.8, audio_top_k: int = 25, audio_repetition_penalty: float = 1.0,
                        forced_text: Optional[torch.Tensor] = None):
        """Streaming form of `generate` (the reference has none).  Decodes in
        chunks of `chunk_steps` hipGraph steps and yields, after each chunk, the audio frames
        that became complete: frame f of the delay pattern is final once generated row
        f + n_vq - 1 exists (`processing_moss_tts.py:515-537`).  Yields lists (one per batch
        row) of LongTensor [n_new_frames, n_vq] (de-delayed, all-pad frames dropped, on the
        device); concatenated per row they equal `split_audio_segments` of the generate()
        output.  A codec decoder can consume each chunk as it arrives."""
        from .processing_moss_tts import apply_de_delay_pattern
        if input_ids.dim() != 3 or input_ids.shape[-1] != self.config.n_vq + 1:
            raise ValueError("`Input_ids`'s shape should be exactly (batch_size, sequence_length, 1 + n_vq).")
        B, T, _ = input_ids.shape
        n_vq, pad = self.config.n_vq, self.config.audio_pad_code
        eng = self.engine(B, T + max_new_tokens)
        seed = int(torch.randint(0, 2 ** 62, (1,)).item())
        sp = sampling_params(text_temperature=text_temperature, text_top_p=text_top_p, text_top_k=text_top_k,
                             audio_temperature=audio_temperature, audio_top_p=audio_top_p, audio_top_k=audio_top_k,
                             audio_repetition_penalty=audio_repetition_penalty, seed=seed)
        starts = (find_last_equal_C(input_ids[..., 0], self.config.im_start_token_id) + 3).tolist()
        sess = eng.session(input_ids, attention_mask, max_new_tokens, sp, forced_text=forced_text)
        sess.poll()
        emitted = [0] * B  # complete frames (pad frames included) already examined per row
        while True:
            final = sess.finished
            gen = sess.fetch()
            out = []
            for b in range(B):
                a = gen[b, int(starts[b]):, 1:]
                n_complete = a.shape[0] - n_vq + 1
                if n_complete <= emitted[b]:
                    out.append(a.new_zeros((0, n_vq)))
                    continue
                frames = apply_de_delay_pattern(a[: n_complete + n_vq - 1])[emitted[b]:n_complete]
                emitted[b] = n_complete
                out.append(frames[~(frames == pad).all(dim=1)])
            yield out
            if final:
                return
            sess.decode(chunk_steps)
