"""MossTTSDelayConfig (mirror of the reference `moss_tts_delay/configuration_moss_tts.py`):
the same fields, defaults and serialisation, so a checkpoint's config.json loads
unchanged; `model_type` stays "moss_tts_delay"."""
from typing import Optional, Union

try:
    from transformers.configuration_utils import PretrainedConfig
    from transformers.models.qwen3 import Qwen3Config
except Exception:  # pragma: no cover - transformers is a hard dependency of the drop-in
    PretrainedConfig = object
    Qwen3Config = None


class MossTTSDelayConfig(PretrainedConfig):
    """Defaults restate `configuration_moss_tts.py:62-77` (n_vq 32, audio vocab 1024, special ids)."""
    model_type = "moss_tts_delay"
    keys_to_ignore_at_inference = ["past_key_values"]

    def __init__(self, language_config: Optional[Union["Qwen3Config", dict]] = None, initializer_range: float = 0.02,
                 n_vq: int = 32, pad_token_id: int = 151643, im_start_token_id: int = 151644,
                 im_end_token_id: int = 151645, audio_vocab_size: int = 1024,
                 audio_user_slot_token_id: int = 151654, audio_assistant_gen_slot_token_id: int = 151656,
                 audio_assistant_delay_slot_token_id: int = 151662, audio_start_token_id: int = 151652,
                 audio_end_token_id: int = 151653, audio_pad_code: int = 1024, sampling_rate: int = 24000,
                 **kwargs):
        if isinstance(language_config, dict):
            language_config = Qwen3Config(**language_config)
        elif language_config is None:
            language_config = Qwen3Config()
        self.language_config = language_config
        self.initializer_range = initializer_range
        self.n_vq = n_vq
        self.audio_vocab_size = audio_vocab_size
        self.audio_user_slot_token_id = audio_user_slot_token_id
        self.audio_assistant_gen_slot_token_id = audio_assistant_gen_slot_token_id
        self.audio_assistant_delay_slot_token_id = audio_assistant_delay_slot_token_id
        self.audio_start_token_id = audio_start_token_id
        self.audio_end_token_id = audio_end_token_id
        self.audio_pad_code = audio_pad_code
        self.sampling_rate = sampling_rate
        self.hidden_size = language_config.hidden_size
        self.vocab_size = language_config.vocab_size
        self.pad_token_id = pad_token_id
        self.im_start_token_id = im_start_token_id
        self.im_end_token_id = im_end_token_id
        super().__init__(**kwargs)

    def to_dict(self):
        out = super().to_dict()
        lc = self.language_config
        out["language_config"] = lc.to_dict() if hasattr(lc, "to_dict") else lc
        return out
