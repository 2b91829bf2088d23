"""MossTTSLocal processor (`moss_tts_local/processing_moss_tts.py`): the Delay processor's
I/O surface with the codes laid out undelayed -- no delay slots in the audio blocks (:465),
at most one audio block per message (:598), generation prompts end on an audio_start row
(:351-356), continuation (truncation) unsupported (:624), decode splits the undelayed codes
(:668-690)."""
from ..processing_moss_tts import AssistantMessage, UserMessage  # noqa: F401
from ..processing_moss_tts import MossTTSDelayProcessor as _DelayProcessor
from .configuration_moss_tts import MossTTSDelayConfig


class MossTTSDelayProcessor(_DelayProcessor):
    delay_pattern = False

    def __init__(self, tokenizer, audio_tokenizer=None, model_config=None, **kwargs):
        super().__init__(tokenizer, audio_tokenizer=audio_tokenizer,
                         model_config=model_config if model_config is not None else MossTTSDelayConfig(), **kwargs)
