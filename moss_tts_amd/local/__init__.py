"""MossTTSLocal drop-in (reference `moss_tts_local/`): configuration and model classes with the
reference's names, state_dict layout and `generate(input_ids, attention_mask,
generation_config)` contract, running on the libmtts.so engine (model_kind MTTS_MODEL_LOCAL)."""
from .configuration_moss_tts import MossTTSDelayConfig
from .modeling_moss_tts import MossTTSDelayModel

__all__ = ["MossTTSDelayConfig", "MossTTSDelayModel"]
