"""MossTTSLocal's MossTTSDelayConfig (mirror of the reference
`moss_tts_local/configuration_moss_tts.py:62-122`): the Delay fields plus the depth-stage
sizes (additional_mlp_ffn_hidden_size, local_ffn_hidden_size, local_hidden_size,
local_num_layers), so a MossTTSLocal checkpoint's config.json loads unchanged."""
from typing import Optional, Union

from ..configuration_moss_tts import MossTTSDelayConfig as _DelayConfig


class MossTTSDelayConfig(_DelayConfig):
    model_type = "moss_tts_delay"

    def __init__(self, language_config: Optional[Union[object, dict]] = None, additional_mlp_ffn_hidden_size: int = 2048,
                 local_ffn_hidden_size: int = 8960, local_hidden_size: int = 1536, local_num_layers: int = 4, **kwargs):
        self.additional_mlp_ffn_hidden_size = additional_mlp_ffn_hidden_size
        self.local_ffn_hidden_size = local_ffn_hidden_size
        self.local_hidden_size = local_hidden_size
        self.local_num_layers = local_num_layers
        super().__init__(language_config=language_config, **kwargs)
