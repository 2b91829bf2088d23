"""The processors' I/O surface (Delay and Local) against golden vectors from the reference's
own processors (tests/golden/make_golden_processor.py, same stub tokenizer): encoded
input_ids / attention_mask per case, the reference's refusals, and _parse_text_codes."""
import json
import os
import sys

import numpy as np
import pytest

torch = pytest.importorskip("torch")
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))

from tokenizer_stub import build_tokenizer  # noqa: E402
from processor_cases import cases  # noqa: E402


@pytest.fixture(scope="module")
def gp():
    g = np.load(os.path.join(HERE, "golden", "golden_processor.npz"))
    meta = json.load(open(os.path.join(HERE, "golden", "golden_processor.json")))
    return g, meta


def processor(kind):
    tok = build_tokenizer()
    if kind == "moss_tts_delay":
        from moss_tts_amd.configuration_moss_tts import MossTTSDelayConfig
        from moss_tts_amd.processing_moss_tts import MossTTSDelayProcessor
    else:
        from moss_tts_amd.local.configuration_moss_tts import MossTTSDelayConfig
        from moss_tts_amd.local.processing_moss_tts import MossTTSDelayProcessor
    return MossTTSDelayProcessor(tokenizer=tok, audio_tokenizer=None, model_config=MossTTSDelayConfig(n_vq=4))


@pytest.mark.parametrize("kind", ["moss_tts_delay", "moss_tts_local"])
def test_processor_encode_matches_reference(gp, kind):
    g, meta = gp
    P = processor(kind)
    for name, (convs, mode) in cases(P).items():
        m = meta[kind][name]
        if m["raises"]:
            with pytest.raises(Exception) as ei:
                P(convs, mode=mode)
            assert type(ei.value).__name__ == m["error"], name
            continue
        out = P(convs, mode=mode)
        want_ids = g[f"{kind}/{name}/input_ids"]
        want_mask = g[f"{kind}/{name}/attention_mask"]
        assert np.array_equal(out["input_ids"].numpy(), want_ids), name
        assert np.array_equal(out["attention_mask"].numpy().astype(np.uint8), want_mask), name


@pytest.mark.parametrize("kind", ["moss_tts_delay", "moss_tts_local"])
def test_parse_text_codes_matches_reference(gp, kind):
    _, meta = gp
    P = processor(kind)
    m = meta[kind]["parse_text"]
    assert P._parse_text_codes(m["start_length"], torch.tensor(m["ids"])) == m["content"]
