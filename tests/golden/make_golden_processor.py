#!/usr/bin/env python3
"""Golden vectors for the processors' I/O surface, from the REFERENCE processors
(`moss_tts_delay/processing_moss_tts.py`, `moss_tts_local/processing_moss_tts.py`) run in this
container with the stub tokenizer of tokenizer_stub.py (no checkpoint / network):

    python tests/golden/make_golden_processor.py

Records, per processor and case, the encoded input_ids / attention_mask of __call__ (generation
and continuation modes, reference audio blocks, multi-turn, left-padded batches, the user
message fields) or the fact that the reference raises, plus _parse_text_codes on synthetic
generation rows.  Outputs tests/golden/golden_processor.npz (allow_pickle=False) + .json."""
import importlib.machinery
import json
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, "/root/reference")
_ta = types.ModuleType("torchaudio")  # the processors import it for codec I/O only
_ta.__spec__ = importlib.machinery.ModuleSpec("torchaudio", None)
sys.modules.setdefault("torchaudio", _ta)

import torch  # noqa: E402

from processor_cases import cases  # noqa: E402
from tokenizer_stub import build_tokenizer  # noqa: E402


def run(mod_name):
    import importlib
    cfg_mod = importlib.import_module(f"{mod_name}.configuration_moss_tts")
    proc_mod = importlib.import_module(f"{mod_name}.processing_moss_tts")
    tok = build_tokenizer()
    P = proc_mod.MossTTSDelayProcessor(tokenizer=tok, audio_tokenizer=None, model_config=cfg_mod.MossTTSDelayConfig(n_vq=4))
    arrays, meta = {}, {}
    for name, (convs, mode) in cases(P).items():
        try:
            out = P(convs, mode=mode)
            arrays[f"{mod_name}/{name}/input_ids"] = out["input_ids"].numpy()
            arrays[f"{mod_name}/{name}/attention_mask"] = out["attention_mask"].numpy().astype(np.uint8)
            meta[name] = {"raises": False}
        except Exception as e:  # the reference's own refusal is part of the contract
            meta[name] = {"raises": True, "error": type(e).__name__}
    # _parse_text_codes on a synthetic generation row: assistant header, audio block, im_end
    gen = ([151644] + tok.encode("assistant\n", add_special_tokens=False) + [151652] + [151656] * 4 +
           ([151662] * 3 if mod_name == "moss_tts_delay" else []) + [151653, 151645])
    meta["parse_text"] = {"ids": gen, "start_length": 3, "content": P._parse_text_codes(3, torch.tensor(gen))}
    return arrays, meta


def main():
    arrays, meta = {}, {}
    for m in ("moss_tts_delay", "moss_tts_local"):
        a, mm = run(m)
        arrays.update(a)
        meta[m] = mm
        print(m, json.dumps(mm)[:300], flush=True)
    np.savez_compressed(os.path.join(HERE, "golden_processor.npz"), **arrays)
    with open(os.path.join(HERE, "golden_processor.json"), "w") as f:
        json.dump(meta, f, indent=1)


if __name__ == "__main__":
    main()
