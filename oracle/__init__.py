"""CPU oracle for the MossTTSDelay decode path -- TEST INFRASTRUCTURE ONLY.

This package is a plain-numpy restatement of the reference algorithm
(xiami2019/MOSS-TTS `moss_tts_delay/*.py` plus the transformers Qwen3 backbone
it calls).  It exists to *check* the HIP engine, never to run in its place:

* only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline`
  leg may import it;
* the product path (`moss_tts_amd`) never imports it and fails loudly when
  the HIP library is missing.

Parity pinning: the restatement is checked against golden vectors produced by
running the reference's own classes in this container
(`tests/golden/make_golden.py`, fixtures in `tests/golden/*.npz`).  The codec
(MOSS-Audio-Tokenizer) is absent from the reference checkout, so there is no
codec oracle: codec parity is "parity unpinned" (see DESIGN.md).
"""

from . import bf16, prng, moss_delay  # noqa: F401
