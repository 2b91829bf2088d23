"""The drop-in contract end to end, the way `clis/moss_tts_app.py` loads and runs the model:

  checkpoint dir = config.json (+ auto_map), model.safetensors (reference state_dict names),
                   tokenizer files, and the two-line shims of INTEGRATION.md §1
  AutoModel.from_pretrained(dir, trust_remote_code=True, torch_dtype=bf16,
                            attn_implementation="sdpa").to("cuda"); model.eval()   (:95-108)
  batch = processor([[processor.build_user_message(text=...)]], mode="generation")  (:211-253, :331)
  model.generate(input_ids, attention_mask, max_new_tokens, audio_temperature, audio_top_p,
                 audio_top_k, audio_repetition_penalty)                              (:336-344)
  processor.decode(outputs)                                                           (:346)

The processor wraps the tokenizer saved in the checkpoint (tests/golden/tokenizer_stub.py, a
character tokenizer with Qwen's special ids) and a tiny HIP codec decoder
(`moss_tts_amd.codec.AudioTokenizerDecoder`) in `processor.audio_tokenizer`: the real codec's
weights are a remote download the reference itself fetches (`processing_moss_tts.py:198-222`).
The generated ids must equal the engine's own generate() with the same sampling parameters and
Philox seed (the model derives the seed from torch's default generator)."""
import json
import os

import pytest

from oracle import codec as K
from tests.test_engine_gpu import case, make_engine

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

SHIMS = {
    "modeling_moss_tts.py": "from moss_tts_amd.modeling_moss_tts import MossTTSDelayModel, "
                            "MossTTSDelayPreTrainedModel  # noqa: F401\n",
    "configuration_moss_tts.py": "from moss_tts_amd.configuration_moss_tts import MossTTSDelayConfig  # noqa: F401\n",
    "processing_moss_tts.py": "from moss_tts_amd.processing_moss_tts import MossTTSDelayProcessor  # noqa: F401\n",
}


def write_checkpoint(path, cfg, W):
    from safetensors.torch import save_file
    from transformers import Qwen3Config
    from moss_tts_amd.configuration_moss_tts import MossTTSDelayConfig
    from tests.golden.tokenizer_stub import build_tokenizer
    lc = Qwen3Config(vocab_size=cfg.vocab, hidden_size=cfg.hidden, intermediate_size=cfg.inter,
                     num_hidden_layers=cfg.layers, num_attention_heads=cfg.n_heads, num_key_value_heads=cfg.n_kv,
                     head_dim=cfg.head_dim, rope_theta=cfg.rope_theta, rms_norm_eps=cfg.eps)
    conf = MossTTSDelayConfig(language_config=lc, n_vq=cfg.n_vq).to_dict()
    conf["architectures"] = ["MossTTSDelayModel"]
    conf["auto_map"] = {"AutoConfig": "configuration_moss_tts.MossTTSDelayConfig",
                        "AutoModel": "modeling_moss_tts.MossTTSDelayModel"}
    with open(os.path.join(path, "config.json"), "w") as f:
        json.dump(conf, f)
    for name, text in SHIMS.items():
        with open(os.path.join(path, name), "w") as f:
            f.write(text)
    save_file({k: torch.from_numpy(v).to(torch.bfloat16).contiguous() for k, v in W.items()},
              os.path.join(path, "model.safetensors"))
    build_tokenizer().save_pretrained(path)


@pytest.fixture(scope="module")
def gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def test_app_loading_sequence(gpu, golden, tmp_path, monkeypatch):
    from transformers import AutoModel, AutoTokenizer
    from moss_tts_amd.codec import AudioTokenizerDecoder, CodecConfig, CodecStageConfig
    from moss_tts_amd.engine import sampling_params
    from moss_tts_amd.processing_moss_tts import MossTTSDelayProcessor
    monkeypatch.setenv("HF_MODULES_CACHE", str(tmp_path / "hf_modules"))  # the remote-code copies
    # the model's engine reserves what make_engine does (same capacity, same launch shapes)
    for k, v in (("MTTS_MAX_BATCH", "4"), ("MTTS_MAX_CTX", "512"), ("MTTS_MAX_PREFILL", "512")):
        monkeypatch.setenv(k, v)
    name = "g_nvq4_bf16"
    g, c, cfg, W = case(golden, name)
    ckpt = tmp_path / "ckpt"
    ckpt.mkdir()
    write_checkpoint(str(ckpt), cfg, W)

    # clis/moss_tts_app.py:95-108
    model = AutoModel.from_pretrained(str(ckpt), trust_remote_code=True, torch_dtype=torch.bfloat16,
                                      attn_implementation="sdpa").to(torch.device("cuda"))
    model.eval()
    assert type(model).__name__ == "MossTTSDelayModel" and type(model).__module__.startswith("moss_tts_amd")
    assert next(model.parameters()).device.type == "cuda"
    kc = K.tiny_codec_cfg(codebook_size=1024)
    codec = AudioTokenizerDecoder(CodecConfig(n_q=kc.n_q, codebook_size=kc.codebook_size, patch=kc.patch,
                                              rope_theta=kc.rope_theta, rms_eps=kc.eps,
                                              stages=[CodecStageConfig(**vars(s)) for s in kc.stages],
                                              max_batch=2, max_frames=256, max_chunk_frames=100), 0)
    codec.init_random(3)
    processor = MossTTSDelayProcessor(tokenizer=AutoTokenizer.from_pretrained(str(ckpt), trust_remote_code=True),
                                      audio_tokenizer=codec,
                                      model_config=model.config)
    processor.audio_tokenizer = processor.audio_tokenizer.to(torch.device("cuda"))  # :110-111

    # clis/moss_tts_app.py:211-253, :331-346
    conversations = [[processor.build_user_message(text="The quick brown fox jumps over the lazy dog again.")]]
    batch = processor(conversations, mode="generation")
    input_ids = batch["input_ids"].to("cuda")
    attention_mask = batch["attention_mask"].to("cuda")
    kw = dict(max_new_tokens=40, audio_temperature=1.7, audio_top_p=0.8, audio_top_k=25, audio_repetition_penalty=1.0)
    torch.manual_seed(1234)
    with torch.no_grad():
        outputs = model.generate(input_ids=input_ids, attention_mask=attention_mask, **kw)
    messages = processor.decode(outputs)
    assert len(outputs) == len(messages) == 1
    # the same generate() on a bare engine: same sampling kwargs, same Philox seed
    torch.manual_seed(1234)
    seed = int(torch.randint(0, 2 ** 62, (1,)).item())
    eng = make_engine(cfg, W, max_ctx=512)
    want = eng.generate_ids(input_ids, attention_mask, kw["max_new_tokens"],
                            sampling_params(text_temperature=1.5, text_top_p=1.0, text_top_k=50,
                                            audio_temperature=1.7, audio_top_p=0.8, audio_top_k=25,
                                            audio_repetition_penalty=1.0, seed=seed)).cpu()
    eng.close()
    start_len, rows = outputs[0]
    T = input_ids.shape[1]
    start = T - int(start_len)
    assert torch.equal(rows.cpu(), want[0, start:])
    # the decoded message carries one waveform per audio segment of the generated codes
    from moss_tts_amd.processing_moss_tts import split_audio_segments
    segs = split_audio_segments(rows[:, 1:].cpu(), cfg.audio_pad_code)
    if messages[0] is not None:
        wavs = messages[0].audio_codes_list
        assert len(wavs) <= len(segs)
        for w in wavs:
            assert w.dtype == torch.float32 and w.dim() == 1
    codec.close()
