"""Processor I/O surface of MossTTSDelay (mirror of the reference
`moss_tts_delay/processing_moss_tts.py`): message templates, chat-template
tokenisation, audio placeholder expansion, delay / de-delay pattern, left
padding, parsing of generate() outputs back into text + audio segments, and the
codec seam (`audio_tokenizer.encode/decode`).

This is host-side integer bookkeeping on small tensors;
the hot path is `MossTTSDelayModel.generate` (modeling_moss_tts.py in this
package).  Names, arguments and error behaviour follow the reference so
`clis/moss_tts_app.py` can use either.
"""
import os
import re
from dataclasses import dataclass
from typing import Any, Dict, List, Optional, Tuple, Union

import torch

try:  # transformers is present wherever the drop-in is used
    from transformers import AutoConfig, AutoModel, AutoTokenizer, BatchFeature
except Exception:  # pragma: no cover
    AutoConfig = AutoModel = AutoTokenizer = None
    BatchFeature = dict

from .configuration_moss_tts import MossTTSDelayConfig

AUDIO_PLACEHOLDER = "<|audio|>"

_USER_TEMPLATE = (
    "<user_inst>\n- Reference(s):\n{reference}\n- Instruction:\n{instruction}\n- Tokens:\n{tokens}\n"
    "- Quality:\n{quality}\n- Sound Event:\n{sound_event}\n- Ambient Sound:\n{ambient_sound}\n"
    "- Language:\n{language}\n- Text:\n{text}\n</user_inst>"
)
USER_MESSAGE_FIELDS = ("text", "reference", "instruction", "tokens", "quality", "sound_event", "ambient_sound",
                       "language")


@dataclass
class Message:
    def to_dict(self) -> Dict[str, Any]:
        raise NotImplementedError


@dataclass
class UserMessage(Message):
    """`processing_moss_tts.py:53-120`: the <user_inst> template; every reference
    (one per speaker, None allowed) becomes "[S<i>]:\\n<|audio|>"."""
    text: Optional[str] = None
    reference: Optional[List[Optional[Union[str, torch.Tensor]]]] = None
    instruction: Optional[str] = None
    tokens: Optional[int] = None
    quality: Optional[str] = None
    sound_event: Optional[str] = None
    ambient_sound: Optional[str] = None
    language: Optional[str] = None

    def __post_init__(self):
        if self.reference is None:
            ref_txt, codes = "None", []
        elif isinstance(self.reference, list):
            present = [(i, r) for i, r in enumerate(self.reference) if r is not None]
            ref_txt = "\n".join(f"[S{i + 1}]:\n{AUDIO_PLACEHOLDER}" for i, _ in present)
            codes = [r for _, r in present]
        else:
            raise TypeError("`reference` should be exactly a list when it is not None.")
        fields = {"reference": ref_txt}
        for k in USER_MESSAGE_FIELDS:
            if k != "reference":
                fields[k] = str(getattr(self, k))
        content = _USER_TEMPLATE
        for k in ("reference", "instruction", "tokens", "quality", "sound_event", "ambient_sound", "language",
                  "text"):
            content = content.replace("{" + k + "}", fields[k])
        self._content = content
        self._audio_codes_list = codes

    def to_dict(self):
        return {"role": "user", "content": self._content, "audio_codes_list": self._audio_codes_list}


@dataclass
class AssistantMessage(Message):
    audio_codes_list: List[Union[str, torch.Tensor]]
    content: str = AUDIO_PLACEHOLDER

    def to_dict(self):
        return {"role": "assistant", "content": self.content, "audio_codes_list": self.audio_codes_list}


# ----------------------------------------------------------------------------
# tokenizer-free statics (exact; pinned by tests/golden fixtures)
# ----------------------------------------------------------------------------
def apply_delay_pattern(codes: torch.Tensor, pad_code: int) -> torch.Tensor:
    """`processing_moss_tts.py:515-525`: [T, n] -> [T+n-1, n], channel i shifted down by i."""
    T, n = codes.shape
    rows = torch.arange(T, device=codes.device)[:, None] + torch.arange(n, device=codes.device)[None, :]
    out = torch.full((T + n - 1, n), pad_code, dtype=codes.dtype, device=codes.device)
    out[rows, torch.arange(n, device=codes.device)[None, :].expand(T, n)] = codes
    return out


def apply_de_delay_pattern(delay_codes: torch.Tensor) -> torch.Tensor:
    """`processing_moss_tts.py:527-537`: inverse of apply_delay_pattern."""
    L, n = delay_codes.shape
    T = L - n + 1
    rows = torch.arange(T, device=delay_codes.device)[:, None] + torch.arange(n, device=delay_codes.device)[None, :]
    return delay_codes[rows, torch.arange(n, device=delay_codes.device)[None, :].expand(T, n)]


def left_pad(seqs: List[torch.Tensor], pad_token_id: int, audio_pad_code: int) -> Dict[str, torch.Tensor]:
    """`processing_moss_tts.py:410-431` (_pad): left pad to the longest sequence; channel 0
    with the text pad id, channels >= 1 with the audio pad code; mask False on pads."""
    L = max(int(s.shape[0]) for s in seqs)
    C = int(seqs[0].shape[1])
    dev = seqs[0].device
    ids = torch.full((len(seqs), L, C), audio_pad_code, dtype=torch.long, device=dev)
    ids[:, :, 0] = pad_token_id
    mask = torch.zeros(len(seqs), L, dtype=torch.bool, device=dev)
    for b, s in enumerate(seqs):
        n = int(s.shape[0])
        ids[b, L - n:] = s.to(torch.long)
        mask[b, L - n:] = True
    return {"input_ids": ids, "attention_mask": mask}


def split_audio_segments(audio_codes: torch.Tensor, pad_code: int, delay: bool = True) -> List[torch.Tensor]:
    """`processing_moss_tts.py:668-685`: de-delay, drop all-pad rows, cut into maximal runs
    of consecutive frames.  (The reference hands break *indices* to torch.split, which
    expects sizes, and raises for more than one segment -- see DESIGN.md; this returns
    the intended runs.)  delay=False: MossTTSLocal's undelayed codes
    (`moss_tts_local/processing_moss_tts.py:668-690`)."""
    a = apply_de_delay_pattern(audio_codes) if delay else audio_codes
    non_pad = ~(a == pad_code).all(dim=1)
    if not bool(non_pad.any()):
        return []
    idx = torch.nonzero(non_pad).squeeze(1)
    breaks = (torch.nonzero(idx[1:] != idx[:-1] + 1).squeeze(1) + 1).tolist()
    bounds = [0] + breaks + [int(idx.numel())]
    return [a[idx[bounds[i]:bounds[i + 1]]] for i in range(len(bounds) - 1)]


def replace_audio_placeholders(content: str, lengths: List[int], n_vq: int, gen_slot_token: str,
                               delay_slot_token: str, audio_start_token: str, audio_end_token: str,
                               delay: bool = True) -> str:
    """`processing_moss_tts.py:433-471` (delay=False: no delay slots, MossTTSLocal :465)."""
    if n_vq < 1:
        raise ValueError(f"n_vq must be >= 1, got {n_vq}")
    n_ph = content.count(AUDIO_PLACEHOLDER)
    if n_ph != len(lengths):
        raise ValueError(f"Number of {AUDIO_PLACEHOLDER} ({n_ph}) does not match lengths ({len(lengths)})")
    it = iter(lengths)

    def block(_m):
        n = next(it)
        if n < 0:
            raise ValueError(f"length must be >= 0, got {n}")
        if n == 0:
            return audio_start_token + audio_end_token
        return audio_start_token + gen_slot_token * n + delay_slot_token * ((n_vq - 1) if delay else 0) + audio_end_token

    return re.sub(re.escape(AUDIO_PLACEHOLDER), block, content)


def merge_consecutive_audio_placeholders(content: str, audio_codes_list: List[torch.Tensor]):
    """`processing_moss_tts.py:473-513`: placeholders separated only by whitespace merge and
    their codes are concatenated along time."""
    ms = list(re.finditer(re.escape(AUDIO_PLACEHOLDER), content))
    if len(ms) <= 1:
        return content, audio_codes_list
    if len(ms) != len(audio_codes_list):
        raise ValueError("Audio placeholders do not match the provided audio codes list.")
    parts, codes, last, i = [], [], 0, 0
    while i < len(ms):
        j = i
        while j + 1 < len(ms) and content[ms[j].end():ms[j + 1].start()].strip() == "":
            j += 1
        parts += [content[last:ms[i].start()], AUDIO_PLACEHOLDER]
        last = ms[j].end()
        codes.append(audio_codes_list[i] if j == i else torch.cat(audio_codes_list[i:j + 1], 0))
        i = j + 1
    parts.append(content[last:])
    return "".join(parts), codes


def loudness_normalize(wav: torch.Tensor, target_dbfs: float = -20, gain_range=(-3.0, 3.0)) -> torch.Tensor:
    """`processing_moss_tts.py:735-748`."""
    wav = wav.to(torch.float32)
    if wav.numel() == 0:
        return wav
    cur = 10.0 * torch.log10(torch.mean(wav ** 2) + 1e-9)
    gain = max(gain_range[0], min(float(target_dbfs - cur), gain_range[1]))
    return wav * (10.0 ** (gain / 20.0))


# ----------------------------------------------------------------------------
class MossTTSDelayProcessor:
    """Mirror of `MossTTSDelayProcessor` (`processing_moss_tts.py:148-930`).  delay_pattern
    False is the MossTTSLocal processor (moss_tts_local/processing_moss_tts.py)."""
    delay_pattern = True

    def __init__(self, tokenizer, audio_tokenizer: Any = None, model_config: Optional[MossTTSDelayConfig] = None,
                 **kwargs):
        self.tokenizer = tokenizer
        self.audio_tokenizer = audio_tokenizer
        self.model_config = model_config if model_config is not None else MossTTSDelayConfig()
        self.imstart_token_id = tokenizer.convert_tokens_to_ids("<|im_start|>")
        self.imend_token_id = tokenizer.convert_tokens_to_ids("<|im_end|>")
        self.newline_token_id = 198

        def tok(i):
            t = tokenizer.convert_ids_to_tokens(int(i))
            return (t[0] if t else "") if isinstance(t, list) else t

        mc = self.model_config
        self.audio_user_slot_token = tok(mc.audio_user_slot_token_id)
        self.audio_assistant_gen_slot_token = tok(mc.audio_assistant_gen_slot_token_id)
        self.audio_assistant_delay_slot_token = tok(mc.audio_assistant_delay_slot_token_id)
        self.audio_start_token = tok(mc.audio_start_token_id)
        self.audio_end_token = tok(mc.audio_end_token_id)

    @classmethod
    def from_pretrained(cls, pretrained_model_name_or_path, *args, **kwargs):
        """`processing_moss_tts.py:193-229`; `codec_path` names the audio tokenizer."""
        trust = kwargs.pop("trust_remote_code", True)
        kwargs.pop("_from_auto", None)
        codec = kwargs.pop("codec_path", "OpenMOSS-Team/MOSS-Audio-Tokenizer")
        cfg = AutoConfig.from_pretrained(pretrained_model_name_or_path, *args, trust_remote_code=trust, **kwargs)
        tk = AutoTokenizer.from_pretrained(pretrained_model_name_or_path, *args, trust_remote_code=trust, **kwargs)
        at = AutoModel.from_pretrained(codec, trust_remote_code=trust, **kwargs)
        return cls(tokenizer=tk, audio_tokenizer=at, model_config=cfg, **kwargs)

    # ---- message helpers ------------------------------------------------------
    @staticmethod
    def build_user_message(text=None, reference=None, instruction=None, tokens=None, quality=None, sound_event=None,
                           ambient_sound=None, language=None) -> Dict:
        if reference is not None and not isinstance(reference, list):
            reference = [reference]
        return UserMessage(text=text, reference=reference, instruction=instruction, tokens=tokens, quality=quality,
                           sound_event=sound_event, ambient_sound=ambient_sound, language=language).to_dict()

    @staticmethod
    def build_assistant_message(audio_codes_list, content: str = AUDIO_PLACEHOLDER) -> Dict:
        return AssistantMessage(audio_codes_list=audio_codes_list, content=content).to_dict()

    def _normalize_message(self, message) -> Dict:
        if isinstance(message, Message):
            return message.to_dict()
        if not isinstance(message, dict):
            raise TypeError("Each message must be a Message or dict.")
        if "role" not in message:
            raise ValueError("Message dict must include a 'role' field.")
        if "content" in message and "audio_codes_list" in message:
            return message
        if message["role"] == "user":
            return self.build_user_message(**{k: message.get(k) for k in USER_MESSAGE_FIELDS})
        if message["role"] == "assistant":
            return self.build_assistant_message(message.get("audio_codes_list", []),
                                                message.get("content", AUDIO_PLACEHOLDER))
        raise ValueError(f"Unsupported role: {message['role']}")

    apply_delay_pattern = staticmethod(apply_delay_pattern)
    apply_de_delay_pattern = staticmethod(apply_de_delay_pattern)

    def _pad(self, input_ids_list: List[torch.Tensor]):
        return left_pad(input_ids_list, self.model_config.pad_token_id, self.model_config.audio_pad_code)

    # ---- encode ---------------------------------------------------------------
    def _get_unified_codes(self, role: str, content: str, audio_codes_list: List[torch.Tensor],
                           truncation: bool) -> torch.Tensor:
        """`processing_moss_tts.py:539-641`: tokenise the templated text and lay the delayed
        audio codes beside the slot tokens; [T, 1+n_vq]."""
        mc = self.model_config
        if role == "user":
            gen_tok = delay_tok = self.audio_user_slot_token
            truncation = False
        else:
            gen_tok, delay_tok = self.audio_assistant_gen_slot_token, self.audio_assistant_delay_slot_token
        n_vq = audio_codes_list[0].shape[1] if audio_codes_list else mc.n_vq
        if len(audio_codes_list) > 1 and AUDIO_PLACEHOLDER in content:
            content, audio_codes_list = merge_consecutive_audio_placeholders(content, audio_codes_list)
        content = replace_audio_placeholders(content, [len(a) for a in audio_codes_list], n_vq, gen_tok, delay_tok,
                                             self.audio_start_token, self.audio_end_token, self.delay_pattern)
        dev = audio_codes_list[0].device if audio_codes_list else None
        text = torch.tensor(self.tokenizer.encode(content), device=dev)
        starts = torch.where(text == mc.audio_start_token_id)[0]
        ends = torch.where(text == mc.audio_end_token_id)[0]
        if len(starts) != len(audio_codes_list) or len(ends) != len(audio_codes_list):
            raise ValueError("Audio placeholders do not match the provided audio codes list.")
        if not self.delay_pattern and len(audio_codes_list) > 1:
            raise AssertionError("MossTTSLocal takes at most one audio block per message")
        if not audio_codes_list:
            audio = torch.full((len(text), n_vq), mc.audio_pad_code, device=text.device, dtype=text.dtype)
        else:
            pieces, prefix = [], 0
            for s, e, codes in zip(starts.tolist(), ends.tolist(), audio_codes_list):
                pieces.append(torch.full((s - prefix + 1, n_vq), mc.audio_pad_code, device=codes.device,
                                         dtype=codes.dtype))
                pieces.append(apply_delay_pattern(codes, mc.audio_pad_code) if self.delay_pattern else codes)
                prefix = e
            if truncation and not self.delay_pattern:
                raise RuntimeError("Truncation generation is not supported at present")
            if truncation:
                pieces[-1] = pieces[-1][: -(n_vq - 1), :]
            else:
                pieces.append(torch.full((len(text) - int(ends[-1]), n_vq), mc.audio_pad_code,
                                         device=audio_codes_list[0].device, dtype=audio_codes_list[0].dtype))
            audio = torch.cat(pieces)
        if text.shape[0] != audio.shape[0]:
            text = text[: audio.shape[0]]
        return torch.cat([text.unsqueeze(1), audio], dim=1)

    def __call__(self, *args, **kwargs):
        """`processing_moss_tts.py:231-354`."""
        conversations = args[0] if args else kwargs.pop("conversations")
        mode = kwargs.pop("mode", "generation")
        apply_chat_template = kwargs.pop("apply_chat_template", True)
        n_vq = kwargs.pop("n_vq", None)
        for k in ("return_tensors", "padding", "truncation"):
            kwargs.pop(k, None)
        if mode not in {"generation", "continuation"}:
            raise RuntimeError
        if isinstance(conversations, (Message, dict)):
            conversations = [conversations]
        truncation = mode == "continuation"
        seqs = []
        for conv in conversations:
            if isinstance(conv, (Message, dict)):
                conv = [conv]
            conv = [self._normalize_message(m) for m in conv]
            if (mode == "generation") ^ (len(conv) % 2 != 0):
                raise ValueError
            if (mode == "generation") ^ (conv[-1]["role"] == "user"):
                raise ValueError
            unified = []
            for i, msg in enumerate(conv):
                content = msg["content"]
                if apply_chat_template:
                    agp = mode == "generation" and i == len(conv) - 1
                    try:
                        content = self.tokenizer.apply_chat_template([{"role": msg["role"], "content": msg["content"]}],
                                                                     add_generation_prompt=agp, tokenize=False)
                    except TypeError:
                        content = self.tokenizer.apply_chat_template([{"role": msg["role"], "content": msg["content"]}],
                                                                     add_generation_prompt=agp)
                content = str(content)
                items = msg.get("audio_codes_list", [])
                codes: List[torch.Tensor] = []
                if items:
                    enc: List[Optional[torch.Tensor]] = [None] * len(items)
                    paths, pos = [], []
                    for j, it in enumerate(items):
                        if isinstance(it, torch.Tensor):
                            if n_vq is not None and it.shape[1] != n_vq:
                                raise RuntimeError("audio_codes's n_vq is not equal to the parameter `n_vq`.")
                            enc[j] = it
                        elif isinstance(it, (str, os.PathLike)):
                            paths.append(str(it))
                            pos.append(j)
                        else:
                            raise TypeError("Each audio item must be a torch.Tensor of codes or a path-like string.")
                    if paths:
                        got = self.encode_audios_from_path(paths, n_vq)
                        if len(got) != len(paths):
                            raise RuntimeError("encode_audios_from_path returned an unexpected number of items.")
                        for p_, c_ in zip(pos, got):
                            enc[p_] = c_
                    codes = list(enc)
                unified.append(self._get_unified_codes(msg["role"], content, codes, truncation))
            u = torch.cat(unified)
            if mode == "generation" and not self.delay_pattern:
                # MossTTSLocal prompts end on an audio_start row (moss_tts_local/processing_moss_tts.py:351-356)
                row = torch.full((1, u.shape[1]), self.model_config.audio_pad_code, dtype=u.dtype, device=u.device)
                row[0, 0] = self.model_config.audio_start_token_id
                u = torch.cat([u, row])
            seqs.append(u)
        return BatchFeature(data=self._pad(seqs))

    # ---- decode ---------------------------------------------------------------
    def _parse_text_codes(self, start_length, text_codes):
        """`processing_moss_tts.py:643-666`."""
        text = self.tokenizer.decode(text_codes)
        prefix = self.tokenizer.decode(text_codes[:start_length])
        text = text[len(prefix):]
        pat = re.compile(rf"(?:{self.audio_start_token})?(?:{self.audio_assistant_gen_slot_token})*"
                         rf"(?:{self.audio_assistant_delay_slot_token})*{self.audio_end_token}")
        return pat.sub(lambda m: AUDIO_PLACEHOLDER if self.audio_assistant_gen_slot_token in m.group(0) else "", text)

    def _parse_audio_codes(self, start_length, audio_codes):
        """`processing_moss_tts.py:668-709`: segments -> one batched codec decode -> trim the
        first segment by the start_length ratio."""
        segs = split_audio_segments(audio_codes, self.model_config.audio_pad_code, self.delay_pattern)
        if not segs:
            return []
        wavs = self.decode_audio_codes(segs)
        if start_length > 0 and wavs:
            n0 = segs[0].shape[0]
            if n0 > 0:
                r = max(0.0, min(float(start_length) / float(n0), 1.0))
                if r >= 1.0:
                    wavs = wavs[1:]
                elif r > 0.0:
                    wavs[0] = wavs[0][..., int(wavs[0].shape[-1] * r):]
        return wavs

    def decode(self, output: List[Tuple[int, torch.Tensor]]):
        """`processing_moss_tts.py:711-733`."""
        msgs = []
        for start_length, gen in output:
            content = self._parse_text_codes(start_length, gen[:, 0])
            audio = self._parse_audio_codes(start_length, gen[:, 1:])
            msgs.append(None if content == "" else AssistantMessage(content=content, audio_codes_list=audio))
        return msgs

    # ---- codec seam -----------------------------------------------------------
    def _get_audio_tokenizer_device(self) -> torch.device:
        at = self.audio_tokenizer
        if at is None:
            return torch.device("cpu")
        d = getattr(at, "device", None)
        if isinstance(d, torch.device):
            return d
        try:
            return next(at.parameters()).device
        except (StopIteration, AttributeError):
            return torch.device("cpu")

    def encode_audios_from_wav(self, wav_list, sampling_rate: int, n_vq: Optional[int] = None):
        """`processing_moss_tts.py:778-852` (resampling needs torchaudio, as in the reference)."""
        if self.audio_tokenizer is None:
            raise RuntimeError("audio_tokenizer is not set on processor.")
        if isinstance(wav_list, torch.Tensor):
            wav_list = [wav_list]
        dev = self._get_audio_tokenizer_device()
        ws = []
        for w in wav_list:
            if w.shape[0] > 1:
                w = torch.mean(w, dim=0, keepdim=True)
            if sampling_rate != self.model_config.sampling_rate:
                import torchaudio
                w = torchaudio.functional.resample(w, sampling_rate, self.model_config.sampling_rate)
            ws.append(loudness_normalize(w.to(dev).squeeze(0)))
        at = self.audio_tokenizer
        if hasattr(at, "batch_encode"):
            enc = at.batch_encode(ws, num_quantizers=n_vq)
        else:
            T = max(int(w.shape[-1]) for w in ws)
            x = torch.zeros(len(ws), 1, T, device=dev)
            m = torch.zeros(len(ws), T, device=dev, dtype=torch.bool)
            for i, w in enumerate(ws):
                x[i, 0, :w.shape[-1]] = w
                m[i, :w.shape[-1]] = True
            enc = at.encode(x, padding_mask=m, num_quantizers=n_vq, return_dict=True)
        codes, lens = enc.audio_codes, enc.audio_codes_lengths
        if codes is None or lens is None:
            raise RuntimeError("audio_tokenizer.encode() returned empty outputs (audio_codes/audio_codes_lengths).")
        return [codes[:, i, :int(lens[i])].transpose(0, 1).contiguous().to(torch.long).cpu()
                for i in range(int(codes.shape[1]))]

    def encode_audios_from_path(self, wav_path_list, n_vq: Optional[int] = None):
        import torchaudio
        if isinstance(wav_path_list, str):
            wav_path_list = [wav_path_list]
        if not wav_path_list:
            raise ValueError("Empty wav_path_list")
        sr_t = int(self.model_config.sampling_rate)
        wavs = []
        for p in wav_path_list:
            w, sr = torchaudio.load(p)
            if int(sr) != sr_t:
                w = torchaudio.functional.resample(w, int(sr), sr_t)
            wavs.append(w)
        return self.encode_audios_from_wav(wavs, sr_t, n_vq)

    def decode_audio_codes(self, audio_tokens_list):
        """`processing_moss_tts.py:880-930`: [(T_i, NQ)] -> padded (NQ, B, T) + mask ->
        audio_tokenizer.decode(..., chunk_duration=8) -> list of fp32 1-D waveforms."""
        if self.audio_tokenizer is None:
            raise RuntimeError("audio_tokenizer is not set on processor.")
        if isinstance(audio_tokens_list, torch.Tensor):
            audio_tokens_list = [audio_tokens_list]
        if not audio_tokens_list:
            return []
        dev = self._get_audio_tokenizer_device()
        cl = [c.transpose(0, 1).contiguous().to(device=dev, dtype=torch.long) for c in audio_tokens_list]
        nq, T = int(cl[0].shape[0]), max(int(c.shape[1]) for c in cl)
        codes = torch.zeros(nq, len(cl), T, device=dev, dtype=torch.long)
        mask = torch.zeros(len(cl), T, device=dev, dtype=torch.bool)
        for i, c in enumerate(cl):
            codes[:, i, :c.shape[1]] = c
            mask[i, :c.shape[1]] = True
        dec = self.audio_tokenizer.decode(codes, padding_mask=mask, return_dict=True, chunk_duration=8)
        if dec.audio is None or dec.audio_lengths is None:
            raise RuntimeError("audio_tokenizer.decode() returned empty outputs (audio/audio_lengths).")
        return [dec.audio[i, 0, :int(dec.audio_lengths[i])].contiguous().to(torch.float32).cpu()
                for i in range(int(dec.audio.shape[0]))]
