"""A self-contained character-level tokenizer with the Qwen special-token ids MOSS-TTS uses
(no network, no checkpoint): printable ASCII one id per character, "\\n" at 198 (the
processors' hard-coded newline id), the audio / chat specials at their config ids, and a
Qwen-style chat template.  Used to run the reference processors (fixture generation) and
this repo's processors (tests) on identical tokenisation."""

SPECIALS = {
    151643: "<|endoftext|>", 151644: "<|im_start|>", 151645: "<|im_end|>", 151652: "<|audio_start|>",
    151653: "<|audio_end|>", 151654: "<|audio_user_slot|>", 151655: "<|unused_155|>", 151656: "<|audio_gen_slot|>",
    151662: "<|audio_delay_slot|>",
}
CHAT_TEMPLATE = ("{% for message in messages %}<|im_start|>{{ message['role'] }}\n{{ message['content'] }}<|im_end|>\n"
                 "{% endfor %}{% if add_generation_prompt %}<|im_start|>assistant\n{% endif %}")
VOCAB_SIZE = 151936


def build_tokenizer():
    from tokenizers import Regex, Tokenizer, decoders, models, pre_tokenizers
    from transformers import PreTrainedTokenizerFast
    vocab = {}
    nid = 0
    for ch in [chr(c) for c in range(32, 127)]:
        if nid == 198:
            nid += 1
        vocab[ch] = nid
        nid += 1
    vocab["\n"] = 198
    vocab["<unk>"] = 300
    for i, s in SPECIALS.items():
        vocab[s] = i
    used = set(vocab.values())
    for i in range(VOCAB_SIZE):
        if i not in used:
            vocab[f"<u{i}>"] = i
    tok = Tokenizer(models.WordLevel(vocab=vocab, unk_token="<unk>"))
    tok.pre_tokenizer = pre_tokenizers.Split(Regex("."), behavior="isolated")
    tok.decoder = decoders.Fuse()
    t = PreTrainedTokenizerFast(tokenizer_object=tok, unk_token="<unk>", chat_template=CHAT_TEMPLATE)
    t.add_special_tokens({"additional_special_tokens": list(SPECIALS.values())})
    return t
