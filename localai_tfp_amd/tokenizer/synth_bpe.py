"""A synthetic byte-level BPE vocabulary the size and shape of Llama-3's (128,000 merged/byte tokens + 256
special tokens = 128,256 ids), for benchmarks and tests that run without network access to a real
tokenizer.json.

The vocabulary is GGUF tokenizer metadata (``tokenizer.ggml.model = "gpt2"``, ``pre = "llama-bpe"``,
tokens / token_type / merges, the Llama-3 special ids and chat template), so it is served by the same
code path as a real Llama-3 GGUF (tokenizer/gguf.py :class:`BPETokenizer`, HF ``tokenizers`` BPE with the
Llama-3 pre-tokenizer regex). What that exercises, and a byte tokenizer does not: a 128k-entry vocabulary
in the BPE merge loop, multi-byte tokens in incremental detokenisation (UTF-8 pieces split across tokens),
stop-string matching over multi-character pieces, and a 128,256-wide logits row in the sampler.

Construction: the 256 GPT-2 byte symbols, then merges that build, left to right, (a) the words of the load
generator's prompt vocabulary and common English words, with and without the leading-space marker, and
(b) pseudo-words drawn from a syllable grammar in a fixed order, until 128,000 tokens exist. Multi-byte
UTF-8 characters (accented Latin, CJK, emoji) get merges too, so decoding single tokens can end inside a
character.
"""
from __future__ import annotations

import functools

import numpy as np

N_REGULAR = 128000
N_SPECIAL = 256
LLAMA3_SPECIALS = {0: "<|begin_of_text|>", 1: "<|end_of_text|>", 6: "<|start_header_id|>",
                   7: "<|end_header_id|>", 8: "<|eom_id|>", 9: "<|eot_id|>", 10: "<|python_tag|>"}
LLAMA3_CHAT_TEMPLATE = (
    "{% set loop_messages = messages %}{% for message in loop_messages %}"
    "{% set content = '<|start_header_id|>' + message['role'] + '<|end_header_id|>\n\n'+ message['content'] | trim"
    " + '<|eot_id|>' %}{% if loop.index0 == 0 %}{% set content = bos_token + content %}{% endif %}"
    "{{ content }}{% endfor %}{% if add_generation_prompt %}{{ '<|start_header_id|>assistant<|end_header_id|>\n\n' }}"
    "{% endif %}")

COMMON = ("the of and to in is was for that on with as by at from his her this which or an be are not have "
          "had it but were they one all there their we has when more been who would will can if no into "
          "other so what some up out time only new about them these may could first than then its two also "
          "model serves tokens fast MI355X paged attention hipGraph decode kernels every request batch xGMI "
          "GPU memory server user assistant system token output input layer weight matrix vector kernel "
          "performance latency throughput hello world question answer Python function return value").split()
UNICODE_WORDS = ["café", "naïve", "über", "señor", "Straße", "日本語", "中文", "한국어", "Ελληνικά", "русский",
                 "😀", "🚀", "✓", "→", "€", "—", "…"]


def _bytes_to_unicode() -> dict[int, str]:
    bs = list(range(ord("!"), ord("~") + 1)) + list(range(ord("¡"), ord("¬") + 1)) + list(range(ord("®"), ord("ÿ") + 1))
    cs = bs[:]
    n = 0
    for b in range(256):
        if b not in bs:
            bs.append(b)
            cs.append(256 + n)
            n += 1
    return {b: chr(c) for b, c in zip(bs, cs)}


def _pseudo_words(rng: np.random.Generator):
    onset = ["", "b", "c", "d", "f", "g", "h", "j", "k", "l", "m", "n", "p", "r", "s", "t", "v", "w", "z",
             "br", "ch", "cl", "cr", "dr", "fl", "gr", "pl", "pr", "sh", "st", "th", "tr", "qu", "sp", "str"]
    nucleus = ["a", "e", "i", "o", "u", "ai", "ea", "ee", "ie", "oo", "ou", "y"]
    coda = ["", "", "n", "r", "s", "t", "l", "m", "nd", "ng", "ck", "st", "rt", "ll", "ss", "x"]
    while True:
        k = int(rng.integers(1, 5))
        w = "".join(onset[rng.integers(len(onset))] + nucleus[rng.integers(len(nucleus))] +
                    coda[rng.integers(len(coda))] for _ in range(k))
        r = float(rng.random())
        if r < 0.15:
            w = w.capitalize()
        elif r < 0.18:
            w = w.upper()
        yield w


@functools.lru_cache(maxsize=2)
def llama3_like_metadata(seed: int = 0) -> dict:
    """GGUF ``tokenizer.*`` metadata of the synthetic vocabulary (cached: building takes ~1 s)."""
    b2u = _bytes_to_unicode()
    tokens: list[str] = [b2u[b] for b in range(256)]
    have = set(tokens)
    merges: list[str] = []

    def add_word(word: str):
        syms = [b2u[b] for b in word.encode("utf-8")]
        cur = syms[0]
        for s in syms[1:]:
            nxt = cur + s
            if nxt not in have:
                if len(tokens) >= N_REGULAR:
                    return
                have.add(nxt)
                tokens.append(nxt)
                merges.append(f"{cur} {s}")
            cur = nxt

    for w in COMMON + UNICODE_WORDS:
        add_word(" " + w)
        add_word(w)
    for d in range(1000):  # numbers: the Llama-3 regex splits digit runs into groups of <= 3
        add_word(str(d))
    for p in ["\n", "\n\n", "  ", "    ", ".", ",", "!", "?", ":", ";", "(", ")", "{", "}", "[", "]", "\"", "'s",
              " (", " \"", "...", "--", "->", "==", "!=", "<=", ">="]:
        add_word(p)
    gen = _pseudo_words(np.random.default_rng(seed))
    while len(tokens) < N_REGULAR:
        w = next(gen)
        add_word(" " + w)
        if len(tokens) < N_REGULAR and len(w) > 3:
            add_word(w)
    names = [LLAMA3_SPECIALS.get(i, f"<|reserved_special_token_{i}|>") for i in range(N_SPECIAL)]
    tokens += names
    ttype = np.ones(len(tokens), np.int32)
    ttype[N_REGULAR:] = 3  # control
    return {
        "tokenizer.ggml.model": "gpt2",
        "tokenizer.ggml.pre": "llama-bpe",
        "tokenizer.ggml.tokens": tokens,
        "tokenizer.ggml.token_type": ttype.tolist(),
        "tokenizer.ggml.merges": merges,
        "tokenizer.ggml.bos_token_id": N_REGULAR + 0,
        "tokenizer.ggml.eos_token_id": N_REGULAR + 9,
        "tokenizer.ggml.add_bos_token": True,
        "tokenizer.chat_template": LLAMA3_CHAT_TEMPLATE,
    }


def llama3_like_tokenizer(seed: int = 0):
    """BPETokenizer over the synthetic Llama-3-sized vocabulary (tokenizer/gguf.py)."""
    from .gguf import BPETokenizer
    return BPETokenizer(llama3_like_metadata(seed))
