"""Whisper tokenizer: byte-level BPE (GPT-2 / tiktoken ranks) plus Whisper's special-token block.

Special-token ids follow from the vocabulary size alone (public model constants): English-only
models (51864 tokens) start at eot = 50256, multilingual ones (>= 51865) shift by one and carry
n_vocab - 51766 language tokens (99; 100 for large-v3) between <|startoftranscript|> and
<|translate|>. Timestamp tokens <|0.00|> .. <|30.00|> follow <|notimestamps|>.

Vocab sources: the token byte strings stored in whisper.cpp's ggml model files (rank order), a
Hugging Face vocab.json (GPT-2 unicode-mapped pieces), or a synthetic byte vocabulary for tests.
Encoding (used for initial prompts) is rank-based byte-pair merging over GPT-2 pre-tokens.
"""
from __future__ import annotations

import json
import os

LANGUAGES = (
    "en zh de es ru ko fr ja pt tr pl ca nl ar sv it id hi fi vi he uk el ms cs ro da hu ta no th ur hr bg lt la "
    "mi ml cy sk te fa lv bn sr az sl kn et mk br eu is hy ne mn bs kk sq sw gl mr pa si km sn yo so af oc ka be "
    "tg sd gu am yi lo uz fo ht ps tk nn mt sa lb my bo tl mg as tt haw ln ha ba jw su yue").split()

_PRETOK = r"""'s|'t|'re|'ve|'m|'ll|'d| ?\p{L}+| ?\p{N}+| ?[^\s\p{L}\p{N}]+|\s+(?!\S)|\s+"""


def _bytes_to_unicode() -> dict[int, str]:
    bs = list(range(ord("!"), ord("~") + 1)) + list(range(ord("¡"), ord("¬") + 1)) + list(range(ord("®"), ord("ÿ") + 1))
    cs = bs[:]
    n = 0
    for b in range(256):
        if b not in bs:
            bs.append(b)
            cs.append(256 + n)
            n += 1
    return dict(zip(bs, (chr(c) for c in cs)))


class WhisperTokenizer:
    def __init__(self, pieces: list[bytes], n_vocab: int):
        self.n_vocab = n_vocab
        self.multilingual = n_vocab >= 51865
        n_lang = n_vocab - 51765 - int(self.multilingual)
        self.eot = 50256 + int(self.multilingual)
        self.sot = self.eot + 1
        self.lang0 = self.sot + 1
        self.n_lang = max(0, n_lang)
        self.translate = self.lang0 + self.n_lang
        self.transcribe = self.translate + 1
        self.solm = self.transcribe + 1
        self.prev = self.solm + 1
        self.nosp = self.prev + 1
        self.no_timestamps = self.nosp + 1
        self.timestamp_begin = self.no_timestamps + 1
        self.pieces = list(pieces[: self.eot])
        self.rank = {p: i for i, p in enumerate(self.pieces)}
        import regex
        self._pat = regex.compile(_PRETOK)

    # ------------------------------------------------------------------ construction
    @classmethod
    def from_ggml_vocab(cls, pieces: list[bytes], n_vocab: int) -> "WhisperTokenizer":
        return cls(pieces, n_vocab)

    @classmethod
    def from_hf_dir(cls, d: str, n_vocab: int) -> "WhisperTokenizer":
        """vocab.json (HF), else tokenizer.json's BPE vocab, else a CTranslate2 vocabulary.json / .txt
        (faster-whisper model directories): byte-level unicode token strings -> ids."""
        if os.path.isfile(os.path.join(d, "vocab.json")):
            with open(os.path.join(d, "vocab.json"), encoding="utf-8") as f:
                vocab = json.load(f)
        elif os.path.isfile(os.path.join(d, "tokenizer.json")):
            with open(os.path.join(d, "tokenizer.json"), encoding="utf-8") as f:
                tj = json.load(f)
            vocab = dict(tj["model"]["vocab"])
            for t in tj.get("added_tokens", []):
                vocab[t["content"]] = t["id"]
        elif os.path.isfile(os.path.join(d, "vocabulary.json")):
            with open(os.path.join(d, "vocabulary.json"), encoding="utf-8") as f:
                vocab = {t: i for i, t in enumerate(json.load(f))}
        else:
            with open(os.path.join(d, "vocabulary.txt"), encoding="utf-8") as f:
                vocab = {t.rstrip("\n"): i for i, t in enumerate(f)}
        dec = {c: b for b, c in _bytes_to_unicode().items()}
        pieces: list[bytes] = [b""] * (max(vocab.values()) + 1)
        for s, i in vocab.items():
            try:
                pieces[i] = bytes(dec[c] for c in s)
            except KeyError:
                pieces[i] = s.encode()
        return cls(pieces, n_vocab)

    @classmethod
    def synthetic(cls, n_vocab: int = 51865) -> "WhisperTokenizer":
        pieces = [bytes([b]) for b in range(256)]
        pieces += [b"<unused%d>" % i for i in range(50256 + int(n_vocab >= 51865) - 256)]
        return cls(pieces, n_vocab)

    # ------------------------------------------------------------------ special tokens
    def language_token(self, lang: str) -> int:
        lang = (lang or "").lower()
        if lang not in LANGUAGES[: self.n_lang]:
            raise ValueError(f"unsupported language {lang!r}")
        return self.lang0 + LANGUAGES.index(lang)

    def language_of(self, tok: int) -> str:
        return LANGUAGES[tok - self.lang0]

    def sot_sequence(self, language: str | None, task: str = "transcribe") -> list[int]:
        seq = [self.sot]
        if self.multilingual:
            seq.append(self.language_token(language or "en"))
            seq.append(self.translate if task == "translate" else self.transcribe)
        return seq

    def is_timestamp(self, t: int) -> bool:
        return t >= self.timestamp_begin

    # ------------------------------------------------------------------ text
    def decode_bytes(self, ids) -> bytes:
        return b"".join(self.pieces[t] for t in ids if 0 <= t < len(self.pieces))

    def decode(self, ids) -> str:
        return self.decode_bytes(ids).decode("utf-8", errors="replace")

    def _bpe(self, word: bytes) -> list[int]:
        if word in self.rank:
            return [self.rank[word]]
        parts = [bytes([b]) for b in word]
        while len(parts) > 1:
            best, bi = None, -1
            for i in range(len(parts) - 1):
                r = self.rank.get(parts[i] + parts[i + 1])
                if r is not None and (best is None or r < best):
                    best, bi = r, i
            if bi < 0:
                break
            parts[bi:bi + 2] = [parts[bi] + parts[bi + 1]]
        return [self.rank.get(p, self.rank.get(p[:1], 0)) for p in parts]

    def encode(self, text: str) -> list[int]:
        out: list[int] = []
        for m in self._pat.findall(text):
            out.extend(self._bpe(m.encode("utf-8")))
        return out
