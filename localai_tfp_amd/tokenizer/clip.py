"""CLIP text tokenizer (byte-level BPE with `</w>` word ends) and a T5 SentencePiece wrapper, for the
diffusion text encoders. Files: Hugging Face `vocab.json` + `merges.txt` (CLIP), `spiece.model`
(T5, via the sentencepiece library). `synthetic()` builds a byte vocabulary for random-init tests.
"""
from __future__ import annotations

import html
import json
import os
import re


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


_PAT = r"""<\|startoftext\|>|<\|endoftext\|>|'s|'t|'re|'ve|'m|'ll|'d|[\p{L}]+|[\p{N}]|[^\s\p{L}\p{N}]+"""


class CLIPTokenizer:
    def __init__(self, encoder: dict[str, int], merges: list[tuple[str, str]], max_len: int = 77,
                 pad_token: str | None = None):
        import regex
        self.encoder = encoder
        self.ranks = {m: i for i, m in enumerate(merges)}
        self.b2u = _bytes_to_unicode()
        self.bos = encoder.get("<|startoftext|>", 49406)
        self.eos = encoder.get("<|endoftext|>", 49407)
        self.pad = encoder.get(pad_token, self.eos) if pad_token else self.eos
        self.max_len = max_len
        self.pat = regex.compile(_PAT, regex.IGNORECASE)
        self.cache: dict[str, list[int]] = {}

    @classmethod
    def from_dir(cls, d: str, pad_token: str | None = None) -> "CLIPTokenizer":
        with open(os.path.join(d, "vocab.json"), encoding="utf-8") as f:
            enc = json.load(f)
        merges = []
        with open(os.path.join(d, "merges.txt"), encoding="utf-8") as f:
            for line in f:
                p = line.split()
                if len(p) == 2 and not line.startswith("#version"):
                    merges.append((p[0], p[1]))
        return cls(enc, merges, pad_token=pad_token)

    @classmethod
    def synthetic(cls, vocab: int = 49408, pad_token: str | None = None) -> "CLIPTokenizer":
        b2u = _bytes_to_unicode()
        enc = {}
        for b in range(256):
            enc[b2u[b]] = len(enc)
        for b in range(256):
            enc[b2u[b] + "</w>"] = len(enc)
        enc["<|startoftext|>"] = vocab - 2
        enc["<|endoftext|>"] = vocab - 1
        return cls(enc, [], pad_token=pad_token)

    def _bpe(self, word: str) -> list[int]:
        if word in self.cache:
            return self.cache[word]
        parts = list(word[:-1]) + [word[-1] + "</w>"]
        while len(parts) > 1:
            best, bi = None, -1
            for i in range(len(parts) - 1):
                r = self.ranks.get((parts[i], parts[i + 1]))
                if r is not None and (best is None or r < best):
                    best, bi = r, i
            if bi < 0:
                break
            parts[bi:bi + 2] = [parts[bi] + parts[bi + 1]]
        ids = []
        for p in parts:
            if p in self.encoder:
                ids.append(self.encoder[p])
            else:  # unknown piece: fall back to its characters
                for ch in p.replace("</w>", ""):
                    ids.append(self.encoder.get(ch, self.encoder.get(ch + "</w>", 0)))
        self.cache[word] = ids
        return ids

    def encode(self, text: str) -> list[int]:
        text = html.unescape(html.unescape(text))
        text = re.sub(r"\s+", " ", text).strip().lower()
        out = []
        for w in self.pat.findall(text):
            u = "".join(self.b2u[b] for b in w.encode("utf-8"))
            out.extend(self._bpe(u))
        return out

    def __call__(self, text: str) -> list[int]:
        """-> exactly max_len ids: <bos> tokens <eos> pad..."""
        ids = [self.bos] + self.encode(text)[: self.max_len - 2] + [self.eos]
        return ids + [self.pad] * (self.max_len - len(ids))


class T5Tokenizer:
    def __init__(self, sp=None, vocab: int = 32128, max_len: int = 256):
        self.sp = sp
        self.vocab = vocab
        self.max_len = max_len
        self.eos = 1
        self.pad = 0

    @classmethod
    def from_file(cls, path: str, max_len: int = 256) -> "T5Tokenizer":
        import sentencepiece as spm
        sp = spm.SentencePieceProcessor()
        sp.Load(path)
        return cls(sp, sp.GetPieceSize(), max_len)

    def encode(self, text: str) -> list[int]:
        if self.sp is not None:
            return list(self.sp.EncodeAsIds(text))
        return [3 + b % (self.vocab - 3) for b in text.encode("utf-8")]

    def __call__(self, text: str) -> list[int]:
        ids = self.encode(text)[: self.max_len - 1] + [self.eos]
        return ids + [self.pad] * (self.max_len - len(ids))
