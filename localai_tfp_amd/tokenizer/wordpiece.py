"""WordPiece tokenizer for BERT-family embedding / rerank models (the reference serves these
through llama.cpp's `bert` GGUF arch and the sentence-transformers/transformers backends).

Two vocabulary conventions are accepted:
  * HF / vocab.txt: word-initial pieces are bare, continuations carry a ``##`` prefix;
  * llama.cpp GGUF: word-initial pieces carry ``▁`` (U+2581), continuations are bare.
"""
from __future__ import annotations

import unicodedata

SPIECE = "▁"


def _is_punct(ch: str) -> bool:
    cp = ord(ch)
    if 33 <= cp <= 47 or 58 <= cp <= 64 or 91 <= cp <= 96 or 123 <= cp <= 126:
        return True
    return unicodedata.category(ch).startswith("P")


def _is_cjk(cp: int) -> bool:
    return (0x4E00 <= cp <= 0x9FFF or 0x3400 <= cp <= 0x4DBF or 0x20000 <= cp <= 0x2A6DF
            or 0x2A700 <= cp <= 0x2CEAF or 0xF900 <= cp <= 0xFAFF or 0x2F800 <= cp <= 0x2FA1F)


def basic_split(text: str, lower: bool = True) -> list[str]:
    """BERT BasicTokenizer: clean, CJK isolation, lowercase + accent strip, punctuation split."""
    out = []
    cur = []
    if lower:
        text = unicodedata.normalize("NFD", text.lower())
    for ch in text:
        cp = ord(ch)
        if cp == 0 or cp == 0xFFFD or (unicodedata.category(ch).startswith("C") and ch not in "\t\n\r"):
            continue
        if lower and unicodedata.category(ch) == "Mn":
            continue
        if ch.isspace():
            if cur:
                out.append("".join(cur))
                cur = []
        elif _is_punct(ch) or _is_cjk(cp):
            if cur:
                out.append("".join(cur))
                cur = []
            out.append(ch)
        else:
            cur.append(ch)
    if cur:
        out.append("".join(cur))
    return out


class WordPieceTokenizer:
    def __init__(self, tokens: list[str], lower: bool = True, unk: str = "[UNK]", cls: str = "[CLS]",
                 sep: str = "[SEP]", pad: str = "[PAD]", max_chars: int = 100):
        self.tokens = list(tokens)
        self.vocab = {t: i for i, t in enumerate(self.tokens)}
        self.gguf_style = not any(t.startswith("##") for t in self.tokens[:5000]) and \
            any(t.startswith(SPIECE) for t in self.tokens)
        self.lower = lower
        self.max_chars = max_chars
        self.unk_token_id = self.vocab.get(unk, 0)
        self.cls_token_id = self.vocab.get(cls, self.vocab.get("<s>"))
        self.sep_token_id = self.vocab.get(sep, self.vocab.get("</s>"))
        self.pad_token_id = self.vocab.get(pad, 0)
        self.bos_token_id, self.eos_token_id = self.cls_token_id, self.sep_token_id
        self.eos_token_ids = [self.sep_token_id]
        self.vocab_size = len(self.tokens)
        self.chat_template = None
        self._special = {i for i in (self.unk_token_id, self.cls_token_id, self.sep_token_id, self.pad_token_id)
                         if i is not None}

    @classmethod
    def from_gguf(cls, md: dict) -> "WordPieceTokenizer":
        toks = [str(t) for t in md["tokenizer.ggml.tokens"]]
        tk = cls(toks)
        for key, attr in (("bos", "cls_token_id"), ("eos", "sep_token_id"), ("seperator", "sep_token_id"),
                          ("separator", "sep_token_id"), ("unknown", "unk_token_id"), ("padding", "pad_token_id")):
            v = md.get(f"tokenizer.ggml.{key}_token_id")
            if v is not None:
                setattr(tk, attr, int(v))
        tk.bos_token_id, tk.eos_token_id = tk.cls_token_id, tk.sep_token_id
        tk.eos_token_ids = [tk.sep_token_id]
        return tk

    @classmethod
    def from_vocab_file(cls, path: str, lower: bool = True) -> "WordPieceTokenizer":
        with open(path, encoding="utf-8") as f:
            return cls([ln.rstrip("\n") for ln in f], lower=lower)

    def _word(self, w: str) -> list[int]:
        if len(w) > self.max_chars:
            return [self.unk_token_id]
        ids = []
        start = 0
        while start < len(w):
            end = len(w)
            hit = None
            while end > start:
                piece = w[start:end]
                if self.gguf_style:
                    key = SPIECE + piece if start == 0 else piece
                else:
                    key = piece if start == 0 else "##" + piece
                hit = self.vocab.get(key)
                if hit is not None:
                    break
                end -= 1
            if hit is None:
                return [self.unk_token_id]
            ids.append(hit)
            start = end
        return ids

    def encode(self, text: str, add_special: bool = True, parse_special: bool = False) -> list[int]:
        ids = []
        for w in basic_split(text, self.lower):
            ids.extend(self._word(w))
        if add_special:
            ids = [self.cls_token_id] + ids + [self.sep_token_id]
        return ids

    def encode_pair(self, a: str, b: str, max_len: int = 512) -> tuple[list[int], list[int]]:
        """[CLS] a [SEP] b [SEP] with token-type ids, truncating the longer side first (rerankers)."""
        ia = self.encode(a, add_special=False)
        ib = self.encode(b, add_special=False)
        while len(ia) + len(ib) + 3 > max_len:
            if len(ib) >= len(ia):
                ib.pop()
            else:
                ia.pop()
        ids = [self.cls_token_id] + ia + [self.sep_token_id] + ib + [self.sep_token_id]
        types = [0] * (len(ia) + 2) + [1] * (len(ib) + 1)
        return ids, types

    def decode(self, ids, skip_special: bool = True) -> str:
        out = []
        for i in ids:
            i = int(i)
            if skip_special and i in self._special:
                continue
            t = self.tokens[i] if 0 <= i < len(self.tokens) else ""
            if self.gguf_style:
                out.append(" " + t[1:] if t.startswith(SPIECE) else t)
            else:
                out.append(t[2:] if t.startswith("##") else " " + t)
        return "".join(out).strip()

    def token_to_piece(self, t: int) -> str:
        return self.decode([t], skip_special=False)

    def token_bytes(self) -> list[bytes]:
        return [self.token_to_piece(i).encode() for i in range(len(self.tokens))]
