"""Tokenizer reconstructed from GGUF metadata (``tokenizer.ggml.*``), the way llama.cpp does for the
reference worker (`common_tokenize`, grpc-server.cpp:1793 / TokenizeString :2603).

* model "gpt2" (byte-level BPE; Llama-3, Qwen2, ...): HF ``tokenizers`` BPE with the
  pre-tokenizer regex selected by ``tokenizer.ggml.pre``, control/user-defined tokens atomic.
* model "llama" (SentencePiece BPE; Llama-2, Mistral, TinyLlama): score-ordered pair merging with
  byte fallback (``<0xXX>``) — llm_tokenizer_spm semantics.
* model "bert" (WordPiece) is handled by the embedding worker (models/bert.py).
"""
from __future__ import annotations

import heapq
import re

import numpy as np

PRE_REGEX = {
    "llama-bpe": r"(?i:'s|'t|'re|'ve|'m|'ll|'d)|[^\r\n\p{L}\p{N}]?\p{L}+|\p{N}{1,3}| ?[^\s\p{L}\p{N}]+[\r\n]*|\s*[\r\n]+|\s+(?!\S)|\s+",
    "llama3": r"(?i:'s|'t|'re|'ve|'m|'ll|'d)|[^\r\n\p{L}\p{N}]?\p{L}+|\p{N}{1,3}| ?[^\s\p{L}\p{N}]+[\r\n]*|\s*[\r\n]+|\s+(?!\S)|\s+",
    "qwen2": r"(?i:'s|'t|'re|'ve|'m|'ll|'d)|[^\r\n\p{L}\p{N}]?\p{L}+|\p{N}| ?[^\s\p{L}\p{N}]+[\r\n]*|\s*[\r\n]+|\s+(?!\S)|\s+",
    "default": r"'s|'t|'re|'ve|'m|'ll|'d| ?\p{L}+| ?\p{N}+| ?[^\s\p{L}\p{N}]+|\s+(?!\S)|\s+",
}

TT_NORMAL, TT_UNKNOWN, TT_CONTROL, TT_USER, TT_UNUSED, TT_BYTE = 1, 2, 3, 4, 5, 6


class _Base:
    def _init_common(self, md: dict):
        self.tokens: list[str] = list(md["tokenizer.ggml.tokens"])
        self.vocab_size = len(self.tokens)
        tt = md.get("tokenizer.ggml.token_type")
        self.token_type = np.asarray(tt, np.int32) if tt is not None else np.ones(self.vocab_size, np.int32)
        self.bos_token_id = md.get("tokenizer.ggml.bos_token_id")
        self.eos_token_id = md.get("tokenizer.ggml.eos_token_id")
        self.unk_token_id = md.get("tokenizer.ggml.unknown_token_id")
        self.pad_token_id = md.get("tokenizer.ggml.padding_token_id")
        self.add_bos = bool(md.get("tokenizer.ggml.add_bos_token", True))
        self.add_eos = bool(md.get("tokenizer.ggml.add_eos_token", False))
        self.chat_template = md.get("tokenizer.chat_template")
        eos = set()
        if self.eos_token_id is not None:
            eos.add(int(self.eos_token_id))
        eot = md.get("tokenizer.ggml.eot_token_id")
        if eot is not None:
            eos.add(int(eot))
        # end-of-generation markers commonly used by chat models
        for i, t in enumerate(self.tokens):
            if self.token_type[i] in (TT_CONTROL, TT_USER) and t in ("<|eot_id|>", "<|im_end|>", "<|end|>", "<end_of_turn>", "<|endoftext|>", "</s>"):
                eos.add(i)
        self.eos_token_ids = sorted(eos)
        self.bos_token = self.tokens[self.bos_token_id] if self.bos_token_id is not None else ""
        self.eos_token = self.tokens[self.eos_token_id] if self.eos_token_id is not None else ""
        self.special_ids = {t: i for i, t in enumerate(self.tokens) if self.token_type[i] in (TT_CONTROL, TT_USER)}

    def token_to_piece(self, t: int) -> str:
        return self.decode([t], skip_special=False)

    def token_bytes(self) -> list[bytes]:
        """Raw bytes each token id emits (b"" for control tokens) — for grammar masking."""
        if getattr(self, "_tb", None) is None:
            self._tb = [b"" if self.token_type[i] in (TT_CONTROL, TT_UNKNOWN, TT_UNUSED) else self._piece_bytes(i)
                        for i in range(self.vocab_size)]
        return self._tb


def _bytes_to_unicode():
    bs = list(range(ord("!"), ord("~") + 1)) + list(range(ord("¡"), ord("¬") + 1)) + list(range(ord("®"), ord("ÿ") + 1))
    cs = bs[:]
    n = 0
    for b in range(256):
        if b not in bs:
            bs.append(b)
            cs.append(256 + n)
            n += 1
    return {chr(c): b for b, c in zip(bs, cs)}


_U2B = _bytes_to_unicode()


class BPETokenizer(_Base):
    def __init__(self, md: dict):
        from tokenizers import AddedToken, Regex, Tokenizer, decoders, models, pre_tokenizers
        self._init_common(md)
        vocab = {t: i for i, t in enumerate(self.tokens)}
        merges = [tuple(m.split(" ", 1)) for m in md.get("tokenizer.ggml.merges", [])]
        bpe = models.BPE(vocab=vocab, merges=merges, ignore_merges=False) if _bpe_has_ignore() else models.BPE(vocab=vocab, merges=merges)
        tk = Tokenizer(bpe)
        pre = str(md.get("tokenizer.ggml.pre", "default"))
        pat = PRE_REGEX.get(pre, PRE_REGEX["llama-bpe"] if pre.startswith("llama") else PRE_REGEX["default"])
        tk.pre_tokenizer = pre_tokenizers.Sequence([
            pre_tokenizers.Split(Regex(pat), behavior="isolated"),
            pre_tokenizers.ByteLevel(add_prefix_space=False, use_regex=False),
        ])
        tk.decoder = decoders.ByteLevel()
        specials = [AddedToken(t, special=True, normalized=False) for t in self.special_ids]
        if specials:
            tk.add_special_tokens(specials)
        self._tk = tk
        self._special_set = set(self.special_ids.values())

    def encode(self, text: str, add_special: bool = True, parse_special: bool = True) -> list[int]:
        if parse_special:
            ids = self._tk.encode(text, add_special_tokens=False).ids
        else:
            ids = []
            for part in re.split("(" + "|".join(map(re.escape, self.special_ids)) + ")", text) if self.special_ids else [text]:
                if part:
                    ids.extend(self._tk.encode(part, add_special_tokens=False).ids)
        if add_special and self.add_bos and self.bos_token_id is not None and (not ids or ids[0] != self.bos_token_id):
            ids = [int(self.bos_token_id)] + ids
        if add_special and self.add_eos and self.eos_token_id is not None:
            ids = ids + [int(self.eos_token_id)]
        return ids

    def decode(self, ids, skip_special: bool = True) -> str:
        return self._tk.decode([int(i) for i in ids], skip_special_tokens=skip_special)

    def stream_bytes(self) -> list[bytes]:
        """Bytes each id contributes to decode(ids, skip_special=True) (b"" for the special / added tokens it
        skips): byte-level BPE text is the concatenation of these, so streamed detokenisation can append bytes
        per token instead of re-decoding a window (engine/sequence.py)."""
        if getattr(self, "_sb", None) is None:
            skip = set(self._special_set)
            self._sb = [b"" if (i in skip or self.token_type[i] in (TT_CONTROL, TT_UNKNOWN, TT_UNUSED))
                        else self._piece_bytes(i) for i in range(self.vocab_size)]
        return self._sb

    def _piece_bytes(self, i: int) -> bytes:
        t = self.tokens[i]
        if self.token_type[i] == TT_USER:
            return t.encode()
        try:
            return bytes(_U2B[c] for c in t)
        except KeyError:
            return t.encode()


def _bpe_has_ignore():
    try:
        from tokenizers import models
        models.BPE(vocab={"a": 0}, merges=[], ignore_merges=False)
        return True
    except TypeError:
        return False


class SPMTokenizer(_Base):
    """SentencePiece-BPE (llama.cpp llm_tokenizer_spm): merge the highest-scoring adjacent pair."""

    def __init__(self, md: dict):
        self._init_common(md)
        sc = md.get("tokenizer.ggml.scores")
        self.scores = np.asarray(sc, np.float32) if sc is not None else np.zeros(self.vocab_size, np.float32)
        self.vocab = {t: i for i, t in enumerate(self.tokens)}
        self.byte_ids = {}
        for i, t in enumerate(self.tokens):
            if self.token_type[i] == TT_BYTE or re.fullmatch(r"<0x[0-9A-Fa-f]{2}>", t):
                self.byte_ids[int(t[3:5], 16)] = i
        self.add_space_prefix = bool(md.get("tokenizer.ggml.add_space_prefix", True))

    def _encode_text(self, text: str) -> list[int]:
        if not text:
            return []
        s = text.replace(" ", "▁")
        syms = list(s)
        n = len(syms)
        prev = list(range(-1, n - 1))
        nxt = list(range(1, n + 1))
        alive = [True] * n
        heap = []

        def push(i):
            j = nxt[i]
            if j >= n:
                return
            tid = self.vocab.get(syms[i] + syms[j])
            if tid is not None:
                heapq.heappush(heap, (-float(self.scores[tid]), i, syms[i] + syms[j]))

        for i in range(n - 1):
            push(i)
        while heap:
            _, i, merged = heapq.heappop(heap)
            j = nxt[i] if i < n else n
            if not alive[i] or j >= n or not alive[j] or syms[i] + syms[j] != merged:
                continue
            syms[i] = merged
            alive[j] = False
            nxt[i] = nxt[j]
            if nxt[j] < n:
                prev[nxt[j]] = i
            if prev[i] >= 0:
                push(prev[i])
            push(i)
        out = []
        i = 0
        while i < n:
            if alive[i]:
                tid = self.vocab.get(syms[i])
                if tid is not None:
                    out.append(tid)
                else:
                    for b in syms[i].encode("utf-8"):
                        bid = self.byte_ids.get(b, self.unk_token_id if self.unk_token_id is not None else 0)
                        out.append(bid)
            i = nxt[i] if alive[i] else i + 1
        return out

    def encode(self, text: str, add_special: bool = True, parse_special: bool = True) -> list[int]:
        ids = []
        pieces = [text]
        if parse_special and self.special_ids:
            pat = "(" + "|".join(map(re.escape, sorted(self.special_ids, key=len, reverse=True))) + ")"
            pieces = re.split(pat, text)
        first = True
        for p in pieces:
            if not p:
                continue
            if parse_special and p in self.special_ids:
                ids.append(self.special_ids[p])
                first = False
                continue
            if first and self.add_space_prefix and not p.startswith(" "):
                p = " " + p
            first = False
            ids.extend(self._encode_text(p))
        if add_special and self.add_bos and self.bos_token_id is not None:
            ids = [int(self.bos_token_id)] + ids
        if add_special and self.add_eos and self.eos_token_id is not None:
            ids.append(int(self.eos_token_id))
        return ids

    def _piece_bytes(self, i: int) -> bytes:
        piece = self.tokens[i]
        if self.token_type[i] == TT_BYTE or re.fullmatch(r"<0x[0-9A-Fa-f]{2}>", piece):
            return bytes([int(piece[3:5], 16)])
        return piece.replace("▁", " ").encode()

    def decode(self, ids, skip_special: bool = True) -> str:
        buf = bytearray()
        for t in ids:
            t = int(t)
            if t < 0 or t >= self.vocab_size:
                continue
            tt = self.token_type[t]
            piece = self.tokens[t]
            if tt == TT_BYTE or (piece.startswith("<0x") and len(piece) == 6 and piece.endswith(">")):
                buf.append(int(piece[3:5], 16))
            elif tt in (TT_CONTROL, TT_UNKNOWN):
                if not skip_special:
                    buf.extend(piece.encode())
            else:
                buf.extend(piece.replace("▁", " ").encode())
        # no leading-space strip: streamed pieces must concatenate to the raw output (token_to_piece)
        return buf.decode("utf-8", errors="replace")


def from_gguf(md: dict):
    model = str(md.get("tokenizer.ggml.model", "gpt2"))
    if model == "llama":
        return SPMTokenizer(md)
    if model in ("gpt2", "bpe"):
        return BPETokenizer(md)
    if model == "bert":
        from .wordpiece import WordPieceTokenizer
        return WordPieceTokenizer.from_gguf(md)
    raise ValueError(f"unsupported tokenizer model {model!r}")
