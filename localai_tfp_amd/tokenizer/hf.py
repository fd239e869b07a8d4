"""Tokenizer of a Hugging Face model directory (``tokenizer.json`` + ``tokenizer_config.json``), for the
safetensors checkpoints the vllm / transformers backends load (reference:
backend/python/transformers/backend.py:68-284 — ``AutoTokenizer.from_pretrained``).

Encoding and decoding run through the HF ``tokenizers`` runtime on the file itself (the exact
pre-tokenizer / normaliser / byte-fallback pipeline of the checkpoint); the GGUF-style fields the
engine and the grammar sampler use (token list, token types, BOS/EOS, per-token bytes, chat template)
are derived from it.
"""
from __future__ import annotations

import json
import os

import numpy as np

from .gguf import _U2B, TT_BYTE, TT_CONTROL, TT_NORMAL, TT_USER, _Base


def _tok_str(v):
    if isinstance(v, dict):
        return v.get("content")
    return v


class HFTokenizer(_Base):
    def __init__(self, d: str):
        from tokenizers import Tokenizer
        self._tk = Tokenizer.from_file(os.path.join(d, "tokenizer.json"))
        tcfg = {}
        p = os.path.join(d, "tokenizer_config.json")
        if os.path.isfile(p):
            with open(p, encoding="utf-8") as f:
                tcfg = json.load(f)
        mcfg = {}
        p = os.path.join(d, "config.json")
        if os.path.isfile(p):
            with open(p, encoding="utf-8") as f:
                mcfg = json.load(f)
        with open(os.path.join(d, "tokenizer.json"), encoding="utf-8") as f:
            spec = json.load(f)
        dec = spec.get("decoder") or {}
        dec_types = {dec.get("type")} | {x.get("type") for x in dec.get("decoders", []) if isinstance(x, dict)}
        self.byte_level = "ByteLevel" in dec_types

        vocab = self._tk.get_vocab(with_added_tokens=True)
        n = max(vocab.values()) + 1
        toks = [""] * n
        for t, i in vocab.items():
            toks[i] = t
        tt = np.full(n, TT_NORMAL, np.int32)
        for i, at in self._tk.get_added_tokens_decoder().items():
            tt[i] = TT_CONTROL if at.special else TT_USER
        if not self.byte_level:
            for i, t in enumerate(toks):
                if len(t) == 6 and t.startswith("<0x") and t.endswith(">"):
                    tt[i] = TT_BYTE

        def tid(s):
            return vocab.get(s) if s else None

        bos = tid(_tok_str(tcfg.get("bos_token")))
        eos = tid(_tok_str(tcfg.get("eos_token")))
        if bos is None and isinstance(mcfg.get("bos_token_id"), int):
            bos = mcfg["bos_token_id"]
        extra_eos = mcfg.get("eos_token_id")
        if eos is None and isinstance(extra_eos, int):
            eos = extra_eos
        if "add_bos_token" in tcfg:
            add_bos = bool(tcfg["add_bos_token"])
        else:  # the post-processor decides (Llama-3 adds <|begin_of_text|>, Qwen adds nothing)
            ids = self._tk.encode("a", add_special_tokens=True).ids
            add_bos = bos is not None and bool(ids) and ids[0] == bos
        ct = tcfg.get("chat_template")
        if isinstance(ct, list):  # [{"name": "default", "template": ...}, ...]
            ct = next((x.get("template") for x in ct if x.get("name") == "default"), ct[0].get("template") if ct else None)
        md = {"tokenizer.ggml.tokens": toks, "tokenizer.ggml.token_type": tt.tolist(),
              "tokenizer.ggml.bos_token_id": bos, "tokenizer.ggml.eos_token_id": eos,
              "tokenizer.ggml.add_bos_token": add_bos, "tokenizer.ggml.add_eos_token": bool(tcfg.get("add_eos_token", False)),
              "tokenizer.chat_template": ct}
        self._init_common(md)
        if isinstance(extra_eos, list):  # generation_config-style multi-EOS (Llama-3.1: <|eot_id|>, <|eom_id|>)
            self.eos_token_ids = sorted(set(self.eos_token_ids) | {int(x) for x in extra_eos})

    def encode(self, text: str, add_special: bool = True, parse_special: bool = True) -> list[int]:
        if parse_special or not self.special_ids:
            ids = list(self._tk.encode(text, add_special_tokens=False).ids)
        else:  # special-token text encoded as plain text
            import re
            ids = []
            for part in re.split("(" + "|".join(map(re.escape, self.special_ids)) + ")", text):
                if not part:
                    continue
                if part in self.special_ids:
                    for ch in part:
                        ids.extend(self._tk.encode(ch, add_special_tokens=False).ids)
                else:
                    ids.extend(self._tk.encode(part, add_special_tokens=False).ids)
        if add_special and self.add_bos and self.bos_token_id is not None and (not ids or ids[0] != self.bos_token_id):
            ids = [int(self.bos_token_id)] + ids
        if add_special and self.add_eos and self.eos_token_id is not None:
            ids = ids + [int(self.eos_token_id)]
        return ids

    def decode(self, ids, skip_special: bool = True) -> str:
        return self._tk.decode([int(i) for i in ids], skip_special_tokens=skip_special)

    def _piece_bytes(self, i: int) -> bytes:
        t = self.tokens[i]
        if self.token_type[i] == TT_USER:
            return t.encode()
        if self.byte_level:
            try:
                return bytes(_U2B[c] for c in t)
            except KeyError:
                return t.encode()
        if self.token_type[i] == TT_BYTE:
            return bytes([int(t[3:5], 16)])
        return t.replace("▁", " ").encode()


def from_hf_dir(d: str) -> HFTokenizer:
    return HFTokenizer(d)
