"""BERT-family encoder for embeddings and cross-encoder reranking.

Parity target: the reference serves these through llama.cpp's `bert` GGUF architecture (embeddings
with mean / CLS pooling + L2 normalisation, grpc-server.cpp send_embedding) and the Python
sentence-transformers / rerankers backends (backend/python/transformers/backend.py:286-322,
backend/python/rerankers/backend.py:72-91).

MI355X path: 16-bit activations (the library's act16 format), GEMMs on hipBLASLt with fused bias
(plain library GEMMs), attention on the fused MFMA flash kernel (attention_dense.hip, key-padding
masks instead of materialised [B, S, S] masks), LayerNorm / residual adds on the norm kernel
(norm.hip) reading the fp32 residual stream once. Weights load from GGUF (llama.cpp `bert` /
`nomic-bert` / `jina-bert-v2` tensor names, any ggml type -> dequantised to 16-bit) or are
random-initialised for `synthetic:bert-*`.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np
import torch
import torch.nn.functional as F

from ..ops import core as K
from ..ops.linear import ACT_DTYPE


@dataclass
class BertConfig:
    vocab: int = 30522
    hidden: int = 768
    n_layers: int = 12
    n_heads: int = 12
    ffn: int = 3072
    max_pos: int = 512
    type_vocab: int = 2
    eps: float = 1e-12
    pooling: str = "mean"  # mean | cls | last | none | rank
    act: str = "gelu"
    name: str = "bert"

    @classmethod
    def from_gguf_metadata(cls, md: dict) -> "BertConfig":
        a = str(md.get("general.architecture", "bert"))

        def g(k, d=None):
            return md.get(f"{a}.{k}", d)
        pool = {0: "none", 1: "mean", 2: "cls", 3: "last", 4: "rank"}.get(int(g("pooling_type", 1) or 1), "mean")
        toks = md.get("tokenizer.ggml.tokens") or []
        return cls(vocab=len(toks) or int(g("vocab_size", 30522)), hidden=int(g("embedding_length")),
                   n_layers=int(g("block_count")), n_heads=int(g("attention.head_count")),
                   ffn=int(g("feed_forward_length")), max_pos=int(g("context_length", 512)),
                   eps=float(g("attention.layer_norm_epsilon", 1e-12)), pooling=pool, name=str(md.get("general.name", a)))


BERT_BASE = BertConfig()
BERT_TINY = BertConfig(vocab=400, hidden=128, n_layers=2, n_heads=2, ffn=512, max_pos=128, name="bert-tiny")


class BertModel:
    def __init__(self, cfg: BertConfig, device="cpu"):
        self.cfg = cfg
        self.device = torch.device(device)
        self.dtype = ACT_DTYPE if self.device.type == "cuda" else torch.float32
        self.w: dict[str, torch.Tensor] = {}
        self.has_cls_head = False

    # ------------------------------------------------------------------ loading
    @classmethod
    def load(cls, cfg: BertConfig, get_tensor, device="cpu") -> "BertModel":
        """get_tensor(name) -> np.float32 array (or None). llama.cpp bert tensor names."""
        m = cls(cfg, device)
        dt = m.dtype

        def put(name, key=None, f32=False):
            a = get_tensor(name)
            if a is None:
                return None
            t = torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32)).to(m.device)
            m.w[key or name] = t if f32 else t.to(dt)
            return m.w[key or name]
        put("token_embd.weight", f32=True)
        put("position_embd.weight", f32=True)
        put("token_types.weight", f32=True)
        put("token_embd_norm.weight", f32=True)
        put("token_embd_norm.bias", f32=True)
        for i in range(cfg.n_layers):
            p = f"blk.{i}."
            q, k, v = (get_tensor(p + f"attn_{x}.weight") for x in "qkv")
            if q is not None:
                m.w[p + "qkv.weight"] = torch.from_numpy(np.concatenate([q, k, v], 0).astype(np.float32)).to(
                    m.device).to(dt)
                bs = [get_tensor(p + f"attn_{x}.bias") for x in "qkv"]
                if bs[0] is not None:
                    m.w[p + "qkv.bias"] = torch.from_numpy(np.concatenate(bs, 0).astype(np.float32)).to(m.device).to(dt)
            else:  # fused qkv (nomic-bert / jina)
                put(p + "attn_qkv.weight", p + "qkv.weight")
                put(p + "attn_qkv.bias", p + "qkv.bias")
            for n in ("attn_output", "ffn_up", "ffn_down", "ffn_gate"):
                put(p + n + ".weight")
                put(p + n + ".bias")
            for n in ("attn_output_norm", "layer_output_norm"):
                put(p + n + ".weight", f32=True)
                put(p + n + ".bias", f32=True)
        # cross-encoder head (rerankers): cls.weight/bias (+ optional cls.output)
        if put("cls.weight") is not None:
            put("cls.bias")
            put("cls.output.weight")
            put("cls.output.bias")
            m.has_cls_head = True
        return m

    # ------------------------------------------------------------------ forward
    def _linear(self, x, name, act: str | None = None):
        W = self.w[name + ".weight"]
        b = self.w.get(name + ".bias")
        y = torch.addmm(b, x, W.t()) if b is not None else x @ W.t()
        if act == "gelu":
            y = F.gelu(y)
        return y

    def _ln(self, h: torch.Tensor, name: str, out: torch.Tensor, residual: torch.Tensor | None = None):
        K.layernorm(h, self.w[name + ".weight"], self.w.get(name + ".bias"), self.cfg.eps, out, residual=residual)
        return out

    def encode(self, ids: list[list[int]], types: list[list[int]] | None = None) -> tuple[torch.Tensor, torch.Tensor]:
        """-> (hidden [B, S, H] fp32 after the final layer, lengths [B])."""
        cfg = self.cfg
        B = len(ids)
        S = max(len(x) for x in ids)
        dev = self.device
        tok = torch.zeros(B, S, dtype=torch.long)
        typ = torch.zeros(B, S, dtype=torch.long)
        lens = torch.tensor([len(x) for x in ids], dtype=torch.int32)
        for b, x in enumerate(ids):
            tok[b, :len(x)] = torch.tensor(x)
            if types is not None:
                typ[b, :len(x)] = torch.tensor(types[b])
        tok, typ = tok.to(dev), typ.to(dev)
        pos = torch.arange(S, device=dev)[None].expand(B, S)
        h = self.w["token_embd.weight"][tok] + self.w["position_embd.weight"][pos]
        if "token_types.weight" in self.w:
            h = h + self.w["token_types.weight"][typ]
        h = h.reshape(B * S, cfg.hidden).contiguous().float()
        x = torch.empty(B * S, cfg.hidden, dtype=self.dtype, device=dev)
        self._ln(h, "token_embd_norm", x)
        hd = cfg.hidden // cfg.n_heads
        lens_d = lens.to(dev)
        attn = torch.empty(B * S, cfg.hidden, dtype=self.dtype, device=dev)
        for i in range(cfg.n_layers):
            p = f"blk.{i}."
            qkv = self._linear(x, p + "qkv")
            H = cfg.hidden
            K.attn_dense(qkv[:, :H], qkv[:, H:2 * H], qkv[:, 2 * H:], attn, B, S, S, cfg.n_heads, cfg.n_heads, hd,
                         1.0 / math.sqrt(hd), causal=False, klen=lens_d)
            o = self._linear(attn, p + "attn_output")
            # post-LN BERT: h = LN(x + attn_out); the fp32 residual sum is formed inside the norm kernel
            h = o.float()
            self._ln(h, p + "attn_output_norm", x, residual=x.float())
            up = self._linear(x, p + "ffn_up", act="gelu")
            down = self._linear(up, p + "ffn_down")
            h = down.float()
            self._ln(h, p + "layer_output_norm", x, residual=x.float())
        return x.float().view(B, S, cfg.hidden), lens

    def embed(self, ids: list[list[int]], normalize: bool = True) -> torch.Tensor:
        hid, lens = self.encode(ids)
        B, S, H = hid.shape
        pool = self.cfg.pooling
        if pool == "cls" or pool == "rank":
            e = hid[:, 0]
        elif pool == "last":
            e = hid[torch.arange(B), (lens - 1).long().to(hid.device)]
        else:  # mean over valid tokens
            mask = (torch.arange(S, device=hid.device)[None] < lens.to(hid.device)[:, None]).float()
            e = (hid * mask[..., None]).sum(1) / mask.sum(1, keepdim=True).clamp_min(1)
        if normalize:
            e = e / e.norm(dim=-1, keepdim=True).clamp_min(1e-12)
        return e

    def rerank_scores(self, pairs_ids: list[list[int]], types: list[list[int]]) -> torch.Tensor:
        """Cross-encoder relevance: classification head on the [CLS] state."""
        hid, _ = self.encode(pairs_ids, types)
        c = hid[:, 0].to(self.dtype)
        y = self._linear(c, "cls")
        if "cls.output.weight" in self.w:
            y = self._linear(torch.tanh(y), "cls.output")
        return y.float()[:, 0]


def synthetic_bert(cfg: BertConfig, seed: int = 0, rerank: bool = False):
    rng = np.random.default_rng(seed)
    H, Fd = cfg.hidden, cfg.ffn
    t = {"token_embd.weight": (cfg.vocab, H), "position_embd.weight": (cfg.max_pos, H),
         "token_types.weight": (cfg.type_vocab, H), "token_embd_norm.weight": (H,), "token_embd_norm.bias": (H,)}
    for i in range(cfg.n_layers):
        p = f"blk.{i}."
        for x in "qkv":
            t[p + f"attn_{x}.weight"] = (H, H)
            t[p + f"attn_{x}.bias"] = (H,)
        t.update({p + "attn_output.weight": (H, H), p + "attn_output.bias": (H,),
                  p + "attn_output_norm.weight": (H,), p + "attn_output_norm.bias": (H,),
                  p + "ffn_up.weight": (Fd, H), p + "ffn_up.bias": (Fd,), p + "ffn_down.weight": (H, Fd),
                  p + "ffn_down.bias": (H,), p + "layer_output_norm.weight": (H,), p + "layer_output_norm.bias": (H,)})
    if rerank:
        t.update({"cls.weight": (H, H), "cls.bias": (H,), "cls.output.weight": (1, H), "cls.output.bias": (1,)})
    cache = {}

    def get(name):
        if name not in t:
            return None
        if name not in cache:
            shape = t[name]
            if name.endswith("norm.weight"):
                cache[name] = np.ones(shape, np.float32)
            elif name.endswith(".bias"):
                cache[name] = np.zeros(shape, np.float32)
            else:
                cache[name] = (rng.standard_normal(shape) * 0.02).astype(np.float32)
        return cache[name]
    return get


def gguf_tensor_source(reader):
    from ..ops.quant import dequantize

    def get(name):
        ti = reader.tensors.get(name)
        if ti is None:
            return None
        a = dequantize(reader.tensor_bytes(name), ti.qtype, ti.shape)  # numpy shape = reversed(ggml shape)
        return a if len(ti.shape) > 1 else a.reshape(-1)
    return get
