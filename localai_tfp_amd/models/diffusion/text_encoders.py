"""Text encoders for the diffusion pipelines: CLIP text transformer (ViT-L/14 "clip_l", OpenCLIP
bigG "clip_g", with the pooled projection) and the T5 v1.1 encoder (T5-XXL for SD3 / Flux).

Parameter names follow the Hugging Face `CLIPTextModelWithProjection` / `T5EncoderModel`
checkpoints (the files sd.cpp's `clip_l_path / clip_g_path / t5xxl_path` options and diffusers'
`text_encoder*` folders hold; reference gosd.cpp:56-162, diffusers backend.py:139-270).
Residual streams are fp32; GEMM inputs 16-bit.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import torch
import torch.nn.functional as F
from torch import nn

from ...ops import core as K
from .nn import attention, cat_w, layernorm16, lin, linear_acc


@dataclass
class CLIPTextConfig:
    vocab: int = 49408
    hidden: int = 768
    layers: int = 12
    heads: int = 12
    ffn: int = 3072
    max_pos: int = 77
    act: str = "quick_gelu"
    proj: int = 768
    eps: float = 1e-5


CLIP_L = CLIPTextConfig()
CLIP_G = CLIPTextConfig(hidden=1280, layers=32, heads=20, ffn=5120, act="gelu", proj=1280)


class _Emb(nn.Module):
    def __init__(self, c: CLIPTextConfig):
        super().__init__()
        self.token_embedding = nn.Embedding(c.vocab, c.hidden)
        self.position_embedding = nn.Embedding(c.max_pos, c.hidden)


class _Attn(nn.Module):
    def __init__(self, d, bias=True):
        super().__init__()
        self.q_proj = nn.Linear(d, d, bias)
        self.k_proj = nn.Linear(d, d, bias)
        self.v_proj = nn.Linear(d, d, bias)
        self.out_proj = nn.Linear(d, d, bias)


class _MLP(nn.Module):
    def __init__(self, d, f):
        super().__init__()
        self.fc1 = nn.Linear(d, f)
        self.fc2 = nn.Linear(f, d)


class _Layer(nn.Module):
    def __init__(self, c: CLIPTextConfig):
        super().__init__()
        self.self_attn = _Attn(c.hidden)
        self.layer_norm1 = nn.LayerNorm(c.hidden, eps=c.eps)
        self.mlp = _MLP(c.hidden, c.ffn)
        self.layer_norm2 = nn.LayerNorm(c.hidden, eps=c.eps)


class _Encoder(nn.Module):
    def __init__(self, c: CLIPTextConfig):
        super().__init__()
        self.layers = nn.ModuleList(_Layer(c) for _ in range(c.layers))


class _TextTransformer(nn.Module):
    def __init__(self, c: CLIPTextConfig):
        super().__init__()
        self.embeddings = _Emb(c)
        self.encoder = _Encoder(c)
        self.final_layer_norm = nn.LayerNorm(c.hidden, eps=c.eps)


class CLIPTextEncoder(nn.Module):
    def __init__(self, c: CLIPTextConfig, with_projection: bool = True):
        super().__init__()
        self.cfg = c
        self.text_model = _TextTransformer(c)
        self.text_projection = nn.Linear(c.hidden, c.proj, bias=False) if with_projection else None
        self._qkv = None

    def _fused(self):
        if self._qkv is None:
            self._qkv = [(cat_w([l.self_attn.q_proj.weight, l.self_attn.k_proj.weight, l.self_attn.v_proj.weight]),
                          torch.cat([l.self_attn.q_proj.bias, l.self_attn.k_proj.bias, l.self_attn.v_proj.bias]))
                         for l in self.text_model.encoder.layers]
        return self._qkv

    @torch.no_grad()
    def forward(self, ids: torch.Tensor, eos_id: int, skip: int = 1):
        """ids [B, S] -> (hidden after layer L-skip [B,S,D] fp32 (skip=1: penultimate, SD3's choice;
        skip=0: final LN output), pooled projection [B, proj] fp32)."""
        c = self.cfg
        tm = self.text_model
        B, S = ids.shape
        dt = tm.embeddings.token_embedding.weight.dtype
        x = (tm.embeddings.token_embedding.weight[ids].float() +
             tm.embeddings.position_embedding.weight[:S].float()).reshape(B * S, c.hidden).contiguous()
        H, D = c.heads, c.hidden // c.heads
        want = len(tm.encoder.layers) - skip
        sel = None
        for i, (l, (wqkv, bqkv)) in enumerate(zip(tm.encoder.layers, self._fused())):
            if i == want:
                sel = x.clone()
            h = layernorm16(x, l.layer_norm1.weight, l.layer_norm1.bias, c.eps, dt)
            qkv = lin(h, wqkv, bqkv)
            o = attention(qkv[:, :c.hidden], qkv[:, c.hidden:2 * c.hidden], qkv[:, 2 * c.hidden:], B, S, S, H, D,
                          causal=True)
            linear_acc(o, l.self_attn.out_proj, x)
            h = layernorm16(x, l.layer_norm2.weight, l.layer_norm2.bias, c.eps, dt)
            u = lin(h, l.mlp.fc1.weight, l.mlp.fc1.bias)
            u = u * torch.sigmoid(1.702 * u) if c.act == "quick_gelu" else F.gelu(u)
            linear_acc(u, l.mlp.fc2, x)
        final = F.layer_norm(x, (c.hidden,), tm.final_layer_norm.weight, tm.final_layer_norm.bias, c.eps)
        if sel is None:
            sel = final
        final3 = final.view(B, S, -1)
        eos_pos = (ids == eos_id).int().argmax(1)
        pooled = final3[torch.arange(B, device=ids.device), eos_pos]
        if self.text_projection is not None:
            pooled = lin(pooled.to(dt), self.text_projection.weight).float()
        return sel.view(B, S, -1), pooled


# ------------------------------------------------------------------------------------------------
# T5 v1.1 encoder

@dataclass
class T5Config:
    vocab: int = 32128
    d_model: int = 4096
    heads: int = 64
    d_kv: int = 64
    d_ff: int = 10240
    layers: int = 24
    buckets: int = 32
    max_distance: int = 128
    eps: float = 1e-6
    ff: str = "gated-gelu"  # T5 v1.1 / Flan (SD3, Flux); "relu" = original T5 (MusicGen's t5-base)

    @classmethod
    def from_hf(cls, d: dict) -> "T5Config":
        ff = d.get("feed_forward_proj", "relu")
        if ff not in ("relu", "gated-gelu"):
            raise NotImplementedError(f"T5 feed_forward_proj {ff!r}")
        return cls(vocab=d.get("vocab_size", 32128), d_model=d["d_model"], heads=d["num_heads"], d_kv=d["d_kv"],
                   d_ff=d["d_ff"], layers=d["num_layers"], buckets=d.get("relative_attention_num_buckets", 32),
                   max_distance=d.get("relative_attention_max_distance", 128),
                   eps=d.get("layer_norm_epsilon", 1e-6), ff=ff)


T5_XXL = T5Config()


class T5RMSNorm(nn.Module):
    def __init__(self, d):
        super().__init__()
        self.weight = nn.Parameter(torch.ones(d))


class _T5Attn(nn.Module):
    def __init__(self, c: T5Config, rel: bool):
        super().__init__()
        inner = c.heads * c.d_kv
        self.q = nn.Linear(c.d_model, inner, bias=False)
        self.k = nn.Linear(c.d_model, inner, bias=False)
        self.v = nn.Linear(c.d_model, inner, bias=False)
        self.o = nn.Linear(inner, c.d_model, bias=False)
        if rel:
            self.relative_attention_bias = nn.Embedding(c.buckets, c.heads)


class _T5SA(nn.Module):
    def __init__(self, c, rel):
        super().__init__()
        self.SelfAttention = _T5Attn(c, rel)
        self.layer_norm = T5RMSNorm(c.d_model)


class _T5DRD(nn.Module):
    def __init__(self, c):
        super().__init__()
        if c.ff == "relu":
            self.wi = nn.Linear(c.d_model, c.d_ff, bias=False)
        else:
            self.wi_0 = nn.Linear(c.d_model, c.d_ff, bias=False)
            self.wi_1 = nn.Linear(c.d_model, c.d_ff, bias=False)
        self.wo = nn.Linear(c.d_ff, c.d_model, bias=False)


class _T5FF(nn.Module):
    def __init__(self, c):
        super().__init__()
        self.DenseReluDense = _T5DRD(c)
        self.layer_norm = T5RMSNorm(c.d_model)


class _T5Block(nn.Module):
    def __init__(self, c, rel):
        super().__init__()
        self.layer = nn.ModuleList([_T5SA(c, rel), _T5FF(c)])


class _T5Stack(nn.Module):
    def __init__(self, c):
        super().__init__()
        self.block = nn.ModuleList(_T5Block(c, i == 0) for i in range(c.layers))
        self.final_layer_norm = T5RMSNorm(c.d_model)


def t5_buckets(rel: torch.Tensor, buckets: int, max_distance: int) -> torch.Tensor:
    n = buckets // 2
    ret = (rel > 0).long() * n
    r = rel.abs()
    max_exact = n // 2
    large = max_exact + (torch.log(r.float().clamp_min(1) / max_exact) / math.log(max_distance / max_exact) *
                         (n - max_exact)).long()
    large = large.clamp(max=n - 1)
    return ret + torch.where(r < max_exact, r, large)


class T5Encoder(nn.Module):
    def __init__(self, c: T5Config):
        super().__init__()
        self.cfg = c
        self.shared = nn.Embedding(c.vocab, c.d_model)
        self.encoder = _T5Stack(c)

    def _rms(self, x, w, dt):
        out = torch.empty(x.shape, dtype=dt, device=x.device)
        if x.is_cuda and dt != torch.float32:
            K.rmsnorm(x, w, self.cfg.eps, out_bf16=out)
        else:
            out.copy_(x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + self.cfg.eps) * w)
        return out

    @torch.no_grad()
    def forward(self, ids: torch.Tensor, mask: torch.Tensor | None = None) -> torch.Tensor:
        """ids [B, S] (mask [B, S]: 1 = token, 0 = padding) -> last hidden state [B, S, d_model] fp32."""
        c = self.cfg
        B, S = ids.shape
        dt = self.shared.weight.dtype
        x = self.shared.weight[ids].float().reshape(B * S, c.d_model).contiguous()
        rel = self.encoder.block[0].layer[0].SelfAttention.relative_attention_bias
        inner = c.heads * c.d_kv
        flash = ids.is_cuda and dt != torch.float32 and c.d_kv <= 128
        if flash:
            # the flash kernel adds T5's bias by key-minus-query offset: one [H, 2S-1] table per forward;
            # padding (right-padded prompts) as per-row key lengths
            offs = torch.arange(-(S - 1), S, device=ids.device)
            rb = rel.weight[t5_buckets(offs, c.buckets, c.max_distance)].t().float().contiguous()  # [H, 2S-1]
            klen = None
            if mask is not None:
                n = mask.to(ids.device).sum(-1).to(torch.int32)
                klen = torch.where(n > 0, n, torch.full_like(n, S)).contiguous()
        else:
            pos = torch.arange(S, device=ids.device)
            bucket = t5_buckets(pos[None, :] - pos[:, None], c.buckets, c.max_distance)
            bias = rel.weight[bucket].permute(2, 0, 1)[None].to(dt)  # [1, H, S, S]
            if mask is not None:
                neg = torch.finfo(dt).min
                bias = bias + torch.where(mask.to(ids.device)[:, None, None, :].bool(), 0.0, neg).to(dt)
        for blk in self.encoder.block:
            sa, ff = blk.layer[0], blk.layer[1]
            a = sa.SelfAttention
            h = self._rms(x, sa.layer_norm.weight, dt)
            if flash:
                q, k, v = (lin(h, w.weight) for w in (a.q, a.k, a.v))
                o = torch.empty(B * S, inner, dtype=q.dtype, device=q.device)
                K.attn_dense(q, k, v, o, B, S, S, c.heads, c.heads, c.d_kv, 1.0, klen=klen, rbias=rb)
            else:
                q, k, v = (lin(h, w.weight).view(B, S, c.heads, c.d_kv).transpose(1, 2) for w in (a.q, a.k, a.v))
                o = F.scaled_dot_product_attention(q, k, v, attn_mask=bias.expand(B, -1, -1, -1).to(q.dtype),
                                                   scale=1.0)
                o = o.transpose(1, 2).reshape(B * S, inner)
            linear_acc(o, a.o, x)
            h = self._rms(x, ff.layer_norm.weight, dt)
            d = ff.DenseReluDense
            if c.ff == "relu":
                act = F.relu(lin(h, d.wi.weight))
            else:
                g = lin(h, d.wi_0.weight)
                u = lin(h, d.wi_1.weight)
                act = torch.empty_like(g)
                K.glu(g, u, act, act="gelu_tanh")
            linear_acc(act, d.wo, x)
        out = self._rms(x, self.encoder.final_layer_norm.weight, torch.float32)
        return out.view(B, S, c.d_model)
