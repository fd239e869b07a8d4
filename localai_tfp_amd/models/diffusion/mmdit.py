"""SD3 / SD3.5 multimodal diffusion transformer (MMDiT) — the denoiser of BASELINE config #5
(Stable-Diffusion-3 /v1/images/generations; reference: sd.cpp via gosd.cpp:56-226 and the diffusers
backend's SD3 pipeline, backend/python/diffusers/backend.py:139-270).

Parameter names follow diffusers' `SD3Transformer2DModel`. MI355X execution plan per step:
* all adaLN modulation vectors of every block (norm1 / norm1_context / norm_out) come from ONE GEMM
  of silu(temb) against the concatenated modulation weights (M = batch, launch-bound otherwise);
* image and context streams keep fp32 residuals; `layernorm_mod` (diffusion.hip) turns them into
  modulated 16-bit GEMM inputs in one pass; gated residual adds (`gate_add`) read the 16-bit GEMM
  output once;
* Q/K/V of each stream come from one fused GEMM; the joint sequence [image ; context] is attended by
  the MFMA flash kernel (head dim 64); the attention output feeds the two output projections as
  strided batched GEMMs (no split copies).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np
import torch
import torch.nn.functional as F
from torch import nn

from ...ops import core as K
from .nn import attention, cat_w, lin, timestep_embedding


@dataclass
class MMDiTConfig:
    patch: int = 2
    in_channels: int = 16
    out_channels: int = 16
    layers: int = 24
    head_dim: int = 64
    heads: int = 24
    joint_dim: int = 4096
    caption_dim: int = 1536
    pooled_dim: int = 2048
    pos_max: int = 192
    sample_size: int = 128
    qk_norm: bool = False
    dual_attention_layers: tuple = ()

    @property
    def dim(self) -> int:
        return self.heads * self.head_dim


SD3_MEDIUM = MMDiTConfig()
SD35_LARGE = MMDiTConfig(layers=38, heads=38, caption_dim=2432, qk_norm=True)
# SD3.5-medium = MMDiT-X: blocks 0..12 add a second, image-only self-attention (attn2) with its own
# three modulation vectors (adaLN 9*D instead of 6*D); position table 384 x 384.
SD35_MEDIUM = MMDiTConfig(layers=24, heads=24, caption_dim=1536, qk_norm=True, pos_max=384,
                          dual_attention_layers=tuple(range(13)))
MMDIT_TEST = MMDiTConfig(layers=2, heads=2, joint_dim=64, caption_dim=128, pooled_dim=64, pos_max=32,
                         sample_size=16)
MMDITX_TEST = MMDiTConfig(layers=3, heads=2, joint_dim=64, caption_dim=128, pooled_dim=64, pos_max=32,
                          sample_size=16, qk_norm=True, dual_attention_layers=(0, 1))


def sincos_2d(dim: int, grid: int, base_size: int, interp: float = 1.0) -> np.ndarray:
    gh = np.arange(grid, dtype=np.float64) / (grid / base_size) / interp
    gw = np.arange(grid, dtype=np.float64) / (grid / base_size) / interp
    mw, mh = np.meshgrid(gw, gh)

    def one(d, pos):
        om = 1.0 / 10000 ** (np.arange(d // 2, dtype=np.float64) / (d / 2.0))
        o = pos.reshape(-1)[:, None] * om[None]
        return np.concatenate([np.sin(o), np.cos(o)], 1)
    return np.concatenate([one(dim // 2, mw), one(dim // 2, mh)], 1).astype(np.float32)


class _Lin(nn.Module):
    def __init__(self, i, o, bias=True):
        super().__init__()
        self.linear = nn.Linear(i, o, bias)


class _PatchEmbed(nn.Module):
    def __init__(self, c: MMDiTConfig):
        super().__init__()
        self.proj = nn.Conv2d(c.in_channels, c.dim, c.patch, c.patch)
        pe = sincos_2d(c.dim, c.pos_max, c.sample_size // c.patch)
        self.register_buffer("pos_embed", torch.from_numpy(pe)[None], persistent=True)


class _TE(nn.Module):
    def __init__(self, i, o):
        super().__init__()
        self.linear_1 = nn.Linear(i, o)
        self.linear_2 = nn.Linear(o, o)


class _TimeText(nn.Module):
    def __init__(self, c):
        super().__init__()
        self.timestep_embedder = _TE(256, c.dim)
        self.text_embedder = _TE(c.pooled_dim, c.dim)


class _Attn(nn.Module):
    def __init__(self, c: MMDiTConfig, pre_only: bool):
        super().__init__()
        d = c.dim
        self.to_q, self.to_k, self.to_v = nn.Linear(d, d), nn.Linear(d, d), nn.Linear(d, d)
        self.add_q_proj, self.add_k_proj, self.add_v_proj = nn.Linear(d, d), nn.Linear(d, d), nn.Linear(d, d)
        self.to_out = nn.ModuleList([nn.Linear(d, d)])
        if not pre_only:
            self.to_add_out = nn.Linear(d, d)
        if c.qk_norm:
            for n in ("norm_q", "norm_k", "norm_added_q", "norm_added_k"):
                m = nn.Module()
                m.weight = nn.Parameter(torch.ones(c.head_dim))
                setattr(self, n, m)


class _SelfAttn(nn.Module):
    """MMDiT-X attn2: image-stream-only self-attention (diffusers `Attention` without added projections)."""

    def __init__(self, c: MMDiTConfig):
        super().__init__()
        d = c.dim
        self.to_q, self.to_k, self.to_v = nn.Linear(d, d), nn.Linear(d, d), nn.Linear(d, d)
        self.to_out = nn.ModuleList([nn.Linear(d, d)])
        if c.qk_norm:
            for n in ("norm_q", "norm_k"):
                m = nn.Module()
                m.weight = nn.Parameter(torch.ones(c.head_dim))
                setattr(self, n, m)


class _FF(nn.Module):
    def __init__(self, d):
        super().__init__()
        proj = nn.Module()
        proj.proj = nn.Linear(d, 4 * d)
        self.net = nn.ModuleList([proj, nn.Identity(), nn.Linear(4 * d, d)])


class _Block(nn.Module):
    def __init__(self, c: MMDiTConfig, pre_only: bool, dual: bool = False):
        super().__init__()
        d = c.dim
        self.pre_only, self.dual = pre_only, dual
        self.norm1 = _Lin(d, (9 if dual else 6) * d)
        if dual:
            self.attn2 = _SelfAttn(c)
        self.norm1_context = _Lin(d, (2 if pre_only else 6) * d)
        self.attn = _Attn(c, pre_only)
        self.ff = _FF(d)
        if not pre_only:
            self.ff_context = _FF(d)


class MMDiT(nn.Module):
    def __init__(self, c: MMDiTConfig):
        super().__init__()
        self.cfg = c
        self.pos_embed = _PatchEmbed(c)
        self.time_text_embed = _TimeText(c)
        self.context_embedder = nn.Linear(c.joint_dim, c.caption_dim if c.caption_dim else c.dim)
        self.transformer_blocks = nn.ModuleList(_Block(c, i == c.layers - 1, i in c.dual_attention_layers)
                                                for i in range(c.layers))
        self.norm_out = _Lin(c.dim, 2 * c.dim)
        self.proj_out = nn.Linear(c.dim, c.patch * c.patch * c.out_channels)
        self._prep = None

    # ------------------------------------------------------------------ fused weights
    def prepare(self):
        """Concatenate per-block weights into the fused layouts the forward pass uses."""
        mods, offs = [], []
        o = 0
        for b in self.transformer_blocks:
            for lin in (b.norm1.linear, b.norm1_context.linear):
                mods.append(lin)
                offs.append(o)
                o += lin.out_features
        mods.append(self.norm_out.linear)
        offs.append(o)
        o += self.norm_out.linear.out_features
        wm = cat_w([m.weight for m in mods])
        bm = torch.cat([m.bias for m in mods]).float()
        fused = []
        for b in self.transformer_blocks:
            a = b.attn
            fused.append((cat_w([a.to_q.weight, a.to_k.weight, a.to_v.weight]),
                          torch.cat([a.to_q.bias, a.to_k.bias, a.to_v.bias]),
                          cat_w([a.add_q_proj.weight, a.add_k_proj.weight, a.add_v_proj.weight]),
                          torch.cat([a.add_q_proj.bias, a.add_k_proj.bias, a.add_v_proj.bias])))
        qkv2 = [(cat_w([b.attn2.to_q.weight, b.attn2.to_k.weight, b.attn2.to_v.weight]),
                 torch.cat([b.attn2.to_q.bias, b.attn2.to_k.bias, b.attn2.to_v.bias])) if b.dual else None
                for b in self.transformer_blocks]
        c = self.cfg
        pw = self.pos_embed.proj.weight.reshape(c.dim, -1).contiguous()  # [D, C*p*p] (c, ph, pw) order
        self._prep = dict(wm=wm, bm=bm, offs=offs, qkv=fused, qkv2=qkv2, pw=pw)
        return self

    def _pos(self, h: int, w: int) -> torch.Tensor:
        c = self.cfg
        top, left = (c.pos_max - h) // 2, (c.pos_max - w) // 2
        pe = self.pos_embed.pos_embed.view(c.pos_max, c.pos_max, -1)
        return pe[top:top + h, left:left + w].reshape(h * w, -1)

    @staticmethod
    def _qk_norm(x: torch.Tensor, w: torch.Tensor, heads: int, eps: float = 1e-6):
        xs = x.float().view(x.shape[0], heads, -1)
        return (xs * torch.rsqrt(xs.pow(2).mean(-1, keepdim=True) + eps) * w.float()).to(x.dtype).view(x.shape[0], -1)

    @torch.no_grad()
    def forward(self, latent: torch.Tensor, t: torch.Tensor, ctx: torch.Tensor, pooled: torch.Tensor) -> torch.Tensor:
        """latent [B, C, H, W] (fp32), t [B] (0..1000), ctx [B, T, joint_dim], pooled [B, pooled_dim]
        -> velocity/eps prediction [B, C, H, W] fp32."""
        if self._prep is None:
            self.prepare()
        P = self._prep
        c = self.cfg
        dt = self.proj_out.weight.dtype
        B, C, Hh, Ww = latent.shape
        p = c.patch
        h, w = Hh // p, Ww // p
        S = h * w
        D = c.dim
        # patchify (conv p x p stride p == GEMM over (c, ph, pw) patches)
        patches = latent.to(dt).view(B, C, h, p, w, p).permute(0, 2, 4, 1, 3, 5).reshape(B * S, C * p * p)
        x = lin(patches, P["pw"], self.pos_embed.proj.bias).float()
        x = (x.view(B, S, D) + self._pos(h, w)[None]).reshape(B * S, D).contiguous()
        # conditioning
        te = self.time_text_embed
        temb = lin(timestep_embedding(t, 256).to(dt), te.timestep_embedder.linear_1.weight,
                        te.timestep_embedder.linear_1.bias)
        temb = lin(F.silu(temb), te.timestep_embedder.linear_2.weight, te.timestep_embedder.linear_2.bias)
        pe = lin(pooled.to(dt), te.text_embedder.linear_1.weight, te.text_embedder.linear_1.bias)
        pe = lin(F.silu(pe), te.text_embedder.linear_2.weight, te.text_embedder.linear_2.bias)
        cond = F.silu((temb.float() + pe.float()).to(dt))
        mod = lin(cond, P["wm"]).float() + P["bm"]  # [B, sum of all modulation widths]
        T = ctx.shape[1]
        cx = lin(ctx.reshape(B * T, -1).to(dt), self.context_embedder.weight, self.context_embedder.bias).float()
        H, hd = c.heads, c.head_dim
        xn = torch.empty(B * S, D, dtype=dt, device=x.device)
        cn = torch.empty(B * T, D, dtype=dt, device=x.device)
        for i, blk in enumerate(self.transformer_blocks):
            o1, o2 = P["offs"][2 * i], P["offs"][2 * i + 1]
            m = mod[:, o1:o1 + (9 if blk.dual else 6) * D]
            sh, sc, g, sh2, sc2, g2 = (m[:, k * D:(k + 1) * D] for k in range(6))
            mc = mod[:, o2:o2 + (2 if blk.pre_only else 6) * D]
            if blk.dual:  # attn2's input is modulated from the block INPUT (same LayerNorm, own shift/scale)
                xn2 = torch.empty_like(xn)
                K.layernorm_mod(x, m[:, 7 * D:8 * D], m[:, 6 * D:7 * D], S, xn2)
            K.layernorm_mod(x, sc, sh, S, xn)
            if blk.pre_only:  # AdaLayerNormContinuous: (scale, shift)
                K.layernorm_mod(cx, mc[:, :D], mc[:, D:2 * D], T, cn)
            else:
                K.layernorm_mod(cx, mc[:, D:2 * D], mc[:, :D], T, cn)
            wq, bq, wcq, bcq = P["qkv"][i]
            qx = lin(xn, wq, bq).view(B, S, 3 * D)
            qc = lin(cn, wcq, bcq).view(B, T, 3 * D)
            a = blk.attn
            if c.qk_norm:
                qx, qc = qx.clone(), qc.clone()
                for tq, nq, nk in ((qx, a.norm_q, a.norm_k), (qc, a.norm_added_q, a.norm_added_k)):
                    f = tq.view(-1, 3 * D)
                    f[:, :D] = self._qk_norm(f[:, :D], nq.weight, H)
                    f[:, D:2 * D] = self._qk_norm(f[:, D:2 * D], nk.weight, H)
            qkv = torch.cat([qx, qc], 1).view(B * (S + T), 3 * D)
            o = attention(qkv[:, :D], qkv[:, D:2 * D], qkv[:, 2 * D:], B, S + T, S + T, H, hd).view(B, S + T, D)
            y = lin(o[:, :S], a.to_out[0].weight, a.to_out[0].bias)
            K.gate_add(x, y.view(B * S, D), g, S)
            if blk.dual:
                w2, b2 = P["qkv2"][i]
                q2 = lin(xn2, w2, b2)
                if c.qk_norm:
                    q2[:, :D] = self._qk_norm(q2[:, :D], blk.attn2.norm_q.weight, H)
                    q2[:, D:2 * D] = self._qk_norm(q2[:, D:2 * D], blk.attn2.norm_k.weight, H)
                o2_ = attention(q2[:, :D], q2[:, D:2 * D], q2[:, 2 * D:], B, S, S, H, hd)
                K.gate_add(x, lin(o2_.reshape(B * S, D), blk.attn2.to_out[0].weight, blk.attn2.to_out[0].bias),
                           m[:, 8 * D:9 * D], S)
            K.layernorm_mod(x, sc2, sh2, S, xn)
            u = F.gelu(lin(xn, blk.ff.net[0].proj.weight, blk.ff.net[0].proj.bias), approximate="tanh")
            K.gate_add(x, lin(u, blk.ff.net[2].weight, blk.ff.net[2].bias), g2, S)
            if not blk.pre_only:
                csh, csc, cg, csh2, csc2, cg2 = (mc[:, k * D:(k + 1) * D] for k in range(6))
                yc = lin(o[:, S:], a.to_add_out.weight, a.to_add_out.bias)
                K.gate_add(cx, yc.reshape(B * T, D), cg, T)
                K.layernorm_mod(cx, csc2, csh2, T, cn)
                u = F.gelu(lin(cn, blk.ff_context.net[0].proj.weight, blk.ff_context.net[0].proj.bias),
                           approximate="tanh")
                K.gate_add(cx, lin(u, blk.ff_context.net[2].weight, blk.ff_context.net[2].bias), cg2, T)
        on = P["offs"][-1]
        K.layernorm_mod(x, mod[:, on:on + D], mod[:, on + D:on + 2 * D], S, xn)
        out = lin(xn, self.proj_out.weight, self.proj_out.bias).float()
        out = out.view(B, h, w, p, p, c.out_channels).permute(0, 5, 1, 3, 2, 4).reshape(B, c.out_channels, Hh, Ww)
        return out
