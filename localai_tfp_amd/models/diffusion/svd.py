"""Stable Video Diffusion (img2vid): the reference's diffusers `StableVideoDiffusionPipeline`
(backend/python/diffusers/backend.py:175-179 load, :338-341 generate + export_to_video), served here
through both GenerateImage (src = start image, dst = video) and the GenerateVideo RPC
(core/backend/video.go:22, backend.proto GenerateVideoRequest).

Components, in diffusers parameter names so `unet/`, `vae/` and `image_encoder/` safetensors load as-is:
* UNetSpatioTemporalConditionModel — every ResNet is a spatial ResnetBlock2D followed by a temporal
  ResNet (3x1x1 convs over frames) and a learned alpha blend; every transformer is a spatial
  BasicTransformerBlock (shared with the SD UNet, models/diffusion/unet.py) followed by a temporal
  block (self-attention over the frames of each pixel) and a learned blend;
* AutoencoderKLTemporalDecoder — the SD VAE encoder and a decoder whose ResNets are spatio-temporal
  too, ending in a temporal 3x1x1 conv;
* CLIPVisionModelWithProjection — image embedding (pooled CLS -> post-LN -> projection).

MI355X layout: activations stay frame-major channels_last [B*F, C, H, W] (memory [B, F, H, W, C]).
The temporal ops need no transposes: that memory IS a channels_last [B, C, F, H*W] tensor, so the
temporal GroupNorm is the GroupNorm kernel over (F*H*W) and the 3x1x1 conv is the implicit-GEMM MFMA
conv kernel (conv.hip) with a (3, 1) filter and (1, 0) padding, residual fused into its epilogue.
Only temporal self-attention regroups tokens (frames of one pixel contiguous) for the flash kernel.
Cross-attention to SVD's single image token reduces exactly to a broadcast add of to_out(to_v(ctx))
(softmax over one key is 1), so it costs one [B, C] GEMM instead of B*H*W attention rows.
Sampler: EulerDiscrete, v-prediction, Karras sigmas (0.002 .. 700), continuous timesteps
0.25 * log(sigma) — the scheduler config SVD checkpoints ship; per-frame CFG scale linspace(min, max).
"""
from __future__ import annotations

import json
import math
import os
from dataclasses import dataclass

import numpy as np
import torch
import torch.nn.functional as F
from torch import nn

from .nn import GroupNorm, attention, cast_module, conv, init_synthetic, layernorm16, linear_acc, timestep_embedding
from .unet import BasicTransformerBlock, Downsample2D, FeedForward, TimestepEmbedding, Upsample2D, Attention
from .vae import VAEConfig, _AttnProc, _Encoder


@dataclass
class SVDConfig:
    in_channels: int = 8
    out_channels: int = 4
    channels: tuple = (320, 640, 1280, 1280)
    heads: tuple = (5, 10, 20, 20)
    layers: int = 2
    transformer_layers: tuple = (1, 1, 1, 1)
    cross_dim: int = 1024
    addition_time_dim: int = 256
    projection_dim: int = 768  # 3 added time ids x addition_time_dim
    groups: int = 32
    num_frames: int = 25
    # VAE (AutoencoderKLTemporalDecoder)
    vae_channels: tuple = (128, 256, 512, 512)
    vae_layers: int = 2
    vae_groups: int = 32
    scaling: float = 0.18215
    # image encoder (CLIP ViT-H/14 with projection)
    clip_hidden: int = 1280
    clip_layers: int = 32
    clip_heads: int = 16
    clip_ffn: int = 5120
    clip_patch: int = 14
    clip_image: int = 224
    clip_act: str = "gelu"

    @property
    def temb_dim(self) -> int:
        return self.channels[0] * 4


SVD_XT = SVDConfig()
SVD = SVDConfig(num_frames=14)
SVD_TEST = SVDConfig(channels=(32, 64), heads=(2, 2), layers=1, transformer_layers=(1, 1), cross_dim=48,
                     addition_time_dim=8, projection_dim=24, groups=8, num_frames=4, vae_channels=(32, 32, 64, 64),
                     vae_layers=1, vae_groups=8, clip_hidden=64, clip_layers=2, clip_heads=4, clip_ffn=128,
                     clip_image=28)
PRESETS = {"svd-xt": SVD_XT, "svd": SVD, "svd-test": SVD_TEST}


# ------------------------------------------------------------------------------------------------
# frame-major channels_last <-> temporal views (free on channels_last GPU tensors)
def tview(x: torch.Tensor, B: int) -> torch.Tensor:
    """[B*F, C, H, W] -> [B, C, F, H*W] over the same memory ([B, F, H, W, C])."""
    BF, C, H, W = x.shape
    return x.permute(0, 2, 3, 1).reshape(B, BF // B, H * W, C).permute(0, 3, 1, 2)


def untview(x4: torch.Tensor, H: int, W: int) -> torch.Tensor:
    B, C, Fr, _ = x4.shape
    return x4.permute(0, 2, 3, 1).reshape(B * Fr, H, W, C).permute(0, 3, 1, 2)


class AlphaBlender(nn.Module):
    """diffusers AlphaBlender with merge_strategy learned / learned_with_images (all frames are video
    frames here: image_only_indicator is all zeros). out = a * spatial + (1 - a) * temporal,
    a = sigmoid(mix_factor), or 1 - sigmoid(mix_factor) with switch_spatial_to_temporal_mix."""

    def __init__(self, alpha: float, switch: bool):
        super().__init__()
        self.mix_factor = nn.Parameter(torch.tensor([alpha]))
        self.switch = switch

    def blend(self, spatial: torch.Tensor, temporal: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
        a = torch.sigmoid(self.mix_factor.float())
        if self.switch:
            a = 1.0 - a
        # temporal + a * (spatial - temporal), no host sync on `a`
        r = torch.lerp(temporal.float(), spatial.float(), a.to(spatial.device))
        if out is None:
            return r.to(spatial.dtype)
        out.copy_(r)
        return out


class Conv3x1(nn.Conv3d):
    """Conv3d with a (3, 1, 1) kernel over frames (padding (1, 0, 0)), run as a (3, 1) 2-D conv over the
    temporal view [B, C, F, H*W] on the implicit-GEMM kernel."""

    def __init__(self, cin, cout):
        super().__init__(cin, cout, (3, 1, 1), padding=(1, 0, 0))

    def run(self, x4: torch.Tensor, **fused) -> torch.Tensor:
        w = self.weight.view(self.out_channels, self.in_channels, 3, 1)
        return conv(x4, self, weight=w, pad=(1, 0, 1, 0), stride=1, dilation=1, **fused)


class Res2D(nn.Module):
    """ResnetBlock2D (optional time embedding), eps configurable."""

    def __init__(self, cin, cout, temb, groups, eps):
        super().__init__()
        self.norm1 = GroupNorm(groups, cin, eps=eps)
        self.conv1 = nn.Conv2d(cin, cout, 3, 1, 1)
        self.time_emb_proj = nn.Linear(temb, cout) if temb else None
        self.norm2 = GroupNorm(groups, cout, eps=eps)
        self.conv2 = nn.Conv2d(cout, cout, 3, 1, 1)
        self.conv_shortcut = nn.Conv2d(cin, cout, 1) if cin != cout else None

    def run(self, x, t=None):
        h = conv(self.norm1.run(x, silu=True), self.conv1, **({"tadd": t} if t is not None else {}))
        sc = conv(x, self.conv_shortcut) if self.conv_shortcut is not None else x
        return conv(self.norm2.run(h, silu=True), self.conv2, residual=sc)


class TemporalResnetBlock(nn.Module):
    def __init__(self, c, temb, groups, eps):
        super().__init__()
        self.norm1 = GroupNorm(groups, c, eps=eps)
        self.conv1 = Conv3x1(c, c)
        self.time_emb_proj = nn.Linear(temb, c) if temb else None
        self.norm2 = GroupNorm(groups, c, eps=eps)
        self.conv2 = Conv3x1(c, c)

    def run(self, x4: torch.Tensor, t: torch.Tensor | None) -> torch.Tensor:
        """x4: temporal view [B, C, F, HW]; t: projected per-frame time embedding [B*F, C] or None.
        GroupNorm statistics span all frames of a sample, as in the 5-D reference."""
        B, C, Fr, _ = x4.shape
        h = self.conv1.run(self.norm1.run(x4, silu=True))
        if t is not None:
            h.permute(0, 2, 3, 1).add_(t.view(B, Fr, 1, C).to(h.dtype))
        return self.conv2.run(self.norm2.run(h, silu=True), residual=x4)


class SpatioTemporalResBlock(nn.Module):
    def __init__(self, cin, cout, temb, groups, eps, temporal_eps=None, merge_factor=0.5, learned_with_images=True):
        super().__init__()
        self.spatial_res_block = Res2D(cin, cout, temb, groups, eps)
        self.temporal_res_block = TemporalResnetBlock(cout, temb, groups, temporal_eps or eps)
        self.time_mixer = AlphaBlender(merge_factor, switch=True)

    def run(self, x, B, ts=None, tt=None):
        h = self.spatial_res_block.run(x, ts)
        h4 = tview(h, B)
        t4 = self.temporal_res_block.run(h4, tt)
        self.time_mixer.blend(h4, t4, out=t4)
        return untview(t4, h.shape[2], h.shape[3])


class TimeEmbed(nn.Module):
    """TimestepEmbedding(in, hidden, out_dim)."""

    def __init__(self, cin, hidden, cout):
        super().__init__()
        self.linear_1 = nn.Linear(cin, hidden)
        self.linear_2 = nn.Linear(hidden, cout)

    def run(self, x):
        return self.linear_2(F.silu(self.linear_1(x)))


class TemporalBasicTransformerBlock(nn.Module):
    def __init__(self, dim, heads, cross_dim):
        super().__init__()
        self.norm_in = nn.LayerNorm(dim)
        self.ff_in = FeedForward(dim)
        self.norm1 = nn.LayerNorm(dim)
        self.attn1 = Attention(dim, heads)
        self.norm2 = nn.LayerNorm(dim)
        self.attn2 = Attention(dim, heads, cross_dim)
        self.norm3 = nn.LayerNorm(dim)
        self.ff = FeedForward(dim)

    def _ff(self, ff, norm, x, dt):
        h = layernorm16(x, norm.weight, norm.bias, 1e-5, dt)
        g = F.linear(h, ff.net[0].proj.weight, ff.net[0].proj.bias)
        inner = g.shape[1] // 2
        linear_acc(g[:, :inner] * F.gelu(g[:, inner:]), ff.net[2], x)

    def run(self, h: torch.Tensor, B: int, Fr: int, S: int, tctx: torch.Tensor) -> torch.Tensor:
        """h: fp32 [B*F*S, C] (frame-major); tctx: 16-bit [B, Sc, cross_dim] (first frame's context)."""
        C = h.shape[1]
        dt = tctx.dtype
        x = h.view(B, Fr, S, C).transpose(1, 2).reshape(B * S * Fr, C).contiguous()  # frames of a pixel together
        self._ff(self.ff_in, self.norm_in, x, dt)
        a1 = self.attn1
        H = a1.heads
        D = C // H
        if a1._qkv is None or a1._qkv.device != a1.to_q.weight.device or a1._qkv.dtype != a1.to_q.weight.dtype:
            a1._qkv = torch.cat([a1.to_q.weight, a1.to_k.weight, a1.to_v.weight])
        y = layernorm16(x, self.norm1.weight, self.norm1.bias, 1e-5, dt)
        qkv = F.linear(y, a1._qkv)
        o = attention(qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:], B * S, Fr, Fr, H, D)
        linear_acc(o, a1.to_out[0], x)
        a2 = self.attn2
        Sc = tctx.shape[1]
        if Sc == 1:
            # one context token: softmax == 1, the output is to_out(to_v(ctx)) for every query row
            v = F.linear(tctx.reshape(B, -1), a2.to_v.weight)
            o = F.linear(v, a2.to_out[0].weight, a2.to_out[0].bias).float()
            x.view(B, S * Fr, C).add_(o[:, None, :])
        else:
            y = layernorm16(x, self.norm2.weight, self.norm2.bias, 1e-5, dt)
            q = F.linear(y, a2.to_q.weight)
            kv = F.linear(tctx.reshape(B * Sc, -1), torch.cat([a2.to_k.weight, a2.to_v.weight]))
            kv = kv.view(B, 1, Sc, 2 * C).expand(B, S, Sc, 2 * C).reshape(B * S * Sc, 2 * C)
            o = attention(q, kv[:, :C], kv[:, C:], B * S, Fr, Sc, H, D)
            linear_acc(o, a2.to_out[0], x)
        self._ff(self.ff, self.norm3, x, dt)
        return x.view(B, S, Fr, C).transpose(1, 2).reshape(B * Fr * S, C)


class TransformerSpatioTemporalModel(nn.Module):
    def __init__(self, c: SVDConfig, dim, heads, layers):
        super().__init__()
        self.norm = GroupNorm(c.groups, dim, eps=1e-6)
        self.proj_in = nn.Linear(dim, dim)
        self.transformer_blocks = nn.ModuleList(BasicTransformerBlock(dim, heads, c.cross_dim) for _ in range(layers))
        self.temporal_transformer_blocks = nn.ModuleList(
            TemporalBasicTransformerBlock(dim, heads, c.cross_dim) for _ in range(layers))
        self.time_pos_embed = TimeEmbed(dim, dim * 4, dim)
        self.time_mixer = AlphaBlender(0.5, switch=False)
        self.proj_out = nn.Linear(dim, dim)

    def run(self, x, B, ctx16, key, tctx):
        BF, C, H, W = x.shape
        Fr, S = BF // B, H * W
        tok = self.norm.run(x).permute(0, 2, 3, 1).reshape(BF * S, C)
        h = F.linear(tok, self.proj_in.weight, self.proj_in.bias).float()
        fid = torch.arange(Fr, device=x.device, dtype=torch.float32).repeat(B)
        femb = self.time_pos_embed.run(timestep_embedding(fid, C, True, 0.0).to(x.dtype)).float()  # [BF, C]
        for blk, tblk in zip(self.transformer_blocks, self.temporal_transformer_blocks):
            h = blk.run(h, BF, S, ctx16, key)
            hm = (h.view(BF, S, C) + femb[:, None, :]).view(BF * S, C)
            hm = tblk.run(hm, B, Fr, S, tctx)
            h = self.time_mixer.blend(h, hm)
        o = F.linear(h.to(x.dtype), self.proj_out.weight, self.proj_out.bias)
        return x + o.view(BF, H, W, C).permute(0, 3, 1, 2)


class _Down(nn.Module):
    def __init__(self, c, cin, cout, heads, tl, cross, down):
        super().__init__()
        self.resnets = nn.ModuleList(SpatioTemporalResBlock(cin if i == 0 else cout, cout, c.temb_dim, c.groups, 1e-5)
                                     for i in range(c.layers))
        self.attentions = nn.ModuleList(TransformerSpatioTemporalModel(c, cout, heads, tl)
                                        for _ in range(c.layers)) if cross else None
        self.downsamplers = nn.ModuleList([Downsample2D(cout)]) if down else None


class _Up(nn.Module):
    def __init__(self, c, cin, cout, prev, heads, tl, cross, up):
        super().__init__()
        n = c.layers + 1
        self.resnets = nn.ModuleList(
            SpatioTemporalResBlock((prev if i == 0 else cout) + (cin if i == n - 1 else cout), cout, c.temb_dim,
                                   c.groups, 1e-5) for i in range(n))
        self.attentions = nn.ModuleList(TransformerSpatioTemporalModel(c, cout, heads, tl)
                                        for _ in range(n)) if cross else None
        self.upsamplers = nn.ModuleList([Upsample2D(cout)]) if up else None


class _Mid(nn.Module):
    def __init__(self, c, ch, heads, tl):
        super().__init__()
        self.resnets = nn.ModuleList([SpatioTemporalResBlock(ch, ch, c.temb_dim, c.groups, 1e-5) for _ in range(2)])
        self.attentions = nn.ModuleList([TransformerSpatioTemporalModel(c, ch, heads, tl)])


class UNetSpatioTemporalConditionModel(nn.Module):
    def __init__(self, c: SVDConfig):
        super().__init__()
        self.cfg = c
        ch = c.channels
        n = len(ch)
        self.conv_in = nn.Conv2d(c.in_channels, ch[0], 3, 1, 1)
        self.time_embedding = TimestepEmbedding(ch[0], c.temb_dim)
        self.add_embedding = TimestepEmbedding(c.projection_dim, c.temb_dim)
        self.down_blocks = nn.ModuleList()
        cout = ch[0]
        for i in range(n):
            cin, cout = cout, ch[i]
            self.down_blocks.append(_Down(c, cin, cout, c.heads[i], c.transformer_layers[i], i < n - 1, i < n - 1))
        self.mid_block = _Mid(c, ch[-1], c.heads[-1], c.transformer_layers[-1])
        self.up_blocks = nn.ModuleList()
        rch, rh, rtl = list(reversed(ch)), list(reversed(c.heads)), list(reversed(c.transformer_layers))
        prev = rch[0]
        for i in range(n):
            cout, cin = rch[i], rch[min(i + 1, n - 1)]
            self.up_blocks.append(_Up(c, cin, cout, prev, rh[i], rtl[i], i > 0, i < n - 1))
            prev = cout
        self.conv_norm_out = GroupNorm(c.groups, ch[0], eps=1e-5)
        self.conv_out = nn.Conv2d(ch[0], c.out_channels, 3, 1, 1)
        self._tproj = None

    def _res(self):
        out = []
        for b in self.down_blocks:
            out += list(b.resnets)
        out += list(self.mid_block.resnets)
        for b in self.up_blocks:
            out += list(b.resnets)
        return out

    def _time_proj(self):
        """Every spatial and temporal time_emb_proj stacked: one GEMM per step for the whole net."""
        w0 = self.conv_in.weight
        if self._tproj is None or self._tproj[0].device != w0.device or self._tproj[0].dtype != w0.dtype:
            lins = []
            for r in self._res():
                lins += [r.spatial_res_block.time_emb_proj, r.temporal_res_block.time_emb_proj]
            self._tproj = (torch.cat([m.weight for m in lins]), torch.cat([m.bias for m in lins]),
                           [m.out_features for m in lins])
        return self._tproj

    @torch.no_grad()
    def forward(self, x: torch.Tensor, t: torch.Tensor, ctx: torch.Tensor, time_ids: torch.Tensor,
                ctx_key=None) -> torch.Tensor:
        """x [B, F, Cin, h, w], t [B] (continuous timesteps), ctx [B, Sc, cross_dim] image embeddings,
        time_ids [B, 3] (fps - 1, motion_bucket_id, noise_aug_strength) -> [B, F, Cout, h, w] fp32."""
        c = self.cfg
        B, Fr = x.shape[:2]
        dt = self.conv_in.weight.dtype
        emb = self.time_embedding.run(timestep_embedding(t, c.channels[0], True, 0.0).to(dt))
        aemb = timestep_embedding(time_ids.reshape(-1), c.addition_time_dim, True, 0.0).reshape(B, -1)
        emb = (emb + self.add_embedding.run(aemb.to(dt))).repeat_interleave(Fr, 0)
        w, b, sizes = self._time_proj()
        ti = iter(F.linear(F.silu(emb), w, b).split(sizes, -1))
        ctx16 = ctx.to(dt).repeat_interleave(Fr, 0)  # [BF, Sc, D]
        tctx = ctx.to(dt)  # first frame's context == every frame's (repeated)
        key = ctx_key if ctx_key is not None else ctx
        ctx16 = ctx16.reshape(-1, ctx.shape[-1]).contiguous()
        h = x.reshape(B * Fr, *x.shape[2:]).to(dt)
        h = h.contiguous(memory_format=torch.channels_last) if h.is_cuda else h
        h = conv(h, self.conv_in)
        skips = [h]
        for blk in self.down_blocks:
            for i, r in enumerate(blk.resnets):
                h = r.run(h, B, next(ti), next(ti))
                if blk.attentions is not None:
                    h = blk.attentions[i].run(h, B, ctx16, key, tctx)
                skips.append(h)
            if blk.downsamplers is not None:
                h = conv(h, blk.downsamplers[0].conv)
                skips.append(h)
        m = self.mid_block
        h = m.resnets[0].run(h, B, next(ti), next(ti))
        h = m.attentions[0].run(h, B, ctx16, key, tctx)
        h = m.resnets[1].run(h, B, next(ti), next(ti))
        for blk in self.up_blocks:
            for i, r in enumerate(blk.resnets):
                h = torch.cat([h, skips.pop()], 1)
                if h.is_cuda:
                    h = h.contiguous(memory_format=torch.channels_last)
                h = r.run(h, B, next(ti), next(ti))
                if blk.attentions is not None:
                    h = blk.attentions[i].run(h, B, ctx16, key, tctx)
            if blk.upsamplers is not None:
                h = conv(h, blk.upsamplers[0].conv, upsample=True)
        h = conv(self.conv_norm_out.run(h, silu=True), self.conv_out)
        return h.float().reshape(B, Fr, *h.shape[1:])


# ------------------------------------------------------------------------------------------------
class _TDMid(nn.Module):
    def __init__(self, ch, groups):
        super().__init__()
        self.resnets = nn.ModuleList([SpatioTemporalResBlock(ch, ch, 0, groups, 1e-6, 1e-5, 0.0) for _ in range(2)])
        self.attentions = nn.ModuleList([_AttnProc(ch, groups)])


class _TDUp(nn.Module):
    def __init__(self, cin, cout, n, groups, up):
        super().__init__()
        self.resnets = nn.ModuleList(SpatioTemporalResBlock(cin if i == 0 else cout, cout, 0, groups, 1e-6, 1e-5, 0.0)
                                     for i in range(n))
        self.upsamplers = nn.ModuleList([Upsample2D(cout)]) if up else None


class TemporalDecoder(nn.Module):
    def __init__(self, c: SVDConfig):
        super().__init__()
        ch = list(reversed(c.vae_channels))
        g = c.vae_groups
        self.conv_in = nn.Conv2d(4, ch[0], 3, 1, 1)
        self.mid_block = _TDMid(ch[0], g)
        self.up_blocks = nn.ModuleList(_TDUp(ch[max(0, i - 1)], ch[i], c.vae_layers + 1, g, i < len(ch) - 1)
                                       for i in range(len(ch)))
        self.conv_norm_out = GroupNorm(g, ch[-1], eps=1e-6)
        self.conv_out = nn.Conv2d(ch[-1], 3, 3, 1, 1)
        self.time_conv_out = Conv3x1(3, 3)

    def run(self, z, B):
        x = conv(z, self.conv_in)
        m = self.mid_block
        x = m.resnets[0].run(x, B)
        x = m.attentions[0].run(x)
        x = m.resnets[1].run(x, B)
        for blk in self.up_blocks:
            for r in blk.resnets:
                x = r.run(x, B)
            if blk.upsamplers is not None:
                x = conv(x, blk.upsamplers[0].conv, upsample=True)
        x = conv(self.conv_norm_out.run(x, silu=True), self.conv_out)
        H, W = x.shape[2:]
        return untview(self.time_conv_out.run(tview(x, B)), H, W)


class AutoencoderKLTemporalDecoder(nn.Module):
    def __init__(self, c: SVDConfig):
        super().__init__()
        self.cfg = c
        vc = VAEConfig(latent=4, channels=c.vae_channels, layers=c.vae_layers, groups=c.vae_groups, scaling=c.scaling,
                       shift=0.0)
        self.encoder = _Encoder(vc)
        self.quant_conv = nn.Conv2d(8, 8, 1)
        self.decoder = TemporalDecoder(c)

    def _nhwc(self, x):
        x = x.to(self.decoder.conv_in.weight.dtype)
        return x.contiguous(memory_format=torch.channels_last) if x.is_cuda else x

    @torch.no_grad()
    def encode_mode(self, img: torch.Tensor) -> torch.Tensor:
        """image [-1, 1] [B, 3, H, W] -> posterior mode (unscaled, as the SVD pipeline conditions on it)."""
        e = self.encoder
        x = conv(self._nhwc(img), e.conv_in)
        for blk in e.down_blocks:
            x = blk.run(x)
        x = e.mid_block.run(x)
        x = conv(conv(e.conv_norm_out.run(x, silu=True), e.conv_out), self.quant_conv)
        return x.float()[:, :4]

    @torch.no_grad()
    def decode(self, z: torch.Tensor, num_frames: int) -> torch.Tensor:
        """z [B*F, 4, h, w] (already divided by the scaling factor), frames of one clip consecutive."""
        return self.decoder.run(self._nhwc(z), z.shape[0] // num_frames).float()


# ------------------------------------------------------------------------------------------------
class ClipImageEncoder(nn.Module):
    """CLIPVisionModelWithProjection (HF names under vision_model.* + visual_projection): pooled CLS
    embedding -> projection. The encoder blocks run on the dense flash-attention kernel."""

    def __init__(self, c: SVDConfig):
        super().__init__()
        H = c.clip_hidden
        self.cfg = c
        vm = nn.Module()
        vm.embeddings = nn.Module()
        vm.embeddings.patch_embedding = nn.Conv2d(3, H, c.clip_patch, c.clip_patch, bias=False)
        vm.embeddings.class_embedding = nn.Parameter(torch.zeros(H))
        vm.embeddings.position_embedding = nn.Embedding((c.clip_image // c.clip_patch) ** 2 + 1, H)
        vm.pre_layrnorm = nn.LayerNorm(H)
        vm.encoder = nn.Module()
        layers = nn.ModuleList()
        for _ in range(c.clip_layers):
            L = nn.Module()
            L.self_attn = nn.Module()
            for n in ("q_proj", "k_proj", "v_proj", "out_proj"):
                setattr(L.self_attn, n, nn.Linear(H, H))
            L.layer_norm1, L.layer_norm2 = nn.LayerNorm(H), nn.LayerNorm(H)
            L.mlp = nn.Module()
            L.mlp.fc1, L.mlp.fc2 = nn.Linear(H, c.clip_ffn), nn.Linear(c.clip_ffn, H)
            layers.append(L)
        vm.encoder.layers = layers
        vm.post_layernorm = nn.LayerNorm(H)
        self.vision_model = vm
        self.visual_projection = nn.Linear(H, c.cross_dim, bias=False)

    MEAN = (0.48145466, 0.4578275, 0.40821073)
    STD = (0.26862954, 0.26130258, 0.27577711)

    @torch.no_grad()
    def embed(self, img: torch.Tensor) -> torch.Tensor:
        """img [-1, 1] [B, 3, H, W] -> [B, cross_dim] (SVD: antialiased resize of the whole frame to the
        CLIP resolution, no crop, then CLIP normalisation)."""
        c = self.cfg
        vm = self.vision_model
        dt = vm.embeddings.patch_embedding.weight.dtype
        x = F.interpolate(img.float(), size=(c.clip_image, c.clip_image), mode="bicubic", align_corners=False,
                          antialias=True)
        x = (x + 1.0) / 2.0
        mean = torch.tensor(self.MEAN, device=x.device)[:, None, None]
        std = torch.tensor(self.STD, device=x.device)[:, None, None]
        x = ((x - mean) / std).to(dt)
        B = x.shape[0]
        H = c.clip_hidden
        pe = F.conv2d(x, vm.embeddings.patch_embedding.weight, stride=c.clip_patch).flatten(2).transpose(1, 2)
        h = torch.cat([vm.embeddings.class_embedding.to(pe.dtype).view(1, 1, H).expand(B, 1, H), pe], 1).float()
        h = h + vm.embeddings.position_embedding.weight.float()[None]
        S = h.shape[1]
        h = F.layer_norm(h, (H,), vm.pre_layrnorm.weight, vm.pre_layrnorm.bias, 1e-5).reshape(B * S, H).contiguous()
        nh = c.clip_heads
        for L in vm.encoder.layers:
            a = L.self_attn
            y = layernorm16(h, L.layer_norm1.weight, L.layer_norm1.bias, 1e-5, dt)
            q, k, v = (F.linear(y, m.weight, m.bias) for m in (a.q_proj, a.k_proj, a.v_proj))
            linear_acc(attention(q, k, v, B, S, S, nh, H // nh), a.out_proj, h)
            y = layernorm16(h, L.layer_norm2.weight, L.layer_norm2.bias, 1e-5, dt)
            u = F.linear(y, L.mlp.fc1.weight, L.mlp.fc1.bias)
            u = F.gelu(u) if c.clip_act == "gelu" else u * torch.sigmoid(1.702 * u)
            linear_acc(u, L.mlp.fc2, h)
        cls = h.view(B, S, H)[:, 0]
        pooled = F.layer_norm(cls, (H,), vm.post_layernorm.weight, vm.post_layernorm.bias, 1e-5)
        return F.linear(pooled.to(dt), self.visual_projection.weight).float()


# ------------------------------------------------------------------------------------------------
def karras_sigmas(n: int, sigma_min: float = 0.002, sigma_max: float = 700.0, rho: float = 7.0) -> list[float]:
    ramp = np.linspace(0, 1, n)
    lo, hi = sigma_min ** (1 / rho), sigma_max ** (1 / rho)
    return [float(s) for s in (hi + ramp * (lo - hi)) ** rho] + [0.0]


@dataclass
class VideoParams:
    width: int = 1024
    height: int = 576
    num_frames: int = 0  # 0: the model's default (14 / 25)
    steps: int = 25
    fps: int = 7
    motion_bucket_id: int = 127
    noise_aug_strength: float = 0.02
    min_guidance: float = 1.0
    max_guidance: float = 3.0
    seed: int = 0
    decode_chunk: int = 8


class SVDPipeline:
    """img2vid: conditioning image -> list of PIL frames."""

    def __init__(self, cfg: SVDConfig, unet, vae, image_encoder, device, dtype):
        self.cfg, self.unet, self.vae, self.image_encoder = cfg, unet, vae, image_encoder
        self.device, self.dtype = torch.device(device), dtype

    @classmethod
    def _build(cls, cfg: SVDConfig, device, sds: dict | None, seed: int = 0):
        dev = torch.device(device)
        dtype = torch.float16 if dev.type == "cuda" else torch.float32
        parts = {"unet": UNetSpatioTemporalConditionModel(cfg), "vae": AutoencoderKLTemporalDecoder(cfg),
                 "image_encoder": ClipImageEncoder(cfg)}
        for i, (name, m) in enumerate(parts.items()):
            if sds is None:
                init_synthetic(m, seed + i)
                for mod in m.modules():  # mixers at their construction default, as an untrained checkpoint
                    if isinstance(mod, AlphaBlender):
                        mod.mix_factor.data.fill_(0.0)
            else:
                missing, unexpected = m.load_state_dict(sds[name], strict=False)
                missing = [k for k in missing if not k.endswith("_mx_conv_pack")]
                if missing:
                    raise ValueError(f"{name}: missing {len(missing)} tensors, e.g. {missing[:4]}")
            cast_module(m.eval(), dev, dtype)
        return cls(cfg, parts["unet"], parts["vae"], parts["image_encoder"], dev, dtype)

    @classmethod
    def synthetic(cls, name: str, device, seed: int = 0) -> "SVDPipeline":
        return cls._build(PRESETS[name], device, None, seed)

    @classmethod
    def from_diffusers(cls, path: str, device) -> "SVDPipeline":
        from safetensors.torch import load_file

        def cfg_of(sub):
            with open(os.path.join(path, sub, "config.json")) as f:
                return json.load(f)

        def sd_of(sub):
            d = os.path.join(path, sub)
            files = sorted(f for f in os.listdir(d) if f.endswith(".safetensors"))
            if not files:
                raise FileNotFoundError(f"{d}: no .safetensors weights")
            pref = [f for f in files if ".fp16." in f] or files
            sd = {}
            for f in pref:
                sd.update(load_file(os.path.join(d, f)))
            return sd
        u, v, ie = cfg_of("unet"), cfg_of("vae"), cfg_of("image_encoder")
        ch = tuple(u["block_out_channels"])
        heads = u.get("num_attention_heads", (5, 10, 20, 20))
        tl = u.get("transformer_layers_per_block", 1)
        cfg = SVDConfig(in_channels=u.get("in_channels", 8), out_channels=u.get("out_channels", 4), channels=ch,
                        heads=tuple(heads) if isinstance(heads, (list, tuple)) else (heads,) * len(ch),
                        layers=u.get("layers_per_block", 2),
                        transformer_layers=tuple(tl) if isinstance(tl, (list, tuple)) else (tl,) * len(ch),
                        cross_dim=u.get("cross_attention_dim", 1024),
                        addition_time_dim=u.get("addition_time_embed_dim", 256),
                        projection_dim=u.get("projection_class_embeddings_input_dim", 768),
                        num_frames=u.get("num_frames", 25), vae_channels=tuple(v["block_out_channels"]),
                        vae_layers=v.get("layers_per_block", 2), scaling=v.get("scaling_factor", 0.18215),
                        clip_hidden=ie["hidden_size"], clip_layers=ie["num_hidden_layers"],
                        clip_heads=ie["num_attention_heads"], clip_ffn=ie["intermediate_size"],
                        clip_patch=ie["patch_size"], clip_image=ie["image_size"],
                        clip_act="gelu" if ie.get("hidden_act", "gelu") == "gelu" else "quick_gelu")
        if ie.get("projection_dim", cfg.cross_dim) != cfg.cross_dim:
            raise ValueError("image encoder projection_dim != unet cross_attention_dim")
        return cls._build(cfg, device, {"unet": sd_of("unet"), "vae": sd_of("vae"), "image_encoder": sd_of("image_encoder")})

    @torch.no_grad()
    def generate(self, image, p: VideoParams) -> list:
        """image: PIL image or [3, H, W] tensor in [-1, 1] -> p.num_frames PIL frames."""
        from PIL import Image
        c = self.cfg
        dev = self.device
        Fr = p.num_frames or c.num_frames
        W, H = (p.width // 64) * 64 or 64, (p.height // 64) * 64 or 64
        if isinstance(image, Image.Image):
            im = image.convert("RGB").resize((W, H), Image.BICUBIC)
            img = torch.from_numpy(np.asarray(im, dtype=np.float32) / 127.5 - 1.0).permute(2, 0, 1)
        else:
            img = F.interpolate(image[None].float(), size=(H, W), mode="bicubic", align_corners=False)[0]
        img = img[None].to(dev)
        gen = torch.Generator(device="cpu").manual_seed(int(p.seed))
        emb = self.image_encoder.embed(img)[:, None, :]  # [1, 1, D]
        noisy = img + p.noise_aug_strength * torch.randn(img.shape, generator=gen).to(dev)
        lat_img = self.vae.encode_mode(noisy)  # [1, 4, h, w]
        h, w = lat_img.shape[2:]
        # classifier-free guidance batch: [uncond (zero image embedding + zero latents), cond]
        ctx = torch.cat([torch.zeros_like(emb), emb])
        cond = torch.cat([torch.zeros_like(lat_img), lat_img])[:, None].expand(2, Fr, 4, h, w)
        tid = torch.tensor([[p.fps - 1, p.motion_bucket_id, p.noise_aug_strength]] * 2, dtype=torch.float32, device=dev)
        gs = torch.linspace(p.min_guidance, p.max_guidance, Fr, device=dev).view(1, Fr, 1, 1, 1)
        sig = karras_sigmas(p.steps)
        x = torch.randn((1, Fr, 4, h, w), generator=gen).to(dev) * math.sqrt(sig[0] ** 2 + 1.0)
        key = object()  # cross-attention K|V of the (fixed) image context cached across steps
        for i in range(p.steps):
            s, sn = sig[i], sig[i + 1]
            cin = 1.0 / math.sqrt(s * s + 1.0)
            xin = torch.cat([(x * cin).expand(2, Fr, 4, h, w), cond], 2)
            t = torch.full((2,), 0.25 * math.log(s), device=dev)
            out = self.unet(xin, t, ctx, tid, ctx_key=key)
            v = out[:1] + gs * (out[1:] - out[:1])
            den = v * (-s / math.sqrt(s * s + 1.0)) + x / (s * s + 1.0)  # v-prediction -> x0
            x = x + (x - den) / s * (sn - s)
        z = x[0] / c.scaling
        frames = []
        for j in range(0, Fr, max(1, p.decode_chunk)):
            chunk = z[j:j + p.decode_chunk]
            frames.append(self.vae.decode(chunk, chunk.shape[0]))
        vid = torch.cat(frames).clamp(-1, 1)
        arr = ((vid + 1.0) * 127.5).round().to(torch.uint8).permute(0, 2, 3, 1).cpu().numpy()
        return [Image.fromarray(a) for a in arr]


__all__ = ["SVDConfig", "SVD", "SVD_XT", "SVD_TEST", "PRESETS", "SVDPipeline", "VideoParams",
           "UNetSpatioTemporalConditionModel", "AutoencoderKLTemporalDecoder", "ClipImageEncoder", "karras_sigmas"]
