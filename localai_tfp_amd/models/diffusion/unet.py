"""UNet2DConditionModel — the denoiser of SD 1.x / 2.x / SDXL (the reference's stablediffusion-ggml
and diffusers backends: gosd.cpp:56-226 txt2img, backend/python/diffusers/backend.py:139-270
StableDiffusionPipeline / StableDiffusionXLPipeline). diffusers parameter names, so a
`unet/diffusion_pytorch_model.safetensors` state dict loads directly.

MI355X execution (NHWC / channels_last 16-bit activations end to end, like the VAE):
* ResNet blocks: GroupNorm+SiLU fused (diffusion.hip groupnorm16) -> MIOpen conv; the time
  embedding projection of EVERY ResNet block of the net comes from one batched GEMM of silu(temb)
  against the concatenated `time_emb_proj` weights (one launch instead of ~22);
* spatial transformers: the token stream of an NHWC feature map is a free [B*H*W, C] view; the
  residual stream is fp32, LayerNorms (norm.hip) emit 16-bit GEMM operands, self-attention Q|K|V is
  one fused GEMM, cross-attention K|V of the (fixed) text context are computed once per block per
  generation and cached across sampler steps, attention runs on the MFMA flash kernel
  (attention_dense.hip; head dims 40/64/80/128) or SDPA for SD1.x's 160-wide heads, GEGLU is one
  GEMM + a fused gate;
* skip connections are concatenated in channels_last (one copy per up-block resnet).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import torch
import torch.nn.functional as F
from torch import nn

from .nn import GroupNorm, attention, cat_w, conv, layernorm16, lin, linear_acc, timestep_embedding


@dataclass
class UNetConfig:
    in_channels: int = 4
    out_channels: int = 4
    channels: tuple = (320, 640, 1280, 1280)
    down_types: tuple = ("CrossAttnDownBlock2D",) * 3 + ("DownBlock2D",)
    up_types: tuple = ("UpBlock2D",) + ("CrossAttnUpBlock2D",) * 3
    layers: int = 2
    heads: tuple = (8, 8, 8, 8)  # attention heads per block (diffusers' `attention_head_dim` for SD1.x)
    transformer_layers: tuple = (1, 1, 1, 1)
    cross_dim: int = 768
    linear_proj: bool = False  # use_linear_projection (SD2 / SDXL)
    groups: int = 32
    addition_embed: str = ""  # "text_time" for SDXL
    addition_time_dim: int = 256
    projection_class_dim: int = 0  # SDXL: 2816 = pooled 1280 + 6 * 256
    mid_transformer_layers: int = 1
    sample_size: int = 64
    extra: dict = field(default_factory=dict)

    @property
    def temb_dim(self) -> int:
        return self.channels[0] * 4


SD15_UNET = UNetConfig()
SDXL_UNET = UNetConfig(channels=(320, 640, 1280), down_types=("DownBlock2D", "CrossAttnDownBlock2D", "CrossAttnDownBlock2D"),
                       up_types=("CrossAttnUpBlock2D", "CrossAttnUpBlock2D", "UpBlock2D"), heads=(5, 10, 20),
                       transformer_layers=(1, 2, 10), cross_dim=2048, linear_proj=True, addition_embed="text_time",
                       projection_class_dim=2816, mid_transformer_layers=10, sample_size=128)
UNET_TEST = UNetConfig(channels=(32, 64), down_types=("CrossAttnDownBlock2D", "DownBlock2D"),
                       up_types=("UpBlock2D", "CrossAttnUpBlock2D"), heads=(2, 2), transformer_layers=(1, 1),
                       cross_dim=32, groups=8, layers=1, sample_size=16)
UNET_XL_TEST = UNetConfig(channels=(32, 64), down_types=("DownBlock2D", "CrossAttnDownBlock2D"),
                          up_types=("CrossAttnUpBlock2D", "UpBlock2D"), heads=(2, 2), transformer_layers=(1, 2),
                          cross_dim=48, groups=8, layers=1, linear_proj=True, addition_embed="text_time",
                          addition_time_dim=8, projection_class_dim=32 + 6 * 8, mid_transformer_layers=2,
                          sample_size=16)


# ------------------------------------------------------------------------------------------------
class TimestepEmbedding(nn.Module):
    def __init__(self, cin, dim):
        super().__init__()
        self.linear_1 = nn.Linear(cin, dim)
        self.linear_2 = nn.Linear(dim, dim)

    def run(self, x):
        return self.linear_2(F.silu(self.linear_1(x)))


class ResnetBlock2D(nn.Module):
    def __init__(self, cin, cout, temb, groups):
        super().__init__()
        self.norm1 = GroupNorm(groups, cin, eps=1e-5)
        self.conv1 = nn.Conv2d(cin, cout, 3, 1, 1)
        self.time_emb_proj = nn.Linear(temb, cout)
        self.norm2 = GroupNorm(groups, cout, eps=1e-5)
        self.conv2 = nn.Conv2d(cout, cout, 3, 1, 1)
        self.conv_shortcut = nn.Conv2d(cin, cout, 1) if cin != cout else None

    def run(self, x, t):
        """t: this block's projected time embedding [B, cout] (batched with all other blocks)."""
        h = conv(self.norm1.run(x, silu=True), self.conv1, tadd=t)
        sc = conv(x, self.conv_shortcut) if self.conv_shortcut is not None else x
        return conv(self.norm2.run(h, silu=True), self.conv2, residual=sc)


class Attention(nn.Module):
    def __init__(self, dim, heads, kv_dim=None):
        super().__init__()
        kv_dim = kv_dim or dim
        self.heads = heads
        self.to_q = nn.Linear(dim, dim, bias=False)
        self.to_k = nn.Linear(kv_dim, dim, bias=False)
        self.to_v = nn.Linear(kv_dim, dim, bias=False)
        self.to_out = nn.ModuleList([nn.Linear(dim, dim)])
        self._qkv = None
        self._kv = None


class GEGLU(nn.Module):
    def __init__(self, dim, inner):
        super().__init__()
        self.proj = nn.Linear(dim, inner * 2)


class FeedForward(nn.Module):
    def __init__(self, dim):
        super().__init__()
        self.net = nn.ModuleList([GEGLU(dim, dim * 4), nn.Identity(), nn.Linear(dim * 4, dim)])


class BasicTransformerBlock(nn.Module):
    def __init__(self, dim, heads, cross_dim):
        super().__init__()
        self.norm1 = nn.LayerNorm(dim)
        self.attn1 = Attention(dim, heads)
        self.norm2 = nn.LayerNorm(dim)
        self.attn2 = Attention(dim, heads, cross_dim)
        self.norm3 = nn.LayerNorm(dim)
        self.ff = FeedForward(dim)

    def run(self, x, B, S, ctx, ctx_key):
        """x: fp32 residual stream [B*S, C]; ctx: 16-bit [B*Sc, cross_dim]."""
        C = x.shape[1]
        H = self.attn1.heads
        D = C // H
        dt = ctx.dtype
        a1 = self.attn1
        if a1._qkv is None or a1._qkv.device != a1.to_q.weight.device or a1._qkv.dtype != a1.to_q.weight.dtype:
            a1._qkv = cat_w([a1.to_q.weight, a1.to_k.weight, a1.to_v.weight])
        h = layernorm16(x, self.norm1.weight, self.norm1.bias, 1e-5, dt)
        qkv = lin(h, a1._qkv)
        o = attention(qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:], B, S, S, H, D)
        linear_acc(o, a1.to_out[0], x)
        a2 = self.attn2
        Sc = ctx.shape[0] // B
        if a2._kv is None or a2._kv[0] is not ctx_key or a2._kv[1].device != ctx.device:
            # text K|V: once per generation, reused every sampler step
            wkv = cat_w([a2.to_k.weight, a2.to_v.weight])
            a2._kv = (ctx_key, lin(ctx, wkv))
        kv = a2._kv[1]
        h = layernorm16(x, self.norm2.weight, self.norm2.bias, 1e-5, dt)
        q = lin(h, a2.to_q.weight)
        o = attention(q, kv[:, :C], kv[:, C:], B, S, Sc, H, D)
        linear_acc(o, a2.to_out[0], x)
        h = layernorm16(x, self.norm3.weight, self.norm3.bias, 1e-5, dt)
        g = lin(h, self.ff.net[0].proj.weight, self.ff.net[0].proj.bias)
        inner = g.shape[1] // 2
        u = g[:, :inner] * F.gelu(g[:, inner:])
        linear_acc(u, self.ff.net[2], x)
        return x


class Transformer2DModel(nn.Module):
    def __init__(self, c: UNetConfig, dim, heads, layers):
        super().__init__()
        self.linear = c.linear_proj
        self.norm = GroupNorm(c.groups, dim, eps=1e-6)
        self.proj_in = nn.Linear(dim, dim) if c.linear_proj else nn.Conv2d(dim, dim, 1)
        self.transformer_blocks = nn.ModuleList(BasicTransformerBlock(dim, heads, c.cross_dim) for _ in range(layers))
        self.proj_out = nn.Linear(dim, dim) if c.linear_proj else nn.Conv2d(dim, dim, 1)

    def _lin(self, t, m):
        if isinstance(m, nn.Linear):
            return lin(t, m.weight, m.bias)
        return lin(t, m.weight.reshape(m.weight.shape[0], -1), m.bias)  # 1x1 conv on NHWC tokens

    def run(self, x, ctx, ctx_key):
        B, C, H, W = x.shape
        tok = self.norm.run(x).permute(0, 2, 3, 1).reshape(B * H * W, C)  # channels_last -> free view
        h = self._lin(tok, self.proj_in).float()
        for blk in self.transformer_blocks:
            h = blk.run(h, B, H * W, ctx, ctx_key)
        o = self._lin(h.to(x.dtype), self.proj_out)
        return x + o.view(B, H, W, C).permute(0, 3, 1, 2)


class Downsample2D(nn.Module):
    def __init__(self, c):
        super().__init__()
        self.conv = nn.Conv2d(c, c, 3, 2, 1)


class Upsample2D(nn.Module):
    def __init__(self, c):
        super().__init__()
        self.conv = nn.Conv2d(c, c, 3, 1, 1)


class DownBlock(nn.Module):
    def __init__(self, c: UNetConfig, cin, cout, heads, tl, cross: bool, down: bool):
        super().__init__()
        self.resnets = nn.ModuleList(ResnetBlock2D(cin if i == 0 else cout, cout, c.temb_dim, c.groups)
                                     for i in range(c.layers))
        self.attentions = nn.ModuleList(Transformer2DModel(c, cout, heads, tl) for _ in range(c.layers)) if cross else None
        self.downsamplers = nn.ModuleList([Downsample2D(cout)]) if down else None


class UpBlock(nn.Module):
    def __init__(self, c: UNetConfig, cin, cout, prev, heads, tl, cross: bool, up: bool):
        super().__init__()
        n = c.layers + 1
        res = []
        for i in range(n):
            skip = cin if i == n - 1 else cout
            rin = prev if i == 0 else cout
            res.append(ResnetBlock2D(rin + skip, cout, c.temb_dim, c.groups))
        self.resnets = nn.ModuleList(res)
        self.attentions = nn.ModuleList(Transformer2DModel(c, cout, heads, tl) for _ in range(n)) if cross else None
        self.upsamplers = nn.ModuleList([Upsample2D(cout)]) if up else None


class MidBlock(nn.Module):
    def __init__(self, c: UNetConfig, ch, heads, tl):
        super().__init__()
        self.resnets = nn.ModuleList([ResnetBlock2D(ch, ch, c.temb_dim, c.groups),
                                      ResnetBlock2D(ch, ch, c.temb_dim, c.groups)])
        self.attentions = nn.ModuleList([Transformer2DModel(c, ch, heads, tl)])


class UNet2DConditionModel(nn.Module):
    def __init__(self, c: UNetConfig):
        super().__init__()
        self.cfg = c
        ch = c.channels
        self.conv_in = nn.Conv2d(c.in_channels, ch[0], 3, 1, 1)
        self.time_embedding = TimestepEmbedding(ch[0], c.temb_dim)
        if c.addition_embed == "text_time":
            self.add_embedding = TimestepEmbedding(c.projection_class_dim, c.temb_dim)
        self.down_blocks = nn.ModuleList()
        cout = ch[0]
        for i, t in enumerate(c.down_types):
            cin, cout = cout, ch[i]
            self.down_blocks.append(DownBlock(c, cin, cout, c.heads[i], c.transformer_layers[i],
                                              t.startswith("CrossAttn"), i < len(ch) - 1))
        self.mid_block = MidBlock(c, ch[-1], c.heads[-1], c.mid_transformer_layers)
        self.up_blocks = nn.ModuleList()
        rch, rheads, rtl = list(reversed(ch)), list(reversed(c.heads)), list(reversed(c.transformer_layers))
        prev = rch[0]
        for i, t in enumerate(c.up_types):
            cout = rch[i]
            cin = rch[min(i + 1, len(ch) - 1)]
            self.up_blocks.append(UpBlock(c, cin, cout, prev, rheads[i], rtl[i], t.startswith("CrossAttn"),
                                          i < len(ch) - 1))
            prev = cout
        self.conv_norm_out = GroupNorm(c.groups, ch[0], eps=1e-5)
        self.conv_out = nn.Conv2d(ch[0], c.out_channels, 3, 1, 1)
        self._tproj = None

    def _resnets(self):
        out = []
        for b in self.down_blocks:
            out += list(b.resnets)
        out += list(self.mid_block.resnets)
        for b in self.up_blocks:
            out += list(b.resnets)
        return out

    def _time_proj(self):
        """All ResNet time_emb_proj weights stacked: one GEMM per step for the whole net."""
        if self._tproj is None or self._tproj[0].device != self.conv_in.weight.device \
                or self._tproj[0].dtype != self.conv_in.weight.dtype:  # (re)built after .to() / cast
            rs = self._resnets()
            w = torch.cat([r.time_emb_proj.weight for r in rs])
            b = torch.cat([r.time_emb_proj.bias for r in rs])
            sizes = [r.time_emb_proj.out_features for r in rs]
            self._tproj = (w, b, sizes)
        return self._tproj

    def _prologue(self, x, t, ctx, added, ctx_key):
        """Time (+SDXL text_time) embedding -> per-ResNet projections (one GEMM), fp16 context, input."""
        c = self.cfg
        dt = self.conv_in.weight.dtype
        B = x.shape[0]
        temb = timestep_embedding(t, c.channels[0], flip_sin_to_cos=True, shift=0.0)
        emb = self.time_embedding.run(temb.to(dt))
        if c.addition_embed == "text_time":
            tid = timestep_embedding(added["time_ids"].reshape(-1), c.addition_time_dim, True, 0.0).reshape(B, -1)
            emb = emb + self.add_embedding.run(torch.cat([added["text_embeds"], tid], -1).to(dt))
        w, b, sizes = self._time_proj()
        tp = lin(F.silu(emb), w, b).split(sizes, -1)
        ti = iter(tp)
        ctx16 = ctx.reshape(-1, ctx.shape[-1]).to(dt).contiguous()
        key = ctx_key if ctx_key is not None else ctx
        h = x.to(dt)
        h = h.contiguous(memory_format=torch.channels_last) if h.is_cuda else h
        return ti, ctx16, key, h

    def _encode(self, h, ti, ctx16, key):
        """conv_in output -> (skip activations, mid-block output): the part ControlNet shares."""
        skips = [h]
        for blk in self.down_blocks:
            for i, r in enumerate(blk.resnets):
                h = r.run(h, next(ti))
                if blk.attentions is not None:
                    h = blk.attentions[i].run(h, ctx16, key)
                skips.append(h)
            if blk.downsamplers is not None:
                h = conv(h, blk.downsamplers[0].conv)
                skips.append(h)
        m = self.mid_block
        h = m.resnets[0].run(h, next(ti))
        h = m.attentions[0].run(h, ctx16, key)
        h = m.resnets[1].run(h, next(ti))
        return skips, h

    @torch.no_grad()
    def forward(self, x: torch.Tensor, t: torch.Tensor, ctx: torch.Tensor, added: dict | None = None,
                ctx_key=None, control: tuple | None = None) -> torch.Tensor:
        """x [B, Cin, h, w] fp32 (scaled input), t [B] timesteps, ctx [B, S, cross_dim] -> eps fp32.
        control = (down residuals, mid residual) from ControlNetModel, added to the skips / mid output."""
        ti, ctx16, key, h = self._prologue(x, t, ctx, added, ctx_key)
        skips, h = self._encode(conv(h, self.conv_in), ti, ctx16, key)
        if control is not None:
            skips = [s + r for s, r in zip(skips, control[0])]
            h = h + control[1]
        for blk in self.up_blocks:
            for i, r in enumerate(blk.resnets):
                s = skips.pop()
                h = torch.cat([h, s], 1)
                if h.is_cuda:
                    h = h.contiguous(memory_format=torch.channels_last)
                h = r.run(h, next(ti))
                if blk.attentions is not None:
                    h = blk.attentions[i].run(h, ctx16, key)
            if blk.upsamplers is not None:
                h = conv(h, blk.upsamplers[0].conv, upsample=True)  # nearest 2x fused into the conv
        h = conv(self.conv_norm_out.run(h, silu=True), self.conv_out)
        return h.float()


def config_from_diffusers(d: dict) -> UNetConfig:
    ch = tuple(d["block_out_channels"])
    ahd = d.get("attention_head_dim", 8)
    nah = d.get("num_attention_heads")
    heads = nah if nah is not None else ahd
    heads = tuple(heads) if isinstance(heads, (list, tuple)) else (heads,) * len(ch)
    tl = d.get("transformer_layers_per_block", 1)
    tl = tuple(tl) if isinstance(tl, (list, tuple)) else (tl,) * len(ch)
    return UNetConfig(in_channels=d.get("in_channels", 4), out_channels=d.get("out_channels", 4), channels=ch,
                      down_types=tuple(d["down_block_types"]),
                      up_types=tuple(d.get("up_block_types") or  # ControlNet configs have no decoder
                                     [t.replace("Down", "Up") for t in reversed(d["down_block_types"])]),
                      layers=d.get("layers_per_block", 2), heads=heads, transformer_layers=tl,
                      cross_dim=d.get("cross_attention_dim", 768), linear_proj=d.get("use_linear_projection", False),
                      groups=d.get("norm_num_groups", 32), addition_embed=d.get("addition_embed_type") or "",
                      addition_time_dim=d.get("addition_time_embed_dim") or 256,
                      projection_class_dim=d.get("projection_class_embeddings_input_dim") or 0,
                      mid_transformer_layers=tl[-1], sample_size=d.get("sample_size", 64))


__all__ = ["UNetConfig", "UNet2DConditionModel", "SD15_UNET", "SDXL_UNET", "UNET_TEST", "UNET_XL_TEST",
           "config_from_diffusers", "math"]
