"""AutoencoderKL (SD1.x/2.x/SDXL: 4 latent channels; SD3/Flux: 16) — decoder for txt2img and
encoder for img2img. diffusers parameter names. NHWC (channels_last) 16-bit activations end to end:
MIOpen convolutions, GroupNorm(+SiLU) from diffusion.hip, nearest 2x upsampling, one single-head
spatial attention in the mid block (head width = channels)."""
from __future__ import annotations

from dataclasses import dataclass

import torch
import torch.nn.functional as F
from torch import nn

from .nn import GroupNorm, attention, conv


@dataclass
class VAEConfig:
    latent: int = 16
    channels: tuple = (128, 256, 512, 512)
    layers: int = 2
    groups: int = 32
    scaling: float = 1.5305
    shift: float = 0.0609
    quant_conv: bool = False


VAE_SD3 = VAEConfig()
VAE_SD15 = VAEConfig(latent=4, scaling=0.18215, shift=0.0, quant_conv=True)
VAE_TEST = VAEConfig(latent=16, channels=(32, 32, 64, 64), layers=1, groups=8)


class Resnet(nn.Module):
    def __init__(self, cin, cout, groups):
        super().__init__()
        self.norm1 = GroupNorm(groups, cin, eps=1e-6)
        self.conv1 = nn.Conv2d(cin, cout, 3, 1, 1)
        self.norm2 = GroupNorm(groups, cout, eps=1e-6)
        self.conv2 = nn.Conv2d(cout, cout, 3, 1, 1)
        self.conv_shortcut = nn.Conv2d(cin, cout, 1) if cin != cout else None

    def run(self, x):
        h = conv(self.norm1.run(x, silu=True), self.conv1)
        sc = conv(x, self.conv_shortcut) if self.conv_shortcut is not None else x
        return conv(self.norm2.run(h, silu=True), self.conv2, residual=sc)


class _AttnProc(nn.Module):
    def __init__(self, c, groups):
        super().__init__()
        self.group_norm = GroupNorm(groups, c, eps=1e-6)
        self.to_q, self.to_k, self.to_v = nn.Linear(c, c), nn.Linear(c, c), nn.Linear(c, c)
        self.to_out = nn.ModuleList([nn.Linear(c, c)])

    def run(self, x):
        B, C, H, W = x.shape
        h = self.group_norm.run(x)
        t = h.permute(0, 2, 3, 1).reshape(B * H * W, C)  # NHWC memory -> free view
        q, k, v = F.linear(t, self.to_q.weight, self.to_q.bias), F.linear(t, self.to_k.weight, self.to_k.bias), \
            F.linear(t, self.to_v.weight, self.to_v.bias)
        o = attention(q, k, v, B, H * W, H * W, 1, C)
        o = F.linear(o, self.to_out[0].weight, self.to_out[0].bias)
        return x + o.view(B, H, W, C).permute(0, 3, 1, 2)


class _Mid(nn.Module):
    def __init__(self, c, groups):
        super().__init__()
        self.resnets = nn.ModuleList([Resnet(c, c, groups), Resnet(c, c, groups)])
        self.attentions = nn.ModuleList([_AttnProc(c, groups)])

    def run(self, x):
        x = self.resnets[0].run(x)
        x = self.attentions[0].run(x)
        return self.resnets[1].run(x)


class _Sampler(nn.Module):
    def __init__(self, c, down: bool):
        super().__init__()
        self.conv = nn.Conv2d(c, c, 3, 2 if down else 1, 0 if down else 1)


class _UpBlock(nn.Module):
    def __init__(self, cin, cout, n, groups, up: bool):
        super().__init__()
        self.resnets = nn.ModuleList(Resnet(cin if i == 0 else cout, cout, groups) for i in range(n))
        self.upsamplers = nn.ModuleList([_Sampler(cout, False)]) if up else None

    def run(self, x):
        for r in self.resnets:
            x = r.run(x)
        if self.upsamplers is not None:
            x = conv(x, self.upsamplers[0].conv, upsample=True)  # nearest 2x fused into the conv
        return x


class _DownBlock(nn.Module):
    def __init__(self, cin, cout, n, groups, down: bool):
        super().__init__()
        self.resnets = nn.ModuleList(Resnet(cin if i == 0 else cout, cout, groups) for i in range(n))
        self.downsamplers = nn.ModuleList([_Sampler(cout, True)]) if down else None

    def run(self, x):
        for r in self.resnets:
            x = r.run(x)
        if self.downsamplers is not None:
            x = conv(x, self.downsamplers[0].conv, pad=(0, 0, 1, 1))  # (top, left, bottom, right)
        return x


class _Decoder(nn.Module):
    def __init__(self, c: VAEConfig):
        super().__init__()
        ch = list(reversed(c.channels))
        self.conv_in = nn.Conv2d(c.latent, ch[0], 3, 1, 1)
        self.mid_block = _Mid(ch[0], c.groups)
        self.up_blocks = nn.ModuleList(
            _UpBlock(ch[max(0, i - 1)] if i else ch[0], ch[i], c.layers + 1, c.groups, i < len(ch) - 1)
            for i in range(len(ch)))
        self.conv_norm_out = GroupNorm(c.groups, ch[-1], eps=1e-6)
        self.conv_out = nn.Conv2d(ch[-1], 3, 3, 1, 1)


class _Encoder(nn.Module):
    def __init__(self, c: VAEConfig):
        super().__init__()
        ch = list(c.channels)
        self.conv_in = nn.Conv2d(3, ch[0], 3, 1, 1)
        self.down_blocks = nn.ModuleList(
            _DownBlock(ch[max(0, i - 1)], ch[i], c.layers, c.groups, i < len(ch) - 1) for i in range(len(ch)))
        self.mid_block = _Mid(ch[-1], c.groups)
        self.conv_norm_out = GroupNorm(c.groups, ch[-1], eps=1e-6)
        self.conv_out = nn.Conv2d(ch[-1], 2 * c.latent, 3, 1, 1)


class AutoencoderKL(nn.Module):
    def __init__(self, c: VAEConfig, with_encoder: bool = True):
        super().__init__()
        self.cfg = c
        self.decoder = _Decoder(c)
        self.encoder = _Encoder(c) if with_encoder else None
        if c.quant_conv:
            self.quant_conv = nn.Conv2d(2 * c.latent, 2 * c.latent, 1)
            self.post_quant_conv = nn.Conv2d(c.latent, c.latent, 1)

    def _nhwc(self, x):
        dt = self.decoder.conv_in.weight.dtype
        x = x.to(dt)
        return x.contiguous(memory_format=torch.channels_last) if x.is_cuda else x

    @torch.no_grad()
    def decode(self, z: torch.Tensor) -> torch.Tensor:
        """latent (model space) [B, latent, h, w] -> image in [-1, 1], [B, 3, 8h, 8w] fp32."""
        c = self.cfg
        z = z / c.scaling + c.shift
        x = self._nhwc(z)
        if c.quant_conv:
            x = conv(x, self.post_quant_conv)
        d = self.decoder
        x = conv(x, d.conv_in)
        x = d.mid_block.run(x)
        for blk in d.up_blocks:
            x = blk.run(x)
        x = conv(d.conv_norm_out.run(x, silu=True), d.conv_out)
        return x.float().clamp(-1, 1)

    @torch.no_grad()
    def encode(self, img: torch.Tensor, sample: bool = False, generator=None) -> torch.Tensor:
        """image [-1, 1] [B, 3, H, W] -> latent in model space (mean of the posterior unless `sample`)."""
        c = self.cfg
        e = self.encoder
        x = conv(self._nhwc(img), e.conv_in)
        for blk in e.down_blocks:
            x = blk.run(x)
        x = e.mid_block.run(x)
        x = conv(e.conv_norm_out.run(x, silu=True), e.conv_out)
        if c.quant_conv:
            x = conv(x, self.quant_conv)
        x = x.float()
        mean, logvar = x[:, :c.latent], x[:, c.latent:]
        z = mean
        if sample:
            z = mean + torch.exp(0.5 * logvar.clamp(-30, 20)) * torch.randn(mean.shape, generator=generator,
                                                                          device=mean.device)
        return (z - c.shift) * c.scaling
