"""ControlNet for the SD1.x / SD2.x / SDXL UNet pipelines.

Reference: the diffusers backend loads `ControlNetModel.from_pretrained(request.ControlNet)` onto the
pipeline and, when a ControlNet is set, feeds the request's `src` image as the control image instead
of an img2img init (backend/python/diffusers/backend.py:239-242, 309-312).

Parameter names follow diffusers' `ControlNetModel` (conv_in / time_embedding / add_embedding /
down_blocks / mid_block, `controlnet_cond_embedding`, `controlnet_down_blocks`, `controlnet_mid_block`),
so a diffusers `controlnet/` folder loads with `load_state_dict`. Execution reuses the UNet's own
NHWC encoder path (`UNet2DConditionModel._prologue/_encode`: one stacked time-projection GEMM, fused
GroupNorm+SiLU ResNets, flash attention), so ControlNet costs one extra UNet encoder pass per step
on the same kernels. Residuals (already multiplied by the conditioning scale) are added into the
UNet's skip activations and mid-block output (`UNet2DConditionModel.forward(control=...)`).
"""
from __future__ import annotations

import json
import os

import torch
import torch.nn.functional as F
from torch import nn

from .nn import conv
from .unet import UNet2DConditionModel, UNetConfig, config_from_diffusers


class ControlNetConditioningEmbedding(nn.Module):
    """Control image [B, 3, H, W] -> [B, ch0, H/8, W/8] (three stride-2 convs, SiLU between)."""

    def __init__(self, out_ch: int, channels=(16, 32, 96, 256), cin: int = 3):
        super().__init__()
        self.conv_in = nn.Conv2d(cin, channels[0], 3, 1, 1)
        self.blocks = nn.ModuleList()
        for a, b in zip(channels[:-1], channels[1:]):
            self.blocks.append(nn.Conv2d(a, a, 3, 1, 1))
            self.blocks.append(nn.Conv2d(a, b, 3, 2, 1))
        self.conv_out = nn.Conv2d(channels[-1], out_ch, 3, 1, 1)

    def run(self, x):
        x = conv(x, self.conv_in, act="silu")
        for b in self.blocks:
            x = conv(x, b, act="silu")
        return conv(x, self.conv_out)


class ControlNetModel(UNet2DConditionModel):
    def __init__(self, c: UNetConfig, cond_channels=(16, 32, 96, 256), cond_in: int = 3):
        super().__init__(c)
        del self.up_blocks, self.conv_norm_out, self.conv_out  # encoder only
        self.controlnet_cond_embedding = ControlNetConditioningEmbedding(c.channels[0], cond_channels, cond_in)
        self.controlnet_down_blocks = nn.ModuleList()
        skip_ch = [c.channels[0]]
        for i, blk in enumerate(self.down_blocks):
            skip_ch += [c.channels[i]] * len(blk.resnets)
            if blk.downsamplers is not None:
                skip_ch.append(c.channels[i])
        for ch in skip_ch:
            self.controlnet_down_blocks.append(nn.Conv2d(ch, ch, 1))
        self.controlnet_mid_block = nn.Conv2d(c.channels[-1], c.channels[-1], 1)

    def _resnets(self):
        out = []
        for b in self.down_blocks:
            out += list(b.resnets)
        return out + list(self.mid_block.resnets)

    @torch.no_grad()
    def forward(self, x, t, ctx, cond: torch.Tensor, scale: float = 1.0, added: dict | None = None, ctx_key=None):
        """x/t/ctx as the UNet's; cond [B, 3, H, W] in [0, 1] -> (down residuals, mid residual)."""
        ti, ctx16, key, h = self._prologue(x, t, ctx, added, ctx_key)
        cd = cond.to(h.dtype)
        cd = cd.contiguous(memory_format=torch.channels_last) if cd.is_cuda else cd
        h = conv(h, self.conv_in, residual=self.controlnet_cond_embedding.run(cd))
        skips, h = self._encode(h, ti, ctx16, key)
        down = [conv(s, zc) * scale for s, zc in zip(skips, self.controlnet_down_blocks)]
        return down, conv(h, self.controlnet_mid_block) * scale


def controlnet_from_diffusers(d: str, device, dtype) -> ControlNetModel:
    from safetensors.torch import load_file

    from .nn import cast_module
    with open(os.path.join(d, "config.json")) as f:
        cfg = json.load(f)
    m = ControlNetModel(config_from_diffusers(cfg), tuple(cfg.get("conditioning_embedding_out_channels",
                                                                  (16, 32, 96, 256))),
                        cfg.get("conditioning_channels", 3))
    sd = {}
    for fn in sorted(os.listdir(d)):
        if fn.endswith(".safetensors"):
            sd.update(load_file(os.path.join(d, fn)))
    missing, _ = m.load_state_dict(sd, strict=False)
    missing = [k for k in missing if "position_ids" not in k]
    if missing:
        raise ValueError(f"{d}: missing ControlNet weights {missing[:5]}")
    return cast_module(m, torch.device(device), dtype).eval()
