"""Sana: linear-attention DiT on a 32x-compressed latent (DC-AE), Gemma-2 text encoder.

Reference: the diffusers backend's `SanaPipeline` (backend/python/diffusers/backend.py:21,218-221:
`from_pretrained(model_dir, variant="bf16", torch_dtype=bf16)`). Parameter names follow diffusers'
`SanaTransformer2DModel` and `AutoencoderDC` (decoder), so the `transformer/` and `vae/` folders load
with `load_state_dict`; `text_encoder/` (Gemma2Model) runs on the repo's LLM engine (last hidden state,
final norm). diffusers is not installed here: parity with its images is unpinned; the tests check the
modules against a float64 re-statement written independently.

Transformer block (per image, N = h*w latent tokens, patch 1):
  adaLN-single: 6 modulation vectors = scale_shift_table[i] + t6 (one linear of the timestep embedding);
  self-attention is ReLU linear attention  o = (V relu(K)^T) relu(Q) / (1^T relu(K)^T relu(Q) + eps),
  cross-attention to the caption is softmax attention on the (unmodulated) residual stream, the FFN is
  GLUMBConv (1x1 expand + SiLU, depthwise 3x3, GLU, 1x1 project) on the 2D token grid.
MI355X execution: LayerNorm+modulation and gated residual adds are the diffusion.hip fused kernels shared
with Flux/SD3; the 1x1 convolutions are GEMMs over NHWC token rows; depthwise 3x3 + SiLU + GLU is one
launch (diffusion.hip mxk_dwconv3_glu); linear attention reduces to two small fp32 batched GEMMs per head;
cross-attention runs on the MFMA flash kernel with key-length masking (attention_dense.hip).

The DC-AE decoder (ResBlocks with BatchNorm / channel RMSNorm, EfficientViT blocks with multi-scale ReLU
linear attention, nearest-upsample + conv stages with channel-repeat shortcuts) runs on PyTorch ops; the
encoder (img2img) is not implemented.
"""
from __future__ import annotations

import json
import math
import os
from dataclasses import dataclass, field

import numpy as np
import torch
import torch.nn.functional as F
from torch import nn

from ... import _native as N
from ...ops import core as K
from .nn import cast_module, cat_w, init_synthetic, lin, timestep_embedding

COMPLEX_HUMAN_INSTRUCTION = [
    "Given a user prompt, generate an 'Enhanced prompt' that provides detailed visual descriptions suitable for "
    "image generation. Evaluate the level of detail in the user prompt:",
    "- If the prompt is simple, focus on adding specifics about colors, shapes, sizes, textures, and spatial "
    "relationships to create vivid and concrete scenes.",
    "- If the prompt is already detailed, refine and enhance the existing details slightly without overcomplicating.",
    "Here are examples of how to transform or refine prompts:",
    "- User Prompt: A cat sleeping -> Enhanced: A small, fluffy white cat curled up in a round shape, sleeping "
    "peacefully on a warm sunny windowsill, surrounded by pots of blooming red flowers.",
    "- User Prompt: A busy city street -> Enhanced: A bustling city street scene at dusk, featuring glowing street "
    "lamps, a diverse crowd of people in colorful clothing, and a double-decker bus passing by towering glass "
    "skyscrapers.",
    "Please generate only the enhanced description for the prompt below and avoid including any additional "
    "commentary or evaluations:",
    "User Prompt: ",
]


@dataclass
class SanaConfig:
    in_channels: int = 32
    heads: int = 70
    head_dim: int = 32
    layers: int = 20
    cross_heads: int = 20
    cross_head_dim: int = 112
    caption_channels: int = 2304
    mlp_ratio: float = 2.5
    attention_bias: bool = False
    patch: int = 1
    sample_size: int = 32
    interpolation_scale: float | None = None
    eps: float = 1e-6
    qk_norm: str | None = None

    @property
    def dim(self) -> int:
        return self.heads * self.head_dim

    @property
    def ffn(self) -> int:
        return int(self.mlp_ratio * self.dim)


SANA_1600M = SanaConfig()
SANA_TEST = SanaConfig(heads=4, head_dim=16, layers=2, cross_heads=2, cross_head_dim=32, caption_channels=64)


class _Lin2(nn.Module):  # TimestepEmbedding / PixArtAlphaTextProjection: linear_1, act, linear_2
    def __init__(self, i, o):
        super().__init__()
        self.linear_1 = nn.Linear(i, o)
        self.linear_2 = nn.Linear(o, o)


class _TimeEmbed(nn.Module):  # AdaLayerNormSingle
    def __init__(self, d):
        super().__init__()
        self.emb = nn.Module()
        self.emb.timestep_embedder = _Lin2(256, d)
        self.linear = nn.Linear(d, 6 * d)


class _RMSB(nn.Module):  # diffusers RMSNorm (optional weight / bias)
    def __init__(self, d, bias=False):
        super().__init__()
        self.weight = nn.Parameter(torch.ones(d))
        if bias:
            self.bias = nn.Parameter(torch.zeros(d))


class _Attention(nn.Module):
    def __init__(self, q_dim, heads, hd, kv_dim, bias, qk_norm=None):
        super().__init__()
        inner = heads * hd
        self.to_q = nn.Linear(q_dim, inner, bias=bias)
        self.to_k = nn.Linear(kv_dim, inner, bias=bias)
        self.to_v = nn.Linear(kv_dim, inner, bias=bias)
        if qk_norm:
            self.norm_q, self.norm_k = _RMSB(inner), _RMSB(inner)
        self.to_out = nn.ModuleList([nn.Linear(inner, q_dim)])


class GLUMBConv(nn.Module):
    def __init__(self, cin, cout, ratio, rms=False):
        super().__init__()
        hid = int(ratio * cin)
        self.conv_inverted = nn.Conv2d(cin, 2 * hid, 1)
        self.conv_depth = nn.Conv2d(2 * hid, 2 * hid, 3, padding=1, groups=2 * hid)
        self.conv_point = nn.Conv2d(hid, cout, 1, bias=False)
        if rms:
            self.norm = _RMSB(cout, bias=True)


class _Block(nn.Module):
    def __init__(self, c: SanaConfig):
        super().__init__()
        d = c.dim
        self.attn1 = _Attention(d, c.heads, c.head_dim, d, c.attention_bias, c.qk_norm)
        self.attn2 = _Attention(d, c.cross_heads, c.cross_head_dim, d, True, c.qk_norm)
        self.ff = GLUMBConv(d, d, c.mlp_ratio)
        self.scale_shift_table = nn.Parameter(torch.randn(6, d) / d ** 0.5)


class _PatchEmbed(nn.Module):
    def __init__(self, c: SanaConfig):
        super().__init__()
        self.proj = nn.Conv2d(c.in_channels, c.dim, c.patch, stride=c.patch)


def sincos_2d(dim: int, h: int, w: int, base: int, interp: float) -> torch.Tensor:
    """diffusers get_2d_sincos_pos_embed for an (h, w) grid -> [h*w, dim] (first half from the column
    coordinate grid, as its meshgrid(w, h) ordering produces)."""
    gh = np.arange(h, dtype=np.float32) / (h / base) / interp
    gw = np.arange(w, dtype=np.float32) / (w / base) / interp
    g = np.stack(np.meshgrid(gw, gh), 0)

    def one(d, pos):
        om = 1.0 / 10000 ** (np.arange(d // 2, dtype=np.float64) / (d / 2.0))
        out = np.einsum("m,d->md", pos.reshape(-1), om)
        return np.concatenate([np.sin(out), np.cos(out)], 1)
    return torch.from_numpy(np.concatenate([one(dim // 2, g[0]), one(dim // 2, g[1])], 1)).float()


def rms_b(x: torch.Tensor, m: _RMSB, eps: float) -> torch.Tensor:
    x = x.float()
    y = x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + eps) * m.weight.float()
    return y + m.bias.float() if hasattr(m, "bias") else y


def dwconv3_glu(x: torch.Tensor, conv: nn.Conv2d, B: int, H: int, W: int, silu_in: bool) -> torch.Tensor:
    """x [B*H*W, 2*Ch] NHWC rows -> [B*H*W, Ch] = dw3x3(x)[:Ch] * silu(dw3x3(x)[Ch:]) (SiLU on the input
    first when silu_in)."""
    C2 = x.shape[1]
    Ch = C2 // 2
    if x.is_cuda:
        w, b = _dw_params(conv)
        out = torch.empty(x.shape[0], Ch, dtype=x.dtype, device=x.device)
        N.ensure_act(x.dtype)
        N.kcall("mxk_dwconv3_glu", x.data_ptr(), w.data_ptr(), b.data_ptr(), out.data_ptr(), B, H, W, Ch,
                int(silu_in), N.stream_ptr())
        return out
    xi = x.float().view(B, H, W, C2).permute(0, 3, 1, 2)
    if silu_in:
        xi = F.silu(xi)
    y = F.conv2d(xi, conv.weight.float(), conv.bias.float(), padding=1, groups=C2)
    y = y[:, :Ch] * F.silu(y[:, Ch:])
    return y.permute(0, 2, 3, 1).reshape(B * H * W, Ch).to(x.dtype)


def _dw_params(conv: nn.Conv2d):
    c = getattr(conv, "_mx_dw", None)
    if c is None:
        c = conv._mx_dw = (conv.weight.detach().float().reshape(conv.weight.shape[0], 9).contiguous(),
                           conv.bias.detach().float().contiguous())
    return c


def linear_attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, B: int, Nt: int, H: int, hd: int,
                     eps: float = 1e-15) -> torch.Tensor:
    """ReLU linear attention over [B*Nt, H*hd] rows (fp32 math) -> [B*Nt, H*hd] in q's dtype."""
    qf = F.relu(q.float()).view(B, Nt, H, hd).permute(0, 2, 1, 3)   # [B, H, N, hd]
    kf = F.relu(k.float()).view(B, Nt, H, hd).permute(0, 2, 1, 3)
    vf = v.float().view(B, Nt, H, hd).permute(0, 2, 1, 3)
    kv = torch.matmul(kf.transpose(-1, -2), vf)                      # [B, H, hd, hd]
    ks = kf.sum(2, keepdim=True)                                     # [B, H, 1, hd]
    num = torch.matmul(qf, kv)                                       # [B, H, N, hd]
    den = (qf * ks).sum(-1, keepdim=True)                            # [B, H, N, 1]
    o = num / (den + eps)
    return o.permute(0, 2, 1, 3).reshape(B * Nt, H * hd).to(q.dtype)


class SanaTransformer(nn.Module):
    def __init__(self, c: SanaConfig):
        super().__init__()
        self.cfg = c
        d = c.dim
        self.patch_embed = _PatchEmbed(c)
        self.time_embed = _TimeEmbed(d)
        self.caption_projection = _Lin2(c.caption_channels, d)
        self.caption_norm = _RMSB(d)
        self.transformer_blocks = nn.ModuleList(_Block(c) for _ in range(c.layers))
        self.scale_shift_table = nn.Parameter(torch.randn(2, d) / d ** 0.5)
        self.proj_out = nn.Linear(d, c.patch * c.patch * c.in_channels)
        self._prep = None

    def prepare(self):
        P = []
        for b in self.transformer_blocks:
            a1, a2, ff = b.attn1, b.attn2, b.ff
            wqkv = cat_w([a1.to_q.weight, a1.to_k.weight, a1.to_v.weight])
            bqkv = torch.cat([a1.to_q.bias, a1.to_k.bias, a1.to_v.bias]) if a1.to_q.bias is not None else None
            P.append(dict(wqkv=wqkv, bqkv=bqkv, wkv2=cat_w([a2.to_k.weight, a2.to_v.weight]),
                          bkv2=torch.cat([a2.to_k.bias, a2.to_v.bias]),
                          w_in=ff.conv_inverted.weight.reshape(ff.conv_inverted.out_channels, -1),
                          w_pt=ff.conv_point.weight.reshape(ff.conv_point.out_channels, -1),
                          table=b.scale_shift_table.detach().float().reshape(1, -1)))
        self._prep = P
        return self

    @torch.no_grad()
    def forward(self, x: torch.Tensor, t: torch.Tensor, ctx: torch.Tensor, klen: torch.Tensor) -> torch.Tensor:
        """x [B, C, H, W] latents, t [B] timesteps (sigma * 1000), ctx [B, T, caption_channels] (padded),
        klen int32 [B] valid caption tokens -> flow velocity [B, C, H, W] fp32."""
        if self._prep is None:
            self.prepare()
        c = self.cfg
        dt = self.proj_out.weight.dtype
        D, p = c.dim, c.patch
        B, C, H, W = x.shape
        h, w = H // p, W // p
        Nt = h * w
        T = ctx.shape[1]
        # patch embed (a p x p stride-p conv = GEMM over patch rows)
        pe = self.patch_embed.proj
        rows = x.reshape(B, C, h, p, w, p).permute(0, 2, 4, 1, 3, 5).reshape(B * Nt, C * p * p)
        hs = lin(rows.to(dt), pe.weight.reshape(D, -1), pe.bias).float()
        if c.interpolation_scale is not None:
            pos = sincos_2d(D, h, w, c.sample_size // p, c.interpolation_scale).to(x.device)
            hs = (hs.view(B, Nt, D) + pos[None]).reshape(B * Nt, D)
        te = self.time_embed
        tf = timestep_embedding(t.float(), 256, shift=0.0).to(dt)
        temb = lin(F.silu(lin(tf, te.emb.timestep_embedder.linear_1.weight, te.emb.timestep_embedder.linear_1.bias)),
                   te.emb.timestep_embedder.linear_2.weight, te.emb.timestep_embedder.linear_2.bias)  # [B, D]
        t6 = (lin(F.silu(temb), te.linear.weight, te.linear.bias)).float()  # [B, 6D]
        cp = self.caption_projection
        e = lin(F.gelu(lin(ctx.reshape(B * T, -1).to(dt), cp.linear_1.weight, cp.linear_1.bias), approximate="tanh"),
                cp.linear_2.weight, cp.linear_2.bias)
        enc = rms_b(e, self.caption_norm, 1e-5).to(dt)  # [B*T, D]
        xn = torch.empty(B * Nt, D, dtype=dt, device=x.device)
        Hq, hd, H2, hd2 = c.heads, c.head_dim, c.cross_heads, c.cross_head_dim
        for i, blk in enumerate(self.transformer_blocks):
            P = self._prep[i]
            m = t6 + P["table"]  # [B, 6D]: shift_msa, scale_msa, gate_msa, shift_mlp, scale_mlp, gate_mlp
            sh1, sc1, g1, sh2, sc2, g2 = (m[:, k * D:(k + 1) * D] for k in range(6))
            K.layernorm_mod(hs, sc1, sh1, Nt, xn, eps=c.eps)
            a1 = blk.attn1
            qkv = lin(xn, P["wqkv"], P["bqkv"])
            q, k, v = qkv[:, :D], qkv[:, D:2 * D], qkv[:, 2 * D:]
            if c.qk_norm:
                q, k = rms_b(q, a1.norm_q, 1e-5).to(dt), rms_b(k, a1.norm_k, 1e-5).to(dt)
            o = linear_attention(q, k, v, B, Nt, Hq, hd)
            K.gate_add(hs, lin(o, a1.to_out[0].weight, a1.to_out[0].bias), g1, Nt)
            # cross-attention on the residual stream (no norm / modulation)
            a2 = blk.attn2
            h16 = hs.to(dt)
            q2 = lin(h16, a2.to_q.weight, a2.to_q.bias)
            kv2 = lin(enc, P["wkv2"], P["bkv2"])
            k2, v2 = kv2[:, :H2 * hd2], kv2[:, H2 * hd2:]
            if c.qk_norm:
                q2, k2 = rms_b(q2, a2.norm_q, 1e-5).to(dt), rms_b(k2, a2.norm_k, 1e-5).to(dt)
            o2 = torch.empty(B * Nt, H2 * hd2, dtype=dt, device=x.device)
            K.attn_dense(q2, k2, v2, o2, B, Nt, T, H2, H2, hd2, hd2 ** -0.5, klen=klen)
            K.gate_add(hs, lin(o2, a2.to_out[0].weight, a2.to_out[0].bias), None, Nt)
            # GLUMBConv feed-forward on the token grid
            K.layernorm_mod(hs, sc2, sh2, Nt, xn, eps=c.eps)
            ff = blk.ff
            u = lin(xn, P["w_in"], ff.conv_inverted.bias)
            g = dwconv3_glu(u, ff.conv_depth, B, h, w, silu_in=True)
            K.gate_add(hs, lin(g, P["w_pt"]), g2, Nt)
        so = (self.scale_shift_table.float().reshape(1, 2, D) + temb.float()[:, None]).reshape(B, 2 * D)
        K.layernorm_mod(hs, so[:, D:], so[:, :D], Nt, xn, eps=1e-6)
        out = lin(xn, self.proj_out.weight, self.proj_out.bias).float()
        return out.view(B, h, w, p, p, C).permute(0, 5, 1, 3, 2, 4).reshape(B, C, H, W)


# ------------------------------------------------------------------------------------------ DC-AE decoder
@dataclass
class DCAEConfig:
    latent: int = 32
    out_channels: int = 3
    head_dim: int = 32
    channels: tuple = (128, 256, 512, 512, 1024, 1024)
    layers: tuple = (3, 3, 3, 3, 3, 3)
    block_types: tuple = ("ResBlock", "ResBlock", "ResBlock", "EfficientViTBlock", "EfficientViTBlock",
                          "EfficientViTBlock")
    norms: tuple = ("batch_norm", "batch_norm", "batch_norm", "rms_norm", "rms_norm", "rms_norm")
    acts: tuple = ("relu", "relu", "relu", "silu", "silu", "silu")
    scales: tuple = ((), (), (), (5,), (5,), (5,))
    interpolate: bool = True
    scaling: float = 0.41407


DCAE_TEST = DCAEConfig(channels=(16, 32, 32), layers=(1, 1, 1), block_types=("ResBlock", "ResBlock", "EfficientViTBlock"),
                       norms=("batch_norm", "rms_norm", "rms_norm"), acts=("relu", "silu", "silu"),
                       scales=((), (), (5,)), head_dim=8, latent=32)


def _norm(kind, c):
    return nn.BatchNorm2d(c) if kind == "batch_norm" else _RMSB(c, bias=True)


def _apply_norm(m, x):
    if isinstance(m, nn.BatchNorm2d):
        return F.batch_norm(x, m.running_mean, m.running_var, m.weight, m.bias, False, 0.0, m.eps)
    return rms_b(x.movedim(1, -1), m, 1e-5).movedim(-1, 1).to(x.dtype)


_ACTS = {"relu": F.relu, "silu": F.silu, "relu6": F.relu6}


class ResBlock(nn.Module):
    def __init__(self, cin, cout, norm, act):
        super().__init__()
        self.act = act
        self.conv1 = nn.Conv2d(cin, cin, 3, padding=1)
        self.conv2 = nn.Conv2d(cin, cout, 3, padding=1, bias=False)
        self.norm = _norm(norm, cout)

    def run(self, x):
        y = self.conv2(_ACTS[self.act](self.conv1(x)))
        return _apply_norm(self.norm, y) + x


class _MSProj(nn.Module):
    def __init__(self, inner, heads, k):
        super().__init__()
        ch = 3 * inner
        self.proj_in = nn.Conv2d(ch, ch, k, padding=k // 2, groups=ch, bias=False)
        self.proj_out = nn.Conv2d(ch, ch, 1, groups=3 * heads, bias=False)


class MSLinearAttention(nn.Module):
    def __init__(self, cin, head_dim, norm, scales, eps=1e-15):
        super().__init__()
        heads = cin // head_dim
        inner = heads * head_dim
        self.head_dim, self.eps = head_dim, eps
        self.to_q = nn.Linear(cin, inner, bias=False)
        self.to_k = nn.Linear(cin, inner, bias=False)
        self.to_v = nn.Linear(cin, inner, bias=False)
        self.to_qkv_multiscale = nn.ModuleList(_MSProj(inner, heads, k) for k in scales)
        self.to_out = nn.Linear(inner * (1 + len(scales)), cin, bias=False)
        self.norm_out = _norm(norm, cin)

    def run(self, x):
        B, _, H, W = x.shape
        xl = x.movedim(1, -1)
        qkv = torch.cat([self.to_q(xl), self.to_k(xl), self.to_v(xl)], -1).movedim(-1, 1)
        ms = [qkv] + [F.conv2d(F.conv2d(qkv, p.proj_in.weight, padding=p.proj_in.padding, groups=p.proj_in.groups),
                               p.proj_out.weight, groups=p.proj_out.groups) for p in self.to_qkv_multiscale]
        h = torch.cat(ms, 1)
        hd = self.head_dim
        h = h.float().reshape(B, -1, 3 * hd, H * W)
        q, k, v = F.relu(h[:, :, :hd]), F.relu(h[:, :, hd:2 * hd]), h[:, :, 2 * hd:]
        if H * W > hd:  # linear attention
            v = F.pad(v, (0, 0, 0, 1), value=1.0)
            o = torch.matmul(torch.matmul(v, k.transpose(-1, -2)), q)
            o = o[:, :, :-1] / (o[:, :, -1:] + self.eps)
        else:  # quadratic (tiny maps)
            s = torch.matmul(k.transpose(-1, -2), q)
            s = s / (s.sum(2, keepdim=True) + self.eps)
            o = torch.matmul(v, s)
        o = o.to(x.dtype).reshape(B, -1, H, W)
        o = self.to_out(o.movedim(1, -1)).movedim(-1, 1)
        return _apply_norm(self.norm_out, o) + x


class EfficientViTBlock(nn.Module):
    def __init__(self, cin, head_dim, norm, scales):
        super().__init__()
        self.attn = MSLinearAttention(cin, head_dim, norm, scales)
        self.conv_out = GLUMBConv(cin, cin, 4, rms=True)

    def run(self, x):
        x = self.attn.run(x)
        f = self.conv_out
        y = F.silu(f.conv_inverted(x))
        y = f.conv_depth(y)
        a, g = y.chunk(2, 1)
        y = f.conv_point(a * F.silu(g))
        return _apply_norm(f.norm, y) + x


class DCUpBlock(nn.Module):
    def __init__(self, cin, cout, interpolate: bool, shortcut: bool = True):
        super().__init__()
        self.interpolate, self.shortcut = interpolate, shortcut
        self.repeats = cout * 4 // cin
        self.conv = nn.Conv2d(cin, cout if interpolate else cout * 4, 3, padding=1)

    def run(self, x):
        if self.interpolate:
            y = self.conv(F.interpolate(x, scale_factor=2, mode="nearest"))
        else:
            y = F.pixel_shuffle(self.conv(x), 2)
        if self.shortcut:
            y = y + F.pixel_shuffle(x.repeat_interleave(self.repeats, 1), 2)
        return y


class _Decoder(nn.Module):
    def __init__(self, c: DCAEConfig):
        super().__init__()
        n = len(c.channels)
        self.conv_in = nn.Conv2d(c.latent, c.channels[-1], 3, padding=1)
        self.in_repeats = c.channels[-1] // c.latent
        ups = []
        for i in reversed(range(n)):
            seq = []
            if i < n - 1 and c.layers[i] > 0:
                seq.append(DCUpBlock(c.channels[i + 1], c.channels[i], c.interpolate))
            for _ in range(c.layers[i]):
                if c.block_types[i] == "ResBlock":
                    seq.append(ResBlock(c.channels[i], c.channels[i], c.norms[i], c.acts[i]))
                else:
                    seq.append(EfficientViTBlock(c.channels[i], c.head_dim, c.norms[i], c.scales[i]))
            ups.insert(0, nn.Sequential(*seq))
        self.up_blocks = nn.ModuleList(ups)
        ch = c.channels[0] if c.layers[0] > 0 else c.channels[1]
        self.norm_out = _RMSB(ch, bias=True)
        self.conv_out = nn.Conv2d(ch, c.out_channels, 3, padding=1) if c.layers[0] > 0 else \
            DCUpBlock(ch, c.out_channels, c.interpolate, shortcut=False)


class AutoencoderDC(nn.Module):
    """diffusers AutoencoderDC, decoder only (`decoder.*` weights)."""

    def __init__(self, c: DCAEConfig):
        super().__init__()
        self.cfg = c
        self.decoder = _Decoder(c)

    @torch.no_grad()
    def decode(self, z: torch.Tensor) -> torch.Tensor:
        d = self.decoder
        dt = d.conv_in.weight.dtype
        z = (z / self.cfg.scaling).to(dt)
        x = d.conv_in(z) + z.repeat_interleave(d.in_repeats, 1)
        for blk in reversed(d.up_blocks):
            for m in blk:
                x = m.run(x)
        x = F.relu(_apply_norm(d.norm_out, x))
        x = d.conv_out(x) if isinstance(d.conv_out, nn.Conv2d) else d.conv_out.run(x)
        return x.float()

    def encode(self, img):
        raise NotImplementedError("Sana img2img needs the DC-AE encoder, which this framework does not implement")


# ------------------------------------------------------------------------------------------------ pipeline
def flow_sigmas(steps: int, shift: float) -> list[float]:
    s = np.linspace(1.0, 1.0 / steps, steps)
    s = shift * s / (1 + (shift - 1) * s)
    return [float(v) for v in s] + [0.0]


class SanaPipeline:
    """Gemma-2 (last hidden state; complex human instruction on the prompt) -> Sana -> DC-AE."""

    def __init__(self, cfg: SanaConfig, tr: SanaTransformer, te, tok, vae: AutoencoderDC, device, shift: float = 3.0,
                 max_tokens: int = 300, chi: bool = True):
        self.cfg, self.tr, self.te, self.tok, self.vae = cfg, tr.prepare(), te, tok, vae
        self.device = torch.device(device)
        self.shift, self.max_tokens, self.chi = shift, max_tokens, chi

    @classmethod
    def synthetic(cls, name: str, device, dtype=None, seed: int = 0) -> "SanaPipeline":
        from ...models.config import tiny_config
        from ...models.llama import LlamaModel
        from ...models.synthetic import synthetic_source
        from ...tokenizer import ByteTokenizer
        dev = torch.device(device)
        dtype = dtype or (torch.bfloat16 if dev.type == "cuda" else torch.float32)
        test = name.endswith("test")
        sc = SANA_TEST if test else SANA_1600M
        dc = DCAE_TEST if test else DCAEConfig()
        gc = tiny_config(arch="gemma2", n_layers=2 if test else 26, hidden=sc.caption_channels,
                         ffn=2 * sc.caption_channels if test else 9216, n_heads=2 if test else 8,
                         n_kv_heads=1 if test else 4, head_dim=32 if test else 256, rope_dim=32 if test else 256,
                         vocab=512 if test else 256000, post_norms=True, embed_scale=sc.caption_channels ** 0.5,
                         ffn_act="gelu", tie_embeddings=True, attn_softcap=50.0, swa_pattern=2, sliding_window=4096)
        te = LlamaModel.load(gc, synthetic_source(gc, "Q8_0", seed=seed + 3), str(dev))

        def build(mod, s):
            with torch.device(dev):
                m = mod()
            init_synthetic(m, seed + s)
            return cast_module(m, dev, dtype).eval()
        tr = build(lambda: SanaTransformer(sc), 1)
        vae = build(lambda: AutoencoderDC(dc), 5)
        return cls(sc, tr, te, ByteTokenizer(gc.vocab), vae, dev, max_tokens=32 if test else 300, chi=not test)

    @classmethod
    def from_diffusers(cls, d: str, device, dtype=None) -> "SanaPipeline":
        from safetensors.torch import load_file
        from ...models.hf import hf_source
        from ...models.llama import LlamaModel
        from ...tokenizer.hf import HFTokenizer
        dev = torch.device(device)
        dtype = dtype or (torch.bfloat16 if dev.type == "cuda" else torch.float32)

        def cfg_of(sub, fn="config.json"):
            with open(os.path.join(d, sub, fn)) as f:
                return json.load(f)

        def load(m, sub, prefix=""):
            sd = {}
            for fn in sorted(os.listdir(os.path.join(d, sub))):
                if fn.endswith(".safetensors"):
                    sd.update(load_file(os.path.join(d, sub, fn)))
            if prefix:
                sd = {k: v for k, v in sd.items() if k.startswith(prefix)}
            missing, _ = m.load_state_dict(sd, strict=False)
            if missing:
                raise ValueError(f"{sub}: missing weights {missing[:5]}")
            return cast_module(m, dev, dtype).eval()
        tc = cfg_of("transformer")
        if tc.get("guidance_embeds"):
            raise ValueError("Sana guidance-distilled transformers (guidance_embeds) are not supported")
        sc = SanaConfig(in_channels=tc.get("in_channels", 32), heads=tc.get("num_attention_heads", 70),
                        head_dim=tc.get("attention_head_dim", 32), layers=tc.get("num_layers", 20),
                        cross_heads=tc.get("num_cross_attention_heads", 20),
                        cross_head_dim=tc.get("cross_attention_head_dim", 112),
                        caption_channels=tc.get("caption_channels", 2304), mlp_ratio=tc.get("mlp_ratio", 2.5),
                        attention_bias=tc.get("attention_bias", False), patch=tc.get("patch_size", 1),
                        sample_size=tc.get("sample_size", 32), interpolation_scale=tc.get("interpolation_scale"),
                        eps=tc.get("norm_eps", 1e-6), qk_norm=tc.get("qk_norm"))
        with torch.device(dev):
            tr = SanaTransformer(sc)
        tr = load(tr, "transformer")
        gcfg, src = hf_source(os.path.join(d, "text_encoder"), "bf16")
        te = LlamaModel.load(gcfg, src, str(dev))
        tok = HFTokenizer(os.path.join(d, "tokenizer"))
        vc = cfg_of("vae")
        n = len(vc.get("decoder_block_out_channels", DCAEConfig.channels))

        def per(v, default):
            v = vc.get(v, default)
            return tuple(v) if isinstance(v, (list, tuple)) else (v,) * n
        dc = DCAEConfig(latent=vc.get("latent_channels", 32), out_channels=vc.get("in_channels", 3),
                        head_dim=vc.get("attention_head_dim", 32),
                        channels=tuple(vc.get("decoder_block_out_channels", DCAEConfig.channels)),
                        layers=per("decoder_layers_per_block", DCAEConfig.layers),
                        block_types=per("decoder_block_types", "ResBlock"), norms=per("decoder_norm_types", "rms_norm"),
                        acts=per("decoder_act_fns", "silu"),
                        scales=tuple(tuple(s) for s in vc.get("decoder_qkv_multiscales", DCAEConfig.scales)),
                        interpolate=vc.get("upsample_block_type", "pixel_shuffle") == "interpolate",
                        scaling=vc.get("scaling_factor", 0.41407))
        with torch.device(dev):
            vae = AutoencoderDC(dc)
        vae = load(vae, "vae", "decoder.")
        shift = 3.0
        sp = os.path.join(d, "scheduler", "scheduler_config.json")
        if os.path.exists(sp):
            with open(sp) as f:
                shift = float(json.load(f).get("flow_shift", 3.0) or 3.0)
        return cls(sc, tr, te, tok, vae, dev, shift=shift)

    @torch.no_grad()
    def encode_prompt(self, prompt: str, chi: bool) -> tuple[torch.Tensor, int]:
        """-> ([max_tokens, C] caption rows (zero padded), valid count). With the complex human instruction the
        rows are BOS + the last max_tokens-1 positions of the instruction+prompt sequence padded to
        len(instruction) + max_tokens - 2, as diffusers selects them."""
        M = self.max_tokens
        if chi:
            pre = "\n".join(COMPLEX_HUMAN_INSTRUCTION)
            n_pre = len(self.tok.encode(pre))
            ids = self.tok.encode(pre + prompt)
            L = n_pre + M - 2
            ids = ids[:L]
            sel = [0] + list(range(L - M + 1, L))
        else:
            ids = self.tok.encode(prompt)[:M]
            sel = list(range(M))
        h = self.te.prompt_hidden(ids or [0])
        out = torch.zeros(M, h.shape[1], dtype=h.dtype, device=h.device)
        valid = [s for s in sel if s < len(ids)]
        out[:len(valid)] = h[torch.tensor(valid, device=h.device)]
        return out, len(valid)

    @torch.no_grad()
    def generate(self, prompt: str, gp, init_image: torch.Tensor | None = None) -> torch.Tensor:
        """-> image [3, H, W] in [0, 1] (fp32, CPU). gp.cfg_scale: guidance (default 4.5)."""
        from . import samplers as Smp
        if init_image is not None:
            raise ValueError("Sana img2img is not supported (no DC-AE encoder)")
        dev = self.device
        f = 2 ** (len(self.vae.cfg.channels) - 1)
        W, H = (gp.width // f) * f, (gp.height // f) * f
        h, w = H // f, W // f
        dt = self.tr.proj_out.weight.dtype
        scale = float(gp.cfg_scale) if gp.cfg_scale and gp.cfg_scale > 0 else 4.5
        c, nc = self.encode_prompt(prompt, self.chi)
        rows, lens = [c], [nc]
        if scale > 1.0:
            u, nu = self.encode_prompt(getattr(gp, "negative", "") or "", False)
            rows, lens = [u, c], [nu, nc]
        ctx = torch.stack(rows).to(dt)
        klen = torch.tensor(lens, dtype=torch.int32, device=dev)
        gen = torch.Generator(device=dev).manual_seed(int(gp.seed) & 0x7FFFFFFFFFFFFFFF)
        sig = flow_sigmas(gp.steps, self.shift)
        z = torch.randn((1, self.cfg.in_channels, h, w), generator=gen, device=dev, dtype=torch.float32)
        nb = ctx.shape[0]

        def denoise(xt: torch.Tensor, sigma: float) -> torch.Tensor:
            xs = xt.expand(nb, -1, -1, -1)
            v = self.tr(xs, torch.full((nb,), sigma * 1000.0, device=dev), ctx, klen)
            if nb == 2:
                v = v[:1] + scale * (v[1:] - v[:1])
            return xt - sigma * v
        sampler = gp.sampler if gp.sampler and gp.sampler != "euler" else "dpm++2m"  # DPMSolverMultistep (2M)
        x = Smp.sample(denoise, z * sig[0], sig, sampler, flow=True, generator=gen)
        img = self.vae.decode(x)[0]
        return ((img + 1) / 2).clamp(0, 1).cpu()
