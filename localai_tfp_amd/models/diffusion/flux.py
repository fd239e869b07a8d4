"""Flux.1 (dev / schnell) rectified-flow transformer + text-to-image pipeline.

Reference: the diffusers backend's Flux pipelines (backend/python/diffusers/backend.py:139-270,
FluxPipeline incl. the fp8 quanto path) and stable-diffusion.cpp's Flux support behind
stablediffusion-ggml (gosd.cpp:56-162, guidance 3.5 in gen_image :164-226); SURVEY.md §2.3 N4/N5,
§2.4 P3.

Parameter names follow diffusers' `FluxTransformer2DModel`, so a diffusers `transformer/` folder
loads with `load_state_dict`. MI355X execution plan per denoising step:
* every adaLN modulation of all 57 blocks + the output norm comes from ONE GEMM of silu(temb)
  against the concatenated modulation weights (M = batch);
* residual streams stay fp32; `layernorm_mod` (diffusion.hip) produces the modulated 16-bit GEMM
  operand in one pass and `gate_add` applies gated residual adds;
* each stream's Q|K|V is one GEMM; per-head QK RMSNorm + 3-axis RoPE run in place on its output in
  one launch (flux.hip); joint [text ; image] attention on the MFMA flash kernel (head dim 128);
* single-stream blocks fuse Q|K|V|MLP-in into one [7D, D] GEMM and read [attn | gelu(mlp)] as one
  strided operand of proj_out.
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

from ... import _native as N
from ...ops import core as K
from .nn import attention, cast_module, cat_w, init_synthetic, lin, linear_f32, timestep_embedding


@dataclass
class FluxConfig:
    in_channels: int = 64
    layers: int = 19  # double-stream blocks
    single_layers: int = 38
    head_dim: int = 128
    heads: int = 24
    joint_dim: int = 4096
    pooled_dim: int = 768
    guidance: bool = True  # flux-dev (guidance-distilled); schnell has no guidance embedder
    axes: tuple = (16, 56, 56)
    theta: float = 10000.0

    @property
    def dim(self) -> int:
        return self.heads * self.head_dim


FLUX_DEV = FluxConfig()
FLUX_SCHNELL = FluxConfig(guidance=False)
FLUX_TEST = FluxConfig(layers=2, single_layers=2, heads=2, joint_dim=64, pooled_dim=32)


class _Lin(nn.Module):
    def __init__(self, i, o):
        super().__init__()
        self.linear = nn.Linear(i, o)


class _TE(nn.Module):
    def __init__(self, i, o):
        super().__init__()
        self.linear_1 = nn.Linear(i, o)
        self.linear_2 = nn.Linear(o, o)

    def run(self, x):
        return lin(F.silu(lin(x, self.linear_1.weight, self.linear_1.bias)), self.linear_2.weight,
                        self.linear_2.bias)


class _Embed(nn.Module):
    def __init__(self, c: FluxConfig):
        super().__init__()
        self.timestep_embedder = _TE(256, c.dim)
        if c.guidance:
            self.guidance_embedder = _TE(256, c.dim)
        self.text_embedder = _TE(c.pooled_dim, c.dim)


class _Norm(nn.Module):
    def __init__(self, d):
        super().__init__()
        self.weight = nn.Parameter(torch.ones(d))


class _Attn(nn.Module):
    def __init__(self, c: FluxConfig, joint: bool):
        super().__init__()
        d = c.dim
        self.to_q, self.to_k, self.to_v = nn.Linear(d, d), nn.Linear(d, d), nn.Linear(d, d)
        self.norm_q, self.norm_k = _Norm(c.head_dim), _Norm(c.head_dim)
        if joint:
            self.add_q_proj, self.add_k_proj, self.add_v_proj = nn.Linear(d, d), nn.Linear(d, d), nn.Linear(d, d)
            self.norm_added_q, self.norm_added_k = _Norm(c.head_dim), _Norm(c.head_dim)
            self.to_out = nn.ModuleList([nn.Linear(d, d)])
            self.to_add_out = nn.Linear(d, d)


class _FF(nn.Module):
    def __init__(self, d):
        super().__init__()
        proj = nn.Module()
        proj.proj = nn.Linear(d, 4 * d)
        self.net = nn.ModuleList([proj, nn.Identity(), nn.Linear(4 * d, d)])


class _Double(nn.Module):
    def __init__(self, c: FluxConfig):
        super().__init__()
        d = c.dim
        self.norm1, self.norm1_context = _Lin(d, 6 * d), _Lin(d, 6 * d)
        self.attn = _Attn(c, True)
        self.ff, self.ff_context = _FF(d), _FF(d)


class _Single(nn.Module):
    def __init__(self, c: FluxConfig):
        super().__init__()
        d = c.dim
        self.norm = _Lin(d, 3 * d)
        self.proj_mlp = nn.Linear(d, 4 * d)
        self.proj_out = nn.Linear(5 * d, d)
        self.attn = _Attn(c, False)


def rope_table(ids: torch.Tensor, axes, theta: float) -> torch.Tensor:
    """ids [L, n_axes] -> [L, 64, 2] (cos, sin) per rotary pair (diffusers FluxPosEmbed order)."""
    parts = []
    for i, d in enumerate(axes):
        freqs = 1.0 / theta ** (torch.arange(0, d, 2, dtype=torch.float64) / d)
        parts.append(ids[:, i].double()[:, None] * freqs[None])
    ang = torch.cat(parts, 1)
    return torch.stack([torch.cos(ang), torch.sin(ang)], -1).float().contiguous()


def qk_norm_rope(qkv: torch.Tensor, D: int, H: int, wq: torch.Tensor, wk: torch.Tensor, cs: torch.Tensor, L: int,
                 eps: float = 1e-6):
    """In place on q (cols [0, D)) and k (cols [D, 2D)) of 16-bit qkv rows; row r uses table row r % L."""
    rows = qkv.shape[0]
    hd = D // H
    if qkv.is_cuda:
        N.ensure_act(qkv.dtype)
        N.kcall("mxk_qk_norm_rope", qkv.data_ptr(), qkv.stride(0), rows, D, H, hd, wq.data_ptr(), wk.data_ptr(),
                cs.data_ptr(), L, float(eps), N.stream_ptr())
        return qkv
    pos = torch.arange(rows) % L
    c, s = cs[pos, :, 0][:, None], cs[pos, :, 1][:, None]  # [rows, 1, 64]
    for j, w in ((0, wq), (1, wk)):
        x = qkv[:, j * D:(j + 1) * D].float().view(rows, H, hd)
        x = x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + eps) * w.float()
        x0, x1 = x[..., 0::2], x[..., 1::2]
        y = torch.stack([x0 * c - x1 * s, x1 * c + x0 * s], -1).reshape(rows, D)
        qkv[:, j * D:(j + 1) * D] = y.to(qkv.dtype)
    return qkv


class FluxTransformer(nn.Module):
    def __init__(self, c: FluxConfig):
        super().__init__()
        self.cfg = c
        d = c.dim
        self.x_embedder = nn.Linear(c.in_channels, d)
        self.time_text_embed = _Embed(c)
        self.context_embedder = nn.Linear(c.joint_dim, d)
        self.transformer_blocks = nn.ModuleList(_Double(c) for _ in range(c.layers))
        self.single_transformer_blocks = nn.ModuleList(_Single(c) for _ in range(c.single_layers))
        self.norm_out = _Lin(d, 2 * d)
        self.proj_out = nn.Linear(d, c.in_channels)
        self._prep = None

    def prepare(self):
        mods, offs, o = [], [], 0
        for b in self.transformer_blocks:
            for lin in (b.norm1.linear, b.norm1_context.linear):
                mods.append(lin)
                offs.append(o)
                o += lin.out_features
        for b in self.single_transformer_blocks:
            mods.append(b.norm.linear)
            offs.append(o)
            o += b.norm.linear.out_features
        mods.append(self.norm_out.linear)
        offs.append(o)
        wm = cat_w([m.weight for m in mods])
        bm = torch.cat([m.bias for m in mods]).float()
        dbl = []
        for b in self.transformer_blocks:
            a = b.attn
            dbl.append((cat_w([a.to_q.weight, a.to_k.weight, a.to_v.weight]),
                        torch.cat([a.to_q.bias, a.to_k.bias, a.to_v.bias]),
                        cat_w([a.add_q_proj.weight, a.add_k_proj.weight, a.add_v_proj.weight]),
                        torch.cat([a.add_q_proj.bias, a.add_k_proj.bias, a.add_v_proj.bias])))
        sgl = []
        for b in self.single_transformer_blocks:
            a = b.attn
            sgl.append((cat_w([a.to_q.weight, a.to_k.weight, a.to_v.weight, b.proj_mlp.weight]),
                        torch.cat([a.to_q.bias, a.to_k.bias, a.to_v.bias, b.proj_mlp.bias])))
        f32 = lambda n: n.weight.float().contiguous()  # noqa: E731
        norms = [(f32(b.attn.norm_q), f32(b.attn.norm_k), f32(b.attn.norm_added_q), f32(b.attn.norm_added_k))
                 for b in self.transformer_blocks]
        snorms = [(f32(b.attn.norm_q), f32(b.attn.norm_k)) for b in self.single_transformer_blocks]
        self._prep = dict(wm=wm, bm=bm, offs=offs, dbl=dbl, sgl=sgl, norms=norms, snorms=snorms)
        return self

    @torch.no_grad()
    def forward(self, x: torch.Tensor, img_ids: torch.Tensor, t: torch.Tensor, ctx: torch.Tensor,
                pooled: torch.Tensor, guidance: torch.Tensor | None = None) -> torch.Tensor:
        """x [B, S, in_ch] packed latents, img_ids [S, 3], t [B] sigma in [0, 1], ctx [B, T, joint_dim],
        pooled [B, pooled_dim], guidance [B] -> velocity [B, S, in_ch] fp32."""
        if self._prep is None:
            self.prepare()
        P, c = self._prep, self.cfg
        dt = self.proj_out.weight.dtype
        B, S, _ = x.shape
        T = ctx.shape[1]
        D, H, L = c.dim, c.heads, T + S
        te = self.time_text_embed
        temb = te.timestep_embedder.run(timestep_embedding(t * 1000.0, 256, shift=0.0).to(dt))
        if c.guidance:
            g = guidance if guidance is not None else torch.full((B,), 3.5, device=x.device)
            temb = temb + te.guidance_embedder.run(timestep_embedding(g * 1000.0, 256, shift=0.0).to(dt))
        temb = temb.float() + te.text_embedder.run(pooled.to(dt)).float()
        mod = lin(F.silu(temb).to(dt), P["wm"]).float() + P["bm"]
        ids = torch.cat([torch.zeros(T, 3, device=img_ids.device, dtype=img_ids.dtype), img_ids], 0)
        cs = rope_table(ids.cpu(), c.axes, c.theta).to(x.device)
        cs_t, cs_i = cs[:T].contiguous(), cs[T:].contiguous()
        h = linear_f32(x.reshape(B * S, -1).to(dt), self.x_embedder).contiguous()
        cx = linear_f32(ctx.reshape(B * T, -1).to(dt), self.context_embedder).contiguous()
        hn = torch.empty(B * S, D, dtype=dt, device=x.device)
        cn = torch.empty(B * T, D, dtype=dt, device=x.device)
        for i, blk in enumerate(self.transformer_blocks):
            o1, o2 = P["offs"][2 * i], P["offs"][2 * i + 1]
            sh, sc, gt, sh2, sc2, g2 = (mod[:, o1 + k * D:o1 + (k + 1) * D] for k in range(6))
            csh, csc, cg, csh2, csc2, cg2 = (mod[:, o2 + k * D:o2 + (k + 1) * D] for k in range(6))
            K.layernorm_mod(h, sc, sh, S, hn)
            K.layernorm_mod(cx, csc, csh, T, cn)
            wq, bq, wcq, bcq = P["dbl"][i]
            nq, nk, naq, nak = P["norms"][i]
            qc = lin(cn, wcq, bcq)  # [B*T, 3D]; table row = r % T, so batches need no loop
            qx = lin(hn, wq, bq)
            qk_norm_rope(qc, D, H, naq, nak, cs_t, T)
            qk_norm_rope(qx, D, H, nq, nk, cs_i, S)
            qkv = torch.cat([qc.view(B, T, 3 * D), qx.view(B, S, 3 * D)], 1)
            f = qkv.view(B * L, 3 * D)
            o = attention(f[:, :D], f[:, D:2 * D], f[:, 2 * D:], B, L, L, H, c.head_dim).view(B, L, D)
            a = blk.attn
            K.gate_add(h, lin(o[:, T:], a.to_out[0].weight, a.to_out[0].bias).reshape(B * S, D), gt, S)
            K.gate_add(cx, lin(o[:, :T], a.to_add_out.weight, a.to_add_out.bias).reshape(B * T, D),
                       cg, T)
            K.layernorm_mod(h, sc2, sh2, S, hn)
            u = F.gelu(lin(hn, blk.ff.net[0].proj.weight, blk.ff.net[0].proj.bias), approximate="tanh")
            K.gate_add(h, lin(u, blk.ff.net[2].weight, blk.ff.net[2].bias), g2, S)
            K.layernorm_mod(cx, csc2, csh2, T, cn)
            u = F.gelu(lin(cn, blk.ff_context.net[0].proj.weight, blk.ff_context.net[0].proj.bias),
                       approximate="tanh")
            K.gate_add(cx, lin(u, blk.ff_context.net[2].weight, blk.ff_context.net[2].bias), cg2, T)
        xs = torch.cat([cx.view(B, T, D), h.view(B, S, D)], 1).reshape(B * L, D).contiguous()
        xn = torch.empty(B * L, D, dtype=dt, device=x.device)
        nb = len(self.transformer_blocks)
        for j, blk in enumerate(self.single_transformer_blocks):
            o1 = P["offs"][2 * nb + j]
            sh, sc, gt = (mod[:, o1 + k * D:o1 + (k + 1) * D] for k in range(3))
            K.layernorm_mod(xs, sc, sh, L, xn)
            w, b = P["sgl"][j]
            y = lin(xn, w, b)  # [B*L, 7D] = q | k | v | mlp_in
            nq, nk = P["snorms"][j]
            qk_norm_rope(y, D, H, nq, nk, cs, L)
            o = attention(y[:, :D], y[:, D:2 * D], y[:, 2 * D:3 * D], B, L, L, H, c.head_dim)
            # proj_out reads [attn | gelu(mlp)]: write both into the q|k slots region as one operand
            cat = y[:, 2 * D:]  # [B*L, 5D] view: v | mlp_in  -> overwritten with attn | gelu(mlp)
            cat[:, D:] = F.gelu(cat[:, D:], approximate="tanh")
            cat[:, :D] = o
            K.gate_add(xs, lin(cat, blk.proj_out.weight, blk.proj_out.bias), gt, L)
        on = P["offs"][-1]
        img = xs.view(B, L, D)[:, T:].reshape(B * S, D).contiguous()
        K.layernorm_mod(img, mod[:, on:on + D], mod[:, on + D:on + 2 * D], S, hn)
        return linear_f32(hn, self.proj_out).view(B, S, -1)


# ------------------------------------------------------------------------------------------------ pipeline
def pack_latents(z: torch.Tensor) -> torch.Tensor:
    B, C, h, w = z.shape
    return z.view(B, C, h // 2, 2, w // 2, 2).permute(0, 2, 4, 1, 3, 5).reshape(B, (h // 2) * (w // 2), C * 4)


def unpack_latents(x: torch.Tensor, h: int, w: int) -> torch.Tensor:
    B, S, C4 = x.shape
    C = C4 // 4
    return x.view(B, h // 2, w // 2, C, 2, 2).permute(0, 3, 1, 4, 2, 5).reshape(B, C, h, w)


def image_ids(h2: int, w2: int, device) -> torch.Tensor:
    ids = torch.zeros(h2, w2, 3)
    ids[..., 1] = torch.arange(h2)[:, None]
    ids[..., 2] = torch.arange(w2)[None, :]
    return ids.view(-1, 3).to(device)


def flux_sigmas(steps: int, seq_len: int, dynamic: bool = True, shift: float = 1.0) -> list[float]:
    """FlowMatchEulerDiscreteScheduler with Flux's resolution-dependent shift (mu from 0.5 at 256
    image tokens to 1.15 at 4096) — or a fixed shift (schnell: 1.0)."""
    s = np.linspace(1.0, 1.0 / steps, steps)
    if dynamic:
        mu = 0.5 + (1.15 - 0.5) / (4096 - 256) * (seq_len - 256)
        m = math.exp(mu)
    else:
        m = shift
    s = m * s / (1 + (m - 1) * s)
    return [float(v) for v in s] + [0.0]


class FluxPipeline:
    """CLIP-L pooled + T5-XXL context -> Flux transformer -> 16-channel VAE (Flux scaling/shift)."""

    def __init__(self, cfg: FluxConfig, tr: FluxTransformer, clip_l, t5, vae, tok_l, tok_t5, device,
                 t5_tokens: int = 512, dynamic_shift: bool = True):
        self.cfg, self.tr, self.clip_l, self.t5, self.vae = cfg, tr.prepare(), clip_l, t5, vae
        self.tok_l, self.tok_t5 = tok_l, tok_t5
        self.device = torch.device(device)
        self.t5_tokens, self.dynamic_shift = t5_tokens, dynamic_shift

    @classmethod
    def synthetic(cls, name: str, device, dtype=None, seed: int = 0) -> "FluxPipeline":
        from ...tokenizer.clip import CLIPTokenizer, T5Tokenizer
        from .pipeline import _CLIP_T1, _T5_T
        from .text_encoders import CLIP_L, T5_XXL, CLIPTextEncoder, T5Encoder
        from .vae import VAE_TEST, AutoencoderKL, VAEConfig
        dev = torch.device(device)
        dtype = dtype or (torch.bfloat16 if dev.type == "cuda" else torch.float32)
        test = name.endswith("test")
        fc = {"flux-dev": FLUX_DEV, "flux-schnell": FLUX_SCHNELL, "flux-test": FLUX_TEST}[name]
        cl_cfg, t5_cfg = (_CLIP_T1, _T5_T) if test else (CLIP_L, T5_XXL)
        vc = VAEConfig(latent=16, channels=VAE_TEST.channels, layers=1, groups=8, scaling=0.3611, shift=0.1159) \
            if test else VAEConfig(scaling=0.3611, shift=0.1159)

        def build(mod, s):
            with torch.device(dev):
                m = mod()
            init_synthetic(m, seed + s)
            return cast_module(m, dev, dtype).eval()
        tr = build(lambda: FluxTransformer(fc), 1)
        cl = build(lambda: CLIPTextEncoder(cl_cfg), 2)
        t5 = build(lambda: T5Encoder(t5_cfg), 4)
        vae = build(lambda: AutoencoderKL(vc), 5)
        nt = 16 if test else 512
        return cls(fc, tr, cl, t5, vae, CLIPTokenizer.synthetic(cl_cfg.vocab), T5Tokenizer(None, t5_cfg.vocab, nt), dev,
                   t5_tokens=nt, dynamic_shift=fc.guidance)

    @classmethod
    def from_diffusers(cls, d: str, device, dtype=None) -> "FluxPipeline":
        """diffusers FluxPipeline directory (transformer / text_encoder / text_encoder_2 / vae / tokenizers)."""
        from safetensors.torch import load_file
        from ...tokenizer.clip import CLIPTokenizer, T5Tokenizer
        from .text_encoders import CLIPTextConfig, CLIPTextEncoder, T5Config, T5Encoder
        from .vae import AutoencoderKL, VAEConfig
        dev = torch.device(device)
        dtype = dtype or (torch.bfloat16 if dev.type == "cuda" else torch.float32)

        def cfg_of(sub):
            with open(os.path.join(d, sub, "config.json")) as f:
                return json.load(f)

        def load(m, sub):
            sd = {}
            for fn in sorted(os.listdir(os.path.join(d, sub))):
                if fn.endswith(".safetensors"):
                    sd.update(load_file(os.path.join(d, sub, fn)))
            missing, _ = m.load_state_dict(sd, strict=False)
            if missing:
                raise ValueError(f"{sub}: missing weights {missing[:5]}")
            return cast_module(m, dev, dtype).eval()
        tc = cfg_of("transformer")
        fc = FluxConfig(in_channels=tc.get("in_channels", 64), layers=tc["num_layers"],
                        single_layers=tc["num_single_layers"], head_dim=tc["attention_head_dim"],
                        heads=tc["num_attention_heads"], joint_dim=tc["joint_attention_dim"],
                        pooled_dim=tc["pooled_projection_dim"], guidance=bool(tc.get("guidance_embeds", False)),
                        axes=tuple(tc.get("axes_dims_rope", (16, 56, 56))))
        tr = load(FluxTransformer(fc), "transformer")
        c = cfg_of("text_encoder")
        cl = load(CLIPTextEncoder(CLIPTextConfig(vocab=c["vocab_size"], hidden=c["hidden_size"],
                                                 layers=c["num_hidden_layers"], heads=c["num_attention_heads"],
                                                 ffn=c["intermediate_size"], max_pos=c["max_position_embeddings"],
                                                 act=c.get("hidden_act", "quick_gelu"),
                                                 proj=c.get("projection_dim", c["hidden_size"]))), "text_encoder")
        c = cfg_of("text_encoder_2")
        t5 = load(T5Encoder(T5Config(vocab=c["vocab_size"], d_model=c["d_model"], heads=c["num_heads"], d_kv=c["d_kv"],
                                     d_ff=c["d_ff"], layers=c["num_layers"])), "text_encoder_2")
        vc = cfg_of("vae")
        vae = load(AutoencoderKL(VAEConfig(latent=vc["latent_channels"], channels=tuple(vc["block_out_channels"]),
                                           layers=vc["layers_per_block"], groups=vc.get("norm_num_groups", 32),
                                           scaling=vc.get("scaling_factor", 0.3611), shift=vc.get("shift_factor") or 0.0,
                                           quant_conv=vc.get("use_quant_conv", False))), "vae")
        tl = CLIPTokenizer.from_dir(os.path.join(d, "tokenizer"))
        tt = T5Tokenizer.from_file(os.path.join(d, "tokenizer_2", "spiece.model"))
        dyn = True
        sp = os.path.join(d, "scheduler", "scheduler_config.json")
        if os.path.exists(sp):
            with open(sp) as f:
                dyn = bool(json.load(f).get("use_dynamic_shifting", True))
        return cls(fc, tr, cl, t5, vae, tl, tt, dev, t5_tokens=512 if fc.guidance else 256, dynamic_shift=dyn)

    @torch.no_grad()
    def encode_prompts(self, prompts: list[str]):
        dev = self.device
        il = torch.tensor([self.tok_l(p) for p in prompts], device=dev)
        _, pooled = self.clip_l(il, self.tok_l.eos, 1)
        it = torch.tensor([self.tok_t5(p) for p in prompts], device=dev)
        return self.t5(it), pooled

    @torch.no_grad()
    def generate(self, prompt: str, gp, init_image: torch.Tensor | None = None) -> torch.Tensor:
        """-> image [3, H, W] in [0, 1] (fp32, CPU). `gp.cfg_scale` is Flux's distilled guidance
        (default 3.5 when unset); schnell ignores it."""
        from . import samplers as Smp
        dev = self.device
        W, H = (gp.width // 16) * 16, (gp.height // 16) * 16
        ctx, pooled = self.encode_prompts([prompt])
        gen = torch.Generator(device=dev).manual_seed(int(gp.seed) & 0x7FFFFFFFFFFFFFFF)
        h, w = H // 8, W // 8
        S = (h // 2) * (w // 2)
        sig = flux_sigmas(gp.steps, S, self.dynamic_shift)
        z = torch.randn((1, 16, h, w), generator=gen, device=dev, dtype=torch.float32)
        ids = image_ids(h // 2, w // 2, dev)
        g = torch.full((1,), float(gp.cfg_scale) if gp.cfg_scale and gp.cfg_scale > 0 else 3.5, device=dev)

        def denoise(xt: torch.Tensor, sigma: float) -> torch.Tensor:
            v = self.tr(pack_latents(xt), ids, torch.full((1,), sigma, device=dev), ctx, pooled, g)
            return xt - sigma * unpack_latents(v, h, w)
        if init_image is not None:  # img2img: start from the noised encoding of the source image
            x0 = self.vae.encode(init_image.to(dev)[None] * 2 - 1)
            x0 = F.interpolate(x0, size=(h, w), mode="bilinear") if x0.shape[2:] != (h, w) else x0
            k = min(len(sig) - 2, int(round((1 - gp.strength) * (len(sig) - 1))))
            sig = sig[k:]
            x = (1 - sig[0]) * x0 + sig[0] * z
        else:
            x = z * sig[0]
        x = Smp.sample(denoise, x, sig, gp.sampler, flow=True, generator=gen)
        img = self.vae.decode(x)[0]
        return ((img + 1) / 2).clamp(0, 1).cpu()
