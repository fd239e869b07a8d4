"""Lumina-Image 2.0: the Unified Next-DiT flow-matching transformer with a Gemma-2 text encoder and the
16-channel (Flux) VAE.

Reference: the diffusers backend's `Lumina2Text2ImgPipeline` (backend/python/diffusers/backend.py:35,
213-216: `from_pretrained(model_dir, torch_dtype=bf16)`). Parameter names follow diffusers'
`Lumina2Transformer2DModel`, so a diffusers `transformer/` folder loads with `load_state_dict`; the
`text_encoder/` folder (a bare `Gemma2Model`) loads into the repo's Llama-family engine (models/hf.py)
and is read at its penultimate layer (hidden_states[-2]). diffusers is not installed here: parity with
its images is unpinned; tests check the loader against the module layout and the transformer against a
plain PyTorch fp32 re-statement of the architecture.

Architecture (per sample; captions keep only their unmasked tokens):
* caption tokens: RMSNorm + linear to the model width, refined by `context_refiner` blocks (no timestep
  modulation); image: 2x2 patches (py, px, c order) -> `x_embedder`, refined by `noise_refiner` blocks;
* joint [caption ; image] sequence through `layers`; every block: RMSNorm pre/post sandwich around
  grouped-query attention (per-head RMSNorm on q/k + 3-axis interleaved RoPE; caption position ids
  (i, 0, 0), image (Tc, row, col)) and a SwiGLU FFN, with tanh-gated adaLN (scale / gate from
  silu(temb) through one linear per block);
* output: LayerNorm (no affine) scaled by 1 + linear(silu(temb)), linear to patch pixels.

MI355X execution: Q|K|V is one GEMM; q/k head RMSNorm + RoPE run in place in one launch
(flux.hip mxk_qk_norm_rope_gqa, head dim 96); attention on the MFMA flash kernel with grouped-query
heads (attention_dense.hip, head dim zero-padded to 128); gate|up is one GEMM.
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
from .nn import cast_module, cat_w, init_synthetic, lin, timestep_embedding

SYSTEM_PROMPT = ("You are an assistant designed to generate superior images with the superior degree of image-text "
                 "alignment based on textual prompts or user prompts.")


@dataclass
class Lumina2Config:
    patch: int = 2
    in_channels: int = 16
    hidden: int = 2304
    layers: int = 26
    refiner_layers: int = 2
    heads: int = 24
    kv_heads: int = 8
    multiple_of: int = 256
    ffn_mult: float | None = None
    eps: float = 1e-5
    axes: tuple = (32, 32, 32)
    axes_lens: tuple = (300, 512, 512)
    cap_dim: int = 2304
    theta: float = 10000.0

    @property
    def head_dim(self) -> int:
        return self.hidden // self.heads

    @property
    def ffn(self) -> int:
        f = 4 * self.hidden
        if self.ffn_mult is not None:
            f = int(self.ffn_mult * f)
        return self.multiple_of * ((f + self.multiple_of - 1) // self.multiple_of)

    @property
    def temb_dim(self) -> int:
        return min(self.hidden, 1024)


LUMINA2 = Lumina2Config()
LUMINA2_TEST = Lumina2Config(hidden=192, layers=2, refiner_layers=1, heads=2, kv_heads=1, multiple_of=64, cap_dim=64)


class _RMS(nn.Module):
    def __init__(self, d):
        super().__init__()
        self.weight = nn.Parameter(torch.ones(d))


class _Attn(nn.Module):
    def __init__(self, c: Lumina2Config):
        super().__init__()
        d, hd = c.hidden, c.head_dim
        self.to_q = nn.Linear(d, c.heads * hd, bias=False)
        self.to_k = nn.Linear(d, c.kv_heads * hd, bias=False)
        self.to_v = nn.Linear(d, c.kv_heads * hd, bias=False)
        self.norm_q, self.norm_k = _RMS(hd), _RMS(hd)
        self.to_out = nn.ModuleList([nn.Linear(c.heads * hd, d, bias=False)])


class _FF(nn.Module):
    def __init__(self, c: Lumina2Config):
        super().__init__()
        self.linear_1 = nn.Linear(c.hidden, c.ffn, bias=False)  # gate
        self.linear_2 = nn.Linear(c.ffn, c.hidden, bias=False)  # down
        self.linear_3 = nn.Linear(c.hidden, c.ffn, bias=False)  # up


class _NormZero(nn.Module):
    def __init__(self, c: Lumina2Config):
        super().__init__()
        self.linear = nn.Linear(c.temb_dim, 4 * c.hidden)
        self.norm = _RMS(c.hidden)


class _Block(nn.Module):
    def __init__(self, c: Lumina2Config, modulation: bool):
        super().__init__()
        self.modulation = modulation
        self.attn = _Attn(c)
        self.feed_forward = _FF(c)
        self.norm1 = _NormZero(c) if modulation else _RMS(c.hidden)
        self.ffn_norm1, self.norm2, self.ffn_norm2 = _RMS(c.hidden), _RMS(c.hidden), _RMS(c.hidden)


class _TE(nn.Module):
    def __init__(self, i, o):
        super().__init__()
        self.linear_1 = nn.Linear(i, o)
        self.linear_2 = nn.Linear(o, o)

    def run(self, x):
        return lin(F.silu(lin(x, self.linear_1.weight, self.linear_1.bias)), self.linear_2.weight, self.linear_2.bias)


class _TimeCaption(nn.Module):
    def __init__(self, c: Lumina2Config):
        super().__init__()
        self.timestep_embedder = _TE(256, c.temb_dim)
        self.caption_embedder = nn.Sequential(_RMS(c.cap_dim), nn.Linear(c.cap_dim, c.hidden))


class _NormOut(nn.Module):
    def __init__(self, c: Lumina2Config):
        super().__init__()
        self.linear_1 = nn.Linear(c.temb_dim, c.hidden)
        self.linear_2 = nn.Linear(c.hidden, c.patch * c.patch * c.in_channels)


def rms(x: torch.Tensor, w: torch.Tensor, eps: float) -> torch.Tensor:
    """fp32 RMSNorm of rows (weight w)."""
    x = x.float()
    return x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + eps) * w.float()


def rope_table(ids: torch.Tensor, axes, theta: float) -> torch.Tensor:
    """ids [L, 3] -> [L, sum(axes)/2, 2] (cos, sin): per axis get_1d_rotary_pos_embed(d, theta) at the id."""
    parts = []
    for i, d in enumerate(axes):
        freqs = 1.0 / theta ** (torch.arange(0, d, 2, dtype=torch.float64)[: d // 2] / d)
        parts.append(ids[:, i].double()[:, None] * freqs[None])
    ang = torch.cat(parts, 1)
    return torch.stack([torch.cos(ang), torch.sin(ang)], -1).float().contiguous()


def position_ids(tc: int, hp: int, wp: int) -> torch.Tensor:
    """Caption tokens (i, 0, 0); image tokens (tc, row, col), rows major."""
    ids = torch.zeros(tc + hp * wp, 3, dtype=torch.int64)
    ids[:tc, 0] = torch.arange(tc)
    ids[tc:, 0] = tc
    ids[tc:, 1] = torch.arange(hp).repeat_interleave(wp)
    ids[tc:, 2] = torch.arange(wp).repeat(hp)
    return ids


def norm_rope_(qkv: torch.Tensor, Hq: int, Hk: int, hd: int, wq: torch.Tensor, wk: torch.Tensor, cs: torch.Tensor,
               eps: float) -> torch.Tensor:
    """In place on the q (cols [0, Hq*hd)) and k (next Hk*hd) heads of 16-bit qkv rows: per-head RMSNorm
    then interleaved-pair RoPE with table row r (cs [rows, hd/2, 2])."""
    rows, L = qkv.shape[0], cs.shape[0]
    if qkv.is_cuda:
        N.ensure_act(qkv.dtype)
        N.kcall("mxk_qk_norm_rope_gqa", qkv.data_ptr(), qkv.stride(0), rows, Hq, Hk, hd, Hq * hd, wq.data_ptr(),
                wk.data_ptr(), cs.data_ptr(), L, float(eps), N.stream_ptr())
        return qkv
    pos = torch.arange(rows) % L
    c, s = cs[pos, :, 0][:, None], cs[pos, :, 1][:, None]
    for o, H, w in ((0, Hq, wq), (Hq * hd, Hk, wk)):
        x = qkv[:, o:o + H * hd].float().view(rows, H, hd)
        x = x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + eps) * w.float()
        x0, x1 = x[..., 0::2], x[..., 1::2]
        qkv[:, o:o + H * hd] = torch.stack([x0 * c - x1 * s, x1 * c + x0 * s], -1).reshape(rows, H * hd).to(qkv.dtype)
    return qkv


class Lumina2Transformer(nn.Module):
    def __init__(self, c: Lumina2Config):
        super().__init__()
        self.cfg = c
        p = c.patch
        self.x_embedder = nn.Linear(p * p * c.in_channels, c.hidden)
        self.time_caption_embed = _TimeCaption(c)
        self.noise_refiner = nn.ModuleList(_Block(c, True) for _ in range(c.refiner_layers))
        self.context_refiner = nn.ModuleList(_Block(c, False) for _ in range(c.refiner_layers))
        self.layers = nn.ModuleList(_Block(c, True) for _ in range(c.layers))
        self.norm_out = _NormOut(c)
        self._prep = None

    def prepare(self):
        blocks = list(self.noise_refiner) + list(self.context_refiner) + list(self.layers)
        f32 = lambda t: t.float().contiguous()  # noqa: E731
        P = {}
        for b in blocks:
            a, ff = b.attn, b.feed_forward
            P[id(b)] = dict(wqkv=cat_w([a.to_q.weight, a.to_k.weight, a.to_v.weight]),
                            nq=f32(a.norm_q.weight), nk=f32(a.norm_k.weight),
                            wgu=cat_w([ff.linear_1.weight, ff.linear_3.weight]))
        # every block's adaLN modulation (and the output norm's scale) from ONE GEMM of silu(temb)
        mods = [b.norm1.linear for b in blocks if b.modulation] + [self.norm_out.linear_1]
        self._mod_w = cat_w([m.weight for m in mods])
        self._mod_b = torch.cat([m.bias for m in mods]).float()
        offs, o = {}, 0
        for b in blocks:
            if b.modulation:
                offs[id(b)] = o
                o += b.norm1.linear.out_features
        self._mod_out = o
        self._prep, self._offs = P, offs
        return self

    def _attn(self, b: _Block, xn: torch.Tensor, cs: torch.Tensor) -> torch.Tensor:
        c = self.cfg
        Hq, Hk, hd = c.heads, c.kv_heads, c.head_dim
        P = self._prep[id(b)]
        L = xn.shape[0]
        qkv = lin(xn, P["wqkv"])
        norm_rope_(qkv, Hq, Hk, hd, P["nq"], P["nk"], cs, c.eps)
        q, k, v = qkv[:, :Hq * hd], qkv[:, Hq * hd:(Hq + Hk) * hd], qkv[:, (Hq + Hk) * hd:]
        o = torch.empty(L, Hq * hd, dtype=xn.dtype, device=xn.device)
        K.attn_dense(q, k, v, o, 1, L, L, Hq, Hk, hd, hd ** -0.5)
        return lin(o, b.attn.to_out[0].weight)

    def _block(self, b: _Block, x: torch.Tensor, cs: torch.Tensor, mod: torch.Tensor | None) -> torch.Tensor:
        """x fp32 [L, D] residual stream (updated and returned)."""
        c, dt = self.cfg, self.x_embedder.weight.dtype
        D = c.hidden
        if b.modulation:
            o = self._offs[id(b)]
            s_msa, g_msa, s_mlp, g_mlp = (mod[o + k * D:o + (k + 1) * D] for k in range(4))
            xn = rms(x, b.norm1.norm.weight, c.eps) * (1 + s_msa)
        else:
            xn = rms(x, b.norm1.weight, c.eps)
        a = self._attn(b, xn.to(dt), cs)
        a = rms(a, b.norm2.weight, c.eps)
        x = x + (torch.tanh(g_msa) * a if b.modulation else a)
        y = rms(x, b.ffn_norm1.weight, c.eps)
        if b.modulation:
            y = y * (1 + s_mlp)
        gu = lin(y.to(dt), self._prep[id(b)]["wgu"])
        F_ = c.ffn
        h = (F.silu(gu[:, :F_].float()) * gu[:, F_:].float()).to(dt)
        f = rms(lin(h, b.feed_forward.linear_2.weight), b.ffn_norm2.weight, c.eps)
        return x + (torch.tanh(g_mlp) * f if b.modulation else f)

    @torch.no_grad()
    def forward(self, x: torch.Tensor, t: torch.Tensor, cap: torch.Tensor) -> torch.Tensor:
        """x [C, H, W] latents, t scalar tensor (0 = noise, 1 = image), cap [Tc, cap_dim] (unmasked caption
        tokens) -> model output [C, H, W] fp32 (the pipeline's velocity is its negation)."""
        if self._prep is None:
            self.prepare()
        c = self.cfg
        dt = self.x_embedder.weight.dtype
        p = c.patch
        C, H, W = x.shape
        hp, wp = H // p, W // p
        tc = cap.shape[0]
        tce = self.time_caption_embed
        temb = tce.timestep_embedder.run(timestep_embedding(t.reshape(1).float(), 256, shift=0.0).to(dt))
        mod = (lin(F.silu(temb), self._mod_w).float() + self._mod_b)[0]
        cn = rms(cap, tce.caption_embedder[0].weight, c.eps).to(dt)
        ctx = lin(cn, tce.caption_embedder[1].weight, tce.caption_embedder[1].bias).float()
        cs = rope_table(position_ids(tc, hp, wp), c.axes, c.theta).to(x.device)
        cs_c, cs_i = cs[:tc].contiguous(), cs[tc:].contiguous()
        img = x.reshape(C, hp, p, wp, p).permute(1, 3, 2, 4, 0).reshape(hp * wp, p * p * C)
        h = lin(img.to(dt), self.x_embedder.weight, self.x_embedder.bias).float()
        for b in self.context_refiner:
            ctx = self._block(b, ctx, cs_c, None)
        for b in self.noise_refiner:
            h = self._block(b, h, cs_i, mod)
        j = torch.cat([ctx, h], 0)
        for b in self.layers:
            j = self._block(b, j, cs, mod)
        so = self._mod_out
        y = F.layer_norm(j[tc:], (c.hidden,), eps=1e-6) * (1 + mod[so:so + c.hidden])
        out = lin(y.to(dt), self.norm_out.linear_2.weight, self.norm_out.linear_2.bias).float()
        return out.view(hp, wp, p, p, C).permute(4, 0, 2, 1, 3).reshape(C, H, W)


def flow_sigmas(steps: int, shift: float, seq_len: int | None = None, dynamic: bool = False) -> list[float]:
    """FlowMatchEulerDiscreteScheduler sigmas: linspace(1, 1/steps) time-shifted (static shift, or Flux-style
    resolution-dependent mu when dynamic)."""
    s = np.linspace(1.0, 1.0 / steps, steps)
    m = math.exp(0.5 + (1.15 - 0.5) / (4096 - 256) * ((seq_len or 256) - 256)) if dynamic else shift
    s = m * s / (1 + (m - 1) * s)
    return [float(v) for v in s] + [0.0]


class Lumina2Pipeline:
    """Gemma-2 (penultimate hidden states) -> Next-DiT -> 16-channel VAE; CFG with per-row renormalisation."""

    def __init__(self, cfg: Lumina2Config, tr: Lumina2Transformer, te, tok, vae, device, shift: float = 6.0,
                 dynamic: bool = False, max_tokens: int = 256, system_prompt: str = SYSTEM_PROMPT):
        self.cfg, self.tr, self.te, self.tok, self.vae = cfg, tr.prepare(), te, tok, vae
        self.device = torch.device(device)
        self.shift, self.dynamic, self.max_tokens, self.system_prompt = shift, dynamic, max_tokens, system_prompt

    @classmethod
    def synthetic(cls, name: str, device, dtype=None, seed: int = 0) -> "Lumina2Pipeline":
        from ...models.config import tiny_config
        from ...models.llama import LlamaModel
        from ...models.synthetic import synthetic_source
        from ...tokenizer import ByteTokenizer
        from .vae import VAE_TEST, AutoencoderKL, VAEConfig
        dev = torch.device(device)
        dtype = dtype or (torch.bfloat16 if dev.type == "cuda" else torch.float32)
        test = name.endswith("test")
        lc = LUMINA2_TEST if test else LUMINA2
        gc = tiny_config(arch="gemma2", n_layers=2 if test else 26, hidden=lc.cap_dim, ffn=2 * lc.cap_dim if test else 9216,
                         n_heads=2 if test else 8, n_kv_heads=1 if test else 4, head_dim=32 if test else 256,
                         rope_dim=32 if test else 256, vocab=512 if test else 256000, post_norms=True,
                         embed_scale=lc.cap_dim ** 0.5, ffn_act="gelu", tie_embeddings=True, attn_softcap=50.0,
                         swa_pattern=2, sliding_window=4096)
        te = LlamaModel.load(gc, synthetic_source(gc, "Q8_0", seed=seed + 3), str(dev))
        vc = VAEConfig(latent=16, channels=VAE_TEST.channels, layers=1, groups=8, scaling=0.3611, shift=0.1159) \
            if test else VAEConfig(scaling=0.3611, shift=0.1159)

        def build(mod, s):
            with torch.device(dev):
                m = mod()
            init_synthetic(m, seed + s)
            return cast_module(m, dev, dtype).eval()
        tr = build(lambda: Lumina2Transformer(lc), 1)
        vae = build(lambda: AutoencoderKL(vc), 5)
        return cls(lc, tr, te, ByteTokenizer(gc.vocab), vae, dev, max_tokens=64 if test else 256)

    @classmethod
    def from_diffusers(cls, d: str, device, dtype=None) -> "Lumina2Pipeline":
        """diffusers Lumina2 directory: transformer / text_encoder (Gemma2Model) / tokenizer / vae / scheduler."""
        from safetensors.torch import load_file
        from ...models.hf import hf_source
        from ...models.llama import LlamaModel
        from ...tokenizer.hf import HFTokenizer
        from .vae import AutoencoderKL, VAEConfig
        dev = torch.device(device)
        dtype = dtype or (torch.bfloat16 if dev.type == "cuda" else torch.float32)

        def cfg_of(sub, fn="config.json"):
            with open(os.path.join(d, sub, fn)) as f:
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
        lc = Lumina2Config(patch=tc.get("patch_size", 2), in_channels=tc.get("in_channels", 16),
                           hidden=tc.get("hidden_size", 2304), layers=tc.get("num_layers", 26),
                           refiner_layers=tc.get("num_refiner_layers", 2), heads=tc.get("num_attention_heads", 24),
                           kv_heads=tc.get("num_kv_heads", 8), multiple_of=tc.get("multiple_of", 256),
                           ffn_mult=tc.get("ffn_dim_multiplier"), eps=tc.get("norm_eps", 1e-5),
                           axes=tuple(tc.get("axes_dim_rope", (32, 32, 32))),
                           axes_lens=tuple(tc.get("axes_lens", (300, 512, 512))), cap_dim=tc.get("cap_feat_dim", 2304))
        with torch.device(dev):
            tr = Lumina2Transformer(lc)
        tr = load(tr, "transformer")
        gcfg, src = hf_source(os.path.join(d, "text_encoder"), "bf16")
        te = LlamaModel.load(gcfg, src, str(dev))
        tok = HFTokenizer(os.path.join(d, "tokenizer"))
        vc = cfg_of("vae")
        with torch.device(dev):
            vae = AutoencoderKL(VAEConfig(latent=vc["latent_channels"], channels=tuple(vc["block_out_channels"]),
                                          layers=vc["layers_per_block"], groups=vc.get("norm_num_groups", 32),
                                          scaling=vc.get("scaling_factor", 0.3611), shift=vc.get("shift_factor") or 0.0,
                                          quant_conv=vc.get("use_quant_conv", False)))
        vae = load(vae, "vae")
        shift, dyn = 6.0, False
        sp = os.path.join(d, "scheduler", "scheduler_config.json")
        if os.path.exists(sp):
            with open(sp) as f:
                sc = json.load(f)
            shift, dyn = float(sc.get("shift", 6.0)), bool(sc.get("use_dynamic_shifting", False))
        return cls(lc, tr, te, tok, vae, dev, shift=shift, dynamic=dyn)

    @torch.no_grad()
    def encode_prompt(self, prompt: str) -> torch.Tensor:
        """-> [Tc, cap_dim] Gemma-2 hidden_states[-2] over the prompt's tokens (BOS included, no padding)."""
        text = f"{self.system_prompt} <Prompt Start> {prompt}" if self.system_prompt else prompt
        ids = self.tok.encode(text)[: self.max_tokens] or [0]
        h = self.te.prompt_hidden(ids, self.te.cfg.n_layers - 1)
        return h.to(self.tr.x_embedder.weight.dtype)

    @torch.no_grad()
    def generate(self, prompt: str, gp, init_image: torch.Tensor | None = None, cfg_normalization: bool = True,
                 cfg_trunc_ratio: float = 1.0) -> torch.Tensor:
        """-> image [3, H, W] in [0, 1] (fp32, CPU). gp.cfg_scale: guidance (default 4.0); gp.negative: the
        unconditional prompt. Defaults as diffusers' Lumina2 pipeline (cfg_normalization, cfg_trunc_ratio 1)."""
        negative_prompt = getattr(gp, "negative", "") or ""
        from . import samplers as Smp
        dev = self.device
        p = self.cfg.patch
        W, H = (gp.width // 16) * 16, (gp.height // 16) * 16
        h, w = H // 8, W // 8
        cond = self.encode_prompt(prompt)
        scale = float(gp.cfg_scale) if gp.cfg_scale and gp.cfg_scale > 0 else 4.0
        uncond = self.encode_prompt(negative_prompt or "") if scale > 1.0 else None
        gen = torch.Generator(device=dev).manual_seed(int(gp.seed) & 0x7FFFFFFFFFFFFFFF)
        sig = flow_sigmas(gp.steps, self.shift, (h // p) * (w // p), self.dynamic)
        z = torch.randn((16, h, w), generator=gen, device=dev, dtype=torch.float32)

        def velocity(xt: torch.Tensor, sigma: float) -> torch.Tensor:
            t = torch.tensor(1.0 - sigma, device=dev)
            vc = self.tr(xt, t, cond)
            if uncond is not None and (1.0 - sigma) <= cfg_trunc_ratio:
                vu = self.tr(xt, t, uncond)
                v = vu + scale * (vc - vu)
                if cfg_normalization:
                    v = v * (vc.norm(dim=-1, keepdim=True) / v.norm(dim=-1, keepdim=True).clamp_min(1e-12))
            else:
                v = vc
            return -v  # Lumina's t = 0 is noise: the flow velocity is the negated output

        def denoise(xt: torch.Tensor, sigma: float) -> torch.Tensor:
            return xt - sigma * velocity(xt[0], sigma)[None]
        if init_image is not None:
            x0 = self.vae.encode(init_image.to(dev)[None] * 2 - 1)
            x0 = F.interpolate(x0, size=(h, w), mode="bilinear") if x0.shape[2:] != (h, w) else x0
            k = min(len(sig) - 2, int(round((1 - gp.strength) * (len(sig) - 1))))
            sig = sig[k:]
            x = (1 - sig[0]) * x0 + sig[0] * z[None]
        else:
            x = z[None] * sig[0]
        x = Smp.sample(denoise, x, sig, gp.sampler, flow=True, generator=gen)
        img = self.vae.decode(x)[0]
        return ((img + 1) / 2).clamp(0, 1).cpu()
