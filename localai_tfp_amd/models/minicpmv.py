"""MiniCPM-V 2.x image path (the `resampler` mmproj of the reference's llama.cpp worker: clip.cpp + the llava image
embedding behind grpc-server.cpp:515-546 / 1192-1210, spliced at `[img-N]`; gallery `minicpm-v-2_6`).

  image -> the source image resized to ~scale_resolution^2 area (multiples of 14) + for large images a grid of slices
  (get_sliced_grid / get_refine_size of the published MiniCPM-V processor; max 9 slices) -> per slice: SigLIP tower
  (patch conv with bias, position ids bucketed into the 70 x 70 table so any slice shape maps onto it, no CLS,
  post-LN) -> resampler (64 learned queries cross-attending to the patch features + 2-D sin-cos positions on the keys,
  LayerNorms, projection) -> [64, LLM hidden] per slice, source first, slices in row-major order.

The towers run on the repo kernels (attention_dense.hip, hipBLASLt; models/vision.ClipVision's blocks); the resampler
is a 64-query cross attention per slice (torch GEMMs + attention_dense.hip). Parity with the reference's llama.cpp is
unpinned (no MiniCPM-V implementation or fixture is available offline): the tower is pinned to transformers'
SiglipVisionModel at the native slice size, the resampler to a torch.nn.MultiheadAttention re-statement.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np
import torch
import torch.nn.functional as F

from ..ops import core as K
from .vision import ClipVision, ClipVisionConfig


@dataclass
class MiniCPMVConfig:
    vision: ClipVisionConfig
    embed_dim: int = 3584       # resampler / LLM hidden
    queries: int = 64
    heads: int = 28
    scale_resolution: int = 448
    max_slices: int = 9
    pos_side: int = 70           # position table side (980 / 14)
    max_size: tuple = (70, 70)   # sin-cos key position cache


MINICPMV_TEST = MiniCPMVConfig(vision=ClipVisionConfig(image_size=56, patch=14, hidden=64, ffn=128, heads=4, layers=2,
                                                       proj_hidden=256, eps=1e-6, act="gelu_tanh",
                                                       mean=(0.5, 0.5, 0.5), std=(0.5, 0.5, 0.5), pad_square=False,
                                                       projector="resampler", name="minicpmv-test"),
                               embed_dim=256, queries=8, heads=4, scale_resolution=56, max_slices=4, pos_side=4,
                               max_size=(8, 8))


# ------------------------------------------------------------------------------------------------ slicing
def ensure_divide(length: float, patch: int) -> int:
    return max(round(length / patch) * patch, patch)


def find_best_resize(size: tuple, scale_resolution: int, patch: int, allow_upscale: bool = False) -> tuple:
    w, h = size
    if w * h > scale_resolution * scale_resolution or allow_upscale:
        r = w / h
        h = int(scale_resolution / math.sqrt(r))
        w = int(h * r)
    return ensure_divide(w, patch), ensure_divide(h, patch)


def get_sliced_grid(size: tuple, scale_resolution: int, max_slices: int):
    w, h = size
    log_ratio = math.log(w / h)
    ratio = w * h / (scale_resolution * scale_resolution)
    multiple = min(math.ceil(ratio), max_slices)
    if multiple <= 1:
        return None
    cands = [i for i in (multiple - 1, multiple, multiple + 1) if i != 1 and i <= max_slices]
    grids = [[m, n // m] for n in cands for m in range(1, n + 1) if n % m == 0]
    best, err = [1, 1], float("inf")
    for g in grids:
        e = abs(log_ratio - math.log(g[0] / g[1]))
        if e < err:
            best, err = g, e
    return best


def get_refine_size(size: tuple, grid, scale_resolution: int, patch: int) -> tuple:
    w, h = size
    gx, gy = grid
    rw, rh = ensure_divide(w, gx), ensure_divide(h, gy)
    bw, bh = find_best_resize((rw / gx, rh / gy), scale_resolution, patch, allow_upscale=True)
    return bw * gx, bh * gy


def slice_image(img, cfg: MiniCPMVConfig) -> list:
    """[source image, slices row-major] (PIL), as the MiniCPM-V processor and clip.cpp uhd_slice_image cut them."""
    from PIL import Image
    P = cfg.vision.patch
    src = img.resize(find_best_resize(img.size, cfg.scale_resolution, P), Image.BICUBIC)
    out = [src]
    grid = get_sliced_grid(img.size, cfg.scale_resolution, cfg.max_slices)
    if grid is not None:
        rw, rh = get_refine_size(img.size, grid, cfg.scale_resolution, P)
        refine = img.resize((rw, rh), Image.BICUBIC)
        sw, sh = rw // grid[0], rh // grid[1]
        for y in range(0, rh, sh):
            for x in range(0, rw, sw):
                out.append(refine.crop((x, y, x + sw, y + sh)))
    return out


# ------------------------------------------------------------------------------------------------ positions
def sincos_2d(embed_dim: int, h: int, w: int) -> torch.Tensor:
    """The MiniCPM-V resampler's key positions [h, w, D] (get_2d_sincos_pos_embed with the w-major meshgrid)."""
    def one(d, pos):
        omega = 1.0 / 10000 ** (np.arange(d // 2, dtype=np.float32) / (d / 2.0))
        out = pos[..., None] * omega
        return np.concatenate([np.sin(out), np.cos(out)], -1)
    gw, gh = np.meshgrid(np.arange(w, dtype=np.float32), np.arange(h, dtype=np.float32))
    emb = np.concatenate([one(embed_dim // 2, gw), one(embed_dim // 2, gh)], -1)
    return torch.from_numpy(emb.astype(np.float32))


def bucket_position_ids(h: int, w: int, side: int) -> torch.Tensor:
    """Slice patch grid (h, w) -> ids into the side x side position table (Idefics2 / MiniCPM-V bucketing)."""
    bounds = torch.arange(1 / side, 1.0, 1 / side)
    fh = torch.arange(0, 1 - 1e-6, 1 / h)
    fw = torch.arange(0, 1 - 1e-6, 1 / w)
    bh = torch.bucketize(fh, bounds, right=True)
    bw = torch.bucketize(fw, bounds, right=True)
    return (bh[:, None] * side + bw[None, :]).flatten()


class MiniCPMVVision(ClipVision):
    """SigLIP slices + resampler. Weights: mmproj GGUF names (v.* tower as models/vision.py, resampler.*)."""

    def __init__(self, cfg: MiniCPMVConfig, sd: dict, device="cpu"):
        self.mcfg = cfg
        super().__init__(cfg.vision, sd, device)
        dev, dt = self.device, self.dtype
        E = cfg.embed_dim

        def f32(k):
            return sd[k].float().to(dev).contiguous()
        self.query = f32("resampler.query")
        kvw = sd.get("resampler.kv.weight")
        self.kv_proj = None if kvw is None else kvw.float().to(dev)
        self.in_w = torch.cat([sd[f"resampler.attn.{x}.weight"] for x in "qkv"]).float().to(dev)
        self.in_b = torch.cat([sd[f"resampler.attn.{x}.bias"] for x in "qkv"]).float().to(dev)
        self.out_w, self.out_b = f32("resampler.attn.out.weight"), f32("resampler.attn.out.bias")
        self.ln = {n: (f32(f"resampler.ln_{n}.weight"), f32(f"resampler.ln_{n}.bias")) for n in ("q", "kv", "post")}
        self.proj = f32("resampler.proj.weight")
        self.pos_cache = sincos_2d(E, *cfg.max_size).to(dev)
        del dt

    @property
    def proj_hidden(self) -> int:
        return self.mcfg.embed_dim

    def _tower(self, px: torch.Tensor) -> torch.Tensor:
        """One slice [3, h, w] -> post-LN patch features [h w / P^2, hidden] fp32."""
        c = self.cfg
        P, H = c.patch, c.hidden
        h, w = px.shape[1] // P, px.shape[2] // P
        x = px[None].to(self.device, torch.float32)
        cols = F.unfold(x, P, stride=P).transpose(1, 2).reshape(-1, 3 * P * P)
        pe = self.patch.f32(cols.to(self.dtype))
        ids = bucket_position_ids(h, w, self.mcfg.pos_side).to(self.device)
        hs = (pe + self.pos[ids]).contiguous()
        S = hs.shape[0]
        hd = H // c.heads
        xa = torch.empty(S, H, dtype=self.dtype, device=self.device)
        attn = torch.empty(S, H, dtype=self.dtype, device=self.device)
        for blk in self.blocks:
            K.layernorm(hs, *blk["ln1"], c.eps, xa)
            qkv = blk["qkv"](xa)
            K.attn_dense(qkv[:, :H], qkv[:, H:2 * H], qkv[:, 2 * H:], attn, 1, S, S, c.heads, c.heads, hd,
                         1.0 / math.sqrt(hd), causal=False)
            blk["out"].acc(attn, hs)
            K.layernorm(hs, *blk["ln2"], c.eps, xa)
            blk["fc2"].acc(self._act(blk["fc1"](xa)), hs)
        return F.layer_norm(hs, (H,), *self.post_ln, c.eps), (h, w)

    def _resample(self, feats: torch.Tensor, hw: tuple) -> torch.Tensor:
        m = self.mcfg
        E, nh = m.embed_dim, m.heads
        x = feats @ self.kv_proj.t() if self.kv_proj is not None else feats
        x = F.layer_norm(x, (E,), *self.ln["kv"], 1e-6)
        q = F.layer_norm(self.query, (E,), *self.ln["q"], 1e-6)
        h, w = hw
        pos = self.pos_cache[:h, :w].reshape(h * w, E) if h <= m.max_size[0] and w <= m.max_size[1] \
            else sincos_2d(E, h, w).to(self.device).reshape(h * w, E)
        wq, wk, wv = self.in_w.split(E)
        bq, bk, bv = self.in_b.split(E)
        qp, kp, vp = q @ wq.t() + bq, (x + pos) @ wk.t() + bk, x @ wv.t() + bv
        hd = E // nh
        o = torch.empty(m.queries, E, dtype=self.dtype, device=self.device)
        K.attn_dense(qp.to(self.dtype), kp.to(self.dtype), vp.to(self.dtype), o, 1, m.queries, kp.shape[0], nh, nh, hd,
                     1.0 / math.sqrt(hd), causal=False)
        y = o.float() @ self.out_w.t() + self.out_b
        y = F.layer_norm(y, (E,), *self.ln["post"], 1e-6)
        return y @ self.proj

    @torch.no_grad()
    def encode_slice(self, img) -> torch.Tensor:
        px = self.normalise(img)
        feats, hw = self._tower(px)
        return self._resample(feats, hw)

    def embed_images(self, images: list) -> list[torch.Tensor]:
        out = []
        for im in images:
            parts = slice_image(self.load_image(im), self.mcfg)
            out.append(torch.cat([self.encode_slice(p) for p in parts], 0))
        return out


def synthetic_minicpmv(cfg: MiniCPMVConfig, seed: int = 0) -> dict:
    from .vision import synthetic_clip
    vc = cfg.vision
    g = torch.Generator().manual_seed(seed + 100)
    E, H = cfg.embed_dim, vc.hidden

    def r(*s, std=0.02):
        return torch.randn(*s, generator=g) * std
    gemma_like = ClipVisionConfig(**{**vc.__dict__, "projector": "gemma3"})
    sd = {k: v for k, v in synthetic_clip(gemma_like, seed).items() if not k.startswith("mm.")}
    sd["v.position_embd.weight"] = r(cfg.pos_side ** 2, H)
    sd.update({"resampler.query": r(cfg.queries, E, std=0.5), "resampler.kv.weight": r(E, H, std=0.1),
               "resampler.attn.out.weight": r(E, E, std=0.1), "resampler.attn.out.bias": r(E),
               "resampler.proj.weight": r(E, E, std=E ** -0.5)})
    for x in "qkv":
        sd[f"resampler.attn.{x}.weight"], sd[f"resampler.attn.{x}.bias"] = r(E, E, std=0.1), r(E)
    for n in ("q", "kv", "post"):
        sd[f"resampler.ln_{n}.weight"], sd[f"resampler.ln_{n}.bias"] = 1 + r(E), r(E)
    return sd
