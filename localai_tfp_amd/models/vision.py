"""CLIP vision tower + multimodal projector (LLaVA), the image path of the reference's llama.cpp
worker (clip.cpp / llava.cpp behind grpc-server.cpp:512-546 `mmproj`, image embedding at
process_images :1192-1210, `[img-N]` prompt splicing :872-944).

  image bytes -> pad to square with the mean colour (LLaVA-1.5) -> bicubic resize -> normalise
  -> patch conv (as one GEMM over unfolded patches) + class token + positions -> pre-LN
  -> N pre-LN transformer blocks (MFMA flash attention, attention_dense.hip; LayerNorm norm.hip;
     GEMMs hipBLASLt) -> drop CLS -> projector (mlp2x_gelu: Linear -> GELU -> Linear)
  -> [n_patches, llm_hidden] embeddings spliced into the LLM prompt.

Weights: a llava `mmproj` GGUF (clip.cpp tensor names: v.patch_embd, v.class_embd,
v.position_embd, v.pre_ln, v.blk.N.{attn_q,attn_k,attn_v,attn_out,ln1,ln2,ffn_down(=fc1),
ffn_up(=fc2)}, mm.0 / mm.2) or `synthetic:<name>`. The GGUF holds the blocks clip.cpp runs
(LLaVA's "penultimate layer" features: the converter drops the last block).
"""
from __future__ import annotations

import base64
import io
import math
from dataclasses import dataclass, field

import numpy as np
import torch
import torch.nn.functional as F

from ..ops import core as K
from ..ops.dense import Dense, model_dtype


@dataclass
class ClipVisionConfig:
    image_size: int = 336
    patch: int = 14
    hidden: int = 1024
    ffn: int = 4096
    heads: int = 16
    layers: int = 23  # blocks present / run (LLaVA-1.5: 24 - 1)
    eps: float = 1e-5
    proj_hidden: int = 4096  # projector output = LLM hidden
    act: str = "quick_gelu"
    mean: tuple = (0.48145466, 0.4578275, 0.40821073)
    std: tuple = (0.26862954, 0.26130258, 0.27577711)
    pad_square: bool = True
    name: str = "clip-vit-l-336"
    # LLaVA-1.6 "anyres": candidate (width, height) canvases (clip.vision.image_grid_pinpoints); empty = 1.5 single crop
    grid_pinpoints: tuple = ()
    # projector (clip.projector_type): "mlp" (LLaVA: CLS token, pre-LN, penultimate-layer features, mlp2x_gelu) or
    # "gemma3" (SigLIP: no CLS / pre-LN, patch bias, post-LN, then avg-pool to tokens_per_image, RMSNorm, projection)
    projector: str = "mlp"
    tokens_per_image: int = 256
    resample: str = "bicubic"
    extra: dict = field(default_factory=dict)

    @property
    def n_patches(self) -> int:
        return (self.image_size // self.patch) ** 2

    @classmethod
    def from_gguf_metadata(cls, md: dict, n_blocks: int) -> "ClipVisionConfig":
        def g(k, d=None):
            return md.get("clip.vision." + k, d)
        return cls(image_size=int(g("image_size", 336)), patch=int(g("patch_size", 14)),
                   hidden=int(g("embedding_length", 1024)), ffn=int(g("feed_forward_length", 4096)),
                   heads=int(g("attention.head_count", 16)), layers=n_blocks,
                   eps=float(g("attention.layer_norm_epsilon", 1e-5)),
                   proj_hidden=int(g("projection_dim", 4096)),
                   act="gelu" if md.get("clip.use_gelu", False) else "quick_gelu",
                   mean=tuple(float(x) for x in g("image_mean", cls.mean)),
                   std=tuple(float(x) for x in g("image_std", cls.std)),
                   name=str(md.get("general.name", "clip")),
                   grid_pinpoints=_pairs(g("image_grid_pinpoints", ())),
                   pad_square=not _pairs(g("image_grid_pinpoints", ())) and
                   str(md.get("clip.projector_type", "mlp")) == "mlp",
                   projector=str(md.get("clip.projector_type", "mlp")),
                   resample="bilinear" if str(md.get("clip.projector_type", "mlp")) == "gemma3" else "bicubic")


def _pairs(v) -> tuple:
    """Flattened [w0, h0, w1, h1, ...] -> ((w0, h0), ...); clip.cpp stops at the first 0."""
    vals = [int(x) for x in (v or ())]
    out = []
    for i in range(0, len(vals) - 1, 2):
        if vals[i] == 0:
            break
        out.append((vals[i], vals[i + 1]))
    return tuple(out)


def select_best_resolution(size: tuple, candidates) -> tuple:
    """clip.cpp select_best_resolution: the (w, h) canvas that keeps the most of the image's pixels after an
    aspect-preserving downscale, ties broken by the least wasted canvas area."""
    ow, oh = size
    best, best_eff, best_waste = None, 0, None
    for w, h in candidates:
        scale = min(w / ow, h / oh)
        dw, dh = int(ow * scale), int(oh * scale)
        eff = min(dw * dh, ow * oh)
        waste = w * h - eff
        if eff > best_eff or (eff == best_eff and (best_waste is None or waste < best_waste)):
            best, best_eff, best_waste = (w, h), eff, waste
    return best


def resize_and_pad(img, target: tuple):
    """clip.cpp resize_and_pad_image: aspect-preserving bicubic resize into the (w, h) canvas, centred on black."""
    from PIL import Image
    tw, th = target
    sw, sh = tw / img.width, th / img.height
    if sw < sh:
        nw, nh = tw, min(math.ceil(img.height * sw), th)
    else:
        nw, nh = min(math.ceil(img.width * sh), tw), th
    r = img.resize((nw, nh), Image.BICUBIC)
    out = Image.new("RGB", (tw, th), (0, 0, 0))
    out.paste(r, ((tw - nw) // 2, (th - nh) // 2))
    return out


CLIP_TEST = ClipVisionConfig(image_size=56, patch=14, hidden=128, ffn=256, heads=4, layers=2, proj_hidden=256,
                             name="clip-test")
CLIP_TEST_ANYRES = ClipVisionConfig(image_size=56, patch=14, hidden=128, ffn=256, heads=4, layers=2, proj_hidden=256,
                                    name="clip-test-anyres", grid_pinpoints=((56, 112), (112, 56), (112, 112)),
                                    pad_square=False)
GEMMA3_TEST = ClipVisionConfig(image_size=56, patch=14, hidden=128, ffn=256, heads=4, layers=2, proj_hidden=256,
                               name="gemma3-test", projector="gemma3", tokens_per_image=4, eps=1e-6, act="gelu_tanh",
                               mean=(0.5, 0.5, 0.5), std=(0.5, 0.5, 0.5), pad_square=False, resample="bilinear")
# Gemma-3 mmproj (gemma-3-*-it mmproj): SigLIP-So400m/14 at 896 px, 4x4 average pool -> 256 tokens
GEMMA3_SIGLIP = ClipVisionConfig(image_size=896, patch=14, hidden=1152, ffn=4304, heads=16, layers=27, proj_hidden=3840,
                                 name="gemma3-siglip", projector="gemma3", tokens_per_image=256, eps=1e-6,
                                 act="gelu_tanh", mean=(0.5, 0.5, 0.5), std=(0.5, 0.5, 0.5), pad_square=False,
                                 resample="bilinear")
# LLaVA-1.6 (llava-v1.6-*-mmproj): ViT-L/14-336 with the 5 anyres canvases of the published configs
LLAVA16 = ClipVisionConfig(name="llava-v1.6-clip", pad_square=False,
                           grid_pinpoints=((336, 672), (672, 336), (672, 672), (1008, 336), (336, 1008)))
SYNTHETIC = {"clip-vit-l-336": ClipVisionConfig(), "clip-test": CLIP_TEST, "clip-test-anyres": CLIP_TEST_ANYRES,
             "llava-v1.6-clip": LLAVA16, "gemma3-test": GEMMA3_TEST, "gemma3-siglip": GEMMA3_SIGLIP}


def synthetic_clip(cfg: ClipVisionConfig, seed: int = 0) -> dict:
    g = torch.Generator().manual_seed(seed)
    H, Fd, P = cfg.hidden, cfg.ffn, cfg.patch

    def r(*s, std=0.02):
        return torch.randn(*s, generator=g) * std
    if cfg.projector == "gemma3":
        sd = {"v.patch_embd.weight": r(H, 3, P, P), "v.patch_embd.bias": r(H),
              "v.position_embd.weight": r(cfg.n_patches, H), "v.post_ln.weight": 1 + r(H), "v.post_ln.bias": r(H),
              "mm.soft_emb_norm.weight": 1 + r(H), "mm.input_projection.weight": r(H, cfg.proj_hidden)}
        for i in range(cfg.layers):
            p = f"v.blk.{i}."
            for n in ("attn_q", "attn_k", "attn_v", "attn_out"):
                sd[p + n + ".weight"], sd[p + n + ".bias"] = r(H, H), r(H)
            sd[p + "ffn_up.weight"], sd[p + "ffn_up.bias"] = r(Fd, H), r(Fd)  # fc1 (gguf-py naming)
            sd[p + "ffn_down.weight"], sd[p + "ffn_down.bias"] = r(H, Fd), r(H)
            for n in ("ln1", "ln2"):
                sd[p + n + ".weight"], sd[p + n + ".bias"] = 1 + r(H), r(H)
        return sd
    sd = {"v.patch_embd.weight": r(H, 3, P, P), "v.class_embd": r(H), "v.position_embd.weight": r(cfg.n_patches + 1, H),
          "v.pre_ln.weight": 1 + r(H), "v.pre_ln.bias": r(H),
          "mm.0.weight": r(cfg.proj_hidden, H), "mm.0.bias": r(cfg.proj_hidden),
          "mm.2.weight": r(cfg.proj_hidden, cfg.proj_hidden), "mm.2.bias": r(cfg.proj_hidden)}
    for i in range(cfg.layers):
        p = f"v.blk.{i}."
        for n in ("attn_q", "attn_k", "attn_v", "attn_out"):
            sd[p + n + ".weight"], sd[p + n + ".bias"] = r(H, H), r(H)
        sd[p + "ffn_down.weight"], sd[p + "ffn_down.bias"] = r(Fd, H), r(Fd)
        sd[p + "ffn_up.weight"], sd[p + "ffn_up.bias"] = r(H, Fd), r(H)
        for n in ("ln1", "ln2"):
            sd[p + n + ".weight"], sd[p + n + ".bias"] = 1 + r(H), r(H)
    return sd


QWEN_VL_PROJECTORS = ("qwen2vl_merger", "qwen2.5vl_merger", "qwen25vl", "qwen2vl")


def load_mmproj(path: str, device="cpu"):
    """An mmproj GGUF (clip.projector_type mlp / gemma3 -> ClipVision; qwen2vl_merger / qwen2.5vl_merger ->
    models/qwen_vl.QwenVLVision) or `synthetic:<name>`."""
    if path.startswith("synthetic:"):
        name = path.split(":", 1)[1]
        if name.startswith("qwen"):
            from .qwen_vl import load_qwen_vl
            return load_qwen_vl(path, device)
        if name.startswith("minicpmv"):
            from .minicpmv import MINICPMV_TEST, MiniCPMVVision, synthetic_minicpmv
            return MiniCPMVVision(MINICPMV_TEST, synthetic_minicpmv(MINICPMV_TEST), device)
        cfg = SYNTHETIC[name]
        return ClipVision(cfg, synthetic_clip(cfg, seed=0), device)
    from ..formats.gguf import GGUFReader
    from ..ops.quant import dequantize
    r = GGUFReader(path)
    if str(r.metadata.get("clip.projector_type", "mlp")) in QWEN_VL_PROJECTORS:
        from .qwen_vl import load_qwen_vl
        return load_qwen_vl(path, device)
    sd = {}
    for name, ti in r.tensors.items():
        a = dequantize(r.tensor_bytes(name), ti.qtype, ti.shape)
        sd[name] = torch.from_numpy(np.ascontiguousarray(a).reshape(tuple(reversed(ti.shape))).copy()).float()
    n_blocks = len({k.split(".")[2] for k in sd if k.startswith("v.blk.")})
    cfg = ClipVisionConfig.from_gguf_metadata(r.metadata, n_blocks)
    if cfg.projector == "resampler":  # MiniCPM-V
        from .minicpmv import MiniCPMVConfig, MiniCPMVVision
        qd = sd["resampler.query"].shape
        cfg.act, cfg.pad_square = "gelu_tanh", False
        side = int(round(sd["v.position_embd.weight"].shape[0] ** 0.5))
        mc = MiniCPMVConfig(vision=cfg, embed_dim=int(qd[1]), queries=int(qd[0]), heads=max(1, int(qd[1]) // 128),
                            scale_resolution=int(r.metadata.get("clip.vision.image_size", 448) or 448), pos_side=side)
        return MiniCPMVVision(mc, sd, device)
    if cfg.projector not in ("mlp", "gemma3"):
        raise NotImplementedError(f"projector type {cfg.projector!r} (supported: mlp / LLaVA-1.5 and -1.6, gemma3, "
                                  f"resampler / MiniCPM-V, qwen2vl_merger / qwen2.5vl_merger)")
    if cfg.projector == "gemma3":
        cfg.proj_hidden = int(sd["mm.input_projection.weight"].shape[1])
        cfg.act = "gelu_tanh"
        n_tok = int(r.metadata.get("clip.vision.mm_tokens_per_image", 256) or 256)
        cfg.tokens_per_image = n_tok
    return ClipVision(cfg, sd, device)


class ClipVision:
    def __init__(self, cfg: ClipVisionConfig, sd: dict, device="cpu"):
        self.cfg = cfg
        self.device = torch.device(device)
        self.dtype = model_dtype(device)
        dt, dev = self.dtype, self.device
        H, P = cfg.hidden, cfg.patch
        self.patch = Dense(sd["v.patch_embd.weight"].reshape(H, 3 * P * P), sd.get("v.patch_embd.bias"), dev, dt)
        self.cls = sd["v.class_embd"].reshape(H).float().to(dev) if "v.class_embd" in sd else None
        self.pos = sd["v.position_embd.weight"].float().to(dev)

        def f32(k):
            return sd[k].float().to(dev).contiguous()
        self.pre_ln = (f32("v.pre_ln.weight"), f32("v.pre_ln.bias")) if "v.pre_ln.weight" in sd else None
        self.post_ln = (f32("v.post_ln.weight"), f32("v.post_ln.bias")) if "v.post_ln.weight" in sd else None
        self.blocks = []
        for i in range(cfg.layers):
            p = f"v.blk.{i}."
            qkv_w = torch.cat([sd[p + f"attn_{x}.weight"] for x in "qkv"], 0)
            qkv_b = torch.cat([sd[p + f"attn_{x}.bias"] for x in "qkv"], 0)
            # fc1 (hidden -> ffn) / fc2: the LLaVA surgery scripts stored fc1 as ffn_down, gguf-py as ffn_up; pick by
            # shape, as clip.cpp does
            a, b = p + "ffn_down", p + "ffn_up"
            if sd[a + ".weight"].shape[1] != H:
                a, b = b, a
            self.blocks.append(dict(
                ln1=(f32(p + "ln1.weight"), f32(p + "ln1.bias")), ln2=(f32(p + "ln2.weight"), f32(p + "ln2.bias")),
                qkv=Dense(qkv_w, qkv_b, dev, dt), out=Dense(sd[p + "attn_out.weight"], sd[p + "attn_out.bias"], dev, dt),
                fc1=Dense(sd[a + ".weight"], sd[a + ".bias"], dev, dt),
                fc2=Dense(sd[b + ".weight"], sd[b + ".bias"], dev, dt)))
        if cfg.projector == "gemma3":
            self.soft_norm = f32("mm.soft_emb_norm.weight")  # (1 + w) as the gguf converter stores it
            self.mm_proj = Dense(sd["mm.input_projection.weight"].t().contiguous(), None, dev, dt)
        elif cfg.projector == "mlp":
            self.mm0 = Dense(sd["mm.0.weight"], sd["mm.0.bias"], dev, dt)
            self.mm2 = Dense(sd["mm.2.weight"], sd["mm.2.bias"], dev, dt)
        # "resampler" (MiniCPM-V): models/minicpmv.py adds its own projector

    # ---------------------------------------------------------------- preprocessing
    @staticmethod
    def load_image(img):
        from PIL import Image
        if isinstance(img, str):
            s = img.split(",", 1)[1] if img.startswith("data:") else img
            img = base64.b64decode(s)
        if isinstance(img, (bytes, bytearray)):
            img = Image.open(io.BytesIO(img))
        return img.convert("RGB")

    def normalise(self, img) -> torch.Tensor:
        c = self.cfg
        x = torch.from_numpy(np.asarray(img, dtype=np.float32) / 255.0).permute(2, 0, 1)
        return (x - torch.tensor(c.mean)[:, None, None]) / torch.tensor(c.std)[:, None, None]

    def anyres_crops(self, img) -> tuple[list, tuple]:
        """LLaVA-1.6 crops (clip.cpp clip_image_preprocess, grid pinpoints): the whole image bicubic-resized to one
        crop, then the best canvas (select_best_resolution) cut into image_size crops in row-major order.
        -> ([crops as [3, S, S]], (grid columns, grid rows))."""
        from PIL import Image
        img = self.load_image(img)
        S = self.cfg.image_size
        w, h = select_best_resolution((img.width, img.height), self.cfg.grid_pinpoints)
        canvas = resize_and_pad(img, (w, h))
        crops = [self.normalise(img.resize((S, S), Image.BICUBIC))]
        for y in range(0, h, S):
            for x in range(0, w, S):
                crops.append(self.normalise(canvas.crop((x, y, x + S, y + S))))
        return crops, (w // S, h // S)

    def preprocess(self, img) -> torch.Tensor:
        """PIL image / encoded bytes / base64 string -> normalised [3, S, S] fp32 (clip_image_preprocess)."""
        from PIL import Image
        img = self.load_image(img)
        c = self.cfg
        if c.pad_square and img.width != img.height:
            side = max(img.width, img.height)
            bg = Image.new("RGB", (side, side), tuple(int(255 * m) for m in c.mean))
            bg.paste(img, ((side - img.width) // 2, (side - img.height) // 2))
            img = bg
        img = img.resize((c.image_size, c.image_size), Image.BILINEAR if c.resample == "bilinear" else Image.BICUBIC)
        x = torch.from_numpy(np.asarray(img, dtype=np.float32) / 255.0).permute(2, 0, 1)
        return (x - torch.tensor(c.mean)[:, None, None]) / torch.tensor(c.std)[:, None, None]

    # ---------------------------------------------------------------- encoder
    def _act(self, y: torch.Tensor) -> torch.Tensor:
        if self.cfg.act == "quick_gelu":
            return y * torch.sigmoid(1.702 * y)
        if self.cfg.act == "gelu_tanh":
            return F.gelu(y, approximate="tanh")
        return F.gelu(y)

    @torch.no_grad()
    def encode(self, pixels: torch.Tensor) -> torch.Tensor:
        """[B, 3, S, S] normalised -> projected patch embeddings [B, n_patches, proj_hidden] fp32."""
        c = self.cfg
        B = pixels.shape[0]
        P, H = c.patch, c.hidden
        x = pixels.to(self.device, torch.float32)
        cols = F.unfold(x, P, stride=P).transpose(1, 2).reshape(-1, 3 * P * P)  # [B*np, 3PP]
        pe = self.patch.f32(cols.to(self.dtype)).view(B, c.n_patches, H)
        h = (torch.cat([self.cls.view(1, 1, H).expand(B, 1, H), pe], 1) if self.cls is not None else pe) + self.pos[None]
        S = h.shape[1]
        h = h.reshape(B * S, H)
        if self.pre_ln is not None:
            h = F.layer_norm(h, (H,), *self.pre_ln, c.eps)
        h = h.contiguous()  # residual stream (fp32)
        hd = H // c.heads
        xa = torch.empty(B * S, H, dtype=self.dtype, device=self.device)
        attn = torch.empty(B * S, H, dtype=self.dtype, device=self.device)
        for blk in self.blocks:
            K.layernorm(h, *blk["ln1"], c.eps, xa)
            qkv = blk["qkv"](xa)
            K.attn_dense(qkv[:, :H], qkv[:, H:2 * H], qkv[:, 2 * H:], attn, B, S, S, c.heads, c.heads, hd,
                         1.0 / math.sqrt(hd), causal=False)
            blk["out"].acc(attn, h)
            K.layernorm(h, *blk["ln2"], c.eps, xa)
            blk["fc2"].acc(self._act(blk["fc1"](xa)), h)
        if c.projector == "gemma3":
            return self._gemma3_project(h, B)
        feats = h.view(B, S, H)[:, 1:].reshape(-1, H).to(self.dtype)
        y = self.mm2.f32(F.gelu(self.mm0(feats)))
        return y.view(B, c.n_patches, c.proj_hidden)

    def _gemma3_project(self, h: torch.Tensor, B: int) -> torch.Tensor:
        """clip.cpp PROJECTOR_TYPE_GEMMA3: post-LN, [side x side] patch grid average-pooled to tokens_per_image,
        RMSNorm with the (1 + w) soft-embedding norm, then x @ mm_input_projection (-> LLM hidden)."""
        c = self.cfg
        H = c.hidden
        h = F.layer_norm(h, (H,), *self.post_ln, c.eps)
        side, ts = c.image_size // c.patch, int(round(c.tokens_per_image ** 0.5))
        k = side // ts
        g = h.view(B, side, side, H).permute(0, 3, 1, 2)
        pooled = F.avg_pool2d(g, k, k).flatten(2).transpose(1, 2).reshape(-1, H)  # [B * tokens, H]
        normed = pooled * torch.rsqrt(pooled.pow(2).mean(-1, keepdim=True) + c.eps) * self.soft_norm
        y = self.mm_proj.f32(normed.to(self.dtype))
        return y.view(B, c.tokens_per_image, c.proj_hidden)

    @property
    def proj_hidden(self) -> int:
        return self.cfg.proj_hidden

    @property
    def tokens_per_image(self) -> int:
        return self.cfg.tokens_per_image if self.cfg.projector == "gemma3" else self.cfg.n_patches

    def embed_images(self, images: list) -> list[torch.Tensor]:
        if not images:
            return []
        if self.cfg.grid_pinpoints:
            return [self.embed_anyres(im) for im in images]
        px = torch.stack([self.preprocess(im) for im in images])
        out = self.encode(px)
        return [out[i] for i in range(out.shape[0])]

    def embed_anyres(self, img) -> torch.Tensor:
        """LLaVA-1.6 as llava.cpp clip_llava_handle_patches runs it: the whole-image crop's n_patches embeddings,
        then the grid crops' embeddings re-ordered into the raster of the whole canvas (grid row, patch row, grid
        column, patch column) — no unpadding and no image_newline rows (llava.cpp: "append without newline tokens")."""
        crops, (gw, gh) = self.anyres_crops(img)
        feats = self.encode(torch.stack(crops))  # [1 + gw gh, n, H]
        side = self.cfg.image_size // self.cfg.patch
        Hp = feats.shape[-1]
        grid = feats[1:].view(gh, gw, side, side, Hp).permute(0, 2, 1, 3, 4).reshape(gh * side * gw * side, Hp)
        return torch.cat([feats[0], grid], 0)


# ------------------------------------------------------------------------------------------------
# prompt splicing (grpc-server.cpp:900-944)
_MEDIA = None


def split_media(prompt: str, n_images: int, n_videos: int) -> list:
    """Prompt -> text pieces and ("img" | "vid", index) markers: `[img-N]` / `[vid-N]` (llama.cpp worker style) or
    the Qwen2-VL chat template's `<|image_pad|>` / `<|video_pad|>` (the i-th pad is medium i, the vLLM style).
    Without any marker the media precede the text (images, then videos)."""
    import re
    global _MEDIA
    if _MEDIA is None:
        _MEDIA = re.compile(r"\[img-([^\]]*)\]|\[vid-([^\]]*)\]|<\|image_pad\|>|<\|video_pad\|>")
    out, pos, ni, nv = [], 0, 0, 0
    for m in _MEDIA.finditer(prompt):
        out.append(prompt[pos:m.start()])
        tok = m.group(0)
        if tok == "<|image_pad|>":
            kind, idx = "img", ni
            ni += 1
        elif tok == "<|video_pad|>":
            kind, idx = "vid", nv
            nv += 1
        else:
            kind = "img" if tok.startswith("[img") else "vid"
            try:
                idx = int(m.group(1) if kind == "img" else m.group(2))
            except ValueError:
                raise ValueError(f"Invalid {'image' if kind == 'img' else 'video'} number id in prompt") from None
        lim = n_images if kind == "img" else n_videos
        if not 0 <= idx < lim:
            raise ValueError(f"{'Image' if kind == 'img' else 'Video'} with id: {idx}, not found.")
        out.append((kind, idx))
        pos = m.end()
    out.append(prompt[pos:])
    if len(out) == 1 and (n_images or n_videos):
        media = [("img", i) for i in range(n_images)] + [("vid", i) for i in range(n_videos)]
        out = [""]
        for md in media:
            out += [md, ""]
        out[-1] = prompt
    return out


def split_prompt(prompt: str, n_images: int) -> list:
    """'a [img-0] b [img-1] c' -> ['a ', 0, ' b ', 1, ' c']; ids must be < n_images."""
    out, pos = [], 0
    while True:
        i = prompt.find("[img-", pos)
        if i < 0:
            break
        j = prompt.find("]", i)
        if j < 0:
            break
        try:
            iid = int(prompt[i + 5:j])
        except ValueError:
            raise ValueError("Invalid image number id in prompt") from None
        if not 0 <= iid < n_images:
            raise ValueError(f"Image with id: {iid}, not found.")
        out.append(prompt[pos:i])
        out.append(iid)
        pos = j + 1
    out.append(prompt[pos:])
    return out
