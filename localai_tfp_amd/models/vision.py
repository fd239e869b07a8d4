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
                   name=str(md.get("general.name", "clip")))


CLIP_TEST = ClipVisionConfig(image_size=56, patch=14, hidden=128, ffn=256, heads=4, layers=2, proj_hidden=256,
                             name="clip-test")
SYNTHETIC = {"clip-vit-l-336": ClipVisionConfig(), "clip-test": CLIP_TEST}


def synthetic_clip(cfg: ClipVisionConfig, seed: int = 0) -> dict:
    g = torch.Generator().manual_seed(seed)
    H, Fd, P = cfg.hidden, cfg.ffn, cfg.patch

    def r(*s, std=0.02):
        return torch.randn(*s, generator=g) * std
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


def load_mmproj(path: str, device="cpu") -> "ClipVision":
    if path.startswith("synthetic:"):
        cfg = SYNTHETIC[path.split(":", 1)[1]]
        return ClipVision(cfg, synthetic_clip(cfg), device)
    from ..formats.gguf import GGUFReader
    from ..ops.quant import dequantize
    r = GGUFReader(path)
    sd = {}
    for name, ti in r.tensors.items():
        a = dequantize(r.tensor_bytes(name), ti.qtype, ti.shape)
        sd[name] = torch.from_numpy(np.ascontiguousarray(a).reshape(tuple(reversed(ti.shape))).copy()).float()
    n_blocks = len({k.split(".")[2] for k in sd if k.startswith("v.blk.")})
    cfg = ClipVisionConfig.from_gguf_metadata(r.metadata, n_blocks)
    if str(r.metadata.get("clip.projector_type", "mlp")) != "mlp":
        raise NotImplementedError(f"projector type {r.metadata.get('clip.projector_type')!r}")
    return ClipVision(cfg, sd, device)


class ClipVision:
    def __init__(self, cfg: ClipVisionConfig, sd: dict, device="cpu"):
        self.cfg = cfg
        self.device = torch.device(device)
        self.dtype = model_dtype(device)
        dt, dev = self.dtype, self.device
        H, P = cfg.hidden, cfg.patch
        self.patch = Dense(sd["v.patch_embd.weight"].reshape(H, 3 * P * P), None, dev, dt)
        self.cls = sd["v.class_embd"].reshape(H).float().to(dev)
        self.pos = sd["v.position_embd.weight"].float().to(dev)

        def f32(k):
            return sd[k].float().to(dev).contiguous()
        self.pre_ln = (f32("v.pre_ln.weight"), f32("v.pre_ln.bias"))
        self.blocks = []
        for i in range(cfg.layers):
            p = f"v.blk.{i}."
            qkv_w = torch.cat([sd[p + f"attn_{x}.weight"] for x in "qkv"], 0)
            qkv_b = torch.cat([sd[p + f"attn_{x}.bias"] for x in "qkv"], 0)
            self.blocks.append(dict(
                ln1=(f32(p + "ln1.weight"), f32(p + "ln1.bias")), ln2=(f32(p + "ln2.weight"), f32(p + "ln2.bias")),
                qkv=Dense(qkv_w, qkv_b, dev, dt), out=Dense(sd[p + "attn_out.weight"], sd[p + "attn_out.bias"], dev, dt),
                fc1=Dense(sd[p + "ffn_down.weight"], sd[p + "ffn_down.bias"], dev, dt),
                fc2=Dense(sd[p + "ffn_up.weight"], sd[p + "ffn_up.bias"], dev, dt)))
        self.mm0 = Dense(sd["mm.0.weight"], sd["mm.0.bias"], dev, dt)
        self.mm2 = Dense(sd["mm.2.weight"], sd["mm.2.bias"], dev, dt)

    # ---------------------------------------------------------------- preprocessing
    def preprocess(self, img) -> torch.Tensor:
        """PIL image / encoded bytes / base64 string -> normalised [3, S, S] fp32 (clip_image_preprocess)."""
        from PIL import Image
        if isinstance(img, str):
            s = img.split(",", 1)[1] if img.startswith("data:") else img
            img = base64.b64decode(s)
        if isinstance(img, (bytes, bytearray)):
            img = Image.open(io.BytesIO(img))
        img = img.convert("RGB")
        c = self.cfg
        if c.pad_square and img.width != img.height:
            side = max(img.width, img.height)
            bg = Image.new("RGB", (side, side), tuple(int(255 * m) for m in c.mean))
            bg.paste(img, ((side - img.width) // 2, (side - img.height) // 2))
            img = bg
        img = img.resize((c.image_size, c.image_size), Image.BICUBIC)
        x = torch.from_numpy(np.asarray(img, dtype=np.float32) / 255.0).permute(2, 0, 1)
        return (x - torch.tensor(c.mean)[:, None, None]) / torch.tensor(c.std)[:, None, None]

    # ---------------------------------------------------------------- encoder
    def _act(self, y: torch.Tensor) -> torch.Tensor:
        if self.cfg.act == "quick_gelu":
            return y * torch.sigmoid(1.702 * y)
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
        h = torch.cat([self.cls.view(1, 1, H).expand(B, 1, H), pe], 1) + self.pos[None]
        S = h.shape[1]
        h = F.layer_norm(h.reshape(B * S, H), (H,), *self.pre_ln, c.eps).contiguous()  # residual stream (fp32)
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
        feats = h.view(B, S, H)[:, 1:].reshape(-1, H).to(self.dtype)
        y = self.mm2.f32(F.gelu(self.mm0(feats)))
        return y.view(B, c.n_patches, c.proj_hidden)

    def embed_images(self, images: list) -> list[torch.Tensor]:
        if not images:
            return []
        px = torch.stack([self.preprocess(im) for im in images])
        out = self.encode(px)
        return [out[i] for i in range(out.shape[0])]


# ------------------------------------------------------------------------------------------------
# prompt splicing (grpc-server.cpp:900-944)
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
