"""Qwen2-VL / Qwen2.5-VL vision tower + patch merger (the `qwen2vl_merger` / `qwen2.5vl_merger` mmproj of the
reference's llama.cpp worker: clip.cpp behind grpc-server.cpp:515-546, images embedded at :1192-1210 and spliced at
`[img-N]`), and the frame-list video input of the vLLM backend (backend/python/vllm/backend.py:238-252).

  image -> aspect-preserving resize to multiples of 28 within [min_pixels, max_pixels] (smart_resize) -> CLIP
  normalisation -> 14 x 14 x 2 (temporal) patches in 2 x 2 merge-group order -> patch GEMM (the Conv3d as one
  [C T P P] -> hidden matrix) -> 2-D rotary positions (row, column halves of head_dim / 2 each) -> blocks reordered
  into 8 x 8-patch windows: RMSNorm -> QKV (bias) -> 2-D RoPE -> attention over the window (full-attention blocks:
  over the image) -> proj -> RMSNorm -> SwiGLU MLP (Qwen2.5) / GELU MLP (Qwen2) -> merger: RMSNorm, 4 patches ->
  one row, Linear -> GELU -> Linear (-> LLM hidden), back to raster order of the merged 2 x 2 groups.

Windows are gathered into one padded batch and run through the repo's flash attention (attention_dense.hip) with
per-window valid lengths; GEMMs hipBLASLt (ops/dense.py). Videos: every 2 consecutive frames form one temporal
patch (grid_t = frames / 2), as the Qwen2-VL processor does; full-attention blocks attend within one temporal
patch, window blocks within a window of one temporal patch (transformers' cu_seqlens).

Weights: transformers' Qwen2_5_VisionTransformerPretrainedModel state dict names (visual.* / model.visual.*),
or a clip.cpp-style GGUF (v.patch_embd.weight + .weight.1 temporal halves, v.blk.N.attn_{q,k,v,out}, ln1 / ln2,
ffn_{gate,up,down}, v.post_ln = merger ln_q, mm.0 / mm.2). GGUF name parity with clip.cpp is unpinned (no qwen2.5vl
mmproj fixture exists offline); the numerics are pinned to transformers (tests/test_vision.py).
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np
import torch
import torch.nn.functional as F

from ..ops import core as K
from ..ops.dense import Dense, model_dtype

CLIP_MEAN = (0.48145466, 0.4578275, 0.40821073)
CLIP_STD = (0.26862954, 0.26130258, 0.27577711)


@dataclass
class QwenVLConfig:
    hidden: int = 1280
    ffn: int = 3420
    heads: int = 16
    depth: int = 32
    patch: int = 14
    temporal: int = 2
    merge: int = 2
    window: int = 112  # px; 0 = no window attention (Qwen2-VL)
    fullatt: tuple = (7, 15, 23, 31)
    out_hidden: int = 3584
    gated_mlp: bool = True  # Qwen2.5-VL SwiGLU; Qwen2-VL: fc1 -> QuickGELU -> fc2 ... (not modelled: use 2.5)
    eps: float = 1e-6
    rope_theta: float = 10000.0
    min_pixels: int = 56 * 56
    max_pixels: int = 28 * 28 * 1280
    name: str = "qwen2.5-vl"

    @property
    def head_dim(self) -> int:
        return self.hidden // self.heads


QWEN25VL_TEST = QwenVLConfig(hidden=64, ffn=96, heads=4, depth=4, window=56, fullatt=(1, 3), out_hidden=256,
                             min_pixels=28 * 28, max_pixels=28 * 28 * 64, name="qwen25vl-test")
QWEN25VL_7B = QwenVLConfig()


def smart_resize(h: int, w: int, factor: int, min_pixels: int, max_pixels: int) -> tuple[int, int]:
    """Qwen2-VL image sizing: both sides multiples of `factor`, area within [min_pixels, max_pixels], aspect kept."""
    hb = max(factor, round(h / factor) * factor)
    wb = max(factor, round(w / factor) * factor)
    if hb * wb > max_pixels:
        beta = math.sqrt(h * w / max_pixels)
        hb = max(factor, math.floor(h / beta / factor) * factor)
        wb = max(factor, math.floor(w / beta / factor) * factor)
    elif hb * wb < min_pixels:
        beta = math.sqrt(min_pixels / (h * w))
        hb = math.ceil(h * beta / factor) * factor
        wb = math.ceil(w * beta / factor) * factor
    return hb, wb


def synthetic_qwen_vl(cfg: QwenVLConfig, seed: int = 0) -> dict:
    g = torch.Generator().manual_seed(seed)
    H, Fd = cfg.hidden, cfg.ffn
    M = H * cfg.merge ** 2

    def r(*s, std=0.02):
        return torch.randn(*s, generator=g) * std
    sd = {"patch_embed.proj.weight": r(H, 3, cfg.temporal, cfg.patch, cfg.patch),
          "merger.ln_q.weight": 1 + r(H), "merger.mlp.0.weight": r(M, M), "merger.mlp.0.bias": r(M),
          "merger.mlp.2.weight": r(cfg.out_hidden, M), "merger.mlp.2.bias": r(cfg.out_hidden)}
    for i in range(cfg.depth):
        p = f"blocks.{i}."
        sd[p + "norm1.weight"], sd[p + "norm2.weight"] = 1 + r(H), 1 + r(H)
        sd[p + "attn.qkv.weight"], sd[p + "attn.qkv.bias"] = r(3 * H, H), r(3 * H)
        sd[p + "attn.proj.weight"], sd[p + "attn.proj.bias"] = r(H, H), r(H)
        for n, (o, i_) in (("gate_proj", (Fd, H)), ("up_proj", (Fd, H)), ("down_proj", (H, Fd))):
            sd[p + f"mlp.{n}.weight"], sd[p + f"mlp.{n}.bias"] = r(o, i_), r(o)
    return sd


def from_gguf_names(sd: dict) -> dict:
    """clip.cpp-style qwen2.5vl mmproj tensor names -> the transformers names this module loads."""
    out = {}
    if "v.patch_embd.weight" in sd:
        w0, w1 = sd["v.patch_embd.weight"], sd.get("v.patch_embd.weight.1", sd["v.patch_embd.weight"])
        out["patch_embed.proj.weight"] = torch.stack([w0, w1], 2)  # [H, 3, T, P, P]
    ren = {"v.post_ln.weight": "merger.ln_q.weight", "mm.0.weight": "merger.mlp.0.weight",
           "mm.0.bias": "merger.mlp.0.bias", "mm.2.weight": "merger.mlp.2.weight", "mm.2.bias": "merger.mlp.2.bias"}
    for k, v in sd.items():
        if k in ren:
            out[ren[k]] = v
        elif k.startswith("v.blk."):
            _, _, i, name, kind = k.split(".", 4)
            p = f"blocks.{i}."
            if name in ("attn_q", "attn_k", "attn_v"):
                out.setdefault(p + f"attn.qkv.{kind}", {})[name] = v
            else:
                m = {"attn_out": "attn.proj", "ln1": "norm1", "ln2": "norm2", "ffn_gate": "mlp.gate_proj",
                     "ffn_up": "mlp.up_proj", "ffn_down": "mlp.down_proj"}[name]
                out[p + f"{m}.{kind}"] = v
    for k in [k for k in out if isinstance(out[k], dict)]:
        d = out[k]
        out[k] = torch.cat([d["attn_q"], d["attn_k"], d["attn_v"]], 0)
    return out


class QwenVLVision:
    """Qwen2.5-VL vision tower + merger on the repo kernels (CPU: the same math in fp32, the numerics oracle)."""

    def __init__(self, cfg: QwenVLConfig, sd: dict, device="cpu"):
        self.cfg = cfg
        self.device = torch.device(device)
        self.dtype = model_dtype(device)
        dt, dev = self.dtype, self.device
        sd = {k.split("visual.", 1)[-1]: v for k, v in sd.items()}
        H, Pp = cfg.hidden, 3 * cfg.temporal * cfg.patch * cfg.patch

        def f32(k):
            return sd[k].float().to(dev).contiguous()
        self.patch = Dense(sd["patch_embed.proj.weight"].reshape(H, Pp), None, dev, dt)
        self.blocks = []
        for i in range(cfg.depth):
            p = f"blocks.{i}."
            blk = dict(n1=f32(p + "norm1.weight"), n2=f32(p + "norm2.weight"),
                       qkv=Dense(sd[p + "attn.qkv.weight"], sd[p + "attn.qkv.bias"], dev, dt),
                       proj=Dense(sd[p + "attn.proj.weight"], sd[p + "attn.proj.bias"], dev, dt),
                       down=Dense(sd[p + "mlp.down_proj.weight"], sd[p + "mlp.down_proj.bias"], dev, dt))
            # gate | up as one GEMM
            blk["gu"] = Dense(torch.cat([sd[p + "mlp.gate_proj.weight"], sd[p + "mlp.up_proj.weight"]], 0),
                              torch.cat([sd[p + "mlp.gate_proj.bias"], sd[p + "mlp.up_proj.bias"]], 0), dev, dt)
            self.blocks.append(blk)
        self.ln_q = f32("merger.ln_q.weight")
        self.mm0 = Dense(sd["merger.mlp.0.weight"], sd["merger.mlp.0.bias"], dev, dt)
        self.mm2 = Dense(sd["merger.mlp.2.weight"], sd["merger.mlp.2.bias"], dev, dt)
        hd = cfg.head_dim // 2
        self.inv_freq = 1.0 / (cfg.rope_theta ** (torch.arange(0, hd, 2, dtype=torch.float32) / hd))

    # ------------------------------------------------------------------ preprocessing
    def patches(self, frames: list) -> tuple[torch.Tensor, tuple]:
        """PIL frames of ONE image (1 frame) or video (>= 2) -> (flattened patches [t h w, C T P P], (t, h, w))."""
        from PIL import Image
        c = self.cfg
        f0 = frames[0]
        hb, wb = smart_resize(f0.height, f0.width, c.patch * c.merge, c.min_pixels, c.max_pixels)
        arr = []
        for im in frames:
            im = im.convert("RGB").resize((wb, hb), Image.BICUBIC)
            x = torch.from_numpy(np.asarray(im, dtype=np.float32) / 255.0).permute(2, 0, 1)
            arr.append((x - torch.tensor(CLIP_MEAN)[:, None, None]) / torch.tensor(CLIP_STD)[:, None, None])
        if len(arr) % c.temporal:  # the processor repeats the last frame to a whole temporal patch
            arr += [arr[-1]] * (c.temporal - len(arr) % c.temporal)
        x = torch.stack(arr)  # [F, C, H, W]
        gt, gh, gw = x.shape[0] // c.temporal, hb // c.patch, wb // c.patch
        m, P = c.merge, c.patch
        x = x.reshape(gt, c.temporal, 3, gh // m, m, P, gw // m, m, P)
        x = x.permute(0, 3, 6, 4, 7, 2, 1, 5, 8)
        return x.reshape(gt * gh * gw, 3 * c.temporal * P * P), (gt, gh, gw)

    def positions(self, grid: tuple) -> torch.Tensor:
        """[(t h w), 2] (row, column) of every patch in merge-group order."""
        t, h, w = grid
        m = self.cfg.merge
        hp = torch.arange(h)[:, None].expand(h, w).reshape(h // m, m, w // m, m).permute(0, 2, 1, 3).flatten()
        wp = torch.arange(w)[None, :].expand(h, w).reshape(h // m, m, w // m, m).permute(0, 2, 1, 3).flatten()
        return torch.stack([hp, wp], -1).repeat(t, 1)

    def windows(self, grid: tuple) -> tuple[torch.Tensor, list]:
        """Merge-group permutation into windows of (window / patch / merge)^2 groups, row-major per frame, and the
        window lengths in patches."""
        c = self.cfg
        t, h, w = grid
        lh, lw = h // c.merge, w // c.merge
        idx = torch.arange(t * lh * lw).reshape(t, lh, lw)
        if not c.window:
            return idx.flatten(), [t * lh * lw * c.merge ** 2]
        ws = c.window // c.merge // c.patch
        ph, pw = (-lh) % ws, (-lw) % ws
        nh, nw = (lh + ph) // ws, (lw + pw) // ws
        pad = F.pad(idx, (0, pw, 0, ph), value=-100)
        win = pad.reshape(t, nh, ws, nw, ws).permute(0, 1, 3, 2, 4).reshape(t, nh * nw, ws, ws)
        order, lens = [], []
        for ti in range(t):
            for j in range(nh * nw):
                v = win[ti, j].flatten()
                v = v[v != -100]
                if v.numel():
                    order.append(v)
                    lens.append(int(v.numel()) * c.merge ** 2)
        return torch.cat(order), lens

    # ------------------------------------------------------------------ encoder
    def _rope(self, x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor) -> torch.Tensor:
        """x [S, heads, hd] fp32, rotate-half form (apply_rotary_pos_emb_vision)."""
        h = x.shape[-1] // 2
        rot = torch.cat([-x[..., h:], x[..., :h]], -1)
        return x * cos[:, None] + rot * sin[:, None]

    def _attend(self, qkv: torch.Tensor, lens: list, cos, sin, out: torch.Tensor):
        """Attention within each segment of `lens` rows (windows or whole frames) of qkv [S, 3 H]."""
        c = self.cfg
        S, H, nh, hd = qkv.shape[0], c.hidden, c.heads, c.head_dim
        q = self._rope(qkv[:, :H].float().view(S, nh, hd), cos, sin)
        k = self._rope(qkv[:, H:2 * H].float().view(S, nh, hd), cos, sin)
        v = qkv[:, 2 * H:].float().view(S, nh, hd)
        L, B = max(lens), len(lens)
        dt = self.dtype
        qb = torch.zeros(B * L, H, dtype=dt, device=qkv.device)
        kb, vb = torch.zeros_like(qb), torch.zeros_like(qb)
        ob = torch.empty(B * L, H, dtype=dt, device=qkv.device)
        rows, r0 = [], 0
        for b, n in enumerate(lens):
            rows.append(torch.arange(b * L, b * L + n))
            r0 += n
        ridx = torch.cat(rows).to(qkv.device)
        qb[ridx] = q.reshape(S, H).to(dt)
        kb[ridx] = k.reshape(S, H).to(dt)
        vb[ridx] = v.reshape(S, H).to(dt)
        ln = torch.tensor(lens, dtype=torch.int32, device=qkv.device)
        K.attn_dense(qb, kb, vb, ob, B, L, L, nh, nh, hd, 1.0 / math.sqrt(hd), causal=False, qlen=ln, klen=ln)
        out.copy_(ob[ridx])

    @torch.no_grad()
    def encode_patches(self, px: torch.Tensor, grid: tuple) -> torch.Tensor:
        """Flattened patches of one image / video -> merged embeddings [t h w / merge^2, out_hidden] fp32."""
        c = self.cfg
        dev, dt = self.device, self.dtype
        S, H = px.shape[0], c.hidden
        U = c.merge ** 2
        h = self.patch.f32(px.to(dev, dt))  # residual stream fp32 [S, H]
        order, wlens = self.windows(grid)
        perm = (order[:, None] * U + torch.arange(U)[None]).flatten().to(dev)
        h = h[perm].contiguous()
        pos = self.positions(grid)[perm.cpu()]
        fr = (pos.float()[..., None] * self.inv_freq).flatten(1)  # [S, hd / 2]: row freqs | column freqs
        emb = torch.cat([fr, fr], -1).to(dev)
        cos, sin = emb.cos(), emb.sin()
        t, gh, gw = grid
        flens = [gh * gw] * t  # "full" attention spans one temporal patch (frame pair) of the image / video
        attn = torch.empty(S, H, dtype=dt, device=dev)
        for i, blk in enumerate(self.blocks):
            x = (h * torch.rsqrt(h.pow(2).mean(-1, keepdim=True) + c.eps) * blk["n1"]).to(dt)
            self._attend(blk["qkv"](x), flens if (i in c.fullatt or not c.window) else wlens, cos, sin, attn)
            blk["proj"].acc(attn, h)
            x = (h * torch.rsqrt(h.pow(2).mean(-1, keepdim=True) + c.eps) * blk["n2"]).to(dt)
            gu = blk["gu"](x).float()
            Fd = gu.shape[1] // 2
            blk["down"].acc((F.silu(gu[:, :Fd]) * gu[:, Fd:]).to(dt), h)
        x = (h * torch.rsqrt(h.pow(2).mean(-1, keepdim=True) + c.eps) * self.ln_q).to(dt).view(S // U, U * H)
        y = self.mm2.f32(F.gelu(self.mm0(x).float()).to(dt))
        return y[torch.argsort(order).to(dev)]

    def embed_images(self, images: list) -> list[torch.Tensor]:
        from .vision import ClipVision
        out = []
        for im in images:
            px, grid = self.patches([ClipVision.load_image(im)])
            out.append(self.encode_patches(px, grid))
        return out

    def embed_video(self, frames: list) -> torch.Tensor:
        """A video as a frame list (vLLM `videos`): PIL images / encoded bytes / base64, or one animated GIF / WebP."""
        import base64
        import io
        from PIL import Image, ImageSequence
        ims = []
        for f in frames:
            if isinstance(f, str):
                f = base64.b64decode(f.split(",", 1)[1] if f.startswith("data:") else f)
            im = Image.open(io.BytesIO(f)) if isinstance(f, (bytes, bytearray)) else f
            if getattr(im, "n_frames", 1) > 1:  # animated GIF / WebP / APNG: every frame
                ims += [fr.convert("RGB") for fr in ImageSequence.Iterator(im)]
            else:
                ims.append(im.convert("RGB"))
        px, grid = self.patches(ims)
        return self.encode_patches(px, grid)

    @property
    def proj_hidden(self) -> int:
        return self.cfg.out_hidden


def load_qwen_vl(path_or_sd, device="cpu", cfg: QwenVLConfig | None = None) -> QwenVLVision:
    """A clip.cpp-style qwen2vl / qwen2.5vl mmproj GGUF, a transformers state dict, or `synthetic:<name>`."""
    if isinstance(path_or_sd, dict):
        return QwenVLVision(cfg or QWEN25VL_7B, path_or_sd, device)
    if path_or_sd.startswith("synthetic:"):
        c = {"qwen25vl-test": QWEN25VL_TEST, "qwen2.5-vl": QWEN25VL_7B}[path_or_sd.split(":", 1)[1]]
        return QwenVLVision(c, synthetic_qwen_vl(c), device)
    from ..formats.gguf import GGUFReader
    from ..ops.quant import dequantize
    r = GGUFReader(path_or_sd)
    raw = {}
    for name, ti in r.tensors.items():
        a = dequantize(r.tensor_bytes(name), ti.qtype, ti.shape)
        raw[name] = torch.from_numpy(np.ascontiguousarray(a).reshape(tuple(reversed(ti.shape))).copy()).float()
    md = r.metadata

    def g(k, d):
        return md.get("clip.vision." + k, d)
    sd = from_gguf_names(raw)
    H = int(g("embedding_length", 1280))
    depth = len({k.split(".")[1] for k in sd if k.startswith("blocks.")})
    n_wa = int(g("n_wa_pattern", 0) or 0)
    fullatt = tuple(int(x) for x in g("wa_layer_indexes", ())) or \
        (tuple(i for i in range(depth) if n_wa and (i + 1) % n_wa == 0))
    c = QwenVLConfig(hidden=H, ffn=int(g("feed_forward_length", 3420)), heads=int(g("attention.head_count", 16)),
                     depth=depth, patch=int(g("patch_size", 14)), window=int(g("window_size", 112) if n_wa or fullatt
                                                                          else 0),
                     fullatt=fullatt, out_hidden=int(sd["merger.mlp.2.weight"].shape[0]),
                     eps=float(g("attention.layer_norm_epsilon", 1e-6)), name=str(md.get("general.name", "qwen-vl")))
    return QwenVLVision(c, sd, device)
