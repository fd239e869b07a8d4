"""WavTokenizer decoder: one 4096-entry codebook at 75 tokens/s -> 24 kHz audio (OuteTTS's audio codec).

Reference: the transformers backend's OuteTTS path (backend/python/transformers/backend.py:205-243, 509-526)
runs `outetts.InterfaceHF`, whose audio side is WavTokenizer (codes -> features -> Vocos-style backbone ->
iSTFT head). Parameter names follow the WavTokenizer checkpoint (`feature_extractor.encodec.quantizer.vq.
layers.0._codebook.embed`, `backbone.*`, `head.out.*`), loaded from safetensors or a PyTorch checkpoint
with `torch.load(weights_only=True)`.

  features = codebook[codes]                                   [T, 512]
  backbone: conv7 embed -> pos_net (2 ResNet, self-attention, 2 ResNet, GroupNorm) -> AdaLayerNorm
            -> N ConvNeXt blocks (depthwise conv7, AdaLayerNorm, MLP GELU, layer scale) -> LayerNorm
  head:     linear -> (log-magnitude, phase) over n_fft/2+1 bins -> iSTFT ("same" padding, Hann window)
The decoder is a once-per-utterance convolutional pass (T ~ 75 x seconds); it runs on PyTorch ops.
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import torch
import torch.nn.functional as F
from torch import nn


@dataclass
class WavTokenizerConfig:
    codebook: int = 4096
    feat_dim: int = 512
    dim: int = 768
    inter_dim: int = 2304
    layers: int = 12
    n_fft: int = 1280
    hop: int = 320
    adanorm: int = 4  # bandwidth embeddings (id 0 used)
    sample_rate: int = 24000


WAVTOKENIZER_75 = WavTokenizerConfig()
WAVTOKENIZER_TEST = WavTokenizerConfig(codebook=64, feat_dim=32, dim=64, inter_dim=96, layers=2, n_fft=64, hop=16)


class _AdaLN(nn.Module):
    def __init__(self, n, d):
        super().__init__()
        self.scale = nn.Embedding(n, d)
        self.shift = nn.Embedding(n, d)

    def run(self, x, cid=0):
        x = F.layer_norm(x, (x.shape[-1],), eps=1e-6)
        return x * self.scale.weight[cid] + self.shift.weight[cid]


class _Res(nn.Module):
    def __init__(self, c):
        super().__init__()
        self.norm1 = nn.GroupNorm(32, c, eps=1e-6)
        self.conv1 = nn.Conv1d(c, c, 3, padding=1)
        self.norm2 = nn.GroupNorm(32, c, eps=1e-6)
        self.conv2 = nn.Conv1d(c, c, 3, padding=1)

    def run(self, x):
        h = self.conv1(F.silu(self.norm1(x)))
        return x + self.conv2(F.silu(self.norm2(h)))


class _Attn(nn.Module):
    def __init__(self, c):
        super().__init__()
        self.norm = nn.GroupNorm(32, c, eps=1e-6)
        self.q, self.k, self.v = nn.Conv1d(c, c, 1), nn.Conv1d(c, c, 1), nn.Conv1d(c, c, 1)
        self.proj_out = nn.Conv1d(c, c, 1)

    def run(self, x):
        h = self.norm(x)
        q, k, v = self.q(h), self.k(h), self.v(h)  # [B, C, T]
        w = torch.softmax(torch.einsum("bct,bcs->bts", q, k) * q.shape[1] ** -0.5, -1)
        return x + self.proj_out(torch.einsum("bts,bcs->bct", w, v))


class _ConvNeXt(nn.Module):
    def __init__(self, c: WavTokenizerConfig):
        super().__init__()
        self.dwconv = nn.Conv1d(c.dim, c.dim, 7, padding=3, groups=c.dim)
        self.norm = _AdaLN(c.adanorm, c.dim)
        self.pwconv1 = nn.Linear(c.dim, c.inter_dim)
        self.pwconv2 = nn.Linear(c.inter_dim, c.dim)
        self.gamma = nn.Parameter(torch.full((c.dim,), 1.0 / c.layers))

    def run(self, x):
        y = self.norm.run(self.dwconv(x).transpose(1, 2))
        y = self.pwconv2(F.gelu(self.pwconv1(y))) * self.gamma
        return x + y.transpose(1, 2)


class _Backbone(nn.Module):
    def __init__(self, c: WavTokenizerConfig):
        super().__init__()
        self.embed = nn.Conv1d(c.feat_dim, c.dim, 7, padding=3)
        self.pos_net = nn.ModuleList([_Res(c.dim), _Res(c.dim), _Attn(c.dim), _Res(c.dim), _Res(c.dim),
                                      nn.GroupNorm(32, c.dim, eps=1e-6)])
        self.norm = _AdaLN(c.adanorm, c.dim)
        self.convnext = nn.ModuleList(_ConvNeXt(c) for _ in range(c.layers))
        self.final_layer_norm = nn.LayerNorm(c.dim, eps=1e-6)


class _Head(nn.Module):
    def __init__(self, c: WavTokenizerConfig):
        super().__init__()
        self.out = nn.Linear(c.dim, c.n_fft + 2)


def istft_same(spec: torch.Tensor, n_fft: int, hop: int) -> torch.Tensor:
    """Vocos' "same"-padded iSTFT: irfft per frame, Hann window, overlap-add, trim (win - hop) / 2 per side,
    divide by the window-square envelope. spec [B, n_fft/2+1, T] complex -> [B, T * hop]."""
    B, _, T = spec.shape
    win = torch.hann_window(n_fft, dtype=torch.float32, device=spec.device)
    frames = torch.fft.irfft(spec, n_fft, dim=1, norm="backward") * win[None, :, None]  # [B, n_fft, T]
    size = (T - 1) * hop + n_fft
    y = F.fold(frames, output_size=(1, size), kernel_size=(1, n_fft), stride=(1, hop))[:, 0, 0]
    env = F.fold(win.square()[None, :, None].expand(1, n_fft, T), output_size=(1, size), kernel_size=(1, n_fft),
                 stride=(1, hop))[0, 0, 0]
    pad = (n_fft - hop) // 2
    return y[:, pad:size - pad] / env[pad:size - pad].clamp_min(1e-11)


class WavTokenizerDecoder(nn.Module):
    def __init__(self, c: WavTokenizerConfig):
        super().__init__()
        self.cfg = c
        self.codebook = nn.Parameter(torch.zeros(c.codebook, c.feat_dim))
        self.backbone = _Backbone(c)
        self.head = _Head(c)

    @torch.no_grad()
    def decode(self, codes: torch.Tensor) -> torch.Tensor:
        """codes int [T] -> audio fp32 [T * hop] at cfg.sample_rate."""
        b = self.backbone
        dt = b.embed.weight.dtype
        x = self.codebook[codes.long().clamp(0, self.cfg.codebook - 1)].to(dt).T[None]  # [1, feat, T]
        x = b.embed(x)
        for m in b.pos_net:
            x = m(x) if isinstance(m, nn.GroupNorm) else m.run(x)
        x = b.norm.run(x.transpose(1, 2)).transpose(1, 2)
        for blk in b.convnext:
            x = blk.run(x)
        x = b.final_layer_norm(x.transpose(1, 2))
        s = self.head.out(x).float().transpose(1, 2)
        mag, ph = s.chunk(2, dim=1)
        mag = torch.exp(mag).clamp(max=1e2)
        return istft_same(torch.polar(mag, ph), self.cfg.n_fft, self.cfg.hop)[0]

    def load_checkpoint_dict(self, sd: dict):
        """WavTokenizer state dict (Lightning `state_dict` or plain) -> this module."""
        sd = sd.get("state_dict", sd)
        out = {}
        for k, v in sd.items():
            if not torch.is_tensor(v):
                continue
            if k.endswith("quantizer.vq.layers.0._codebook.embed"):
                out["codebook"] = v.reshape(v.shape[-2], v.shape[-1])
            elif k.startswith(("backbone.", "head.out.")):
                out[k] = v
        if "codebook" not in out:
            raise ValueError("WavTokenizer checkpoint: codebook (feature_extractor.encodec.quantizer.vq.layers.0."
                             "_codebook.embed) not found")
        missing, _ = self.load_state_dict(out, strict=False)
        if missing:
            raise ValueError(f"WavTokenizer checkpoint: missing {missing[:5]}")
        return self


def config_from_state(sd: dict) -> WavTokenizerConfig:
    sd = sd.get("state_dict", sd)
    cb = next(v for k, v in sd.items() if k.endswith("_codebook.embed"))
    n = 0
    while f"backbone.convnext.{n}.dwconv.weight" in sd:
        n += 1
    dim = sd["backbone.embed.weight"].shape[0]
    nf = sd["head.out.weight"].shape[0] - 2
    return WavTokenizerConfig(codebook=cb.shape[-2], feat_dim=cb.shape[-1], dim=dim,
                              inter_dim=sd["backbone.convnext.0.pwconv1.weight"].shape[0], layers=n, n_fft=nf,
                              hop=nf // 4, adanorm=sd["backbone.norm.scale.weight"].shape[0])


def load_wavtokenizer(path: str, device="cpu", dtype=torch.float32) -> WavTokenizerDecoder:
    """A safetensors file or a PyTorch checkpoint (loaded with weights_only=True; nothing is unpickled)."""
    if os.path.isdir(path):
        cands = [f for f in sorted(os.listdir(path)) if f.endswith((".safetensors", ".ckpt", ".pt", ".pth", ".bin"))]
        if not cands:
            raise FileNotFoundError(f"{path}: no WavTokenizer checkpoint")
        path = os.path.join(path, cands[0])
    if path.endswith(".safetensors"):
        from safetensors.torch import load_file
        sd = load_file(path)
    else:
        sd = torch.load(path, map_location="cpu", weights_only=True)
    c = config_from_state(sd)
    m = WavTokenizerDecoder(c).load_checkpoint_dict(sd)
    return m.to(device=device, dtype=dtype).eval()
