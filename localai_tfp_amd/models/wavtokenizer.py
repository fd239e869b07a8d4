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

import math
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


# ------------------------------------------------------------------------------------------------ encoder

def _pad_reflect(x: torch.Tensor, left: int, right: int) -> torch.Tensor:
    """Reflect padding that also works when the input is shorter than the pad (zero-extend first, as EnCodec)."""
    n = x.shape[-1]
    m = max(left, right)
    extra = 0
    if n <= m:
        extra = m - n + 1
        x = F.pad(x, (0, extra))
    y = F.pad(x, (left, right), mode="reflect")
    return y[..., : y.shape[-1] - extra]


def _sconv(x: torch.Tensor, w: torch.Tensor, b, stride: int = 1, dilation: int = 1) -> torch.Tensor:
    """EnCodec SConv1d, non-causal: reflect padding split around the input plus the extra right padding that
    makes the last frame whole."""
    k = (w.shape[-1] - 1) * dilation + 1
    pad_total = k - stride
    L = x.shape[-1]
    n_frames = (L - k + pad_total) / stride + 1
    extra = (math.ceil(n_frames) - 1) * stride + (k - pad_total) - L
    pr = pad_total // 2
    return F.conv1d(_pad_reflect(x, pad_total - pr, pr + extra), w, b, stride, dilation=dilation)


class WavTokenizerEncoder:
    """WavTokenizer's feature extractor for speaker creation (OuteTTS `create_speaker`): the EnCodec SEANet
    encoder (`feature_extractor.encodec.encoder.model.*`: conv 7, [residual block (ELU, conv 3, ELU, conv 1, 1x1
    shortcut), ELU, strided conv 2r] per ratio, 2-layer LSTM with skip, ELU, conv 7 to the feature width) and the
    nearest entry of the one 4096-code codebook. audio (24 kHz) -> codes at sample_rate / hop per second. The
    layer list is read from the checkpoint's keys (index kinds: conv / residual block / LSTM; gaps are ELUs), so
    ratios and widths follow the file."""

    def __init__(self, sd: dict, codebook: torch.Tensor, device="cpu"):
        from .tts import fold_weight_norm
        sd = sd.get("state_dict", sd)
        P = "feature_extractor.encodec.encoder.model."
        enc = fold_weight_norm({k[len(P):]: v.float() for k, v in sd.items() if k.startswith(P)})
        if not enc:
            raise ValueError("WavTokenizer checkpoint: no encoder (feature_extractor.encodec.encoder.model.*)")
        self.dev = torch.device(device)
        self.w = {k: v.to(self.dev) for k, v in enc.items()}
        n = 1 + max(int(k.split(".", 1)[0]) for k in enc)
        self.layers = []
        for i in range(n):
            if f"{i}.conv.conv.weight" in enc:
                k = enc[f"{i}.conv.conv.weight"].shape[-1]
                self.layers.append(("conv", f"{i}.conv.conv", k // 2 if k % 2 == 0 else 1))
            elif f"{i}.block.1.conv.conv.weight" in enc:
                self.layers.append(("res", f"{i}.", 1))
            elif f"{i}.lstm.weight_ih_l0" in enc:
                C = enc[f"{i}.lstm.weight_ih_l0"].shape[1]
                nl = sum(1 for k in enc if k.startswith(f"{i}.lstm.weight_ih_l"))
                lstm = torch.nn.LSTM(C, C, nl)
                with torch.no_grad():
                    for name, p in lstm.named_parameters():
                        p.copy_(enc[f"{i}.lstm.{name}"])
                from ..ops.rnn import LSTMStack
                lstm = lstm.to(self.dev).eval()
                self.layers.append(("lstm", (lstm, LSTMStack(lstm)), 1))
            else:
                self.layers.append(("elu", None, 1))
        self.codebook = codebook.float().to(self.dev)

    def _res(self, x, p):
        w = self.w
        h = _sconv(F.elu(x), w[p + "block.1.conv.conv.weight"], w.get(p + "block.1.conv.conv.bias"))
        h = _sconv(F.elu(h), w[p + "block.3.conv.conv.weight"], w.get(p + "block.3.conv.conv.bias"))
        sc = x if (p + "shortcut.conv.conv.weight") not in w else _sconv(
            x, w[p + "shortcut.conv.conv.weight"], w.get(p + "shortcut.conv.conv.bias"))
        return sc + h

    @torch.no_grad()
    def features(self, audio: torch.Tensor) -> torch.Tensor:
        x = audio.float().to(self.dev).view(1, 1, -1)
        for kind, p, stride in self.layers:
            if kind == "conv":
                x = _sconv(x, self.w[p + ".weight"], self.w.get(p + ".bias"), stride)
            elif kind == "res":
                x = self._res(x, p)
            elif kind == "lstm":
                lstm, scan = p
                xf = x.permute(2, 0, 1).contiguous()  # [T, 1, C]
                y = scan(xf) if x.is_cuda else lstm(xf)[0]
                x = (y + xf).permute(1, 2, 0)
            else:
                x = F.elu(x)
        return x[0].t()  # [T, feat]

    @torch.no_grad()
    def encode(self, audio: torch.Tensor) -> list[int]:
        f = self.features(audio)
        cb = self.codebook
        d = (f * f).sum(1, keepdim=True) - 2 * f @ cb.t() + (cb * cb).sum(1)[None]
        return d.argmin(1).tolist()


def load_wavtokenizer_encoder(path: str, codebook: torch.Tensor, device="cpu") -> WavTokenizerEncoder:
    if os.path.isdir(path):
        cands = [f for f in sorted(os.listdir(path)) if f.endswith((".safetensors", ".ckpt", ".pt", ".pth", ".bin"))]
        path = os.path.join(path, cands[0])
    if path.endswith(".safetensors"):
        from safetensors.torch import load_file
        sd = load_file(path)
    else:
        sd = torch.load(path, map_location="cpu", weights_only=True)
    return WavTokenizerEncoder(sd, codebook, device)


def synthetic_encoder_state(c: WavTokenizerConfig, ratios=(2, 2, 2, 2), n_filters: int = 8, seed: int = 0) -> dict:
    """Random SEANet encoder weights in the checkpoint's names (tests): hop = prod(ratios)."""
    g = torch.Generator().manual_seed(seed)

    def r(*shape):
        return torch.randn(*shape, generator=g) * (1.0 / math.sqrt(shape[1] * shape[-1]))
    P = "feature_extractor.encodec.encoder.model."
    sd, i, ch = {}, 0, n_filters
    sd[f"{P}{i}.conv.conv.weight"], sd[f"{P}{i}.conv.conv.bias"] = r(ch, 1, 7), torch.zeros(ch)
    i += 1
    for ratio in reversed(ratios):
        sd[f"{P}{i}.block.1.conv.conv.weight"], sd[f"{P}{i}.block.1.conv.conv.bias"] = r(ch // 2, ch, 3), torch.zeros(ch // 2)
        sd[f"{P}{i}.block.3.conv.conv.weight"], sd[f"{P}{i}.block.3.conv.conv.bias"] = r(ch, ch // 2, 1), torch.zeros(ch)
        sd[f"{P}{i}.shortcut.conv.conv.weight"], sd[f"{P}{i}.shortcut.conv.conv.bias"] = r(ch, ch, 1), torch.zeros(ch)
        i += 2  # residual block, ELU
        sd[f"{P}{i}.conv.conv.weight"], sd[f"{P}{i}.conv.conv.bias"] = r(2 * ch, ch, 2 * ratio), torch.zeros(2 * ch)
        ch *= 2
        i += 1
    for layer in range(2):
        for n, shape in (("weight_ih", (4 * ch, ch)), ("weight_hh", (4 * ch, ch))):
            sd[f"{P}{i}.lstm.{n}_l{layer}"] = r(*shape)
        sd[f"{P}{i}.lstm.bias_ih_l{layer}"] = torch.zeros(4 * ch)
        sd[f"{P}{i}.lstm.bias_hh_l{layer}"] = torch.zeros(4 * ch)
    i += 2  # LSTM, ELU
    sd[f"{P}{i}.conv.conv.weight"], sd[f"{P}{i}.conv.conv.bias"] = r(c.feat_dim, ch, 7), torch.zeros(c.feat_dim)
    return sd
