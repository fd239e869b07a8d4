"""Coqui XTTS-v2 (the reference's `coqui` backend with an XTTS model: backend/python/coqui/backend.py:60-83 —
`TTS(model)`, `tts_to_file(text, speaker_wav=AudioPath, language=...)`, or a named speaker via `voice`).

The pipeline, inference only (Coqui TTS `Xtts.inference`, XTTS-v2 `config.json` `model_args`):

1. Voice conditioning, once per reference clip:
   * GPT conditioning latents: the 22.05 kHz clip in 6 s chunks, each a log-mel (80 HTK-scale Slaney-normalised
     bins, n_fft 2048, hop 256, window 1024, f_max 8 kHz) divided by `mel_stats`. Each chunk runs the
     conditioning encoder: a 1x1 conv, then 6 attention blocks (GroupNorm32, 1x1-conv qkv, the legacy head
     split, and a residual on the normed input). Then a 2-layer Perceiver resampler (32 latents; the keys /
     values include the latents; GEGLU FF; RMSNorm). The chunk results are averaged, giving [1, 32, 1024].
   * speaker embedding: a 16 kHz clip, pre-emphasis, a 64-bin log-mel, an instance norm, then a ResNet with
     squeeze-excitation blocks ([3, 4, 6, 3] x [32, 64, 128, 256], BatchNorm after ReLU), attentive statistics
     pooling and a linear layer to 512. The result is L2-normalised.
2. The GPT-2 code LM (30 layers x 1024, 16 heads, gelu_new, its own learned text / audio position tables, no
   wpe). The prefix is [conditioning latents | start_text + BPE text + stop_text]. Audio codes (1024 + start /
   stop) are sampled with top-k 50, top-p 0.85, temperature 0.75 and repetition penalty 10 until the stop code.
   The trunk is the Bark GPT core of this framework (models/bark.py `_GPT`: MFMA flash attention over a dense KV
   cache, with the decode step replayed as one HIP graph). Logits come from final_norm then mel_head, after the
   GPT-2 ln_f.
3. Latents: one teacher-forced pass over [start | codes | stop | stop] gives the final-normed hidden states of
   [start | codes].
4. HiFi-GAN decoder: the latents are interpolated x4 (the 1024-sample code stride against a 256-sample hop) and
   by 24000 / 22050. Then conv_pre plus cond_layer(g), and 4 upsamplings (8, 8, 2, 2; k = 2r) each followed by
   + conds[i](g). The MRF ResBlock1 kernels are 3 / 7 / 11 with dilations 1 / 3 / 5, then conv_post and tanh.
   The result is a 24 kHz waveform. On the GPU the convolutions run on conv.hip as in the VITS vocoder
   (models/tts.py).

Checkpoints: an XTTS model directory holds config.json (`"model": "xtts"`), model.pth (its `"model"` state dict
in Coqui's names: `gpt.*`, `hifigan_decoder.*`, `mel_stats`), vocab.json, optionally speakers_xtts.pth (named
voices) and mel_stats.pth. Everything is read with `torch.load(weights_only=True)`, and a file that needs the
unsafe loader is refused. The `tokenizers` library reads the BPE vocabulary. Text is lower-cased, digits are
spelled out in English, the text becomes `[lang]text`, and spaces become `[SPACE]`. Parity with Coqui's XTTS
output is unpinned: `TTS` is not importable here, and no checkpoint is available offline. The tests run
synthetic weights of the same layout (tests/test_xtts.py).
"""
from __future__ import annotations

import json
import logging
import math
import os
import re
from dataclasses import dataclass

import numpy as np
import torch
import torch.nn.functional as F

from .bark import _GPT
from .tts import fold_weight_norm

log = logging.getLogger("localai_tfp_amd.xtts")


@dataclass
class XttsConfig:
    gpt_layers: int = 30
    gpt_dim: int = 1024
    gpt_heads: int = 16
    text_tokens: int = 6681
    audio_tokens: int = 1026
    start_text: int = 261
    stop_text: int = 0
    start_audio: int = 1024
    stop_audio: int = 1025
    max_audio_tokens: int = 605
    max_text_tokens: int = 402
    code_stride: int = 1024
    cond_heads: int = 16
    cond_blocks: int = 6
    perceiver_latents: int = 32
    perceiver_depth: int = 2
    perceiver_heads: int = 8
    perceiver_dim_head: int = 64
    input_sr: int = 22050
    output_sr: int = 24000
    output_hop: int = 256
    d_vector: int = 512
    upsample_initial: int = 512
    upsample_rates: tuple = (8, 8, 2, 2)
    upsample_kernels: tuple = (16, 16, 4, 4)
    resblock_kernels: tuple = (3, 7, 11)
    resblock_dilations: tuple = ((1, 3, 5), (1, 3, 5), (1, 3, 5))
    spk_layers: tuple = (3, 4, 6, 3)
    spk_filters: tuple = (32, 64, 128, 256)
    spk_mels: int = 64
    # generation (Coqui XTTS-v2 config defaults)
    temperature: float = 0.75
    top_k: int = 50
    top_p: float = 0.85
    repetition_penalty: float = 10.0
    length_penalty: float = 1.0
    cond_len_s: float = 30.0
    cond_chunk_s: float = 6.0

    @classmethod
    def from_json(cls, cfg: dict) -> "XttsConfig":
        ma = cfg.get("model_args") or {}
        c = cls()
        m = {"gpt_layers": "gpt_layers", "gpt_dim": "gpt_n_model_channels", "gpt_heads": "gpt_n_heads",
             "text_tokens": "gpt_number_text_tokens", "audio_tokens": "gpt_num_audio_tokens",
             "start_text": "gpt_start_text_token", "stop_text": "gpt_stop_text_token",
             "start_audio": "gpt_start_audio_token", "stop_audio": "gpt_stop_audio_token",
             "max_audio_tokens": "gpt_max_audio_tokens", "max_text_tokens": "gpt_max_text_tokens",
             "code_stride": "gpt_code_stride_len", "input_sr": "input_sample_rate", "output_sr": "output_sample_rate",
             "output_hop": "output_hop_length", "d_vector": "d_vector_dim"}
        for k, src in m.items():
            if ma.get(src) is not None:
                setattr(c, k, type(getattr(c, k))(ma[src]))
        for k in ("temperature", "top_k", "top_p", "repetition_penalty", "length_penalty"):
            if cfg.get(k) is not None:
                setattr(c, k, type(getattr(c, k))(cfg[k]))
        if cfg.get("gpt_cond_len") is not None:
            c.cond_len_s = float(cfg["gpt_cond_len"])
        if cfg.get("gpt_cond_chunk_len") is not None:
            c.cond_chunk_s = float(cfg["gpt_cond_chunk_len"])
        return c


# ------------------------------------------------------------------------------------------------ audio features

def mel_filters(sr: int, n_fft: int, n_mels: int, fmin: float = 0.0, fmax: float | None = None,
                slaney_norm: bool = False) -> torch.Tensor:
    """HTK-scale triangular filters [n_fft // 2 + 1, n_mels] (torchaudio's MelSpectrogram default scale), area-
    normalised when slaney_norm (its norm="slaney")."""
    fmax = sr / 2 if fmax is None else fmax

    def hz2mel(f):
        return 2595.0 * np.log10(1.0 + np.asarray(f, np.float64) / 700.0)

    def mel2hz(m):
        return 700.0 * (10.0 ** (np.asarray(m, np.float64) / 2595.0) - 1.0)

    freqs = np.linspace(0, sr / 2, n_fft // 2 + 1)
    pts = mel2hz(np.linspace(hz2mel(fmin), hz2mel(fmax), n_mels + 2))
    fdiff = np.diff(pts)
    slopes = pts[None, :] - freqs[:, None]
    down = -slopes[:, :-2] / fdiff[:-1]
    up = slopes[:, 2:] / fdiff[1:]
    fb = np.maximum(0.0, np.minimum(down, up))
    if slaney_norm:
        fb *= (2.0 / (pts[2:n_mels + 2] - pts[:n_mels]))[None, :]
    return torch.from_numpy(fb.astype(np.float32))


def power_mel(x: torch.Tensor, fb: torch.Tensor, n_fft: int, hop: int, win: int, window: str = "hann") -> torch.Tensor:
    """x [T] fp32 -> mel power [n_mels, frames] (centered reflect-padded STFT, |X|^2, filterbank)."""
    w = (torch.hann_window(win, device=x.device) if window == "hann" else torch.hamming_window(win, device=x.device))
    spec = torch.stft(x, n_fft, hop_length=hop, win_length=win, window=w, center=True, pad_mode="reflect",
                      return_complex=True)
    return fb.to(x.device).t() @ spec.abs().pow(2)


def resample(x: np.ndarray, sr: int, target: int) -> np.ndarray:
    from ..utils.audio import resample as _rs
    return np.asarray(_rs(np.asarray(x, np.float32), sr, target), np.float32)


# ------------------------------------------------------------------------------------------------ conditioning

def _legacy_attention(qkv: torch.Tensor, heads: int) -> torch.Tensor:
    """Tortoise QKVAttentionLegacy: qkv [B, 3 H C, T] with the per-head [q | k | v] channel layout."""
    B, W, T = qkv.shape
    ch = W // (3 * heads)
    q, k, v = qkv.reshape(B * heads, 3 * ch, T).split(ch, dim=1)
    scale = 1.0 / math.sqrt(math.sqrt(ch))
    w = torch.softmax(torch.einsum("bct,bcs->bts", q * scale, k * scale).float(), dim=-1).to(qkv.dtype)
    return torch.einsum("bts,bcs->bct", w, v).reshape(B, -1, T)


class _SpeakerEncoder:
    """ResNet-SE speaker encoder (16 kHz audio -> L2-normalised 512-d embedding)."""

    def __init__(self, sd: dict, p: str, cfg: XttsConfig, device):
        self.dev = torch.device(device)
        self.cfg = cfg
        g = lambda k: sd[p + k].float().to(self.dev)  # noqa: E731
        self.g, self.has = g, lambda k: (p + k) in sd  # noqa: E731
        fb = sd.get(p + "torch_spec.1.mel_scale.fb")
        self.fb = fb.float().to(self.dev) if fb is not None else mel_filters(16000, 512, cfg.spk_mels).to(self.dev)
        pre = sd.get(p + "torch_spec.0.filter")
        self.coef = float(-pre.flatten()[0]) if pre is not None else 0.97

    def _bn(self, x, name):
        g = self.g
        return F.batch_norm(x, g(name + ".running_mean"), g(name + ".running_var"), g(name + ".weight"),
                            g(name + ".bias"), False, 0.0, 1e-5)

    def _block(self, x, name, stride):
        g = self.g
        out = F.conv2d(x, g(name + ".conv1.weight"), None, stride, 1)
        out = self._bn(F.relu(out), name + ".bn1")
        out = self._bn(F.conv2d(out, g(name + ".conv2.weight"), None, 1, 1), name + ".bn2")
        y = out.mean(dim=(2, 3))
        y = torch.sigmoid(F.linear(F.relu(F.linear(y, g(name + ".se.fc.0.weight"), g(name + ".se.fc.0.bias"))),
                                   g(name + ".se.fc.2.weight"), g(name + ".se.fc.2.bias")))
        out = out * y[:, :, None, None]
        res = x
        if self.has(name + ".downsample.0.weight"):
            res = self._bn(F.conv2d(x, g(name + ".downsample.0.weight"), None, stride), name + ".downsample.1")
        return F.relu(out + res)

    @torch.no_grad()
    def __call__(self, wav16: torch.Tensor) -> torch.Tensor:
        """wav16 [T] fp32 (16 kHz) -> [1, 512] (L2-normalised)."""
        x = wav16.float().to(self.dev)
        # pre-emphasis y[t] = x[t] - coef x[t - 1], the sample before the first reflected (x[-1] = x[1])
        x = torch.cat([x[:1] - self.coef * x[1:2], x[1:] - self.coef * x[:-1]])
        m = power_mel(x, self.fb, 512, 160, 400, "hamming")
        m = torch.log(m + 1e-6)
        m = F.instance_norm(m[None]).unsqueeze(1)  # [1, 1, 64, frames]
        g = self.g
        h = self._bn(F.relu(F.conv2d(m, g("conv1.weight"), None, 1, 1)), "bn1")
        for li, n in enumerate(self.cfg.spk_layers):
            for bi in range(n):
                h = self._block(h, f"layer{li + 1}.{bi}", (1 if li == 0 else 2) if bi == 0 else 1)
        h = h.reshape(1, -1, h.shape[-1])  # [1, C * F', T']
        w = F.conv1d(h, g("attention.0.weight"), g("attention.0.bias"))
        w = self._bn(F.relu(w), "attention.2")
        w = torch.softmax(F.conv1d(w, g("attention.3.weight"), g("attention.3.bias")), dim=2)
        mu = (h * w).sum(2)
        sg = torch.sqrt((((h * h) * w).sum(2) - mu * mu).clamp(min=1e-5))
        e = F.linear(torch.cat([mu, sg], 1), g("fc.weight"), g("fc.bias"))
        return F.normalize(e, p=2, dim=1)


class _Conditioner:
    """GPT conditioning: conditioning encoder + Perceiver resampler (mel [1, 80, T] -> [1, 32, D])."""

    def __init__(self, sd: dict, cfg: XttsConfig, device):
        self.dev, self.cfg = torch.device(device), cfg
        self.g = lambda k: sd[k].float().to(self.dev)  # noqa: E731

    def _perceiver_attn(self, x, ctx, pre):
        g, c = self.g, self.cfg
        H, dh = c.perceiver_heads, c.perceiver_dim_head
        kv_in = torch.cat([x, ctx], dim=1)  # cross attention with the queries included in the keys
        q = F.linear(x, g(pre + "to_q.weight"))
        k, v = F.linear(kv_in, g(pre + "to_kv.weight")).chunk(2, dim=-1)
        B, N, _ = q.shape
        q = q.view(B, N, H, dh).transpose(1, 2)
        k = k.reshape(B, -1, H, dh).transpose(1, 2)
        v = v.reshape(B, -1, H, dh).transpose(1, 2)
        a = torch.softmax((q @ k.transpose(-1, -2)) * dh ** -0.5, dim=-1) @ v
        return F.linear(a.transpose(1, 2).reshape(B, N, H * dh), g(pre + "to_out.weight"))

    @torch.no_grad()
    def __call__(self, mel: torch.Tensor) -> torch.Tensor:
        g, c = self.g, self.cfg
        P = "gpt.conditioning_encoder."
        h = F.conv1d(mel.float().to(self.dev), g(P + "init.weight"), g(P + "init.bias"))
        for i in range(c.cond_blocks):
            b = f"{P}attn.{i}."
            xn = F.group_norm(h, 32, g(b + "norm.weight"), g(b + "norm.bias"), 1e-5)
            qkv = F.conv1d(xn, g(b + "qkv.weight"), g(b + "qkv.bias"))
            a = _legacy_attention(qkv, c.cond_heads)
            h = xn + F.conv1d(a, g(b + "proj_out.weight"), g(b + "proj_out.bias"))
        ctx = h.transpose(1, 2)  # [1, T, D]
        Q = "gpt.conditioning_perceiver."
        lat = g(Q + "latents")[None]
        for i in range(c.perceiver_depth):
            lat = self._perceiver_attn(lat, ctx, f"{Q}layers.{i}.0.") + lat
            y = F.linear(lat, g(f"{Q}layers.{i}.1.0.weight"), g(f"{Q}layers.{i}.1.0.bias"))
            a, gate = y.chunk(2, dim=-1)
            lat = F.linear(F.gelu(gate) * a, g(f"{Q}layers.{i}.1.2.weight"), g(f"{Q}layers.{i}.1.2.bias")) + lat
        gamma = g(Q + "norm.gamma")
        return F.normalize(lat, dim=-1) * math.sqrt(lat.shape[-1]) * gamma  # RMSNorm


# ------------------------------------------------------------------------------------------------ GPT

class _XttsGPT(_GPT):
    """GPT-2 code LM on the Bark GPT core: HF Conv1D weights transposed into Linear layout, positions added by
    the caller (text / audio tables), logits = mel_head(final_norm(ln_f(h)))."""

    def __init__(self, sd: dict, cfg: XttsConfig, device, dtype):
        core = {}
        for i in range(cfg.gpt_layers):
            s, d = f"gpt.gpt.h.{i}.", f"layers.{i}."
            core[d + "layernorm_1.weight"], core[d + "layernorm_1.bias"] = sd[s + "ln_1.weight"], sd[s + "ln_1.bias"]
            core[d + "layernorm_2.weight"], core[d + "layernorm_2.bias"] = sd[s + "ln_2.weight"], sd[s + "ln_2.bias"]
            core[d + "attn.att_proj.weight"] = sd[s + "attn.c_attn.weight"].t()
            core[d + "attn.att_proj.bias"] = sd[s + "attn.c_attn.bias"]
            core[d + "attn.out_proj.weight"] = sd[s + "attn.c_proj.weight"].t()
            core[d + "attn.out_proj.bias"] = sd[s + "attn.c_proj.bias"]
            core[d + "mlp.in_proj.weight"] = sd[s + "mlp.c_fc.weight"].t()
            core[d + "mlp.in_proj.bias"] = sd[s + "mlp.c_fc.bias"]
            core[d + "mlp.out_proj.weight"] = sd[s + "mlp.c_proj.weight"].t()
            core[d + "mlp.out_proj.bias"] = sd[s + "mlp.c_proj.bias"]
        core["layernorm_final.weight"], core["layernorm_final.bias"] = sd["gpt.gpt.ln_f.weight"], sd["gpt.gpt.ln_f.bias"]
        core["input_embeds_layer.weight"] = sd["gpt.mel_embedding.weight"]
        core["lm_head.weight"] = sd["gpt.mel_head.weight"]
        D = cfg.gpt_dim
        core["position_embeds_layer.weight"] = torch.zeros(1, D)
        super().__init__(core, "", {"num_heads": cfg.gpt_heads, "hidden_size": D, "num_layers": cfg.gpt_layers,
                                    "gelu_approx": "tanh"}, device, dtype, True)
        dev = self.device
        self.text_emb = sd["gpt.text_embedding.weight"].float().to(dev)
        self.text_pos = sd["gpt.text_pos_embedding.emb.weight"].float().to(dev)
        self.mel_pos = sd["gpt.mel_pos_embedding.emb.weight"].float().to(dev)
        self.final_norm = (sd["gpt.final_norm.weight"].float().to(dev), sd["gpt.final_norm.bias"].float().to(dev))
        self.mel_head_b = sd["gpt.mel_head.bias"].float().to(dev)

    def head_logits(self, h: torch.Tensor) -> torch.Tensor:
        hn = F.layer_norm(h.float(), (self.D,), self.final_norm[0], self.final_norm[1], 1e-5)
        return F.linear(hn.to(self.dtype), self.heads[0]).float() + self.mel_head_b

    def latents(self, h: torch.Tensor) -> torch.Tensor:
        return F.layer_norm(h.float(), (self.D,), self.final_norm[0], self.final_norm[1], 1e-5)

    def audio_emb(self, codes: torch.Tensor, pos0: int = 0) -> torch.Tensor:
        codes = codes.to(self.device).long()
        return self.emb[0][codes].float() + self.mel_pos[pos0:pos0 + codes.shape[-1]]

    def text_embed(self, ids: torch.Tensor) -> torch.Tensor:
        ids = ids.to(self.device).long()
        return self.text_emb[ids] + self.text_pos[: ids.shape[-1]]

    def decode_logits(self, tok: torch.Tensor, apos: torch.Tensor, pos: torch.Tensor, cache) -> torch.Tensor:
        """One audio code (int64 [1]) at audio position apos / sequence position pos (device int64 [1]) -> logits
        [1, V] fp32; shape-static, captured as one HIP graph by the sampling loop."""
        x = (self.emb[0].index_select(0, tok).float() + self.mel_pos.index_select(0, apos))[None]
        return self.head_logits(self.decode_trunk(x, pos, cache))[:, -1]


def _sample(logits: torch.Tensor, prev: torch.Tensor, n_prev: int, c: XttsConfig, gen) -> torch.Tensor:
    """HF generate's chain for one row: repetition penalty over the codes so far, temperature, top-k, top-p,
    multinomial. logits [1, V] fp32 (modified), prev int64 [>= n_prev] device history."""
    if c.repetition_penalty != 1.0 and n_prev:
        idx = prev[:n_prev].view(1, -1)
        sc = logits.gather(1, idx)
        sc = torch.where(sc < 0, sc * c.repetition_penalty, sc / c.repetition_penalty)
        logits.scatter_(1, idx, sc)
    x = logits / max(c.temperature, 1e-5)
    if 0 < c.top_k < x.shape[-1]:
        kth = torch.topk(x, c.top_k, dim=-1).values[:, -1:]
        x = x.masked_fill(x < kth, float("-inf"))
    if 0 < c.top_p < 1:
        sv, si = torch.sort(x, descending=True, dim=-1)
        cp = torch.softmax(sv, -1).cumsum(-1)
        drop = cp > c.top_p
        drop[:, 1:] = drop[:, :-1].clone()
        drop[:, 0] = False
        x = x.masked_fill(torch.zeros_like(drop).scatter(1, si, drop), float("-inf"))
    return torch.multinomial(torch.softmax(x, -1), 1, generator=gen).view(-1)


# ------------------------------------------------------------------------------------------------ vocoder

class _HifiDecoder:
    """XTTS HiFi-GAN: latents [1, T, 1024] + speaker embedding [1, 512] -> 24 kHz waveform."""

    def __init__(self, sd: dict, cfg: XttsConfig, device):
        self.cfg, self.dev = cfg, torch.device(device)
        P = "hifigan_decoder.waveform_decoder."
        self.w = {k[len(P):]: v.float().to(self.dev) for k, v in sd.items() if k.startswith(P)}
        self.plan = None

    def _conv(self, x, name, dilation=1, padding=0):
        return F.conv1d(x, self.w[name + ".weight"], self.w.get(name + ".bias"), dilation=dilation, padding=padding)

    def _gpu_plan(self):
        from types import SimpleNamespace
        from ..ops import conv as CV
        from .encodec import _ConvT
        c, dt = self.cfg, torch.float16
        cf = SimpleNamespace(use_causal_conv=False, pad_mode="constant", trim_right_ratio=1.0)

        def c1(name):
            w = self.w[name + ".weight"]
            b = self.w.get(name + ".bias")
            w4 = w[:, :, None, :].to(dt).contiguous()
            return (w4, b.float() if b is not None else None, CV.pack_weight(w4, dt), int(w.shape[2]))
        for r, k in zip(c.upsample_rates, c.upsample_kernels):
            if k != 2 * r or r % 2:
                return None
        ups = [_ConvT(self.w[f"ups.{i}.weight"], self.w.get(f"ups.{i}.bias"), r, cf, self.dev, dt)
               for i, r in enumerate(c.upsample_rates)]
        nk = len(c.resblock_kernels)
        res = {}
        for i in range(len(ups)):
            for j, dils in enumerate(c.resblock_dilations):
                pre = f"resblocks.{i * nk + j}."
                res[i * nk + j] = [(c1(f"{pre}convs1.{n}"), c1(f"{pre}convs2.{n}")) for n in range(len(dils))]
        return dict(pre=c1("conv_pre"), post=c1("conv_post"), ups=ups, res=res)

    @torch.no_grad()
    def __call__(self, lat: torch.Tensor, g: torch.Tensor) -> torch.Tensor:
        c = self.cfg
        z = F.interpolate(lat.float().transpose(1, 2), scale_factor=c.code_stride / c.output_hop, mode="linear")
        if c.output_sr != c.input_sr:
            z = F.interpolate(z, scale_factor=c.output_sr / c.input_sr, mode="linear")
        gg = g.float().to(self.dev)[:, :, None]  # [1, 512, 1]
        cond = self._conv(gg, "cond_layer")  # [1, C0, 1]
        conds = [self._conv(gg, f"conds.{i}") for i in range(len(c.upsample_rates))]
        if self.dev.type == "cuda":
            if self.plan is None:
                self.plan = self._gpu_plan() or False
            if self.plan:
                return self._gpu(z, cond, conds)
        x = self._conv(z, "conv_pre", padding=3) + cond
        nk = len(c.resblock_kernels)
        for i, (r, k) in enumerate(zip(c.upsample_rates, c.upsample_kernels)):
            x = F.leaky_relu(x, 0.1)
            x = F.conv_transpose1d(x, self.w[f"ups.{i}.weight"], self.w.get(f"ups.{i}.bias"), stride=r,
                                   padding=(k - r) // 2)
            x = x + conds[i]
            acc = None
            for j, (rk, dils) in enumerate(zip(c.resblock_kernels, c.resblock_dilations)):
                pre = f"resblocks.{i * nk + j}."
                h = x
                for n, d in enumerate(dils):
                    t = self._conv(F.leaky_relu(h, 0.1), f"{pre}convs1.{n}", d, (rk * d - d) // 2)
                    t = self._conv(F.leaky_relu(t, 0.1), f"{pre}convs2.{n}", 1, (rk - 1) // 2)
                    h = h + t
                acc = h if acc is None else acc + h
            x = acc / nk
        x = F.leaky_relu(x, 0.01)
        return torch.tanh(self._conv(x, "conv_post", padding=3))[0, 0]

    def _gpu(self, z, cond, conds):
        from .tts import VitsModel
        c, P = self.cfg, self.plan
        c1 = VitsModel._c1
        nk = len(c.resblock_kernels)
        x = c1(z.transpose(1, 2).to(torch.float16).contiguous(), P["pre"], tadd=cond[:, :, 0].float())
        for i in range(len(P["ups"])):
            x = P["ups"][i](F.leaky_relu(x, 0.1).contiguous())
            x = (x.float() + conds[i][:, :, 0][:, None, :]).to(torch.float16)
            acc = None
            for j, dils in enumerate(c.resblock_dilations):
                h = x
                for (cw1, cw2), d in zip(P["res"][i * nk + j], dils):
                    t = c1(F.leaky_relu(h, 0.1).contiguous(), cw1, dil=d, act="leaky")
                    h = c1(t, cw2, residual=h)
                acc = h.float() if acc is None else acc + h.float()
            x = (acc / nk).to(torch.float16)
        y = c1(F.leaky_relu(x, 0.01).contiguous(), P["post"], act="tanh")
        return y.float()[0, :, 0]


# ------------------------------------------------------------------------------------------------ text

_ONES = ["zero", "one", "two", "three", "four", "five", "six", "seven", "eight", "nine", "ten", "eleven", "twelve",
         "thirteen", "fourteen", "fifteen", "sixteen", "seventeen", "eighteen", "nineteen"]
_TENS = ["", "", "twenty", "thirty", "forty", "fifty", "sixty", "seventy", "eighty", "ninety"]


def _num_en(n: int) -> str:
    if n < 20:
        return _ONES[n]
    if n < 100:
        return _TENS[n // 10] + ("" if n % 10 == 0 else " " + _ONES[n % 10])
    for div, name in ((10 ** 9, "billion"), (10 ** 6, "million"), (1000, "thousand"), (100, "hundred")):
        if n >= div:
            rest = n % div
            return _num_en(n // div) + " " + name + ("" if rest == 0 else " " + _num_en(rest))
    return str(n)


class XttsTokenizer:
    """VoiceBpeTokenizer: English-style cleaning (lower-case, symbols, digits spelled out), `[lang]` prefix,
    spaces as `[SPACE]`, then the BPE vocabulary (tokenizers library)."""

    def __init__(self, vocab_path: str | None = None, tok=None):
        if tok is None:
            from tokenizers import Tokenizer
            tok = Tokenizer.from_file(vocab_path)
        self.tok = tok

    @staticmethod
    def clean(text: str) -> str:
        t = text.lower().replace("&", " and ").replace("%", " percent ").replace("@", " at ")
        t = re.sub(r"\d+", lambda m: " " + _num_en(int(m.group(0))) + " " if len(m.group(0)) < 13 else m.group(0), t)
        t = re.sub(r'[\\"()<>\[\]{}*_~^|#]', "", t)
        return re.sub(r"\s+", " ", t).strip()

    def encode(self, text: str, lang: str = "en") -> list[int]:
        lang = (lang or "en").split("-")[0].lower()
        lang = "zh-cn" if lang == "zh" else lang
        t = f"[{lang}]" + self.clean(text)
        return self.tok.encode(t.replace(" ", "[SPACE]")).ids


# ------------------------------------------------------------------------------------------------ model

class Xtts:
    def __init__(self, cfg: XttsConfig, sd: dict, tokenizer: XttsTokenizer, device="cpu", speakers: dict | None = None):
        self.cfg = cfg
        self.device = torch.device(device)
        self.dtype = torch.float16 if self.device.type == "cuda" else torch.float32
        sd = fold_weight_norm(sd)
        self.gpt = _XttsGPT(sd, cfg, self.device, self.dtype)
        self.cond = _Conditioner(sd, cfg, self.device)
        self.spk = _SpeakerEncoder(sd, "hifigan_decoder.speaker_encoder.", cfg, self.device)
        self.dec = _HifiDecoder(sd, cfg, self.device)
        ms = sd.get("mel_stats")
        self.mel_stats = (ms.float() if ms is not None else torch.ones(80)).to(self.device)
        self.cond_fb = mel_filters(cfg.input_sr, 2048, 80, 0.0, 8000.0, slaney_norm=True).to(self.device)
        self.tokenizer = tokenizer
        self.speakers = speakers or {}
        self.sample_rate = cfg.output_sr

    # -------------------------------------------------------------- conditioning
    @torch.no_grad()
    def conditioning(self, wav: np.ndarray, sr: int) -> tuple[torch.Tensor, torch.Tensor]:
        """Reference clip -> (GPT conditioning latents [1, 32, D], speaker embedding [1, 512])."""
        c = self.cfg
        a22 = torch.from_numpy(resample(wav, sr, c.input_sr)[: int(c.cond_len_s * c.input_sr)]).to(self.device)
        chunk = int(c.cond_chunk_s * c.input_sr)
        embs = []
        for i in range(0, max(1, a22.numel()), chunk):
            seg = a22[i:i + chunk]
            if seg.numel() < 0.33 * c.input_sr and embs:
                continue
            mel = power_mel(seg, self.cond_fb, 2048, 256, 1024)
            mel = torch.log(mel.clamp(min=1e-5)) / self.mel_stats[:, None]
            embs.append(self.cond(mel[None]))
        lat = torch.stack(embs).mean(0)
        a16 = torch.from_numpy(resample(wav, sr, 16000)).to(self.device)
        return lat, self.spk(a16)

    def voice(self, audio_path: str = "", speaker: str = "") -> tuple[torch.Tensor, torch.Tensor]:
        if audio_path:
            from ..utils.audio import load_audio
            return self.conditioning(load_audio(audio_path, 22050), 22050)
        if speaker:
            if speaker not in self.speakers:
                raise ValueError(f"unknown XTTS speaker {speaker!r} (known: {', '.join(sorted(self.speakers)[:8])})")
            s = self.speakers[speaker]
            return (s["gpt_cond_latent"].float().to(self.device).view(1, -1, self.cfg.gpt_dim),
                    s["speaker_embedding"].float().to(self.device).view(1, -1))
        raise ValueError("XTTS needs a voice: a reference clip (AudioPath / speaker_wav) or a named speaker")

    # -------------------------------------------------------------- synthesis
    @torch.no_grad()
    def codes(self, lat: torch.Tensor, text_ids: list[int], seed: int = 0, max_new: int | None = None) -> list[int]:
        c, gpt = self.cfg, self.gpt
        if len(text_ids) + 2 > c.max_text_tokens:
            raise ValueError(f"text too long for XTTS ({len(text_ids)} tokens, max {c.max_text_tokens - 2})")
        t = torch.tensor([c.start_text] + list(text_ids) + [c.stop_text])
        prefix = torch.cat([lat.float().to(self.device), gpt.text_embed(t)[None]], 1)  # [1, S0, D]
        start = gpt.audio_emb(torch.tensor([c.start_audio]))[None]
        x = torch.cat([prefix, start], 1)
        S = x.shape[1]
        max_new = min(max_new or c.max_audio_tokens, c.max_audio_tokens)
        cache = gpt.new_cache(1, S + max_new + 1)
        logits = gpt.head_logits(gpt.trunk(x, 0, cache))[:, -1]
        gen = torch.Generator(device=self.device).manual_seed(int(seed))
        hist = torch.full((max_new + 1,), c.start_audio, dtype=torch.long, device=self.device)
        n_hist = 1
        out = []
        graph = None
        tok = torch.zeros(1, dtype=torch.long, device=self.device)
        apos = torch.zeros(1, dtype=torch.long, device=self.device)
        pos = torch.zeros(1, dtype=torch.long, device=self.device)
        g_out = None
        if self.device.type == "cuda":
            side = torch.cuda.Stream()
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                gpt.decode_logits(tok, apos, torch.full((1,), S, dtype=torch.long, device=self.device), cache)
            torch.cuda.current_stream().wait_stream(side)
            pos.fill_(S)
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph):
                g_out = gpt.decode_logits(tok, apos, pos, cache)
        for i in range(max_new):
            nxt = _sample(logits.clone(), hist, n_hist, c, gen)
            v = int(nxt)
            if v == c.stop_audio:
                break
            out.append(v)
            hist[n_hist] = v
            n_hist += 1
            if i + 1 == max_new:
                break
            if graph is not None:
                tok.copy_(nxt)
                apos.fill_(i + 1)
                pos.fill_(S + i)
                graph.replay()
                logits = g_out.clone()
            else:
                xe = gpt.audio_emb(nxt.view(1), i + 1)[None]
                logits = gpt.head_logits(gpt.trunk(xe, S + i, cache))[:, -1]
        return out

    @torch.no_grad()
    def gpt_latents(self, lat: torch.Tensor, text_ids: list[int], codes: list[int]) -> torch.Tensor:
        """Teacher-forced pass: final-normed hidden states of [start | codes] -> [1, len(codes) + 1, D]."""
        c, gpt = self.cfg, self.gpt
        t = torch.tensor([c.start_text] + list(text_ids) + [c.stop_text])
        a = torch.tensor([c.start_audio] + list(codes) + [c.stop_audio, c.stop_audio])
        x = torch.cat([lat.float().to(self.device), gpt.text_embed(t)[None], gpt.audio_emb(a)[None]], 1)
        h = gpt.trunk(x, 0, None)
        return gpt.latents(h[:, -a.numel():][:, :-2])

    @torch.no_grad()
    def synthesize(self, text: str, language: str = "en", audio_path: str = "", speaker: str = "", seed: int = 0,
                   voice=None, max_new: int | None = None) -> np.ndarray:
        lat, spk = voice if voice is not None else self.voice(audio_path, speaker)
        ids = self.tokenizer.encode(text.strip(), language)
        codes = self.codes(lat, ids, seed, max_new)
        if not codes:
            raise ValueError("XTTS produced no audio codes")
        wav = self.dec(self.gpt_latents(lat, ids, codes), spk)
        return wav.float().cpu().numpy()


def is_xtts_dir(d: str) -> bool:
    try:
        cfg = json.load(open(os.path.join(d, "config.json"), encoding="utf-8"))
    except (OSError, ValueError):
        return False
    return "xtts" in str(cfg.get("model", "")).lower()


def _load(path: str):
    try:
        return torch.load(path, map_location="cpu", weights_only=True)
    except Exception as ex:
        raise ValueError(f"XTTS file {os.path.basename(path)} not loadable with the weights-only loader: {ex}") from ex


def load_xtts(d: str, device="cpu") -> Xtts:
    cfg_j = json.load(open(os.path.join(d, "config.json"), encoding="utf-8"))
    cfg = XttsConfig.from_json(cfg_j)
    ck_path = next((os.path.join(d, n) for n in ("model.pth", "model_file.pth", "best_model.pth")
                    if os.path.exists(os.path.join(d, n))), None)
    if ck_path is None:
        raise FileNotFoundError(f"XTTS checkpoint (model.pth) not found in {d}")
    ck = _load(ck_path)
    sd = ck.get("model", ck) if isinstance(ck, dict) else None
    if not isinstance(sd, dict):
        raise ValueError("XTTS checkpoint holds no state dict")
    missing = [k for k in ("gpt.gpt.ln_f.weight", "gpt.mel_head.weight", "gpt.conditioning_encoder.init.weight",
                           "hifigan_decoder.waveform_decoder.conv_pre.weight") if not any(
        kk == k or kk.startswith(k.rsplit(".", 1)[0] + ".") for kk in sd)]
    if missing:
        raise ValueError(f"XTTS checkpoint {os.path.basename(ck_path)} lacks {', '.join(missing)}")
    if "mel_stats" not in sd and os.path.exists(os.path.join(d, "mel_stats.pth")):
        sd = dict(sd, mel_stats=_load(os.path.join(d, "mel_stats.pth")))
    cfg.gpt_layers = sum(1 for k in sd if k.startswith("gpt.gpt.h.") and k.endswith(".ln_1.weight"))
    vocab = os.path.join(d, "vocab.json")
    speakers = {}
    sp = os.path.join(d, "speakers_xtts.pth")
    if os.path.exists(sp):
        try:
            speakers = _load(sp)
        except ValueError as ex:
            log.warning("%s", ex)
    return Xtts(cfg, sd, XttsTokenizer(vocab), device, speakers)


# ------------------------------------------------------------------------------------------------ synthetic

def tiny_config() -> XttsConfig:
    """A small XTTS of the same layout (tests / smoke): 2 GPT layers of 64, 2 conditioning blocks."""
    return XttsConfig(gpt_layers=2, gpt_dim=64, gpt_heads=4, text_tokens=300, audio_tokens=66, start_text=261,
                      stop_text=0, start_audio=64, stop_audio=65, max_audio_tokens=40, max_text_tokens=64,
                      cond_heads=4, cond_blocks=2, perceiver_latents=8, perceiver_depth=2, perceiver_heads=2,
                      perceiver_dim_head=16, d_vector=32, upsample_initial=32, spk_layers=(1, 1, 1, 1),
                      spk_filters=(4, 8, 8, 8), spk_mels=64)


def synthetic_state_dict(c: XttsConfig, seed: int = 0) -> dict:
    """Random weights in Coqui's XTTS names (Conv1D GPT-2 layout, weight-norm-free HiFi-GAN)."""
    g = torch.Generator().manual_seed(seed)

    def r(*shape, s=0.05):
        return torch.randn(*shape, generator=g) * s
    D, sd = c.gpt_dim, {}
    for i in range(c.gpt_layers):
        p = f"gpt.gpt.h.{i}."
        sd[p + "ln_1.weight"], sd[p + "ln_1.bias"] = torch.ones(D), torch.zeros(D)
        sd[p + "ln_2.weight"], sd[p + "ln_2.bias"] = torch.ones(D), torch.zeros(D)
        sd[p + "attn.c_attn.weight"], sd[p + "attn.c_attn.bias"] = r(D, 3 * D), r(3 * D)
        sd[p + "attn.c_proj.weight"], sd[p + "attn.c_proj.bias"] = r(D, D), r(D)
        sd[p + "mlp.c_fc.weight"], sd[p + "mlp.c_fc.bias"] = r(D, 4 * D), r(4 * D)
        sd[p + "mlp.c_proj.weight"], sd[p + "mlp.c_proj.bias"] = r(4 * D, D), r(D)
    sd["gpt.gpt.ln_f.weight"], sd["gpt.gpt.ln_f.bias"] = torch.ones(D), torch.zeros(D)
    sd["gpt.final_norm.weight"], sd["gpt.final_norm.bias"] = torch.ones(D), torch.zeros(D)
    sd["gpt.text_embedding.weight"] = r(c.text_tokens, D, s=0.5)
    sd["gpt.mel_embedding.weight"] = r(c.audio_tokens, D, s=0.5)
    sd["gpt.text_pos_embedding.emb.weight"] = r(c.max_text_tokens + 2, D)
    sd["gpt.mel_pos_embedding.emb.weight"] = r(c.max_audio_tokens + 3, D)
    sd["gpt.mel_head.weight"], sd["gpt.mel_head.bias"] = r(c.audio_tokens, D, s=0.3), torch.zeros(c.audio_tokens)
    sd["gpt.conditioning_encoder.init.weight"], sd["gpt.conditioning_encoder.init.bias"] = r(D, 80, 1), r(D)
    for i in range(c.cond_blocks):
        p = f"gpt.conditioning_encoder.attn.{i}."
        sd[p + "norm.weight"], sd[p + "norm.bias"] = torch.ones(D), torch.zeros(D)
        sd[p + "qkv.weight"], sd[p + "qkv.bias"] = r(3 * D, D, 1), r(3 * D)
        sd[p + "proj_out.weight"], sd[p + "proj_out.bias"] = r(D, D, 1), r(D)
    inner = c.perceiver_heads * c.perceiver_dim_head
    ff = int(D * 4 * 2 / 3)
    sd["gpt.conditioning_perceiver.latents"] = r(c.perceiver_latents, D, s=1.0)
    for i in range(c.perceiver_depth):
        p = f"gpt.conditioning_perceiver.layers.{i}."
        sd[p + "0.to_q.weight"], sd[p + "0.to_kv.weight"], sd[p + "0.to_out.weight"] = r(inner, D), r(2 * inner, D), r(D, inner)
        sd[p + "1.0.weight"], sd[p + "1.0.bias"] = r(2 * ff, D), r(2 * ff)
        sd[p + "1.2.weight"], sd[p + "1.2.bias"] = r(D, ff), r(D)
    sd["gpt.conditioning_perceiver.norm.gamma"] = torch.ones(D)
    sd["mel_stats"] = torch.rand(80, generator=g) + 1.0
    # HiFi-GAN
    P = "hifigan_decoder.waveform_decoder."
    ch = c.upsample_initial
    sd[P + "conv_pre.weight"], sd[P + "conv_pre.bias"] = r(ch, D, 7), r(ch)
    sd[P + "cond_layer.weight"], sd[P + "cond_layer.bias"] = r(ch, c.d_vector, 1), r(ch)
    nk = len(c.resblock_kernels)
    for i, (u, k) in enumerate(zip(c.upsample_rates, c.upsample_kernels)):
        ci, co = ch // (2 ** i), ch // (2 ** (i + 1))
        sd[P + f"ups.{i}.weight"], sd[P + f"ups.{i}.bias"] = r(ci, co, k, s=0.1), r(co)
        sd[P + f"conds.{i}.weight"], sd[P + f"conds.{i}.bias"] = r(co, c.d_vector, 1), r(co)
        for j, (rk, dils) in enumerate(zip(c.resblock_kernels, c.resblock_dilations)):
            for n in range(len(dils)):
                q = P + f"resblocks.{i * nk + j}."
                sd[q + f"convs1.{n}.weight"], sd[q + f"convs1.{n}.bias"] = r(co, co, rk, s=0.1), r(co)
                sd[q + f"convs2.{n}.weight"], sd[q + f"convs2.{n}.bias"] = r(co, co, rk, s=0.1), r(co)
    sd[P + "conv_post.weight"] = r(1, ch // (2 ** len(c.upsample_rates)), 7)
    # speaker encoder
    S = "hifigan_decoder.speaker_encoder."

    def bn(name, n):
        sd[name + ".weight"], sd[name + ".bias"] = torch.ones(n), torch.zeros(n)
        sd[name + ".running_mean"], sd[name + ".running_var"] = torch.zeros(n), torch.ones(n)
    f = c.spk_filters
    sd[S + "conv1.weight"] = r(f[0], 1, 3, 3, s=0.3)
    bn(S + "bn1", f[0])
    cin = f[0]
    for li, (n, co) in enumerate(zip(c.spk_layers, f)):
        for bi in range(n):
            p = S + f"layer{li + 1}.{bi}"
            stride = (1 if li == 0 else 2) if bi == 0 else 1
            sd[p + ".conv1.weight"] = r(co, cin, 3, 3, s=0.2)
            bn(p + ".bn1", co)
            sd[p + ".conv2.weight"] = r(co, co, 3, 3, s=0.2)
            bn(p + ".bn2", co)
            sd[p + ".se.fc.0.weight"], sd[p + ".se.fc.0.bias"] = r(max(1, co // 8), co), r(max(1, co // 8))
            sd[p + ".se.fc.2.weight"], sd[p + ".se.fc.2.bias"] = r(co, max(1, co // 8)), r(co)
            if stride != 1 or cin != co:
                sd[p + ".downsample.0.weight"] = r(co, cin, 1, 1, s=0.3)
                bn(p + ".downsample.1", co)
            cin = co
    outc = f[-1] * (c.spk_mels // 8)
    sd[S + "attention.0.weight"], sd[S + "attention.0.bias"] = r(128, outc, 1), r(128)
    bn(S + "attention.2", 128)
    sd[S + "attention.3.weight"], sd[S + "attention.3.bias"] = r(outc, 128, 1), r(outc)
    sd[S + "fc.weight"], sd[S + "fc.bias"] = r(c.d_vector, 2 * outc), r(c.d_vector)
    return sd


def synthetic_tokenizer(c: XttsConfig) -> XttsTokenizer:
    """A character-level stand-in for vocab.json (tests): `[en]`, `[SPACE]`, a-z, digits, punctuation."""
    from tokenizers import Regex, Tokenizer, models, pre_tokenizers
    vocab = {"[STOP]": 0, "[UNK]": 1, "[SPACE]": 2, "[en]": 3}
    for ch in "abcdefghijklmnopqrstuvwxyz0123456789.,!?'-":
        vocab[ch] = len(vocab)
    tok = Tokenizer(models.WordLevel(vocab, unk_token="[UNK]"))
    tok.pre_tokenizer = pre_tokenizers.Split(Regex(r"\[SPACE\]|\[en\]|."), behavior="isolated")
    return XttsTokenizer(tok=tok)


def synthetic_xtts(device="cpu", seed: int = 0, speakers: bool = True) -> Xtts:
    c = tiny_config()
    sd = synthetic_state_dict(c, seed)
    spk = {"Synthetic Voice": {"gpt_cond_latent": torch.randn(1, c.perceiver_latents, c.gpt_dim) * 0.5,
                               "speaker_embedding": F.normalize(torch.randn(1, c.d_vector, 1), dim=1)}} if speakers else {}
    return Xtts(c, sd, synthetic_tokenizer(c), device, spk)
