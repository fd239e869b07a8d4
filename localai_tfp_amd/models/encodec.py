"""EnCodec neural audio codec — the decoder half (codes -> waveform) that MusicGen and Bark speak through.

Structure (Hugging Face ``EncodecModel`` names, ``audio_encoder.*`` inside a MusicGen checkpoint):
residual vector quantiser (sum of per-codebook embeddings) -> SEANet decoder:
conv(k7) -> 2-layer LSTM (+skip) -> per upsampling ratio r: ELU, ConvTranspose1d(k=2r, stride r),
residual unit (ELU, conv k3, ELU, conv k1, + 1x1 shortcut) -> ELU -> conv(k7) -> audio.

MI355X mapping: activations stay [B, T, C] rows (channels-last 1-D), every Conv1d is an H = 1 conv on the
implicit-GEMM MFMA kernel (ops/conv.py) with bias, ELU and the residual add fused into its epilogue, and
every ConvTranspose1d(k = 2r, stride r) is rewritten at load time as ONE ordinary conv: output phase
phi of frame m is x[m-1] . w[phi + r] + x[m] . w[phi], so a k = 2 conv with r*Cout output channels over
the zero-padded input produces the r phases of each frame side by side — which, in [B, T, C] rows, IS
the upsampled [B, r*(T+1), Cout] sequence (no scatter, no col2im). Weight norm (g * v / ||v||) is folded
at load. The LSTM runs through PyTorch (MIOpen RNN) in fp32. CPU tensors run the same graph on the fp32
PyTorch reference of each op (the oracle: transformers ``EncodecModel.decode``).

Reference: backend/go/bark/gobark.cpp:22-80 (bark.cpp's encodec), backend/python/transformers/
backend.py:452-507 (MusicGen's ``audio_encoder.decode``).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import torch
import torch.nn.functional as F

from ..ops import conv as CV


@dataclass
class EncodecConfig:
    audio_channels: int = 1
    num_filters: int = 32
    upsampling_ratios: list = field(default_factory=lambda: [8, 5, 4, 2])
    hidden_size: int = 128
    codebook_size: int = 1024
    codebook_dim: int | None = None
    kernel_size: int = 7
    last_kernel_size: int = 7
    residual_kernel_size: int = 3
    dilation_growth_rate: int = 2
    num_residual_layers: int = 1
    num_lstm_layers: int = 2
    compress: int = 2
    use_causal_conv: bool = True
    pad_mode: str = "reflect"
    trim_right_ratio: float = 1.0
    use_conv_shortcut: bool = True
    sampling_rate: int = 24000

    @classmethod
    def from_dict(cls, d: dict) -> "EncodecConfig":
        c = cls()
        for k in c.__dataclass_fields__:
            if k in d and d[k] is not None:
                setattr(c, k, d[k])
        if d.get("norm_type", "weight_norm") != "weight_norm":
            raise NotImplementedError(f"EnCodec norm_type {d.get('norm_type')!r} (only weight_norm checkpoints)")
        return c


def _wn(sd: dict, p: str) -> torch.Tensor:
    """Weight of a (possibly weight-normed) conv: g * v / ||v|| with the norm over all dims but 0."""
    for g_name, v_name in ((p + "parametrizations.weight.original0", p + "parametrizations.weight.original1"),
                           (p + "weight_g", p + "weight_v")):
        if v_name in sd:
            g, v = sd[g_name].float(), sd[v_name].float()
            n = v.reshape(v.shape[0], -1).norm(dim=1).reshape(-1, *([1] * (v.dim() - 1)))
            return g * v / n
    return sd[p + "weight"].float()


class _Conv:
    """One EnCodec Conv1d (asymmetric / causal padding, reflect or zero) as an H = 1 conv."""

    def __init__(self, w: torch.Tensor, b: torch.Tensor | None, stride: int, dilation: int, cfg: EncodecConfig,
                 device, dtype):
        co, ci, k = w.shape
        self.k, self.stride, self.dil = k, stride, dilation
        self.w = w[:, :, None, :].to(device, dtype)  # [Cout, Cin, 1, K]
        self.b = b.float().to(device) if b is not None else None
        self.packed = CV.pack_weight(self.w, dtype) if torch.device(device).type == "cuda" else None
        self.causal, self.pad_mode = cfg.use_causal_conv, cfg.pad_mode
        self.eff_k = (k - 1) * dilation + 1
        self.pad_total = self.eff_k - stride

    def __call__(self, x: torch.Tensor, act: str | None = None, residual: torch.Tensor | None = None):
        """x [B, T, C] rows -> [B, T', Cout] rows."""
        L = x.shape[1]
        n_frames = math.ceil((L - self.eff_k + self.pad_total) / self.stride + 1) - 1
        extra = n_frames * self.stride + self.eff_k - self.pad_total - L
        if self.causal:
            pl, pr = self.pad_total, extra
        else:
            pr0 = self.pad_total // 2
            pl, pr = self.pad_total - pr0, pr0 + extra
        pad = (0, pl, 0, pr)
        if self.pad_mode == "reflect" and (pl or pr):
            x = _reflect_rows(x, pl, pr)
            pad = (0, 0, 0, 0)
        xin = x[:, None].permute(0, 3, 1, 2)  # NCHW-shaped view of [B, 1, T, C] rows (channels_last)
        res = residual[:, None].permute(0, 3, 1, 2) if residual is not None else None
        y = CV.conv2d(xin, weight=self.w, bias=self.b, stride=self.stride, pad=pad, dilation=self.dil, act=act,
                      residual=res, packed=self.packed)
        return y.permute(0, 2, 3, 1)[:, 0]


def _reflect_rows(x: torch.Tensor, pl: int, pr: int) -> torch.Tensor:
    """Reflect-pad [B, T, C] rows along T (HF _pad1d: zero-extend first when T <= max pad)."""
    L = x.shape[1]
    extra = 0
    if L <= max(pl, pr):
        extra = max(pl, pr) - L + 1
        x = torch.cat([x, x.new_zeros(x.shape[0], extra, x.shape[2])], 1)
    n = x.shape[1]
    idx = torch.arange(-pl, n + pr, device=x.device).abs()
    idx = torch.where(idx >= n, 2 * (n - 1) - idx, idx)
    y = x[:, idx]
    return y[:, :y.shape[1] - extra] if extra else y


class _ConvT:
    """ConvTranspose1d(k = 2r, stride r) as one k = 2 conv producing the r output phases per frame."""

    def __init__(self, w: torch.Tensor, b: torch.Tensor | None, stride: int, cfg: EncodecConfig, device, dtype):
        ci, co, k = w.shape
        r = stride
        if k != 2 * r:
            raise NotImplementedError(f"EnCodec ConvTranspose1d kernel {k} != 2 x stride {r}")
        # W'[(phi, co), ci, 0, tap]: tap 0 sees x[m-1] -> w[ci, co, phi + r]; tap 1 sees x[m] -> w[ci, co, phi]
        w_hi = w[:, :, r:].permute(2, 1, 0)  # [r, co, ci]
        w_lo = w[:, :, :r].permute(2, 1, 0)
        wp = torch.stack([w_hi, w_lo], -1).reshape(r * co, ci, 1, 2)
        bp = b.float().repeat(r) if b is not None else None
        self.r, self.co = r, co
        self.conv = _Conv.__new__(_Conv)
        self.conv.w = wp.to(device, dtype)
        self.conv.b = bp.to(device) if bp is not None else None
        self.conv.packed = CV.pack_weight(self.conv.w, dtype) if torch.device(device).type == "cuda" else None
        pad_total = k - r
        self.trim_r = math.ceil(pad_total * cfg.trim_right_ratio) if cfg.use_causal_conv else pad_total // 2
        self.trim_l = pad_total - self.trim_r

    def __call__(self, x: torch.Tensor) -> torch.Tensor:
        B, L, _ = x.shape
        xin = x[:, None].permute(0, 3, 1, 2)
        y = CV.conv2d(xin, weight=self.conv.w, bias=self.conv.b, stride=1, pad=(0, 1, 0, 1),
                      packed=self.conv.packed)  # [B, r*co, 1, L+1]
        y = y.permute(0, 2, 3, 1).reshape(B, (L + 1) * self.r, self.co)
        return y[:, self.trim_l:y.shape[1] - self.trim_r]


class EncodecDecoder:
    """codes [B, n_q, T] -> waveform [B, audio_channels, samples] (fp32)."""

    def __init__(self, cfg: EncodecConfig, sd: dict, device="cpu", dtype=None, prefix: str = ""):
        self.cfg = cfg
        self.device = torch.device(device)
        self.dtype = dtype or (torch.float16 if self.device.type == "cuda" else torch.float32)
        dev, dt = self.device, self.dtype
        P = prefix
        # RVQ codebooks
        self.codebooks = []
        i = 0
        while f"{P}quantizer.layers.{i}.codebook.embed" in sd:
            self.codebooks.append(sd[f"{P}quantizer.layers.{i}.codebook.embed"].float().to(dev))
            i += 1
        if not self.codebooks:
            raise ValueError(f"no EnCodec codebooks under {P}quantizer.layers.*")
        D = f"{P}decoder.layers."

        def conv(idx, stride=1, dilation=1, sub=""):
            p = f"{D}{idx}.{sub}conv."
            return _Conv(_wn(sd, p), sd.get(p + "bias"), stride, dilation, cfg, dev, dt)

        scaling = 2 ** len(cfg.upsampling_ratios)
        self.plan = []  # (kind, module(s))
        li = 0
        self.plan.append(("conv", conv(li)))
        li += 1
        lp = f"{D}{li}.lstm."
        nl = cfg.num_lstm_layers
        dim = scaling * cfg.num_filters
        lstm = torch.nn.LSTM(dim, dim, nl)
        with torch.no_grad():
            for name, prm in lstm.named_parameters():
                prm.copy_(sd[lp + name].float())
        self.lstm = lstm.to(dev).eval()
        from ..ops.rnn import LSTMStack
        self.lstm_scan = LSTMStack(self.lstm)  # the recurrence on the repo's cooperative scan kernel (audio.hip)
        self.plan.append(("lstm", None))
        li += 1
        for ratio in cfg.upsampling_ratios:
            li += 1  # ELU (fused into the transposed conv's input below)
            p = f"{D}{li}.conv."
            ct = _ConvT(_wn(sd, p), sd.get(p + "bias"), ratio, cfg, dev, dt)
            li += 1
            self.plan.append(("convt", ct))
            for j in range(cfg.num_residual_layers):
                dil = cfg.dilation_growth_rate ** j
                c1 = conv(li, 1, dil, "block.1.")
                c2 = conv(li, 1, 1, "block.3.")
                sc = conv(li, 1, 1, "shortcut.") if cfg.use_conv_shortcut else None
                self.plan.append(("res", (c1, c2, sc)))
                li += 1
        li += 1  # final ELU
        self.plan.append(("final", conv(li)))

    @torch.no_grad()
    def quantized(self, codes: torch.Tensor) -> torch.Tensor:
        """codes [B, n_q, T] -> summed codebook embeddings [B, T, D] fp32."""
        out = None
        for q in range(codes.shape[1]):
            e = self.codebooks[q][codes[:, q].to(self.device)]
            out = e if out is None else out + e
        return out

    @torch.no_grad()
    def decode(self, codes: torch.Tensor) -> torch.Tensor:
        x = self.quantized(codes).to(self.dtype).contiguous()
        for kind, mod in self.plan:
            if kind == "conv":
                x = mod(x)
            elif kind == "lstm":
                xf = x.float().transpose(0, 1)  # [T, B, C]
                y = self.lstm_scan(xf) + xf
                x = y.transpose(0, 1).to(self.dtype).contiguous()
            elif kind == "convt":
                x = mod(F.elu(x))
            elif kind == "res":
                c1, c2, sc = mod
                h = c1(F.elu(x), act="elu")  # the ELU in front of the k1 conv rides c1's epilogue
                skip = sc(x) if sc is not None else x
                x = c2(h, residual=skip)
            else:
                x = mod(F.elu(x))
        return x.float().permute(0, 2, 1).contiguous()


def from_state_dict(cfg_dict: dict, sd: dict, device="cpu", prefix: str = "", dtype=None) -> EncodecDecoder:
    return EncodecDecoder(EncodecConfig.from_dict(cfg_dict), sd, device, dtype, prefix)
