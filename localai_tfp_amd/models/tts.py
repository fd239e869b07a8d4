"""VITS text-to-speech (the architecture behind the reference's `piper` voices and Coqui/MMS VITS
models): relative-position transformer text encoder -> (stochastic) duration predictor -> monotonic
length regulation -> reverse normalising flow -> HiFi-GAN vocoder.

Parity targets: the reference's `piper` backend (backend/go/tts/piper.go:20-49, go-piper ->
piper C++ -> onnxruntime VITS) and the Python `coqui` / `transformers` (VitsModel) TTS backends.
Weights load from a Hugging Face VITS directory (config.json + model.safetensors + vocab.json, e.g.
the MMS-TTS voices; weight-norm parametrisations are folded at load) or `synthetic:vits-*`
(random init). Piper .onnx voices load through models/piper.py (initializer renaming, no onnx runtime).

MI355X path: the encoder, flows and vocoder run as fp32 conv/GEMM ops on the GPU (MIOpen /
hipBLASLt — plain library convolutions), the WaveNet gate (tanh(a) * sigmoid(b) over the two
channel halves) is one fused pass in csrc/kernels/audio.hip, and the expanded prior is built with
one gather instead of the [T_out, T_in] alignment-matrix matmul of the HF implementation.
"""
from __future__ import annotations

import json
import math
import os
from dataclasses import dataclass, field

import numpy as np
import torch
import torch.nn.functional as F

from ..ops import conv as CV


@dataclass
class VitsConfig:
    vocab: int = 38
    hidden: int = 192
    n_layers: int = 6
    n_heads: int = 2
    ffn: int = 768
    ffn_kernel: int = 3
    window: int = 4
    flow_size: int = 192
    eps: float = 1e-5
    sdp: bool = True  # stochastic duration predictor
    dp_filter: int = 256
    dp_kernel: int = 3
    dds_layers: int = 3
    dds_channels: int = 2
    flow_bins: int = 10
    tail_bound: float = 5.0
    dp_flows: int = 4
    prior_flows: int = 4
    prior_wn_layers: int = 4
    wn_kernel: int = 5
    wn_dilation: int = 1
    upsample_initial: int = 512
    upsample_rates: tuple = (8, 8, 2, 2)
    upsample_kernels: tuple = (16, 16, 4, 4)
    resblock_kernels: tuple = (3, 7, 11)
    resblock_dilations: tuple = ((1, 3, 5), (1, 3, 5), (1, 3, 5))
    slope: float = 0.1
    n_speakers: int = 1
    spk_dim: int = 0
    sample_rate: int = 16000
    noise_scale: float = 0.667
    noise_scale_duration: float = 0.8
    speaking_rate: float = 1.0
    name: str = "vits"
    extra: dict = field(default_factory=dict)

    @classmethod
    def from_hf(cls, c: dict) -> "VitsConfig":
        return cls(vocab=c["vocab_size"], hidden=c["hidden_size"], n_layers=c["num_hidden_layers"],
                   n_heads=c["num_attention_heads"], ffn=c["ffn_dim"], ffn_kernel=c.get("ffn_kernel_size", 3),
                   window=c.get("window_size", 4) or 0, flow_size=c["flow_size"], eps=c.get("layer_norm_eps", 1e-5),
                   sdp=c.get("use_stochastic_duration_prediction", True),
                   dp_filter=c.get("duration_predictor_filter_channels", 256),
                   dp_kernel=c.get("duration_predictor_kernel_size", 3),
                   dds_layers=c.get("depth_separable_num_layers", 3),
                   dds_channels=c.get("depth_separable_channels", 2),
                   flow_bins=c.get("duration_predictor_flow_bins", 10),
                   tail_bound=c.get("duration_predictor_tail_bound", 5.0),
                   dp_flows=c.get("duration_predictor_num_flows", 4),
                   prior_flows=c.get("prior_encoder_num_flows", 4),
                   prior_wn_layers=c.get("prior_encoder_num_wavenet_layers", 4),
                   wn_kernel=c.get("wavenet_kernel_size", 5), wn_dilation=c.get("wavenet_dilation_rate", 1),
                   upsample_initial=c["upsample_initial_channel"], upsample_rates=tuple(c["upsample_rates"]),
                   upsample_kernels=tuple(c["upsample_kernel_sizes"]),
                   resblock_kernels=tuple(c["resblock_kernel_sizes"]),
                   resblock_dilations=tuple(tuple(d) for d in c["resblock_dilation_sizes"]),
                   slope=c.get("leaky_relu_slope", 0.1), n_speakers=c.get("num_speakers", 1),
                   spk_dim=c.get("speaker_embedding_size", 0), sample_rate=c.get("sampling_rate", 16000),
                   noise_scale=c.get("noise_scale", 0.667), noise_scale_duration=c.get("noise_scale_duration", 0.8),
                   speaking_rate=c.get("speaking_rate", 1.0), name=c.get("_name_or_path", "vits") or "vits")

    def to_hf(self) -> dict:
        """HF VitsConfig kwargs (tests build a transformers VitsModel oracle from the same config)."""
        return dict(vocab_size=self.vocab, hidden_size=self.hidden, num_hidden_layers=self.n_layers,
                    num_attention_heads=self.n_heads, ffn_dim=self.ffn, ffn_kernel_size=self.ffn_kernel,
                    window_size=self.window, flow_size=self.flow_size, layer_norm_eps=self.eps,
                    use_stochastic_duration_prediction=self.sdp, duration_predictor_filter_channels=self.dp_filter,
                    duration_predictor_kernel_size=self.dp_kernel, depth_separable_num_layers=self.dds_layers,
                    depth_separable_channels=self.dds_channels, duration_predictor_flow_bins=self.flow_bins,
                    duration_predictor_tail_bound=self.tail_bound, duration_predictor_num_flows=self.dp_flows,
                    prior_encoder_num_flows=self.prior_flows, prior_encoder_num_wavenet_layers=self.prior_wn_layers,
                    wavenet_kernel_size=self.wn_kernel, wavenet_dilation_rate=self.wn_dilation,
                    upsample_initial_channel=self.upsample_initial, upsample_rates=list(self.upsample_rates),
                    upsample_kernel_sizes=list(self.upsample_kernels),
                    resblock_kernel_sizes=list(self.resblock_kernels),
                    resblock_dilation_sizes=[list(d) for d in self.resblock_dilations], leaky_relu_slope=self.slope,
                    num_speakers=self.n_speakers, speaker_embedding_size=self.spk_dim,
                    sampling_rate=self.sample_rate, noise_scale=self.noise_scale,
                    noise_scale_duration=self.noise_scale_duration, speaking_rate=self.speaking_rate)


VITS_TEST = VitsConfig(name="vits-test", vocab=40, hidden=64, n_layers=2, n_heads=2, ffn=128, flow_size=32,
                       dp_filter=64, prior_wn_layers=2, upsample_initial=64, upsample_rates=(4, 4),
                       upsample_kernels=(8, 8), resblock_kernels=(3, 5), resblock_dilations=((1, 3), (1, 3)))
VITS_BASE = VitsConfig(name="vits-base")  # MMS-TTS / piper-medium sized (~36M params)
SYNTHETIC = {"vits-test": VITS_TEST, "vits-base": VITS_BASE}


# ------------------------------------------------------------------------------------------------
# weights
def fold_weight_norm(sd: dict) -> dict:
    """weight = g * v / ||v|| (norm over all but dim 0), for both the legacy `weight_g/weight_v` and
    the `parametrizations.weight.original0/1` layouts."""
    out = {}
    for k, v in sd.items():
        if k.endswith(".weight_g") or k.endswith(".parametrizations.weight.original0"):
            base = k[: -len(".weight_g")] if k.endswith(".weight_g") else k[: -len(".parametrizations.weight.original0")]
            vv = sd.get(base + ".weight_v", sd.get(base + ".parametrizations.weight.original1"))
            dims = tuple(range(1, vv.dim()))
            out[base + ".weight"] = v * vv / vv.norm(dim=dims, keepdim=True)
        elif k.endswith(".weight_v") or k.endswith(".parametrizations.weight.original1"):
            continue
        else:
            out[k] = v
    return out


def synthetic_vits(cfg: VitsConfig, seed: int = 0) -> dict:
    """Random-init state dict with the HF VitsModel names (built from a transformers VitsModel when
    available so the layout is exact; otherwise that import failing is an error)."""
    from transformers import VitsConfig as HC, VitsModel
    torch.manual_seed(seed)
    m = VitsModel(HC(**cfg.to_hf())).eval()
    sd = {k: v.detach().float().clone() for k, v in m.state_dict().items()}
    return fold_weight_norm(sd)


def load_vits(path: str, device="cpu"):
    """-> (VitsModel, tokenizer). `path`: HF VITS directory or synthetic:<name>."""
    if path.startswith("synthetic:"):
        cfg = SYNTHETIC[path.split(":", 1)[1]]
        return VitsModel(cfg, synthetic_vits(cfg), device), CharTokenizer.synthetic(cfg.vocab)
    cj = json.load(open(os.path.join(path, "config.json")))
    cfg = VitsConfig.from_hf(cj)
    from safetensors.torch import load_file
    st = [f for f in os.listdir(path) if f.endswith(".safetensors")]
    if st:
        sd = {}
        for f in sorted(st):
            sd.update(load_file(os.path.join(path, f)))
    else:
        sd = torch.load(os.path.join(path, "pytorch_model.bin"), map_location="cpu", weights_only=True)
    sd = fold_weight_norm({k: v.float() for k, v in sd.items()})
    return VitsModel(cfg, sd, device), CharTokenizer.from_dir(path)


class CharTokenizer:
    """VitsTokenizer semantics without a phonemizer: lower-case (optional), drop characters missing
    from the vocab, intersperse the blank id 0 (add_blank)."""

    def __init__(self, vocab: dict, add_blank: bool = True, lower: bool = True):
        self.vocab = vocab
        self.add_blank = add_blank
        self.lower = lower

    @classmethod
    def from_dir(cls, path: str) -> "CharTokenizer":
        vocab = json.load(open(os.path.join(path, "vocab.json")))
        tc = os.path.join(path, "tokenizer_config.json")
        cfg = json.load(open(tc)) if os.path.exists(tc) else {}
        return cls(vocab, cfg.get("add_blank", True), cfg.get("normalize", True))

    @classmethod
    def synthetic(cls, n: int) -> "CharTokenizer":
        chars = ["_"] + list(" abcdefghijklmnopqrstuvwxyz',.?!-") + [str(i) for i in range(10)]
        return cls({c: i for i, c in enumerate(chars[:n])})

    def encode(self, text: str) -> list[int]:
        t = text.lower() if self.lower else text
        ids = [self.vocab[c] for c in t if c in self.vocab]
        if self.add_blank:
            out = [0] * (2 * len(ids) + 1)
            out[1::2] = ids
            return out
        return ids


# ------------------------------------------------------------------------------------------------
def _leaky(x: torch.Tensor, slope: float) -> torch.Tensor:
    return F.leaky_relu(x, slope)


def _wn_gate(x: torch.Tensor, H: int) -> torch.Tensor:
    if x.is_cuda:
        from ..ops import core as K
        return K.wavenet_gate(x, H)
    return torch.tanh(x[:, :H]) * torch.sigmoid(x[:, H:])


def rq_spline_inverse(x, uw, uh, ud, tail: float, min_w=1e-3, min_h=1e-3, min_d=1e-3):
    """Inverse of the unconstrained monotone rational-quadratic spline (identity outside
    [-tail, tail], linear tails). x [...], uw/uh [..., K], ud [..., K-1]."""
    K = uw.shape[-1]
    inside = (x >= -tail) & (x <= tail)
    const = math.log(math.exp(1 - min_d) - 1)
    ud = F.pad(ud, (1, 1), value=const)
    w = F.softmax(uw, -1)
    w = min_w + (1 - min_w * K) * w
    cw = F.pad(torch.cumsum(w, -1), (1, 0))
    cw = 2 * tail * cw - tail
    cw[..., 0], cw[..., -1] = -tail, tail
    w = cw[..., 1:] - cw[..., :-1]
    d = min_d + F.softplus(ud)
    h = F.softmax(uh, -1)
    h = min_h + (1 - min_h * K) * h
    ch = F.pad(torch.cumsum(h, -1), (1, 0))
    ch = 2 * tail * ch - tail
    ch[..., 0], ch[..., -1] = -tail, tail
    h = ch[..., 1:] - ch[..., :-1]
    loc = ch.clone()
    loc[..., -1] += 1e-6
    idx = (torch.sum(x[..., None] >= loc, -1) - 1).clamp(0, K - 1)[..., None]
    icw, iw = cw.gather(-1, idx)[..., 0], w.gather(-1, idx)[..., 0]
    ich, ih = ch.gather(-1, idx)[..., 0], h.gather(-1, idx)[..., 0]
    delta = (h / w).gather(-1, idx)[..., 0]
    d0, d1 = d.gather(-1, idx)[..., 0], d[..., 1:].gather(-1, idx)[..., 0]
    i1 = d0 + d1 - 2 * delta
    i2 = x - ich
    i3 = i2 * i1
    a = ih * (delta - d0) + i3
    b = ih * d0 - i3
    c = -delta * i2
    disc = (b * b - 4 * a * c).clamp_min(0)
    root = (2 * c) / (-b - torch.sqrt(disc))
    y = root * iw + icw
    return torch.where(inside, y, x)


class VitsModel:
    """Inference-only VITS with weights in a flat dict (HF VitsModel names, weight norm folded)."""

    def __init__(self, cfg: VitsConfig, sd: dict, device="cpu"):
        self.cfg = cfg
        self.device = torch.device(device)
        self.w = {k: v.to(self.device, torch.float32).contiguous() for k, v in sd.items()}

    def p(self, k):
        return self.w[k]

    def pb(self, k):
        return self.w.get(k)

    def conv(self, x, name, **kw):
        if x.is_cuda:  # fp32 im2col + library GEMM (the text encoder / flows / duration predictor; no MIOpen)
            return CV.conv1d_gemm(x, self.w[name + ".weight"], self.w.get(name + ".bias"), **kw)
        return F.conv1d(x, self.w[name + ".weight"], self.w.get(name + ".bias"), **kw)

    # ---------------------------------------------------------------- text encoder
    def _rel_emb(self, emb, L):
        W = self.cfg.window
        pad = max(L - (W + 1), 0)
        if pad:
            emb = F.pad(emb, (0, 0, pad, pad))
        s = max(W + 1 - L, 0)
        return emb[:, s:s + 2 * L - 1]

    def attention(self, x, pre):
        c = self.cfg
        B, L, D = x.shape
        H, hd = c.n_heads, D // c.n_heads
        q = F.linear(x, self.p(pre + "q_proj.weight"), self.pb(pre + "q_proj.bias")) * hd ** -0.5
        k = F.linear(x, self.p(pre + "k_proj.weight"), self.pb(pre + "k_proj.bias"))
        v = F.linear(x, self.p(pre + "v_proj.weight"), self.pb(pre + "v_proj.bias"))
        q, k, v = (t.view(B, L, H, hd).transpose(1, 2).reshape(B * H, L, hd) for t in (q, k, v))
        s = q @ k.transpose(1, 2)
        if c.window:
            rk = self._rel_emb(self.p(pre + "emb_rel_k"), L)  # [1, 2L-1, hd]
            rl = q @ rk.transpose(1, 2)  # [BH, L, 2L-1]: column L-1+(j-i) is the key-offset logit
            idx = (torch.arange(L, device=x.device)[None, :] - torch.arange(L, device=x.device)[:, None]) + L - 1
            s = s + rl.gather(2, idx[None].expand(B * H, L, L))
        pr = s.softmax(-1)
        o = pr @ v
        if c.window:
            rv = self._rel_emb(self.p(pre + "emb_rel_v"), L)
            idx = (torch.arange(L, device=x.device)[None, :] - torch.arange(L, device=x.device)[:, None]) + L - 1
            rel = x.new_zeros(B * H, L, 2 * L - 1).scatter_(2, idx[None].expand(B * H, L, L), pr)
            o = o + rel @ rv
        o = o.view(B, H, L, hd).transpose(1, 2).reshape(B, L, D)
        return F.linear(o, self.p(pre + "out_proj.weight"), self.pb(pre + "out_proj.bias"))

    def ffn(self, x, pre):
        k = self.cfg.ffn_kernel
        pl, pr = (k - 1) // 2, k // 2
        h = x.transpose(1, 2)
        h = F.relu(self.conv(F.pad(h, (pl, pr)), pre + "conv_1"))
        h = self.conv(F.pad(h, (pl, pr)), pre + "conv_2")
        return h.transpose(1, 2)

    def text_encoder(self, ids: torch.Tensor):
        c = self.cfg
        x = F.embedding(ids, self.p("text_encoder.embed_tokens.weight")) * math.sqrt(c.hidden)
        for i in range(c.n_layers):
            pre = f"text_encoder.encoder.layers.{i}."
            x = F.layer_norm(x + self.attention(x, pre + "attention."), (c.hidden,),
                             self.p(pre + "layer_norm.weight"), self.p(pre + "layer_norm.bias"), c.eps)
            x = F.layer_norm(x + self.ffn(x, pre + "feed_forward."), (c.hidden,),
                             self.p(pre + "final_layer_norm.weight"), self.p(pre + "final_layer_norm.bias"), c.eps)
        stats = self.conv(x.transpose(1, 2), "text_encoder.project")  # [B, 2F, L]
        m, logs = stats.split(c.flow_size, 1)
        return x.transpose(1, 2), m, logs

    # ---------------------------------------------------------------- duration
    def dds(self, x, pre, g=None):
        c = self.cfg
        if g is not None:
            x = x + g
        ch = x.shape[1]
        for i in range(c.dds_layers):
            dil = c.dp_kernel ** i
            if x.is_cuda:
                h = CV.depthwise_conv1d(x, self.p(f"{pre}convs_dilated.{i}.weight"),
                                        self.p(f"{pre}convs_dilated.{i}.bias"), dilation=dil,
                                        padding=(c.dp_kernel * dil - dil) // 2)
            else:
                h = F.conv1d(x, self.p(f"{pre}convs_dilated.{i}.weight"), self.p(f"{pre}convs_dilated.{i}.bias"),
                             groups=ch, dilation=dil, padding=(c.dp_kernel * dil - dil) // 2)
            h = F.gelu(F.layer_norm(h.transpose(1, 2), (ch,), self.p(f"{pre}norms_1.{i}.weight"),
                                    self.p(f"{pre}norms_1.{i}.bias"), 1e-5).transpose(1, 2))
            h = self.conv(h, f"{pre}convs_pointwise.{i}")
            h = F.gelu(F.layer_norm(h.transpose(1, 2), (ch,), self.p(f"{pre}norms_2.{i}.weight"),
                                    self.p(f"{pre}norms_2.{i}.bias"), 1e-5).transpose(1, 2))
            x = x + h
        return x

    def conv_flow_inv(self, z, pre, g):
        c = self.cfg
        half = c.dds_channels // 2
        a, b = z[:, :half], z[:, half:]
        h = self.conv(a, pre + "conv_pre")
        h = self.dds(h, pre + "conv_dds.", g)
        h = self.conv(h, pre + "conv_proj")
        B, _, L = a.shape
        h = h.reshape(B, half, -1, L).permute(0, 1, 3, 2)
        K = c.flow_bins
        s = math.sqrt(c.hidden)
        b = rq_spline_inverse(b, h[..., :K] / s, h[..., K:2 * K] / s, h[..., 2 * K:], c.tail_bound)
        return torch.cat([a, b], 1)

    def log_durations(self, x, g=None, noise_scale_duration: float = 0.8, gen=None):
        c = self.cfg
        if not c.sdp:
            pre = "duration_predictor."
            if g is not None:
                x = x + self.conv(g, pre + "cond")
            h = F.relu(self.conv(x, pre + "conv_1", padding=c.dp_kernel // 2))
            h = F.layer_norm(h.transpose(1, 2), (c.dp_filter,), self.p(pre + "norm_1.weight"),
                             self.p(pre + "norm_1.bias"), c.eps).transpose(1, 2)
            h = F.relu(self.conv(h, pre + "conv_2", padding=c.dp_kernel // 2))
            h = F.layer_norm(h.transpose(1, 2), (c.dp_filter,), self.p(pre + "norm_2.weight"),
                             self.p(pre + "norm_2.bias"), c.eps).transpose(1, 2)
            return self.conv(h, pre + "proj")
        pre = "duration_predictor."
        h = self.conv(x, pre + "conv_pre")
        if g is not None:
            h = h + self.conv(g, pre + "cond")
        h = self.dds(h, pre + "conv_dds.")
        h = self.conv(h, pre + "conv_proj")
        B, _, L = x.shape
        z = torch.randn(B, 2, L, generator=gen, device="cpu").to(x.device) * noise_scale_duration
        # reverse flows: the conv flows in reverse order, then the elementwise affine; the last conv
        # flow (flows[1]) is skipped as in VITS inference ("remove a useless vflow")
        order = list(range(c.dp_flows, 1, -1))
        for fi in order:
            z = torch.flip(z, [1])
            z = self.conv_flow_inv(z, f"{pre}flows.{fi}.", h)
        z = torch.flip(z, [1])
        t, ls = self.p(pre + "flows.0.translate"), self.p(pre + "flows.0.log_scale")
        z = (z - t) * torch.exp(-ls)
        return z[:, :1]

    # ---------------------------------------------------------------- flow + vocoder
    def wavenet(self, x, pre, n_layers, g=None):
        c = self.cfg
        H = c.hidden
        out = torch.zeros_like(x)
        gc = self.conv(g, pre + "cond_layer") if g is not None else None
        for i in range(n_layers):
            dil = c.wn_dilation ** i
            h = self.conv(x, f"{pre}in_layers.{i}", dilation=dil, padding=(c.wn_kernel * dil - dil) // 2)
            if gc is not None:
                h = h + gc[:, i * 2 * H:(i + 1) * 2 * H]
            acts = _wn_gate(h, H)
            rs = self.conv(acts, f"{pre}res_skip_layers.{i}")
            if i < n_layers - 1:
                x = x + rs[:, :H]
                out = out + rs[:, H:]
            else:
                out = out + rs
        return out

    def flow_inv(self, z, g=None):
        c = self.cfg
        half = c.flow_size // 2
        for i in reversed(range(c.prior_flows)):
            z = torch.flip(z, [1])
            pre = f"flow.flows.{i}."
            a, b = z[:, :half], z[:, half:]
            h = self.conv(a, pre + "conv_pre")
            h = self.wavenet(h, pre + "wavenet.", c.prior_wn_layers, g)
            m = self.conv(h, pre + "conv_post")
            z = torch.cat([a, b - m], 1)
        return z

    def _vocoder_plan(self):
        """HiFi-GAN convolutions as conv.hip convs over [B, T, C] 16-bit rows (built once): transposed convs
        (k = 2r, padding r/2) as one k = 2 conv producing the r output phases per frame (models/encodec.py)."""
        from types import SimpleNamespace
        from .encodec import _ConvT
        c = self.cfg
        dt = torch.float16
        cf = SimpleNamespace(use_causal_conv=False, pad_mode="constant", trim_right_ratio=1.0)

        def c1(name):
            w = self.w[name + ".weight"]
            b = self.w.get(name + ".bias")
            w4 = w[:, :, None, :].to(dt).contiguous()
            return (w4, b.float() if b is not None else None, CV.pack_weight(w4, dt), int(w.shape[2]))
        if c.slope != 0.1:
            return None  # the fused epilogue's leaky slope is 0.1
        ups = []
        for i, (r, k) in enumerate(zip(c.upsample_rates, c.upsample_kernels)):
            if k != 2 * r or r % 2:
                return None  # not the k = 2r, padding r/2 HiFi-GAN geometry: library path
            ups.append(_ConvT(self.w[f"decoder.upsampler.{i}.weight"], self.w.get(f"decoder.upsampler.{i}.bias"), r, cf,
                              self.device, dt))
        nk = len(c.resblock_kernels)
        res = {}
        for i in range(len(ups)):
            for j, dils in enumerate(c.resblock_dilations):
                pre = f"decoder.resblocks.{i * nk + j}."
                res[i * nk + j] = [(c1(f"{pre}convs1.{n}"), c1(f"{pre}convs2.{n}")) for n in range(len(dils))]
        return dict(pre=c1("decoder.conv_pre"), post=c1("decoder.conv_post"), ups=ups, res=res,
                    cond=c1("decoder.cond") if "decoder.cond.weight" in self.w else None)

    @staticmethod
    def _c1(x, cw, dil=1, act=None, residual=None, tadd=None):
        """One stride-1 'same' Conv1d on conv.hip: x [B, T, C] 16-bit rows -> [B, T, Cout] rows."""
        w4, b, packed, k = cw
        p = dil * (k - 1) // 2
        xin = x[:, None].permute(0, 3, 1, 2)
        res = residual[:, None].permute(0, 3, 1, 2) if residual is not None else None
        y = CV.conv2d(xin, weight=w4, bias=b, stride=1, pad=(0, p, 0, dil * (k - 1) - p), dilation=dil, act=act,
                      residual=res, tadd=tadd, packed=packed)
        return y.permute(0, 2, 3, 1)[:, 0]

    def vocoder(self, z, g=None):
        c = self.cfg
        if self.device.type == "cuda":
            if not hasattr(self, "_vplan"):
                self._vplan = self._vocoder_plan()
            if self._vplan is not None:
                return self._vocoder_gpu(z, g)
        return self._vocoder_ref(z, g)

    def _vocoder_gpu(self, z, g=None):
        c, P = self.cfg, self._vplan
        nk = len(c.resblock_kernels)
        tadd = None
        if g is not None and P["cond"] is not None:
            w4, b, _, _ = P["cond"]
            tadd = CV.conv1d_gemm(g, w4[:, :, 0].float(), b)[:, :, 0]  # [B, C] per-utterance channel offset
        x = self._c1(z.transpose(1, 2).to(torch.float16).contiguous(), P["pre"], tadd=tadd)
        for i in range(len(P["ups"])):
            x = P["ups"][i](F.leaky_relu(x, c.slope).contiguous())
            acc = None
            for j, dils in enumerate(c.resblock_dilations):
                h = x
                for (cw1, cw2), d in zip(P["res"][i * nk + j], dils):
                    t = self._c1(F.leaky_relu(h, c.slope).contiguous(), cw1, dil=d, act="leaky")
                    h = self._c1(t, cw2, residual=h)
                acc = h.float() if acc is None else acc + h.float()
            x = (acc / nk).to(torch.float16)
        y = self._c1(F.leaky_relu(x, 0.01).contiguous(), P["post"], act="tanh")
        return y.float().transpose(1, 2)

    def _vocoder_ref(self, z, g=None):
        c = self.cfg
        x = self.conv(z, "decoder.conv_pre", padding=3)
        if g is not None:
            x = x + self.conv(g, "decoder.cond")
        nk = len(c.resblock_kernels)
        for i, (r, k) in enumerate(zip(c.upsample_rates, c.upsample_kernels)):
            x = _leaky(x, c.slope)
            x = F.conv_transpose1d(x, self.p(f"decoder.upsampler.{i}.weight"), self.p(f"decoder.upsampler.{i}.bias"),
                                   stride=r, padding=(k - r) // 2)
            acc = None
            for j, (rk, dils) in enumerate(zip(c.resblock_kernels, c.resblock_dilations)):
                pre = f"decoder.resblocks.{i * nk + j}."
                h = x
                for n, d in enumerate(dils):
                    t = self.conv(_leaky(h, c.slope), f"{pre}convs1.{n}", dilation=d, padding=(rk * d - d) // 2)
                    t = self.conv(_leaky(t, c.slope), f"{pre}convs2.{n}", padding=(rk - 1) // 2)
                    h = h + t
                acc = h if acc is None else acc + h
            x = acc / nk
        x = F.leaky_relu(x, 0.01)
        return torch.tanh(F.conv1d(x, self.p("decoder.conv_post.weight"), None, padding=3))

    # ---------------------------------------------------------------- full synthesis
    @torch.no_grad()
    def synthesize(self, ids: list[int], speaker: int | None = None, speaking_rate: float | None = None,
                   noise_scale: float | None = None, noise_scale_duration: float | None = None,
                   seed: int | None = 0) -> np.ndarray:
        """token ids -> float32 waveform at cfg.sample_rate."""
        c = self.cfg
        gen = torch.Generator().manual_seed(seed) if seed is not None else None
        ids_t = torch.tensor([ids], dtype=torch.long, device=self.device)
        g = None
        if c.n_speakers > 1 and speaker is not None:
            g = self.p("embed_speaker.weight")[int(speaker) % c.n_speakers][None, :, None]
        x, m, logs = self.text_encoder(ids_t)
        nsd = c.noise_scale_duration if noise_scale_duration is None else noise_scale_duration
        logw = self.log_durations(x, g, nsd, gen)
        rate = speaking_rate or c.speaking_rate
        dur = torch.ceil(torch.exp(logw) / rate)[0, 0].long()  # [L]
        T = max(int(dur.sum()), 1)
        # monotonic alignment as a gather: output frame t copies the token whose span covers t
        tok = torch.repeat_interleave(torch.arange(dur.numel(), device=self.device), dur.clamp_min(0))
        if tok.numel() == 0:
            tok = torch.zeros(1, dtype=torch.long, device=self.device)
        mp, lp = m[:, :, tok], logs[:, :, tok]
        ns = c.noise_scale if noise_scale is None else noise_scale
        eps = torch.randn(mp.shape, generator=gen, device="cpu").to(self.device)
        z = mp + eps * torch.exp(lp) * ns
        z = self.flow_inv(z, g)
        wav = self.vocoder(z, g)
        assert T == z.shape[-1]
        return wav[0, 0].float().cpu().numpy()
