"""Shared building blocks of the diffusion stack (text encoders, MMDiT, VAE, UNet).

Parameters live in `torch.nn.Module`s named like the public Hugging Face / diffusers checkpoints so a
`state_dict` loads directly from safetensors; the forward passes run on this library's kernels:
hipBLASLt GEMMs (F.linear / addmm with fp32 accumulate into residual streams), attention on the
MFMA flash kernel (attention_dense.hip, head dim <= 128; larger heads — only the VAE mid-block's
single 512-wide head — use PyTorch SDPA), adaLN / gated residual / GroupNorm kernels
(diffusion.hip), and convolutions on the implicit-GEMM MFMA kernel (conv.hip, ops/conv.py) over
channels_last (NHWC) activations, with bias / time-embedding / residual / SiLU / 2x upsampling fused.

Linear weights may also be `QParam`s — ggml block-quantised matrices from a GGUF checkpoint kept in their
block format on the GPU (stable-diffusion.cpp's Q4_0 / Q8_0 / K-quant files; reference gosd.cpp:56-162)
and run through the quantised GEMM (`ops.linear.qmatmul`) instead of being densified at load. Every
linear of the diffusion models goes through `lin` / `cat_w`, which accept either kind.
"""
from __future__ import annotations

import math
import os

import torch
import torch.nn.functional as F
from torch import nn

from ...ops import conv as CV
from ...ops import core as K
from ...ops import linear as L
from ...ops.linear import _fp32_out_ok


class QParam:
    """A [N, K] linear weight held block-quantised (ops.linear.QWeight, ggml row layout) in place of an
    nn.Linear's dense parameter. `dtype` is the pipeline's compute dtype (activations in and out)."""

    def __init__(self, qw: "L.QWeight", dtype):
        self.qw, self.dtype = qw, dtype

    @classmethod
    def from_ggml(cls, raw, qtype: int, N_: int, K_: int, device, dtype):
        """QParam, or a dense tensor when the block format / shape has no quantised kernel."""
        qw = L.QWeight.from_ggml(raw, qtype, N_, K_, device, dense_dtype=dtype)
        if not qw.is_quant and torch.device(device).type != "cpu":
            return qw.data.to(dtype)
        return cls(qw, dtype)  # CPU: the ggml bytes, dequantised by the reference GEMM

    @property
    def shape(self):
        return torch.Size((self.qw.N, self.qw.K))

    @property
    def device(self):
        return self.qw.device

    def dim(self) -> int:
        return 2

    def nbytes(self) -> int:
        return self.qw.nbytes() if self.qw.data.numel() else int(getattr(self.qw._raw, "nbytes", 0))

    def dense(self) -> torch.Tensor:
        if self.qw.data.is_cuda:
            return self.qw.dequant_gpu(self.dtype if self.dtype in (torch.bfloat16, torch.float16) else torch.float32)
        return self.qw.dense_f32().to(self.dtype)

    def linear(self, x: torch.Tensor, b: torch.Tensor | None = None) -> torch.Tensor:
        lead, K_ = x.shape[:-1], x.shape[-1]
        x2 = x.reshape(-1, K_)
        cdt = x2.dtype
        if x2.is_cuda and cdt not in (torch.bfloat16, torch.float16):
            x2 = x2.to(self.dtype if self.dtype in (torch.bfloat16, torch.float16) else torch.bfloat16)
        x2 = x2.contiguous()
        out = torch.empty(x2.shape[0], self.qw.N, dtype=x2.dtype, device=x2.device)
        L.qmatmul(self.qw, x2, L.EPI_BF16, out)
        if b is not None:
            out += b.to(out.dtype)
        return out.to(cdt).view(*lead, self.qw.N)

    @staticmethod
    def concat(ws: list["QParam"]):
        q = L.concat_rows([w.qw for w in ws])
        return QParam(q, ws[0].dtype) if q is not None else None


def lin(x: torch.Tensor, w, b: torch.Tensor | None = None) -> torch.Tensor:
    """F.linear over a dense weight or a QParam."""
    if isinstance(w, QParam):
        return w.linear(x, b)
    return F.linear(x, w, b)


def cat_w(ws: list) -> "torch.Tensor | QParam":
    """Row-concatenation of linear weights for a fused GEMM (Q|K|V, all adaLN modulations, ...): quantised
    weights of one block format stay quantised; a mix is densified."""
    if not any(isinstance(w, QParam) for w in ws):
        return torch.cat(ws)
    if all(isinstance(w, QParam) for w in ws):
        q = QParam.concat(ws)
        if q is not None:
            return q
    return torch.cat([w.dense() if isinstance(w, QParam) else w for w in ws])


def attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, B: int, Sq: int, Sk: int, H: int, D: int,
              scale: float | None = None, causal: bool = False, klen=None) -> torch.Tensor:
    """q: [B*Sq, H*D] rows (any row stride), k/v: [B*Sk, H*D] -> [B*Sq, H*D] (q dtype)."""
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    if q.is_cuda and D in (64, 128, 512):  # D = 512: the VAE mid-block's single head
        out = torch.empty(B * Sq, H * D, dtype=q.dtype, device=q.device)
        return K.attn_dense(q, k, v, out, B, Sq, Sk, H, H, D, scale, causal, klen=klen)
    qh = q.reshape(B, Sq, H, D).transpose(1, 2)
    kh = k.reshape(B, Sk, H, D).transpose(1, 2)
    vh = v.reshape(B, Sk, H, D).transpose(1, 2)
    mask = None
    if klen is not None:
        mask = (torch.arange(Sk, device=q.device)[None, :] < klen.to(q.device).view(B, 1))[:, None, None, :]
    o = F.scaled_dot_product_attention(qh, kh, vh, attn_mask=mask, is_causal=causal and mask is None, scale=scale)
    return o.transpose(1, 2).reshape(B * Sq, H * D)


def linear_acc(x: torch.Tensor, lin: nn.Linear, acc: torch.Tensor) -> torch.Tensor:
    """acc (fp32) += lin(x): the residual add runs as GEMM beta = 1 where the build supports fp32 out."""
    if isinstance(lin.weight, QParam):
        acc.add_(lin.weight.linear(x, lin.bias).float())
        return acc
    if x.is_cuda and x.dtype != torch.float32 and _fp32_out_ok(x.dtype) and acc.is_contiguous():
        if lin.bias is not None:
            acc.add_(lin.bias)
        torch.addmm(acc, x, lin.weight.t(), out_dtype=torch.float32, out=acc)
        return acc
    acc.add_(F.linear(x, lin.weight, lin.bias).float())
    return acc


def linear_f32(x: torch.Tensor, lin: nn.Linear) -> torch.Tensor:
    if isinstance(lin.weight, QParam):
        return lin.weight.linear(x, lin.bias).float()
    if x.is_cuda and x.dtype != torch.float32 and _fp32_out_ok(x.dtype):
        out = torch.empty(x.shape[0], lin.out_features, dtype=torch.float32, device=x.device)
        if lin.bias is not None:
            out.copy_(lin.bias.float().expand_as(out))
            torch.addmm(out, x, lin.weight.t(), out_dtype=torch.float32, out=out)
        else:
            torch.mm(x, lin.weight.t(), out_dtype=torch.float32, out=out)
        return out
    return F.linear(x, lin.weight, lin.bias).float()


def layernorm16(x: torch.Tensor, w, b, eps: float, dtype) -> torch.Tensor:
    out = torch.empty(x.shape, dtype=dtype, device=x.device)
    K.layernorm(x, w, b, eps, out)
    return out


def timestep_embedding(t: torch.Tensor, dim: int, flip_sin_to_cos: bool = True, shift: float = 0.0,
                       max_period: float = 10000.0) -> torch.Tensor:
    """Sinusoidal timestep features (diffusers `Timesteps`)."""
    half = dim // 2
    ex = -math.log(max_period) * torch.arange(half, dtype=torch.float32, device=t.device) / (half - shift)
    a = t.float()[:, None] * torch.exp(ex)[None, :]
    emb = torch.cat([torch.sin(a), torch.cos(a)], -1)
    if flip_sin_to_cos:
        emb = torch.cat([emb[:, half:], emb[:, :half]], -1)
    return emb


class GroupNorm(nn.GroupNorm):
    """GroupNorm (+ fused SiLU) on NHWC 16-bit activations (diffusion.hip); fp32 parameters."""

    def run(self, x: torch.Tensor, silu: bool = False) -> torch.Tensor:
        return K.groupnorm16(x, self.weight, self.bias, self.num_groups, self.eps, silu)


_VENDOR_CONV = os.environ.get("MX_CONV", "").lower() == "miopen"  # A/B switch for benchmarks only


def conv(x: torch.Tensor, m: nn.Conv2d, **fused) -> torch.Tensor:
    """m(x) with optional fused epilogue / prologue (ops/conv.py: tadd, residual, act, upsample, pad)."""
    if _VENDOR_CONV and x.is_cuda:
        return _vendor_conv(x, m, **fused)
    if x.is_cuda and x.dtype in (torch.float16, torch.bfloat16):
        return CV.conv2d(x, m, **fused)
    if not fused:
        return F.conv2d(x, m.weight, m.bias, m.stride, m.padding)
    return CV.conv2d(x, m, **fused)


def _vendor_conv(x, m, upsample=False, pad=None, tadd=None, residual=None, act=None):
    """The same fused op as unfused PyTorch/MIOpen calls (MX_CONV=miopen; benchmark baseline)."""
    if upsample:
        x = F.interpolate(x, scale_factor=2.0, mode="nearest").contiguous(memory_format=torch.channels_last)
    if pad is not None:
        t, l, b, r = pad
        x = F.pad(x, (l, r, t, b))
        y = F.conv2d(x, m.weight, m.bias, m.stride, 0)
    else:
        y = F.conv2d(x, m.weight, m.bias, m.stride, m.padding)
    if tadd is not None:
        y = y + tadd.to(y.dtype)[:, :, None, None]
    if residual is not None:
        y = y + residual
    if act == "silu":
        y = F.silu(y)
    return y


def cast_module(m: nn.Module, device, dtype) -> nn.Module:
    """Weights to `dtype` on `device`; norm parameters stay fp32 (the norm kernels read fp32)."""
    m.to(device)
    for mod in m.modules():
        keep32 = isinstance(mod, (nn.LayerNorm, nn.GroupNorm)) or type(mod).__name__.endswith("RMSNorm")
        for p in mod.parameters(recurse=False):
            p.data = p.data.float() if keep32 else p.data.to(dtype)
        for n, bf in mod.named_buffers(recurse=False):
            setattr(mod, n, bf.float())
    for mod in m.modules():
        if isinstance(mod, nn.Conv2d) and torch.device(device).type == "cuda":
            mod.weight.data = mod.weight.data.contiguous(memory_format=torch.channels_last)
    return m


def init_synthetic(m: nn.Module, seed: int = 0, std: float = 0.02):
    """Random-init weights in place (benchmarks / tests; no checkpoint download). Norm weights 1,
    biases 0, other tensors N(0, std) scaled by fan-in for linears/convs."""
    g = torch.Generator(device=next(m.parameters()).device).manual_seed(seed)
    with torch.no_grad():
        for name, p in m.named_parameters():
            if name.endswith("bias"):
                p.zero_()
            elif p.dim() == 1:
                p.fill_(1.0)
            else:
                fan_in = p[0].numel() if p.dim() > 1 else 1
                s = std if "embed" in name and p.dim() == 2 and "linear" not in name else 1.0 / math.sqrt(fan_in)
                p.normal_(0.0, s, generator=g)
    return m
