"""2-D convolution on the implicit-GEMM MFMA kernel (csrc/kernels/conv.hip) for NHWC 16-bit tensors.

``conv2d(x, m, ...)`` takes an NCHW-shaped tensor stored channels_last (the layout every diffusion
module in this package keeps its activations in) and a ``torch.nn.Conv2d`` (or weight/bias), and
fuses what the UNet / VAE / ControlNet blocks do around a convolution into the kernel:

* ``upsample=True``   nearest-2x upsampling of the input (``conv(interpolate(x, 2))``), never materialised;
* ``pad=(t, l, b, r)`` asymmetric zero padding (the VAE encoder's ``F.pad(x, (0, 1, 0, 1))`` + stride 2);
* ``tadd``            a per-image channel vector added after the bias (ResNet time embedding);
* ``residual``        an NHWC tensor of the output's shape added in the epilogue (ResNet skip);
* ``act="silu"|"gelu"|"elu"|"leaky"|"tanh"`` SiLU / exact (erf) GELU / ELU / leaky ReLU (0.1) / tanh on the result;
* ``dilation``        filter dilation (EnCodec residual units).

The packed weight ([Cout, KH*KW*Cp] with Cp = Cin rounded up to 8 and k rounded up to 64, zero padded)
is built once per module and cached on it, keyed by the parameter's storage, dtype and version counter
(LoRA merges at load time and device casts rebuild it). CPU tensors run the fp32 PyTorch reference
(F.conv2d), which is the oracle for the GPU tests.

Reference parity: the convolutions of stablediffusion-ggml / diffusers (`backend/go/image/
stablediffusion-ggml/gosd.cpp:164-226`, `backend/python/diffusers/backend.py`) — here on MFMA instead of
ggml's im2col + GEMM or MIOpen.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from .. import _native as N

_ZERO: dict = {}
_ACT = {None: 0, "silu": 1, "gelu": 2, "elu": 3, "leaky": 4, "tanh": 5}


def _zero_page(device) -> torch.Tensor:
    z = _ZERO.get(device)
    if z is None:
        z = _ZERO[device] = torch.zeros(64, dtype=torch.uint8, device=device)
    return z


def pack_weight(w: torch.Tensor, dtype) -> tuple[torch.Tensor, int]:
    """[Cout, Cin, KH, KW] -> ([Cout, Kp] dtype, Cp): k = (kh*KW + kw)*Cp + ci, zero padded."""
    co, ci, kh, kw = w.shape
    cp = -(-ci // 8) * 8
    t = w.detach().permute(0, 2, 3, 1)  # [Cout, KH, KW, Cin]
    if cp != ci:
        t = F.pad(t, (0, cp - ci))
    t = t.reshape(co, kh * kw * cp)
    kp = -(-t.shape[1] // 64) * 64
    if kp != t.shape[1]:
        t = F.pad(t, (0, kp - t.shape[1]))
    return t.to(dtype).contiguous(), cp


def _packed(m, weight: torch.Tensor, dtype):
    key = (weight.data_ptr(), weight.dtype, weight.device, weight._version, dtype)
    c = getattr(m, "_mx_conv_pack", None) if m is not None else None
    if c is not None and c[0] == key:
        return c[1], c[2]
    wp, cp = pack_weight(weight, dtype)
    if m is not None:
        m._mx_conv_pack = (key, wp, cp)
    return wp, cp


def _bias32(m, bias):
    if bias is None:
        return None
    if bias.dtype == torch.float32 and bias.is_contiguous():
        return bias
    key = (bias.data_ptr(), bias.dtype, bias._version)
    c = getattr(m, "_mx_conv_bias", None) if m is not None else None
    if c is not None and c[0] == key:
        return c[1]
    b = bias.detach().float().contiguous()
    if m is not None:
        m._mx_conv_bias = (key, b)
    return b


def _reference(x, weight, bias, stride, pad, upsample, tadd, residual, act, dilation=1):
    xf = x.float()
    if upsample:
        xf = F.interpolate(xf, scale_factor=2.0, mode="nearest")
    t, l, b, r = pad
    if t == b and l == r:
        y = F.conv2d(xf, weight.float(), None if bias is None else bias.float(), stride, (t, l), dilation)
    else:
        y = F.conv2d(F.pad(xf, (l, r, t, b)), weight.float(), None if bias is None else bias.float(), stride, 0,
                     dilation)
    if tadd is not None:
        y = y + tadd.float()[:, :, None, None]
    if residual is not None:
        y = y + residual.float()
    if act == "silu":
        y = F.silu(y)
    elif act == "gelu":
        y = F.gelu(y)
    elif act == "elu":
        y = F.elu(y)
    elif act == "leaky":
        y = F.leaky_relu(y, 0.1)
    elif act == "tanh":
        y = torch.tanh(y)
    return y.to(x.dtype)


def conv2d(x: torch.Tensor, m: torch.nn.Conv2d | None = None, *, weight: torch.Tensor | None = None,
           bias: torch.Tensor | None = None, stride: int | None = None, padding: int | None = None,
           pad: tuple | None = None, upsample: bool = False, tadd: torch.Tensor | None = None,
           residual: torch.Tensor | None = None, act: str | None = None, out: torch.Tensor | None = None,
           packed: tuple | None = None, dilation: int | None = None, cfg: int = -1) -> torch.Tensor:
    """y = act(conv(up(x)) + bias + tadd + residual); x [N, C, H, W] channels_last 16-bit on GPU.
    ``packed``: a (weight, Cp) pair from :func:`pack_weight` for callers without a module to cache on."""
    if m is not None:
        weight = m.weight if weight is None else weight
        bias = m.bias if bias is None else bias
        stride = m.stride[0] if stride is None else stride
        if dilation is None:
            dh, dw = m.dilation
            if dh != dw and m.kernel_size[0] > 1 and m.kernel_size[1] > 1:
                raise ValueError("conv2d: per-axis dilation is not supported")
            dilation = max(dh, dw)
        if pad is None and padding is None:
            padding = m.padding[0]
    stride = 1 if stride is None else int(stride)
    dil = 1 if dilation is None else int(dilation)
    if pad is None:
        p = int(padding or 0)
        pad = (p, p, p, p)
    if not x.is_cuda:
        return _reference(x, weight, bias, stride, pad, upsample, tadd, residual, act, dil)
    n, c, h, w = x.shape
    co, ci, kh, kw = weight.shape
    if ci != c:
        raise ValueError(f"conv2d: input has {c} channels, weight expects {ci}")
    if x.dtype not in (torch.float16, torch.bfloat16):
        raise ValueError(f"conv2d: 16-bit activations required, got {x.dtype}")
    wp, cp = packed if packed is not None else _packed(m, weight, x.dtype)
    xin = x.permute(0, 2, 3, 1)  # NHWC view
    if cp != c:
        xin = F.pad(xin, (0, cp - c))
    if not xin.is_contiguous():
        xin = xin.contiguous()
    hl, wl = (2 * h, 2 * w) if upsample else (h, w)
    t, l, b, r = pad
    ho = (hl + t + b - dil * (kh - 1) - 1) // stride + 1
    wo = (wl + l + r - dil * (kw - 1) - 1) // stride + 1
    if out is None:
        out = torch.empty((n, co, ho, wo), dtype=x.dtype, device=x.device, memory_format=torch.channels_last)
    y = out.permute(0, 2, 3, 1)
    if not y.is_contiguous():
        raise ValueError("conv2d: `out` must be channels_last contiguous")
    res = None
    if residual is not None:
        if residual.shape != out.shape:
            raise ValueError(f"conv2d: residual {tuple(residual.shape)} vs output {tuple(out.shape)}")
        res = residual.permute(0, 2, 3, 1)
        if not res.is_contiguous() or res.dtype != x.dtype:
            res = res.to(x.dtype).contiguous()
    ta, ldt = None, co
    if tadd is not None:
        ta = tadd.float().reshape(-1, co)
        if ta.shape[0] not in (1, n):
            raise ValueError(f"conv2d: tadd rows {ta.shape[0]} vs batch {n}")
        ldt = 0 if ta.shape[0] == 1 else co  # one row broadcast over the batch
        if not ta.is_contiguous():
            ta = ta.contiguous()
    b32 = _bias32(m, bias)
    N.ensure_act(x.dtype)
    N.kcall("mxk_conv2d", xin.data_ptr(), n, h, w, cp, wp.data_ptr(), co, kh, kw, wp.shape[1], stride, dil, t, l,
            int(upsample), ho, wo, N.ptr(b32), N.ptr(ta), ldt, N.ptr(res), co, y.data_ptr(), co,
            _ACT[act], _zero_page(x.device).data_ptr(), int(cfg), N.stream_ptr())
    return out


# ---- Conv1d / ConvTranspose1d over [B, C, T] tensors (TTS vocoders, Kokoro) on the same kernel ------------------
# A Conv1d is the H = 1 case of conv2d: the input goes to [B, T, C] 16-bit rows once, the kernel writes
# [B, T', Cout] rows, and the result comes back as a [B, Cout, T'] view in the caller's dtype. Weights are
# packed once per (caller cache, name).

def conv1d_weights(w: torch.Tensor, b: torch.Tensor | None, dtype=torch.float16):
    """[Cout, Cin, K] weight -> (w4 [Cout, Cin, 1, K], fp32 bias, packed) for :func:`conv1d`."""
    w4 = w[:, :, None, :].to(dtype).contiguous()
    return w4, (b.float().contiguous() if b is not None else None), pack_weight(w4, dtype)


def conv1d(x: torch.Tensor, cw, stride: int = 1, padding: int = 0, dilation: int = 1, act: str | None = None,
           pad_r: int | None = None) -> torch.Tensor:
    """y = act(conv1d(x) + bias); x [B, C, T] any float dtype on the GPU, cw from :func:`conv1d_weights`.
    Zero padding `padding` on the left and `pad_r` (default the same) on the right."""
    w4, b32, packed = cw
    dt = w4.dtype
    B, C, T = x.shape
    rows = torch.empty((B, T, C), dtype=dt, device=x.device)
    rows.copy_(x.transpose(1, 2))
    pr = padding if pad_r is None else pad_r
    y = conv2d(rows[:, None].permute(0, 3, 1, 2), weight=w4, bias=b32, stride=stride, pad=(0, padding, 0, pr),
               dilation=dilation, act=act, packed=packed)  # [B, Cout, 1, T'] channels_last
    return y[:, :, 0, :].to(x.dtype)


def conv_transpose1d_weights(w: torch.Tensor, b: torch.Tensor | None, stride: int, dtype=torch.float16):
    """ConvTranspose1d weight [Cin, Cout, K = 2 stride] -> the k = 2 conv producing the `stride` output phases
    of each input frame (W'[(phi, co), ci, 0, tap]: tap 0 sees x[m-1] -> w[ci, co, phi + r], tap 1 sees x[m]
    -> w[ci, co, phi])."""
    ci, co, k = w.shape
    r = stride
    if k != 2 * r:
        raise ValueError(f"conv_transpose1d: kernel {k} != 2 x stride {r}")
    wp = torch.stack([w[:, :, r:].permute(2, 1, 0), w[:, :, :r].permute(2, 1, 0)], -1).reshape(r * co, ci, 1, 2)
    wp = wp.to(dtype).contiguous()
    bp = b.float().repeat(r).contiguous() if b is not None else None
    return wp, bp, pack_weight(wp, dtype), r, co


def conv_transpose1d(x: torch.Tensor, cwt, padding: int) -> torch.Tensor:
    """ConvTranspose1d(k = 2r, stride r, padding p) of x [B, Cin, T] -> [B, Cout, (T - 1) r - 2p + 2r]."""
    wp, bp, packed, r, co = cwt
    B, C, T = x.shape
    rows = torch.empty((B, T, C), dtype=wp.dtype, device=x.device)
    rows.copy_(x.transpose(1, 2))
    y = conv2d(rows[:, None].permute(0, 3, 1, 2), weight=wp, bias=bp, stride=1, pad=(0, 1, 0, 1),
               packed=packed)  # [B, r*co, 1, T+1]: frame m, phase phi
    y = y.permute(0, 2, 3, 1).reshape(B, (T + 1) * r, co)  # the full output: sample m r + phi
    # the full (unpadded) transposed conv has (T - 1) r + 2r = (T + 1) r samples; padding p trims p per side
    return y[:, padding:y.shape[1] - padding].transpose(1, 2).to(x.dtype)


def conv1d_gemm(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor | None = None, stride: int = 1, padding: int = 0,
                dilation: int = 1) -> torch.Tensor:
    """Conv1d [B, C, T] -> [B, Cout, T'] in the input's precision as an im2col view + one library GEMM (fp32
    where 16-bit operands would move a rounding decision, e.g. the VITS duration predictor / flows: no MIOpen)."""
    B, C, T = x.shape
    co, ci, k = w.shape
    xp = F.pad(x, (padding, padding)) if padding else x
    span = dilation * (k - 1) + 1
    cols = xp.unfold(2, span, stride)  # [B, C, T', span]
    if dilation > 1:
        cols = cols[..., ::dilation]
    To = cols.shape[2]
    a = cols.permute(0, 2, 1, 3).reshape(B * To, C * k)  # rows = output positions, (c, tap) columns
    y = a @ w.reshape(co, ci * k).t()
    if b is not None:
        y = y + b
    return y.view(B, To, co).transpose(1, 2)


def depthwise_conv1d(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor | None = None, padding: int = 0,
                     dilation: int = 1) -> torch.Tensor:
    """Depthwise (groups = C) stride-1 Conv1d [B, C, T] -> [B, C, T'] as a per-channel tap sum (fp32, no MIOpen)."""
    k = w.shape[-1]
    xp = F.pad(x, (padding, padding)) if padding else x
    cols = xp.unfold(2, dilation * (k - 1) + 1, 1)
    if dilation > 1:
        cols = cols[..., ::dilation]
    y = (cols * w.reshape(1, -1, 1, k)).sum(-1)
    return y + b[:, None] if b is not None else y
