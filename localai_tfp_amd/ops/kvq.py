"""Block-quantised paged KV cache (llama.cpp `cache_type_k / cache_type_v` q8_0 / q4_0 / q4_1 / q5_0 / q5_1 /
iq4_nl, grpc-server.cpp:2338-2341): host-side format table, the reference quantiser / dequantiser (the numerics oracle
of csrc/kernels/kvq.hip and the CPU engine path), and the cache-tensor tagging the attention wrappers read.

A quantised layer cache is a uint8 tensor [num_blocks, Hkv, block_size, row_bytes]: one row per (token, KV head)
holding the D / 32 blocks of that head vector in the csrc/kernels/kvq.h layout (codes, 5-bit high bits, f16 scales),
with exactly llama.cpp's bytes per block. The tensors carry their format as a `kvf` attribute (KVCache.layer sets it
on every view it hands out).
"""
from __future__ import annotations

import numpy as np
import torch

# ids shared with csrc/kernels/kvq.h (0 / 1 are the bf16 / fp8 e4m3 caches)
KVF_BF16, KVF_FP8, KVF_Q8_0, KVF_Q4_0, KVF_Q4_1, KVF_Q5_0, KVF_Q5_1, KVF_IQ4_NL = range(8)
FORMATS = {"q8_0": KVF_Q8_0, "q4_0": KVF_Q4_0, "q4_1": KVF_Q4_1, "q5_0": KVF_Q5_0, "q5_1": KVF_Q5_1,
           "iq4_nl": KVF_IQ4_NL}
NAMES = {v: k for k, v in FORMATS.items()}
IQ4NL = np.array([-127, -104, -83, -65, -49, -35, -22, -10, 1, 13, 25, 38, 53, 69, 89, 113], np.float32)
# llama.cpp bytes per 32-element block (ggml_type_size): the row layout here stores the same bytes
BLOCK_BYTES = {KVF_Q8_0: 34, KVF_Q4_0: 18, KVF_Q4_1: 20, KVF_Q5_0: 22, KVF_Q5_1: 24, KVF_IQ4_NL: 18}


def _geom(kvf: int, D: int):
    q8 = kvf == KVF_Q8_0
    hb = kvf in (KVF_Q5_0, KVF_Q5_1)
    mn = kvf in (KVF_Q4_1, KVF_Q5_1)
    cb = D if q8 else D // 2
    hbb = D // 8 if hb else 0
    sb = (D // 32) * (4 if mn else 2)
    return cb, hbb, sb, q8, hb, mn


def row_bytes(kvf: int, D: int) -> int:
    cb, hbb, sb, *_ = _geom(kvf, D)
    return cb + hbb + sb


def kv_format(t: torch.Tensor) -> int:
    f = getattr(t, "kvf", None)
    if f is not None:
        return int(f)
    return KVF_FP8 if t.dtype == torch.float8_e4m3fn else KVF_BF16


def tag(t: torch.Tensor, kvf: int) -> torch.Tensor:
    t.kvf = kvf
    return t


def _f16(x):
    return np.asarray(x, np.float32).astype(np.float16)


def quantize_rows(x: torch.Tensor | np.ndarray, kvf: int) -> np.ndarray:
    """fp32 rows [n, D] -> uint8 rows [n, row_bytes] (llama.cpp quantize_row_*_ref; iq4_nl as ggml-cuda's KV copy)."""
    x = np.asarray(x.float().cpu() if isinstance(x, torch.Tensor) else x, np.float32)
    n, D = x.shape
    cb, hbb, sb, q8, hb, mn = _geom(kvf, D)
    b = x.reshape(n, D // 32, 32)
    amax_i = np.abs(b).argmax(-1)
    vmax = np.take_along_axis(b, amax_i[..., None], -1)[..., 0]
    amax = np.abs(vmax)
    m = np.zeros_like(amax)
    with np.errstate(divide="ignore", invalid="ignore"):
        if kvf == KVF_Q8_0:
            d = amax / 127.0
            idv = np.where(d != 0, 1.0 / d, 0.0).astype(np.float32)
            q = np.rint(b * idv[..., None]).astype(np.int32)  # roundf: half away from zero vs rint half-even
            r = b * idv[..., None]
            q = np.where(np.abs(r - np.trunc(r)) == 0.5, np.trunc(r) + np.sign(r), q).astype(np.int32)
        elif kvf in (KVF_Q4_0, KVF_Q5_0):
            neg, off, qmax = (-8.0, 8.5, 15) if kvf == KVF_Q4_0 else (-16.0, 16.5, 31)
            d = vmax / neg
            idv = np.where(d != 0, 1.0 / d, 0.0).astype(np.float32)
            q = np.minimum(qmax, np.trunc((b * idv[..., None] + off).astype(np.float32)).astype(np.int32))
        elif kvf in (KVF_Q4_1, KVF_Q5_1):
            qmax = 15 if kvf == KVF_Q4_1 else 31
            lo, hi = b.min(-1), b.max(-1)
            d = (hi - lo) / qmax
            m = lo
            idv = np.where(d != 0, 1.0 / d, 0.0).astype(np.float32)
            q = np.minimum(qmax, np.trunc(((b - lo[..., None]) * idv[..., None] + 0.5).astype(np.float32)).astype(np.int32))
        else:  # iq4_nl
            d = vmax / IQ4NL[0]
            idv = np.where(d != 0, 1.0 / d, 0.0).astype(np.float32)
            s = b * idv[..., None]
            # nearest codebook entry; a tie goes to the upper entry (ggml best_index_int8)
            q = (15 - np.abs(s[..., None] - IQ4NL)[..., ::-1].argmin(-1)).astype(np.int32)
            v = IQ4NL[q]
            w = b * b
            sqx, sq2 = (w * v * b).sum(-1), (w * v * v).sum(-1)
            d = np.where(sq2 > 0, sqx / np.where(sq2 > 0, sq2, 1), d)
    out = np.zeros((n, cb + hbb + sb), np.uint8)
    if q8:
        out[:, :cb] = (q.reshape(n, D) & 0xFF).astype(np.uint8)
    else:
        qq = q.reshape(n, D)
        out[:, :cb] = ((qq[:, 0::2] & 0xF) | ((qq[:, 1::2] & 0xF) << 4)).astype(np.uint8)
    if hb:
        bits = ((q.reshape(n, D) >> 4) & 1).astype(np.uint8).reshape(n, D // 8, 8)
        out[:, cb:cb + hbb] = (bits << np.arange(8, dtype=np.uint8)).sum(-1).astype(np.uint8)
    if mn:
        sc = np.stack([_f16(d), _f16(m)], -1).reshape(n, -1)
    else:
        sc = _f16(d).reshape(n, -1)
    out[:, cb + hbb:] = sc.view(np.uint8).reshape(n, sb)
    return out


def dequantize_rows(u: torch.Tensor | np.ndarray, kvf: int, D: int) -> np.ndarray:
    """uint8 rows [n, row_bytes] -> fp32 [n, D]."""
    u = np.asarray(u.cpu() if isinstance(u, torch.Tensor) else u, np.uint8)
    n = u.shape[0]
    cb, hbb, sb, q8, hb, mn = _geom(kvf, D)
    sc = np.ascontiguousarray(u[:, cb + hbb:]).view(np.float16).astype(np.float32)
    if mn:
        d, m = sc[:, 0::2], sc[:, 1::2]
    else:
        d, m = sc, np.zeros_like(sc)
    if q8:
        q = u[:, :cb].view(np.int8).astype(np.float32)
    else:
        c = u[:, :cb]
        q = np.empty((n, D), np.int32)
        q[:, 0::2] = c & 0xF
        q[:, 1::2] = c >> 4
        if hb:
            bits = (u[:, cb:cb + hbb][..., None] >> np.arange(8, dtype=np.uint8)) & 1
            q |= bits.reshape(n, D).astype(np.int32) << 4
        q = q.astype(np.float32)
    q = q.reshape(n, D // 32, 32)
    if kvf == KVF_Q4_0:
        q = q - 8
    elif kvf == KVF_Q5_0:
        q = q - 16
    elif kvf == KVF_IQ4_NL:
        q = IQ4NL[q.astype(np.int32)]
    return (q * d[..., None] + m[..., None]).reshape(n, D).astype(np.float32)


def dequant_cache(c: torch.Tensor, kvf: int, D: int) -> torch.Tensor:
    """Quantised cache rows [..., row_bytes] -> fp32 [..., D] (CPU reference path)."""
    sh = c.shape
    return torch.from_numpy(dequantize_rows(c.reshape(-1, sh[-1]), kvf, D)).view(*sh[:-1], D)
