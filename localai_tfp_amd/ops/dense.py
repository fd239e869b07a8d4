"""Dense 16-bit layers for the non-LLM model families (BERT, Whisper, CLIP/T5 text encoders, UNet /
MMDiT, VAE, TTS): plain library GEMMs on hipBLASLt with the bias folded into the
GEMM, fp32 accumulation into the residual stream, and the library's act16 activations.

On CPU everything runs in fp32 (the numerics oracle for the tests)."""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F

from .linear import ACT_DTYPE, _fp32_out_ok


def model_dtype(device) -> torch.dtype:
    return ACT_DTYPE if torch.device(device).type == "cuda" else torch.float32


def to_dev(a, device, dtype) -> torch.Tensor:
    if isinstance(a, torch.Tensor):
        return a.to(device=device, dtype=dtype).contiguous()
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32)).to(device).to(dtype).contiguous()


class Dense:
    """y = x W^T + b with W [N, K] in the model dtype; bias kept in both dtypes."""

    __slots__ = ("w", "b", "b32", "wt")

    def __init__(self, w, b=None, device="cpu", dtype=torch.float32):
        self.w = to_dev(w, device, dtype)
        self.wt = self.w.t()
        self.b = to_dev(b, device, dtype) if b is not None else None
        self.b32 = to_dev(b, device, torch.float32) if b is not None else None

    @property
    def n(self) -> int:
        return self.w.shape[0]

    def __call__(self, x: torch.Tensor, act: str | None = None) -> torch.Tensor:
        y = torch.addmm(self.b, x, self.wt) if self.b is not None else x @ self.wt
        if act == "gelu":
            y = F.gelu(y)
        elif act == "silu":
            y = F.silu(y)
        elif act == "gelu_tanh":
            y = F.gelu(y, approximate="tanh")
        return y

    def f32(self, x: torch.Tensor) -> torch.Tensor:
        """fp32 output (hipBLASLt 16-bit x 16-bit -> fp32 where the build supports it)."""
        if x.dtype == torch.float32:
            return self(x)
        out = torch.empty(x.shape[0], self.n, dtype=torch.float32, device=x.device)
        if _fp32_out_ok(x.dtype):
            if self.b32 is not None:
                out.copy_(self.b32.expand_as(out))
                torch.addmm(out, x, self.wt, out_dtype=torch.float32, out=out)
            else:
                torch.mm(x, self.wt, out_dtype=torch.float32, out=out)
            return out
        out.copy_(self(x))
        return out

    def acc(self, x: torch.Tensor, acc: torch.Tensor) -> torch.Tensor:
        """acc (fp32) += x W^T + b — the residual add fused as GEMM beta = 1."""
        if x.dtype != torch.float32 and _fp32_out_ok(x.dtype) and acc.is_contiguous():
            if self.b32 is not None:
                acc.add_(self.b32)
            torch.addmm(acc, x, self.wt, out_dtype=torch.float32, out=acc)
            return acc
        acc.add_(self(x).float())
        return acc


def layernorm(x: torch.Tensor, w, b, eps: float, out_dtype) -> torch.Tensor:
    """fp32 [M, H] -> layer-normed in out_dtype (norm.hip on GPU)."""
    from . import core as K
    out = torch.empty(x.shape, dtype=out_dtype, device=x.device)
    K.layernorm(x, w, b, eps, out)
    return out
