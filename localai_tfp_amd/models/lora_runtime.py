"""Runtime LoRA for the Llama-family engine: adapters stay separate from the (quantised) base weights.

Reference: llama.cpp keeps each `params.lora_adapters` entry as its own tensors and adds `scale * alpha / r *
B (A x)` beside every adapted matmul at inference (backend/cpp/llama/grpc-server.cpp:2402-2410) — the base GGUF
bytes are never rewritten. The merge path (models/lora.py `with_adapters`) folds adapters into the weights at
load, which re-quantises every adapted tensor (Q8_0 by default: ~2x the bytes per decode token, or a second
4-bit rounding with requant="same"). This module is the reference's behaviour: `lora_requant: runtime`.

MI355X form: per adapted projection the adapters of the same input are concatenated along the rank, so one
skinny [M, K] x [K, R] GEMM (hipBLASLt, 16-bit operands, fp32 accumulation) produces every adapter's
low-rank activations, and one [M, R] x [R, N] GEMM per projection part adds the scaled update into the
projection's output (the q|k|v columns, the interleaved gate|up rows before the gated activation, or the fp32
residual stream for o_proj / down). Scales are folded into B at load. All launches are plain stream work, so
the decode step still captures into one hipGraph.
"""
from __future__ import annotations

import logging

import numpy as np
import torch

log = logging.getLogger("localai_tfp_amd.models.lora")

# GGUF tensor names of the per-layer projections an adapter may target
PROJ = ("attn_q", "attn_k", "attn_v", "attn_output", "ffn_gate", "ffn_up", "ffn_down")


class LoraProj:
    """Low-rank update of one input: A_cat [R, K] (all adapters' A stacked), and per output part (name, column
    offset in the projection's output, B_scaled [n, R] zero-padded outside the part's adapters' rank slices)."""

    def __init__(self, A: torch.Tensor, parts: list[tuple[str, int, torch.Tensor]]):
        self.A = A
        self.parts = parts

    def low_rank(self, x: torch.Tensor) -> torch.Tensor:
        """x [M, K] (16-bit or fp32) -> t [M, R]."""
        return torch.matmul(x.to(self.A.dtype), self.A.t())


class LayerLora:
    """Runtime LoRA of one decoder layer: qkv (input: the attention-normed rows), o (input: attention output),
    gate_up (input: the FFN-normed rows), down (input: the gated activation)."""

    def __init__(self):
        self.qkv: LoraProj | None = None
        self.o: LoraProj | None = None
        self.gate_up: LoraProj | None = None
        self.down: LoraProj | None = None

    @property
    def any(self) -> bool:
        return any(p is not None for p in (self.qkv, self.o, self.gate_up, self.down))


def _proj(pairs: list[tuple[str, int, np.ndarray, np.ndarray, float]], dtype, device) -> LoraProj:
    """pairs: (part name, column offset, A [r, K], B [n, r], mult) -> one LoraProj with the ranks stacked."""
    R = sum(a.shape[0] for _, _, a, _, _ in pairs)
    K = pairs[0][2].shape[1]
    A = np.zeros((R, K), np.float32)
    parts: dict[tuple[str, int, int], np.ndarray] = {}
    r0 = 0
    for name, off, a, b, s in pairs:
        r = a.shape[0]
        A[r0:r0 + r] = a
        key = (name, off, b.shape[0])
        Bp = parts.setdefault(key, np.zeros((b.shape[0], R), np.float32))
        Bp[:, r0:r0 + r] += s * b
        r0 += r
    At = torch.from_numpy(A).to(device, dtype)
    out = [(name, off, torch.from_numpy(B).to(device, dtype)) for (name, off, _), B in parts.items()]
    return LoraProj(At, out)


def build(model, adapters, l0: int = 0) -> int:
    """Attach runtime LoRA to a loaded LlamaModel (single rank; a pipeline stage holds blocks l0..l0+len(layers)).
    Returns the number of adapted projections on this model."""
    cfg = model.cfg
    dev = model.device
    dtype = torch.float32 if dev.type == "cpu" else torch.float16
    qd, kvd = model.n_heads * cfg.head_dim, model.n_kv * cfg.head_dim
    F = cfg.ffn
    offs = {"attn_q": ("qkv", 0), "attn_k": ("qkv", qd), "attn_v": ("qkv", qd + kvd), "attn_output": ("o", 0),
            "ffn_gate": ("gate_up", 0), "ffn_up": ("gate_up", F), "ffn_down": ("down", 0)}
    per_layer: dict[int, dict[str, list]] = {}
    n = 0
    for ad in adapters:
        for name, (a, b) in ad.pairs.items():
            parts = name.split(".")
            if len(parts) != 4 or parts[0] != "blk" or parts[2] not in PROJ or parts[3] != "weight":
                raise ValueError(f"LoRA target {name!r}: not a decoder-layer projection")
            li, proj = int(parts[1]), parts[2]
            if li >= cfg.n_layers:
                raise ValueError(f"LoRA target {name!r}: the model has {cfg.n_layers} layers")
            if not l0 <= li < l0 + len(model.layers):
                continue  # another pipeline stage's block
            grp, off = offs[proj]
            per_layer.setdefault(li - l0, {}).setdefault(grp, []).append((proj, off, np.asarray(a, np.float32),
                                                                     np.asarray(b, np.float32), ad.mult(a.shape[0])))
            n += 1
    for li, groups in per_layer.items():
        ll = LayerLora()
        for grp, pairs in groups.items():
            setattr(ll, grp, _proj(pairs, dtype, dev))
        model.layers[li].lora = ll
    return n


def add_qkv(lp: LoraProj, x: torch.Tensor, qkv: torch.Tensor):
    """qkv fp32 [M, qd + 2 kvd] += the q / k / v updates of the normed rows x."""
    t = lp.low_rank(x)
    for _, off, B in lp.parts:
        qkv[:, off:off + B.shape[0]] += torch.matmul(t, B.t()).float()


def add_residual(lp: LoraProj, x: torch.Tensor, h: torch.Tensor):
    """fp32 residual rows h += the o_proj / down update of x."""
    t = lp.low_rank(x)
    for _, off, B in lp.parts:
        h[:, off:off + B.shape[0]] += torch.matmul(t, B.t()).float()


def add_gate_up(lp: LoraProj, x: torch.Tensor, y: torch.Tensor, F: int):
    """Pre-activation gate|up rows y [M, 2F] in the fused layout (gate / up interleaved in 16-column groups,
    ops/linear.py interleave_gate_up) += the gate (columns 0..F) / up (F..2F) updates of x."""
    t = lp.low_rank(x)
    M = y.shape[0]
    yv = y.view(M, F // 16, 2, 16)
    for name, off, B in lp.parts:
        d = torch.matmul(t, B.t()).to(y.dtype).view(M, F // 16, 16)
        yv[:, :, 0 if off == 0 else 1, :] += d


def add_parts(lp: LoraProj, x: torch.Tensor, outs: dict):
    """Separate gate / up outputs (16-bit [M, F] each) += their updates (outs: part name -> tensor)."""
    t = lp.low_rank(x)
    for name, _, B in lp.parts:
        o = outs[name]
        o += torch.matmul(t, B.t()).to(o.dtype)
