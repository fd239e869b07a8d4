"""LoRA adapters for the LLM worker, merged into the GGUF weights as they are loaded.

Reference: the llama-cpp backend passes `LoraAdapter` (relative to the model directory) with
`LoraScale` (default 1.0) into llama.cpp's `params.lora_adapters` (backend/cpp/llama/grpc-server.cpp:
2402-2410); llama.cpp reads llama.cpp-format adapter GGUFs (`general.type = adapter`,
`adapter.lora.alpha`, tensors `<base name>.lora_a` [r, K] / `.lora_b` [N, r]) and scales each
adapter by `scale * alpha / r`.

Two modes (model option `lora_requant`): `runtime` (default, models/lora_runtime.py) keeps the adapters beside
the untouched base weights as llama.cpp does; the merge modes fold every adapter into the base weight once at
load — `W' = W + sum_i scale_i * alpha_i / r_i * B_i @ A_i` — and re-quantise (no extra launches per token).
Merge `requant="q8_0"`: merged K-quant tensors are stored as Q8_0 (a second 4-bit rounding would
cost more accuracy than the adapter adds; Q8_0 stays on the native MFMA GEMM / GEMV kernels and only
the adapted tensors grow). `requant="same"` keeps the base block format (Q4_K / Q6_K / Q8_0 — same
bytes and kernels as without LoRA, like llama.cpp's `export-lora`). F32/F16/BF16 and formats without
a quantiser merge into F32 (loaded as dense bf16 on the GPU). Tensor parallelism shards after the merge, so TP ranks see merged shards.

Also read: HF PEFT `adapter_model.safetensors` (+ `adapter_config.json` for `lora_alpha`), names
`base_model.model.model.layers.N.self_attn.q_proj.lora_A.weight` mapped to GGUF names; q/k rows
get the same rotary-half permutation llama.cpp's converter applies to Llama-family q/k weights.
"""
from __future__ import annotations

import json
import logging
import os
import re

import numpy as np

from ..formats.gguf import GGUFReader, QType
from ..ops import quant as Q

log = logging.getLogger("localai_tfp_amd.models.lora")

_HF = {"self_attn.q_proj": "attn_q", "self_attn.k_proj": "attn_k", "self_attn.v_proj": "attn_v",
       "self_attn.o_proj": "attn_output", "mlp.gate_proj": "ffn_gate", "mlp.up_proj": "ffn_up",
       "mlp.down_proj": "ffn_down"}
_PERMUTE_ARCHS = {"llama", "mistral", "granite", "deci", "smollm", "codellama", "minicpm"}
_REQUANT = {QType.Q4_K: Q.quantize_q4_k, QType.Q6_K: Q.quantize_q6_k, QType.Q8_0: Q.quantize_q8_0}


class Adapter:
    """name -> (A [r, K] fp32, B [N, r] fp32) plus the effective multiplier scale*alpha/r."""

    def __init__(self, pairs: dict[str, tuple[np.ndarray, np.ndarray]], alpha: float, scale: float, path: str):
        self.pairs, self.alpha, self.scale, self.path = pairs, alpha, scale, path

    def mult(self, r: int) -> float:
        return self.scale * (self.alpha / r if self.alpha else 1.0)


def load_adapter(path: str, scale: float = 1.0, cfg=None) -> Adapter:
    if os.path.isdir(path):
        for fn in ("adapter_model.safetensors",):
            if os.path.isfile(os.path.join(path, fn)):
                path = os.path.join(path, fn)
                break
        else:
            raise ValueError(f"{path}: no adapter_model.safetensors in directory")
    if path.endswith(".safetensors"):
        return _load_peft(path, scale, cfg)
    r = GGUFReader(path)
    if str(r.metadata.get("general.type", "adapter")) != "adapter" or \
            str(r.metadata.get("adapter.type", "lora")) != "lora":
        raise ValueError(f"{path}: not a LoRA adapter GGUF")
    pairs = {}
    for n, ti in r.tensors.items():
        if n.endswith(".lora_a"):
            base = n[:-7]
            tb = r.tensors.get(base + ".lora_b")
            if tb is None:
                raise ValueError(f"{path}: {n} without lora_b")
            a = Q.dequantize(r.tensor_bytes(n), ti.qtype, ti.shape)
            b = Q.dequantize(r.tensor_bytes(base + ".lora_b"), tb.qtype, tb.shape)
            pairs[base] = (a.reshape(a.shape[-2], -1), b.reshape(b.shape[-2], -1))
    return Adapter(pairs, float(r.metadata.get("adapter.lora.alpha", 0.0)), scale, path)


def _permute_rows(w: np.ndarray, n_head: int) -> np.ndarray:
    """HF rotary-half row order -> GGUF interleaved-pair order (llama.cpp convert permute)."""
    return w.reshape(n_head, 2, w.shape[0] // n_head // 2, *w.shape[1:]).swapaxes(1, 2).reshape(w.shape)


def _load_peft(path: str, scale: float, cfg) -> Adapter:
    from safetensors.numpy import load_file
    sd = load_file(path)
    alpha = 0.0
    cj = os.path.join(os.path.dirname(path), "adapter_config.json")
    if os.path.isfile(cj):
        with open(cj) as f:
            alpha = float(json.load(f).get("lora_alpha", 0.0))
    pairs = {}
    rx = re.compile(r"(?:.*\.)?layers\.(\d+)\.(self_attn\.[qkvo]_proj|mlp\.(?:gate|up|down)_proj)\.lora_A(?:\.default)?\.weight$")
    permute = cfg is not None and getattr(cfg, "arch", "llama") in _PERMUTE_ARCHS
    for k, a in sd.items():
        m = rx.match(k)
        if not m:
            if k.endswith("lora_A.weight") or k.endswith("lora_A.default.weight"):
                log.warning("LoRA: unmapped PEFT tensor %s", k)
            continue
        b = sd[k.replace("lora_A", "lora_B")]
        name = f"blk.{m.group(1)}.{_HF[m.group(2)]}.weight"
        b = b.astype(np.float32)
        if permute and m.group(2) in ("self_attn.q_proj", "self_attn.k_proj"):
            nh = cfg.n_heads if m.group(2) == "self_attn.q_proj" else cfg.n_kv_heads
            b = _permute_rows(b, nh)
        pairs[name] = (a.astype(np.float32), b)
    return Adapter(pairs, alpha, scale, path)


def merged_tensor(raw, qtype: int, shape, deltas: list[np.ndarray], requant: str = "q8_0"):
    """Base ggml tensor + dense deltas [N, K] -> (raw bytes, qtype, ggml shape) of the merged weight."""
    K_, N_ = int(shape[0]), int(np.prod(shape[1:]))
    w = Q.dequantize(raw, qtype, shape).reshape(N_, K_).astype(np.float32)
    for d in deltas:
        w += d
    qt = QType(qtype)
    # requant "q8_0" (default): every block-quantised base (Q4_K, Q5_K, Q4_0, IQ*, ...) comes back as
    # Q8_0 when K allows it, never as 4-byte F32; "same": keep the base type where it can be re-encoded
    dense = qt in (QType.F32, QType.F16, QType.BF16)
    if requant == "f32":  # exact merge, dense fp32 (the runtime path's numerics oracle)
        return np.ascontiguousarray(w).view(np.uint8).reshape(N_, -1), int(QType.F32), shape
    if requant != "same" and not dense and K_ % 32 == 0:
        qt = QType.Q8_0
    if qt in _REQUANT and K_ % (32 if qt == QType.Q8_0 else 256) == 0:
        return _REQUANT[qt](w).reshape(N_, -1), int(qt), shape
    return np.ascontiguousarray(w).view(np.uint8).reshape(N_, -1), int(QType.F32), shape


def with_adapters(get_tensor, adapters: list[Adapter], requant: str = "q8_0"):
    """Wrap a `get_tensor(name) -> (raw, qtype, shape)` source so LoRA'd tensors come back merged."""
    targets: dict[str, list[tuple[np.ndarray, np.ndarray, float]]] = {}
    for ad in adapters:
        for name, (a, b) in ad.pairs.items():
            targets.setdefault(name, []).append((a, b, ad.mult(a.shape[0])))
    missing = [n for n in targets if get_tensor(n) is None]
    if missing:
        raise ValueError(f"LoRA targets not in the base model: {missing[:4]}")
    # only the most recent merges are kept: the model loader asks for a tensor at most twice in a row
    # (an existence check, then the load), so holding every merged tensor would multiply peak host RAM
    cache: dict = {}

    def get(name):
        t = get_tensor(name)
        if t is None or name not in targets:
            return t
        if name not in cache:
            while len(cache) >= 2:
                cache.pop(next(iter(cache)))
            raw, qt, shape = t
            K_, N_ = int(shape[0]), int(np.prod(shape[1:]))
            deltas = []
            for a, b, s in targets[name]:
                if a.shape[1] != K_ or b.shape[0] != N_:
                    raise ValueError(f"LoRA {name}: A {a.shape} / B {b.shape} vs weight [{N_}, {K_}]")
                deltas.append(s * (b @ a))
            cache[name] = merged_tensor(raw, qt, shape, deltas, requant)
        return cache[name]
    get.lora_targets = len(targets)
    return get
