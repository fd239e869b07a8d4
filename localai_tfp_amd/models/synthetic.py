"""Synthetic random-init checkpoints of real architectures (no network to fetch weights).

``llama_tensor_plan`` reproduces llama.cpp's Q4_K_M type recipe (llama_tensor_get_type): Q4_K
everywhere, Q6_K for output.weight and for attn_v / ffn_down on the "more bits" layers
(i < n/8, i >= 7n/8, or (i - n/8) % 3 == 2), F32 norms. ``synthetic_source`` returns a
``get_tensor`` callable producing random blocks in the quantised domain (valid fp16 scales,
uniform codes, element std ~0.02) — same bytes-per-weight and kernels as a real Q4_K_M file.
``write_synthetic_gguf`` streams such a model (plus a tokenizer) to disk for the end-to-end tests.
"""
from __future__ import annotations

import numpy as np

from ..formats.gguf import GGUFWriter, QType, tensor_nbytes
from ..ops.quant import random_quantized
from .config import LlamaConfig


def _more_bits(i: int, n: int) -> bool:
    return i < n // 8 or i >= 7 * n // 8 or (i - n // 8) % 3 == 2


def llama_tensor_plan(cfg: LlamaConfig, ftype: str = "Q4_K_M"):
    """[(name, ggml_shape, qtype)] for a Llama-architecture GGUF."""
    H, F, V = cfg.hidden, cfg.ffn, cfg.vocab
    qd, kvd = cfg.q_dim, cfg.kv_dim
    base = {"Q4_K_M": QType.Q4_K, "Q3_K_M": QType.Q3_K, "Q6_K": QType.Q6_K, "Q8_0": QType.Q8_0,
            "F16": QType.F16}[ftype]
    hi = QType.Q6_K if ftype == "Q4_K_M" else base
    # Q3_K_M (llama.cpp's mix, approximately): attn_v / ffn_down in Q5_K on the "more bits" layers and Q4_K
    # elsewhere, attn_output Q4_K, output Q6_K, the rest Q3_K
    mid = QType.Q4_K if ftype == "Q3_K_M" else None
    if ftype == "Q3_K_M":
        hi = QType.Q5_K
    out = [("token_embd.weight", (H, V), base)]
    L = cfg.n_layers
    for i in range(L):
        p = f"blk.{i}."
        mb = _more_bits(i, L)
        out += [
            (p + "attn_norm.weight", (H,), QType.F32),
            (p + "attn_q.weight", (H, qd), base),
            (p + "attn_k.weight", (H, kvd), base),
            (p + "attn_v.weight", (H, kvd), hi if mb else (mid or base)),
            (p + "attn_output.weight", (qd, H), mid or base),
            (p + "ffn_norm.weight", (H,), QType.F32),
        ]
        if cfg.n_expert:
            E, Fe = cfg.n_expert, cfg.expert_ffn
            out += [
                (p + "ffn_gate_inp.weight", (H, E), QType.F32),
                (p + "ffn_gate_exps.weight", (H, Fe, E), base),
                (p + "ffn_up_exps.weight", (H, Fe, E), base),
                (p + "ffn_down_exps.weight", (Fe, H, E), hi if mb else base),
            ]
            if cfg.expert_shared_ffn:
                Fs = cfg.expert_shared_ffn
                out += [(p + "ffn_gate_inp_shexp.weight", (H,), QType.F32),
                        (p + "ffn_gate_shexp.weight", (H, Fs), base), (p + "ffn_up_shexp.weight", (H, Fs), base),
                        (p + "ffn_down_shexp.weight", (Fs, H), hi if mb else base)]
        else:
            out += [
                (p + "ffn_gate.weight", (H, F), base),
                (p + "ffn_up.weight", (H, F), base),
                (p + "ffn_down.weight", (F, H), hi if mb else (mid or base)),
            ]
        if cfg.post_norms:
            out += [(p + "post_attention_norm.weight", (H,), QType.F32),
                    (p + "post_ffw_norm.weight", (H,), QType.F32)]
        if cfg.qk_norm:
            out += [(p + "attn_q_norm.weight", (cfg.head_dim,), QType.F32),
                    (p + "attn_k_norm.weight", (cfg.head_dim,), QType.F32)]
        if cfg.qkv_bias:
            out += [(p + "attn_q.bias", (qd,), QType.F32), (p + "attn_k.bias", (kvd,), QType.F32),
                    (p + "attn_v.bias", (kvd,), QType.F32)]
    out.append(("output_norm.weight", (H,), QType.F32))
    if not cfg.tie_embeddings:
        out.append(("output.weight", (H, V), QType.Q6_K if ftype in ("Q4_K_M", "Q3_K_M") else base))
    return out


def _gen(rng, name, shape, qt, cfg):
    n = int(np.prod(shape))
    if qt == QType.F32:
        return _gen_f32(rng, name, n).view(np.uint8)
    std = 0.02
    if name.startswith("token_embd"):
        std = 1.0 / np.sqrt(cfg.hidden) * 4
    return random_quantized(rng, qt, n // shape[0], shape[0], std=std)


def _gen_f32(rng, name, n):
    if name.endswith("norm.weight"):
        return (1.0 + 0.05 * rng.standard_normal(n, dtype=np.float32)).astype(np.float32)
    if "gate_inp" in name:  # router: logits with a spread large enough to make top-k choices distinct
        return (0.5 * rng.standard_normal(n, dtype=np.float32)).astype(np.float32)
    return (0.02 * rng.standard_normal(n, dtype=np.float32)).astype(np.float32)


def synthetic_source(cfg: LlamaConfig, ftype: str = "Q4_K_M", seed: int = 0, shard_gen: bool = False):
    """get_tensor(name) -> (raw, qtype, ggml_shape). shard_gen=True also exposes
    get_tensor.shard(name, split, rank, size) -> (raw, qtype, N, K), which generates ONLY that rank's
    tensor-parallel slice (same shapes and block formats, independent random values): a 70B model on 8
    ranks then costs each rank 1/8 of the generation time and host memory. Slices are not slices of
    get_tensor(name) — TP-vs-TP=1 parity checks use the plain source."""
    plan = {n: (s, q) for n, s, q in llama_tensor_plan(cfg, ftype)}
    order = {n: i for i, n in enumerate(plan)}

    def get_tensor(name):
        if name not in plan:
            return None
        shape, qt = plan[name]
        rng = np.random.default_rng(seed * 100003 + order[name])
        return _gen(rng, name, shape, qt, cfg), int(qt), shape

    def shard(name, split, rank, size):
        shape, qt = plan[name]
        K, N = int(shape[0]), int(np.prod(shape[1:]))
        kind = split[0]
        if kind == "col_heads":
            n_heads, hd = split[1], split[2]
            N = (n_heads // size if n_heads >= size else 1) * hd
        elif kind == "col":
            N //= size
        elif kind == "row":
            K //= size
        rng = np.random.default_rng((seed * 100003 + order[name]) * 64 + rank + 1)
        raw = _gen(rng, name, [K, N], qt, cfg)
        return np.asarray(raw).view(np.uint8).reshape(N, -1), int(qt), N, K

    get_tensor.plan = plan
    if shard_gen:
        get_tensor.shard = shard
    return get_tensor


def gguf_metadata(cfg: LlamaConfig, ftype: str = "Q4_K_M") -> dict:
    a = cfg.arch
    md = {
        "general.architecture": a,
        "general.name": cfg.name,
        "general.file_type": {"Q4_K_M": 15, "Q6_K": 18, "Q8_0": 7, "F16": 1}[ftype],
        f"{a}.block_count": cfg.n_layers,
        f"{a}.context_length": cfg.ctx_train,
        f"{a}.embedding_length": cfg.hidden,
        f"{a}.feed_forward_length": cfg.ffn,
        f"{a}.attention.head_count": cfg.n_heads,
        f"{a}.attention.head_count_kv": cfg.n_kv_heads,
        f"{a}.attention.layer_norm_rms_epsilon": float(cfg.rms_eps),
        f"{a}.rope.freq_base": float(cfg.rope_base),
        f"{a}.rope.dimension_count": cfg.rope_dim,
        f"{a}.vocab_size": cfg.vocab,
    }
    if cfg.n_expert:
        md[f"{a}.expert_count"] = cfg.n_expert
        md[f"{a}.expert_used_count"] = cfg.n_expert_used
        md[f"{a}.expert_feed_forward_length"] = cfg.expert_ffn
        if cfg.expert_shared_ffn:
            md[f"{a}.expert_shared_feed_forward_length"] = cfg.expert_shared_ffn
    if cfg.arch == "gemma2":
        md[f"{a}.attn_logit_softcapping"] = float(cfg.attn_softcap)
        md[f"{a}.final_logit_softcapping"] = float(cfg.final_softcap)
        md[f"{a}.attention.sliding_window"] = cfg.sliding_window
    if cfg.arch == "gemma3":
        md[f"{a}.attention.sliding_window"] = cfg.sliding_window
        md[f"{a}.attention.sliding_window_pattern"] = cfg.swa_pattern
        if cfg.rope_scale != 1.0:
            md[f"{a}.rope.scaling.type"] = cfg.rope_scaling
            md[f"{a}.rope.scaling.factor"] = float(1.0 / cfg.rope_scale)
    if cfg.head_dim * cfg.n_heads != cfg.hidden:
        md[f"{a}.attention.key_length"] = cfg.head_dim
        md[f"{a}.attention.value_length"] = cfg.head_dim
    return md


def write_synthetic_gguf(path, cfg: LlamaConfig, ftype: str = "Q4_K_M", seed: int = 0, tokenizer_md: dict | None = None):
    src = synthetic_source(cfg, ftype, seed)
    w = GGUFWriter(path)
    for k, v in gguf_metadata(cfg, ftype).items():
        w.add(k, v)
    for k, v in (tokenizer_md or {}).items():
        w.add(k, v)
    for name, (shape, qt) in src.plan.items():
        w.add_tensor(name, (lambda n=name: src(n)[0].tobytes()), shape=shape, qtype=qt)
    return w.write()
