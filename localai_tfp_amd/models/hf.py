"""Hugging Face safetensors LLM checkpoints for the `vllm` / `transformers` backends.

Reference: backend/python/vllm/backend.py:81-141 (``LLM(model=...)`` on an HF repo directory),
backend/python/transformers/backend.py:68-284 (``AutoModelForCausalLM.from_pretrained``). Here an HF
model directory (``config.json`` + ``*.safetensors`` [+ ``model.safetensors.index.json``] +
``tokenizer.json``) is mapped onto the same :class:`~.llama.LlamaModel` graph the GGUF path uses:

* ``config.json`` -> :class:`~.config.LlamaConfig` (Llama / Mistral / Mixtral, Qwen2 / Qwen3 and their
  MoE variants, Gemma 1/2/3 text, Phi-3), including the rope_scaling variants (linear, YaRN, llama3);
* HF tensor names -> the GGUF names the model loader consumes, with the conversions llama.cpp's
  convert_hf_to_gguf applies: Q/K rows permuted to adjacent-pair rotary order for NORM-rope
  architectures, Gemma RMSNorm weights stored as (1 + w), per-expert tensors stacked;
* weights stay bf16 by default (the precision the reference's vLLM / transformers backends serve;
  hipBLASLt GEMMs), or are quantised at load into a GPU-native block format with the ``quant`` option
  (q8_0 — 8.5 bits, within the dequant error of the bf16 checkpoint — q4_k / q6_k), so the qmm / qmv
  kernels stream them like any GGUF model; ``f16`` / ``f32`` keep other dense copies;
* GPTQ (AutoGPTQ / optimum ``quant_method: gptq``, 2/4/8-bit, ``g_idx`` act-order, v1 zero-point
  convention or ``checkpoint_format: gptq_v2``) and AWQ (``quant_method: awq``, GEMM packing, 4-bit)
  checkpoints — what vLLM's ``quantization: gptq / awq`` and exllama2 load
  (backend/python/vllm/backend.py:106-107) — are dequantised at load from their packed
  ``qweight / qzeros / scales [/ g_idx]`` tensors, then served like any other checkpoint (bf16 by default,
  or re-blocked with ``quant``). Parity with AutoGPTQ / AutoAWQ kernels is unpinned (not installed here);
  the formulas are pinned by tests/test_hf_gptq.py's independent packer;
* EXL2 (exllamav2, the reference's exllama2 backend: backend/python/exllama2/backend.py:49-56): per-group 2-8-bit
  codes behind a row permutation (``q_weight / q_scale / q_scale_max / q_groups / q_invperm``), dequantised the
  same way (:func:`dequant_exl2`; exllamav2 is not importable here, parity unpinned).
"""
from __future__ import annotations

import json
import logging
import os
from collections import OrderedDict

import numpy as np
import torch

from ..formats.gguf import QType
from .config import NEOX_ARCHS, LlamaConfig

log = logging.getLogger("localai_tfp_amd.models.hf")

HF_ARCH = {
    "LlamaForCausalLM": "llama", "MistralForCausalLM": "llama", "MixtralForCausalLM": "llama",
    "Qwen2ForCausalLM": "qwen2", "Qwen3ForCausalLM": "qwen3", "Qwen2MoeForCausalLM": "qwen2moe",
    "Qwen3MoeForCausalLM": "qwen3moe", "GemmaForCausalLM": "gemma", "Gemma2ForCausalLM": "gemma2",
    "Gemma3ForCausalLM": "gemma3", "Gemma3ForConditionalGeneration": "gemma3", "Phi3ForCausalLM": "phi3",
}
QUANTS = {"q8_0": QType.Q8_0, "q4_k": QType.Q4_K, "q6_k": QType.Q6_K, "f16": QType.F16, "bf16": QType.BF16,
          "f32": QType.F32}


def is_hf_dir(path: str) -> bool:
    if not (os.path.isdir(path) and os.path.isfile(os.path.join(path, "config.json"))):
        return False
    return any(f.endswith(".safetensors") for f in os.listdir(path))


def config_from_hf(hc: dict) -> LlamaConfig:
    if "text_config" in hc and "hidden_size" not in hc:  # Gemma 3 multimodal wrapper: the text tower
        hc = {**hc["text_config"], "architectures": hc.get("architectures")}
    archs = hc.get("architectures") or []
    arch = next((HF_ARCH[a] for a in archs if a in HF_ARCH), None)
    if arch is None:
        mt = hc.get("model_type", "llama")
        arch = {"mistral": "llama", "mixtral": "llama", "qwen2_moe": "qwen2moe", "qwen3_moe": "qwen3moe",
                "gemma3_text": "gemma3"}.get(mt, mt)
    hidden = int(hc["hidden_size"])
    n_heads = int(hc["num_attention_heads"])
    head_dim = int(hc.get("head_dim") or hidden // n_heads)
    # rope: transformers <= 4.x writes rope_theta + rope_scaling, 5.x a rope_parameters dict (Gemma 3: one
    # per layer type, "full_attention" / "sliding_attention")
    rp = hc.get("rope_parameters") or {}
    rp_local = {}
    if "full_attention" in rp:
        rp_local = rp.get("sliding_attention") or {}
        rp = rp["full_attention"] or {}
    rs = hc.get("rope_scaling") or rp or {}
    rtype = str(rs.get("rope_type", rs.get("type", "none")) or "none")
    rope_theta = float(hc.get("rope_theta") or rp.get("rope_theta") or 10000.0)
    cfg = LlamaConfig(
        arch=arch, n_layers=int(hc["num_hidden_layers"]), hidden=hidden, ffn=int(hc.get("intermediate_size", 4 * hidden)),
        n_heads=n_heads, n_kv_heads=int(hc.get("num_key_value_heads") or n_heads), head_dim=head_dim,
        vocab=int(hc["vocab_size"]), ctx_train=int(hc.get("max_position_embeddings", 4096)),
        rope_base=rope_theta,
        rope_dim=int(head_dim * float(hc.get("partial_rotary_factor", 1.0))),
        rms_eps=float(hc.get("rms_norm_eps", 1e-6)), tie_embeddings=bool(hc.get("tie_word_embeddings", False)),
        qkv_bias=bool(hc.get("attention_bias", arch in ("qwen2", "qwen2moe"))),
        name=str(hc.get("_name_or_path") or arch))
    if rtype == "linear":
        cfg.rope_scaling, cfg.rope_scale = "linear", 1.0 / float(rs.get("factor", 1.0))
    elif rtype == "yarn":
        cfg.rope_scaling, cfg.rope_scale = "yarn", 1.0 / float(rs.get("factor", 1.0))
        cfg.rope_orig_ctx = int(rs.get("original_max_position_embeddings", 0) or 0)
    elif rtype == "llama3":
        cfg.rope_llama3 = {k: rs[k] for k in ("factor", "low_freq_factor", "high_freq_factor",
                                              "original_max_position_embeddings") if k in rs}
    if arch.startswith("gemma"):
        cfg.embed_scale = hidden ** 0.5
        cfg.ffn_act = "gelu"
        cfg.tie_embeddings = True
        qs = hc.get("query_pre_attn_scalar")
        if qs and arch != "gemma":
            cfg.attn_scale = float(qs) ** -0.5
    if arch == "gemma2":
        cfg.post_norms = True
        cfg.attn_softcap = float(hc.get("attn_logit_softcapping") or 0.0)
        cfg.final_softcap = float(hc.get("final_logit_softcapping") or 0.0)
        cfg.sliding_window = int(hc.get("sliding_window") or 0)
        cfg.swa_pattern = 2
    if arch == "gemma3":
        cfg.post_norms = True
        cfg.sliding_window = int(hc.get("sliding_window") or 0)
        cfg.swa_pattern = int(hc.get("sliding_window_pattern", 6) or 6)
        cfg.rope_base_local = float(hc.get("rope_local_base_freq") or rp_local.get("rope_theta") or 10000.0)
        cfg.final_softcap = float(hc.get("final_logit_softcapping") or 0.0)
    ne = int(hc.get("num_local_experts") or hc.get("num_experts") or 0)
    if ne:
        cfg.n_expert = ne
        cfg.n_expert_used = int(hc.get("num_experts_per_tok", 2))
        cfg.expert_ffn = int(hc.get("moe_intermediate_size") or cfg.ffn)
        cfg.expert_shared_ffn = int(hc.get("shared_expert_intermediate_size") or 0)
        cfg.moe_renorm = bool(hc.get("norm_topk_prob", arch != "qwen2moe"))
    cfg.qk_norm = arch in ("qwen3", "qwen3moe", "gemma3")
    return cfg


AWQ_ORDER = (0, 2, 4, 6, 1, 3, 5, 7)  # AWQ GEMM packing: nibble i of an int32 holds column 8c + AWQ_ORDER[i]


def _unpack_rows(qw: np.ndarray, bits: int) -> np.ndarray:
    """int32 [R, C] packed along rows (GPTQ qweight: 32/bits values of consecutive k per word, low bits first)
    -> uint8 [R * 32/bits, C]."""
    u = np.ascontiguousarray(qw).view(np.uint32)
    per, mask = 32 // bits, (1 << bits) - 1
    out = np.empty((u.shape[0] * per, u.shape[1]), np.uint8)
    for j in range(per):
        out[j::per] = (u >> (bits * j)) & mask
    return out


def _unpack_cols(qw: np.ndarray, bits: int, order=None) -> np.ndarray:
    """int32 [R, C] packed along columns (GPTQ qzeros, AWQ qweight / qzeros) -> uint8 [R, C * 32/bits];
    `order`: the column each bit-field holds within its group of 32/bits (AWQ)."""
    u = np.ascontiguousarray(qw).view(np.uint32)
    per, mask = 32 // bits, (1 << bits) - 1
    out = np.empty((u.shape[0], u.shape[1] * per), np.uint8)
    for i in range(per):
        out[:, (order[i] if order else i)::per] = (u >> (bits * i)) & mask
    return out


def dequant_gptq(qweight, qzeros, scales, g_idx=None, bits: int = 4, group_size: int = 128, v2: bool = False):
    """GPTQ linear -> fp32 weight [N, K] (out, in): W[k, n] = s[g(k), n] * (q[k, n] - (z[g(k), n] + 1)), the +1 being
    AutoGPTQ's v1 zero-point storage (none for gptq_v2)."""
    if bits not in (2, 4, 8):
        raise ValueError(f"GPTQ {bits}-bit weights are not supported (2 / 4 / 8)")
    N = scales.shape[1]
    q = _unpack_rows(qweight, bits).astype(np.float32)
    K = q.shape[0]
    z = _unpack_cols(qzeros, bits)[:, :N].astype(np.float32) + (0.0 if v2 else 1.0)
    g = (np.asarray(g_idx, np.int64) if g_idx is not None else np.arange(K) // (group_size if group_size > 0 else K))
    s = np.asarray(scales, np.float32)
    return np.ascontiguousarray((s[g] * (q - z[g])).T)


def dequant_awq(qweight, qzeros, scales, bits: int = 4, group_size: int = 128):
    """AWQ (GEMM packing) linear -> fp32 weight [N, K]: W[k, n] = s[k // g, n] * (q[k, n] - z[k // g, n])."""
    if bits != 4:
        raise ValueError(f"AWQ {bits}-bit weights are not supported (4-bit GEMM packing)")
    q = _unpack_cols(qweight, 4, AWQ_ORDER).astype(np.float32)
    K = q.shape[0]
    z = _unpack_cols(qzeros, 4, AWQ_ORDER).astype(np.float32)
    g = np.arange(K) // (group_size if group_size > 0 else K)
    s = np.asarray(scales, np.float32)
    return np.ascontiguousarray((s[g] * (q - z[g])).T)


EXL2_BITS = (2, 3, 4, 5, 6, 8)


def _exl2_groupsize(K: int, G: int) -> int:
    """exllamav2's group size: the smallest power of two whose G groups cover the K input rows."""
    gs = 1
    while gs * G < K:
        gs *= 2
    return gs


def dequant_exl2(q_weight, q_scale, q_scale_max, q_groups, q_invperm):
    """exllamav2 EXL2 linear -> fp32 weight [N, K] (out, in).

    Layout (exllamav2's QMatrix tensors, reference backend/python/exllama2/backend.py:49-56 loads them):
      q_groups    int16 [2 G]: per row group (bits b_g, first int32 row of its codes in q_weight); group g covers the
                  permuted input rows [g gs, (g + 1) gs), gs = _exl2_groupsize(K, G);
      q_weight    int32 [*, N]: each column's codes of a group as one little-endian bitstream of b_g-bit fields, row
                  after row (so 32 / b_g rows per word for b in {2, 4, 8}; 16 rows in 3 words at 6 bits, 32 rows in
                  3 / 5 words at 3 / 5 bits), code value c -> c - 2^(b_g - 1);
      q_scale     int32 [G, N / 8]: a 4-bit scale code s per (group, column), column n in nibble n % 8;
      q_scale_max fp16 [G]: the group's scale = ((s + 1) / 16)^2 * q_scale_max[g];
      q_invperm   int16 [K]: packed row of input feature j (the codes are stored in a permuted row order that sorts the
                  groups by bit width) — W[:, j] = W_packed[:, q_invperm[j]].
    exllamav2 is not importable here: the layout is re-stated from its format, parity with its kernels is unpinned
    (tests/test_hf_gptq.py packs EXL2 tensors independently)."""
    qw = np.ascontiguousarray(q_weight).view(np.uint32)
    N = qw.shape[1]
    qg = np.asarray(q_groups).astype(np.int64) & 0xFFFF
    G = qg.size // 2
    bits, start = qg[0::2], qg[1::2]
    inv = np.asarray(q_invperm).astype(np.int64) & 0xFFFF
    K = inv.size
    gs = _exl2_groupsize(K, G)
    sc = np.ascontiguousarray(q_scale).view(np.uint32)
    snib = np.empty((G, N), np.float32)
    for i in range(8):
        snib[:, i::8] = ((sc >> np.uint32(4 * i)) & 0xF)[:, : (N - i + 7) // 8]
    scale = ((snib + 1.0) / 16.0) ** 2 * np.asarray(q_scale_max, np.float32).reshape(G, 1)
    wp = np.empty((K, N), np.float32)  # [packed row, column]
    g = 0
    while g < G:  # runs of consecutive groups with one bit width decode as one bitstream
        b = int(bits[g])
        if b not in EXL2_BITS:
            raise ValueError(f"EXL2 group with {b}-bit codes")
        h = g
        while h + 1 < G and int(bits[h + 1]) == b and int(start[h + 1]) == int(start[g]) + (h + 1 - g) * gs * b // 32:
            h += 1
        r_run0, r_run1 = g * gs, min(K, (h + 1) * gs)
        for r0 in range(r_run0, r_run1, 1024):  # 1024-row chunks (whole words: 1024 b / 32) bound the bit arrays
            r1 = min(r_run1, r0 + 1024)
            w0 = int(start[g]) + (r0 - r_run0) * b // 32
            words = qw[w0: w0 + -(-(r1 - r0) * b // 32)]  # [words, N]
            stream = np.unpackbits(np.ascontiguousarray(words.T).view(np.uint8), axis=1, bitorder="little")
            fields = stream[:, : (r1 - r0) * b].reshape(N, r1 - r0, b)
            codes = np.zeros((N, r1 - r0), np.int32)
            for t in range(b):
                codes |= fields[..., t].astype(np.int32) << t
            codes -= 1 << (b - 1)
            wp[r0:r1] = codes.T.astype(np.float32) * scale[np.arange(r0, r1) // gs]
        g = h + 1
    return np.ascontiguousarray(wp[inv].T)


class _SafetensorsDir:
    """Lazy tensor access over one or more .safetensors shards (fp32 numpy out). With a GPTQ / AWQ
    quantization_config, `<linear>.weight` is served dequantised from `<linear>.qweight / qzeros / scales`."""

    def __init__(self, d: str, qcfg: dict | None = None):
        from safetensors import safe_open
        idx = os.path.join(d, "model.safetensors.index.json")
        if os.path.isfile(idx):
            with open(idx) as f:
                wm = json.load(f)["weight_map"]
            files = sorted(set(wm.values()))
        else:
            files = sorted(f for f in os.listdir(d) if f.endswith(".safetensors"))
            wm = None
        self._h = {f: safe_open(os.path.join(d, f), framework="pt") for f in files}
        self.where = {}
        for f, h in self._h.items():
            for k in h.keys():
                self.where[k] = f
        if wm:
            self.where.update({k: v for k, v in wm.items() if v in self._h})
        self.qcfg = qcfg or {}
        self.qmethod = str(self.qcfg.get("quant_method", "") or "").lower()
        if any(k.endswith(".q_invperm") for k in self.where):
            self.qmethod = "exl2"  # exllamav2 EXL2 (per-group mixed 2-8-bit codes behind a row permutation)
        if self.qmethod and self.qmethod not in ("gptq", "awq", "exl2"):
            raise ValueError(f"quantization_config.quant_method {self.qmethod!r} is not supported (gptq / awq / exl2)")

    def _packed(self, k):
        if not (self.qmethod and k.endswith(".weight") and k not in self.where):
            return False
        return k[: -len("weight")] + ("q_weight" if self.qmethod == "exl2" else "qweight") in self.where

    def __contains__(self, k):
        return k in self.where or bool(self._packed(k))

    def raw(self, k):
        t = self._h[self.where[k]].get_tensor(k)
        # numpy has no bfloat16: GPTQ / AWQ checkpoints that store scales in bf16 are widened first
        return (t.float() if t.is_floating_point() and t.dtype != torch.float16 else t).numpy()

    def get(self, k) -> np.ndarray:
        if self._packed(k):
            b = k[: -len("weight")]
            if self.qmethod == "exl2":
                return dequant_exl2(self.raw(b + "q_weight"), self.raw(b + "q_scale"), self.raw(b + "q_scale_max"),
                                    self.raw(b + "q_groups"), self.raw(b + "q_invperm"))
            c = self.qcfg
            bits, gs = int(c.get("bits", c.get("w_bit", 4))), int(c.get("group_size", c.get("q_group_size", 128)))
            if self.qmethod == "gptq":
                gi = self.raw(b + "g_idx") if b + "g_idx" in self.where else None
                return dequant_gptq(self.raw(b + "qweight"), self.raw(b + "qzeros"), self.raw(b + "scales"), gi, bits, gs,
                                    v2=str(c.get("checkpoint_format", "")).lower() == "gptq_v2")
            return dequant_awq(self.raw(b + "qweight"), self.raw(b + "qzeros"), self.raw(b + "scales"), bits, gs)
        return self._h[self.where[k]].get_tensor(k).float().numpy()


def _permute_qk(w: np.ndarray, n_head: int) -> np.ndarray:
    """HF half-split rotary rows -> GGUF adjacent-pair rows (llama.cpp convert_hf_to_gguf permute)."""
    return w.reshape(n_head, 2, w.shape[0] // n_head // 2, *w.shape[1:]).swapaxes(1, 2).reshape(w.shape)


def hf_source(model_dir: str, quant: str = "q8_0"):
    """-> (LlamaConfig, get_tensor) for LlamaModel.load; get_tensor(gguf_name) -> (raw, qtype, ggml_shape)."""
    from ..ops.quant import QUANTIZERS
    with open(os.path.join(model_dir, "config.json")) as f:
        hc = json.load(f)
    cfg = config_from_hf(hc)
    st = _SafetensorsDir(model_dir, hc.get("quantization_config") or (hc.get("text_config") or {}).get("quantization_config"))
    if str(quant or "").lower() in ("gptq", "awq", "gptq_marlin", "awq_marlin", "marlin", "exl2"):
        quant = "bf16"  # vLLM's quantization names: the checkpoint's own format is read from config.json
    qt = QUANTS.get(str(quant or "q8_0").lower())
    if qt is None:
        raise ValueError(f"unknown quantization {quant!r} (choose from {sorted(QUANTS)})")
    pre = "model.language_model." if any(k.startswith("model.language_model.") for k in st.where) else "model."
    if "embed_tokens.weight" in st:  # a bare base model (e.g. a diffusers text_encoder/ Gemma2Model)
        pre = ""
    gemma = cfg.arch.startswith("gemma")
    permute = cfg.arch not in NEOX_ARCHS

    def norm_src(hf):
        return lambda: st.get(hf) + (1.0 if gemma else 0.0)

    m: dict[str, tuple] = {}  # gguf name -> (kind, loader)
    m["token_embd.weight"] = ("w", lambda: st.get(pre + "embed_tokens.weight"))
    m["output_norm.weight"] = ("v", norm_src(pre + "norm.weight"))
    if "lm_head.weight" in st and not cfg.tie_embeddings:
        m["output.weight"] = ("w", lambda: st.get("lm_head.weight"))
    for i in range(cfg.n_layers):
        hp, gp = f"{pre}layers.{i}.", f"blk.{i}."
        a, mlp = hp + "self_attn.", hp + "mlp."
        m[gp + "attn_norm.weight"] = ("v", norm_src(hp + "input_layernorm.weight"))
        if cfg.post_norms:  # Gemma 2/3: post-attention norm, pre/post feed-forward norms
            m[gp + "post_attention_norm.weight"] = ("v", norm_src(hp + "post_attention_layernorm.weight"))
            m[gp + "ffn_norm.weight"] = ("v", norm_src(hp + "pre_feedforward_layernorm.weight"))
            m[gp + "post_ffw_norm.weight"] = ("v", norm_src(hp + "post_feedforward_layernorm.weight"))
        else:
            m[gp + "ffn_norm.weight"] = ("v", norm_src(hp + "post_attention_layernorm.weight"))
        if a + "qkv_proj.weight" in st:
            m[gp + "attn_qkv.weight"] = ("w", (lambda k: lambda: st.get(k))(a + "qkv_proj.weight"))
        else:
            for hn, gn, nh in (("q_proj", "attn_q", cfg.n_heads), ("k_proj", "attn_k", cfg.n_kv_heads),
                               ("v_proj", "attn_v", 0)):
                def ld(k=a + hn + ".weight", nh=nh):
                    w = st.get(k)
                    return _permute_qk(w, nh) if (permute and nh) else w
                m[gp + gn + ".weight"] = ("w", ld)
                if a + hn + ".bias" in st:
                    def ldb(k=a + hn + ".bias", nh=nh):
                        b = st.get(k)
                        return _permute_qk(b, nh) if (permute and nh) else b
                    m[gp + gn + ".bias"] = ("v", ldb)
        m[gp + "attn_output.weight"] = ("w", (lambda k: lambda: st.get(k))(a + "o_proj.weight"))
        if cfg.qk_norm:
            m[gp + "attn_q_norm.weight"] = ("v", norm_src(a + "q_norm.weight"))
            m[gp + "attn_k_norm.weight"] = ("v", norm_src(a + "k_norm.weight"))
        if cfg.n_expert:
            moe = hp + ("block_sparse_moe." if hp + "block_sparse_moe.gate.weight" in st else "mlp.")
            m[gp + "ffn_gate_inp.weight"] = ("v", (lambda k: lambda: st.get(k))(moe + "gate.weight"))
            names = (("w1", "w3", "w2") if moe.endswith("block_sparse_moe.")
                     else ("gate_proj", "up_proj", "down_proj"))
            for hn, gn in zip(names, ("ffn_gate_exps", "ffn_up_exps", "ffn_down_exps")):
                m[gp + gn + ".weight"] = ("e", (lambda pfx, hn: lambda: np.stack(
                    [st.get(f"{pfx}experts.{e}.{hn}.weight") for e in range(cfg.n_expert)]))(moe, hn))
            if cfg.expert_shared_ffn:
                for hn, gn in (("gate_proj", "ffn_gate_shexp"), ("up_proj", "ffn_up_shexp"),
                               ("down_proj", "ffn_down_shexp")):
                    m[gp + gn + ".weight"] = ("w", (lambda k: lambda: st.get(k))(f"{moe}shared_expert.{hn}.weight"))
                if moe + "shared_expert_gate.weight" in st:
                    m[gp + "ffn_gate_inp_shexp.weight"] = ("v", (lambda k: lambda: st.get(k))(moe + "shared_expert_gate.weight"))
        elif mlp + "gate_up_proj.weight" in st:  # Phi-3: fused gate|up rows
            m[gp + "ffn_up.weight"] = ("w", (lambda k: lambda: st.get(k))(mlp + "gate_up_proj.weight"))
            m[gp + "ffn_down.weight"] = ("w", (lambda k: lambda: st.get(k))(mlp + "down_proj.weight"))
        else:
            for hn, gn in (("gate_proj", "ffn_gate"), ("up_proj", "ffn_up"), ("down_proj", "ffn_down")):
                m[gp + gn + ".weight"] = ("w", (lambda k: lambda: st.get(k))(mlp + hn + ".weight"))

    cache: OrderedDict = OrderedDict()  # the model loader asks for some tensors twice (existence checks)

    def convert(name):
        kind, ld = m[name]
        x = np.ascontiguousarray(ld(), dtype=np.float32)
        if kind == "v" or x.ndim == 1:
            return x.reshape(-1), int(QType.F32), list(reversed(x.shape))
        K = x.shape[-1]
        rows = int(np.prod(x.shape[:-1]))
        shape = list(reversed(x.shape))
        q = qt
        if q in (QType.Q4_K, QType.Q6_K) and K % 256:
            q = QType.Q8_0
        if q == QType.Q8_0 and K % 32:
            q = QType.F16
        if q in QUANTIZERS:
            raw = QUANTIZERS[q](x.reshape(rows, K)).reshape(rows, -1)
            return raw, int(q), shape
        if q == QType.F16:
            return x.astype(np.float16).view(np.uint8).reshape(rows, -1), int(q), shape
        if q == QType.BF16:
            u = x.view(np.uint32)
            b = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)
            return b.view(np.uint8).reshape(rows, -1), int(q), shape
        return x.view(np.uint8).reshape(rows, -1), int(QType.F32), shape

    def get_tensor(name):
        if name not in m:
            return None
        if name in cache:
            cache.move_to_end(name)
            return cache[name]
        try:
            v = convert(name)
        except KeyError:  # optional tensor absent from this checkpoint
            m.pop(name, None)
            return None
        cache[name] = v
        while len(cache) > 6:
            cache.popitem(last=False)
        return v

    log.info("HF checkpoint %s: %s, %d layers, weights quantised to %s", model_dir, cfg.arch, cfg.n_layers,
             QType(qt).name)
    return cfg, get_tensor
