"""Model acquisition for the LLM worker: GGUF files (llama.cpp's format, what the reference's
llama-cpp backend loads) or `synthetic:<arch>` random-init checkpoints of a named architecture
(bench / tests — there is no network to fetch real weights)."""
from __future__ import annotations

import logging
import os

import numpy as np

from ..formats.gguf import GGUFReader
from . import config as C
from .config import LlamaConfig
from .llama import LlamaModel

log = logging.getLogger("localai_tfp_amd.models")

SYNTHETIC = {"llama3-8b": C.LLAMA3_8B, "llama3-70b": C.LLAMA3_70B, "llama32-1b": C.LLAMA32_1B,
             "qwen3-8b": C.QWEN3_8B, "qwen3-30b-a3b": C.QWEN3_30B_A3B, "mixtral-8x7b": C.MIXTRAL_8X7B,
             "tiny": C.tiny_config(),
             "tiny-draft": C.tiny_config(n_layers=1, name="tiny-draft"),
             "tiny-4l": C.tiny_config(n_layers=4, name="tiny-4l"),  # layer-split tests  # speculative-decoding draft for "tiny"
             "tiny-moe": C.tiny_config(arch="qwen3moe", n_expert=8, n_expert_used=2, expert_ffn=256, qk_norm=True)}
SUPPORTED_ARCHS = {"llama", "mistral", "qwen2", "qwen2vl", "qwen3", "qwen2moe", "qwen3moe", "phi3", "gemma", "gemma2", "gemma3", "granite", "internlm2", "deci", "exaone", "olmo", "minicpm",
                   "smollm", "codellama"}


def gguf_source(reader: GGUFReader):
    def get_tensor(name):
        ti = reader.tensors.get(name)
        if ti is None:
            return None
        return reader.tensor_bytes(name), ti.qtype, ti.shape
    return get_tensor


def load_llm(model: str, device="cpu", tp_rank: int = 0, tp_size: int = 1, tp_group=None, overrides: dict | None = None):
    """-> (LlamaModel, tokenizer, LlamaConfig, metadata dict)"""
    from ..tokenizer import ByteTokenizer, from_gguf
    ov = overrides or {}
    rec = _load_recurrent(model, device, tp_size)
    if rec is not None:
        if ov.get("lora"):
            raise NotImplementedError("LoRA adapters are not supported for recurrent (Mamba / RWKV) models")
        return rec
    if model.startswith("synthetic:"):
        from .synthetic import synthetic_source
        key = model.split(":", 1)[1]
        cfg = SYNTHETIC[key]
        import copy
        cfg = copy.deepcopy(cfg)
        _apply_overrides(cfg, ov)
        src = _lora_source(synthetic_source(cfg, "Q4_K_M", seed=1), ov, cfg, tp_size)
        m = _lora_attach(LlamaModel.load(cfg, src, device, tp_rank, tp_size, tp_group), ov, cfg, tp_size)
        return m, ByteTokenizer(cfg.vocab), cfg, {}
    from .hf import QUANTS, hf_source, is_hf_dir
    if is_hf_dir(model):  # vllm / transformers backends: HF safetensors directory (models/hf.py)
        # bf16 by default, as the reference's vLLM / transformers backends serve HF checkpoints; `quant:
        # q8_0 | q4_k | q6_k` opts into the quantised kernels
        q = str(ov.get("hf_quant") or "bf16").lower()
        if q not in QUANTS:
            log.warning("quantization %r is not a load-time format here; using bf16", q)
            q = "bf16"
        cfg, get = hf_source(model, q)
        _apply_overrides(cfg, ov)
        m = _lora_attach(LlamaModel.load(cfg, _lora_source(get, ov, cfg, tp_size), device, tp_rank, tp_size, tp_group),
                         ov, cfg, tp_size)
        try:
            from ..tokenizer import from_hf_dir
            tok = from_hf_dir(model)
        except Exception as ex:  # tokenizer.json is optional for synthetic / test checkpoints
            log.warning("no usable tokenizer in %s (%s); byte-level fallback", model, ex)
            tok = ByteTokenizer(cfg.vocab)
        return m, tok, cfg, {"tokenizer.chat_template": getattr(tok, "chat_template", None)}
    if not os.path.isfile(model):
        raise FileNotFoundError(model)
    r = GGUFReader(model)
    md = dict(r.metadata)
    arch = str(md.get("general.architecture", "llama"))
    if arch not in SUPPORTED_ARCHS:
        log.warning("architecture %r not in the tested set; trying the Llama graph", arch)
    cfg = LlamaConfig.from_gguf_metadata(md)
    if f"{arch}.rope.scaling.type" not in md and "rope_freqs.weight" in r.tensors:
        from ..ops.quant import dequantize
        ti = r.tensors["rope_freqs.weight"]
        cfg.extra["rope_freqs"] = dequantize(r.tensor_bytes("rope_freqs.weight"), ti.qtype, ti.shape).tolist()
    _apply_overrides(cfg, ov)
    m = _lora_attach(LlamaModel.load(cfg, _lora_source(gguf_source(r), ov, cfg, tp_size), device, tp_rank, tp_size,
                                     tp_group), ov, cfg, tp_size)
    try:
        tok = from_gguf(md)
    except Exception as ex:
        log.warning("no usable tokenizer in %s (%s); byte-level fallback", model, ex)
        tok = ByteTokenizer(cfg.vocab)
    return m, tok, cfg, md


def _lora_mode(ov: dict, tp_size: int, cfg: LlamaConfig | None = None) -> str:
    """`lora_requant`: runtime (default: adapters kept beside the untouched base weights, as llama.cpp applies them)
    | q8_0 | same | f32 (merged into the weights at load). Tensor parallelism merges (shards are cut after it), and
    so do post-norm (Gemma 2/3) blocks, whose o / down outputs are normalised before the residual add."""
    m = str(ov.get("lora_requant") or "runtime").lower()
    if m == "runtime" and (tp_size > 1 or (cfg is not None and cfg.post_norms)):
        log.info("LoRA: %s load merges the adapters (Q8_0)", "tensor parallel" if tp_size > 1 else "post-norm model")
        m = "q8_0"
    return m


def _lora_source(get_tensor, ov: dict, cfg: LlamaConfig, tp_size: int = 1):
    """overrides["lora"] = [(adapter path, scale), ...] -> a source yielding LoRA-merged weights (merge modes),
    or the base source unchanged (runtime mode: _lora_attach after the load)."""
    if not ov.get("lora") or _lora_mode(ov, tp_size, cfg) == "runtime":
        return get_tensor
    from .lora import load_adapter, with_adapters
    ads = [load_adapter(p, s, cfg) for p, s in ov["lora"]]
    src = with_adapters(get_tensor, ads, _lora_mode(ov, tp_size, cfg))
    log.info("LoRA: %d adapter(s), %d weight tensors merged", len(ads), src.lora_targets)
    return src


def _lora_attach(m, ov: dict, cfg: LlamaConfig, tp_size: int = 1, l0: int = 0):
    """Runtime LoRA: the adapters beside the loaded base weights (models/lora_runtime.py)."""
    if not ov.get("lora") or _lora_mode(ov, tp_size, cfg) != "runtime":
        return m
    from .lora import load_adapter
    from .lora_runtime import build
    ads = [load_adapter(p, s, cfg) for p, s in ov["lora"]]
    n = build(m, ads, l0)
    log.info("LoRA: %d adapter(s) applied at runtime to %d projections (base weights unchanged)", len(ads), n)
    return m


def _apply_overrides(cfg: LlamaConfig, ov: dict):
    if ov.get("rope_freq_base"):
        cfg.rope_base = float(ov["rope_freq_base"])
    if ov.get("rope_freq_scale"):
        cfg.rope_scale = float(ov["rope_freq_scale"])
        if cfg.rope_scaling == "none":
            cfg.rope_scaling = "linear"
    if ov.get("rope_scaling"):
        cfg.rope_scaling = str(ov["rope_scaling"])
    if ov.get("rms_norm_eps"):
        cfg.rms_eps = float(ov["rms_norm_eps"])
    if ov.get("context_size"):
        cfg.ctx_train = max(cfg.ctx_train, int(ov["context_size"])) if ov.get("extend_context") else cfg.ctx_train


RECURRENT_ARCHS = {"mamba", "rwkv6"}


def _load_recurrent(model: str, device, tp_size: int):
    """Recurrent checkpoints: Mamba (models/mamba.py: `synthetic:mamba-*`, an HF MambaForCausalLM
    directory, GGUF arch `mamba`) and RWKV-6 (models/rwkv.py: `synthetic:rwkv6-*`, GGUF arch
    `rwkv6`). None for everything else."""
    from . import mamba as M
    from ..tokenizer import ByteTokenizer, from_gguf
    if model.startswith("synthetic:rwkv"):
        from . import rwkv as RW
        key = model.split(":", 1)[1]
        cfg = {"rwkv6-7b": RW.RWKV6_WORLD_7B, "rwkv6-1b6": RW.RWKV6_WORLD_1B6, "rwkv6-tiny": RW.tiny_rwkv_config()}[key]
        import copy
        cfg = copy.deepcopy(cfg)
        m = RW.RwkvModel.load(cfg, RW.synthetic_rwkv_source(cfg, seed=1), device)
        return m, ByteTokenizer(cfg.vocab), cfg, {}
    if model.startswith("synthetic:mamba"):
        key = model.split(":", 1)[1]
        cfg = {"mamba-130m": M.MAMBA_130M, "mamba-1.4b": M.MAMBA_1_4B, "mamba-2.8b": M.MAMBA_2_8B,
               "mamba-tiny": M.tiny_mamba_config()}[key]
        import copy
        cfg = copy.deepcopy(cfg)
        return M.MambaModel.load(cfg, M.synthetic_mamba_source(cfg, seed=1), device), ByteTokenizer(cfg.vocab), cfg, {}
    if os.path.isdir(model) and os.path.isfile(os.path.join(model, "config.json")):
        import json
        with open(os.path.join(model, "config.json")) as f:
            if json.load(f).get("model_type") != "mamba":
                return None
        if tp_size > 1:
            raise ValueError("tensor parallelism is not supported for Mamba models")
        cfg, get = M.hf_mamba_source(model)
        tok = ByteTokenizer(cfg.vocab)
        try:
            from ..tokenizer import from_hf_dir
            tok = from_hf_dir(model)
        except Exception as ex:  # tokenizer.json is optional for synthetic / test checkpoints
            log.warning("no usable tokenizer in %s (%s); byte-level fallback", model, ex)
        return M.MambaModel.load(cfg, get, device), tok, cfg, {}
    if os.path.isfile(model):
        try:
            r = GGUFReader(model)
        except Exception:
            return None
        md = dict(r.metadata)
        if str(md.get("general.architecture")) not in RECURRENT_ARCHS:
            return None
        if tp_size > 1:
            raise ValueError("tensor parallelism is not supported for Mamba models")
        if str(md.get("general.architecture")) == "rwkv6":
            from . import rwkv as RW
            cfg = RW.RwkvConfig.from_gguf_metadata(md)
            m = RW.RwkvModel.load(cfg, gguf_source(r), device)
        else:
            cfg = M.MambaConfig.from_gguf_metadata(md)
            m = M.MambaModel.load(cfg, gguf_source(r), device)
        try:
            tok = from_gguf(md)
        except Exception as ex:
            log.warning("no usable tokenizer in %s (%s); byte-level fallback", model, ex)
            tok = ByteTokenizer(cfg.vocab)
        return m, tok, cfg, md
    return None
