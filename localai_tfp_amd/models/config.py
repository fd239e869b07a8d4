"""Architecture hyper-parameters read from GGUF metadata (or built for synthetic checkpoints)."""
from __future__ import annotations

from dataclasses import dataclass, field

# llama.cpp rope type per architecture: NORM (adjacent pairs) vs NEOX (half split)
NEOX_ARCHS = {"qwen2", "qwen2vl", "qwen2moe", "qwen3", "qwen3moe", "phi2", "phi3", "gemma", "gemma2", "gemma3", "starcoder2",
              "falcon", "gptneox", "stablelm", "olmo2", "bert", "nomic-bert", "jina-bert-v2"}
# qwen2vl (Qwen2-VL / Qwen2.5-VL text model): M-RoPE, whose three position components coincide for text tokens, so
# it runs as NEOX RoPE (image embeddings take the next sequential positions, as the reference's llava path decodes them)
BIAS_QKV_ARCHS = {"qwen2", "qwen2vl", "qwen2moe"}


@dataclass
class LlamaConfig:
    arch: str = "llama"
    n_layers: int = 32
    hidden: int = 4096
    ffn: int = 14336
    n_heads: int = 32
    n_kv_heads: int = 8
    head_dim: int = 128
    vocab: int = 128256
    ctx_train: int = 8192
    rope_base: float = 500000.0
    rope_dim: int = 128
    rope_scaling: str = "none"
    rope_scale: float = 1.0
    rope_orig_ctx: int = 0
    rope_llama3: dict | None = None
    rms_eps: float = 1e-5
    tie_embeddings: bool = False
    qkv_bias: bool = False
    embed_scale: float = 1.0
    # mixture of experts (Mixtral = llama arch with experts, qwen2moe, qwen3moe)
    n_expert: int = 0
    n_expert_used: int = 0
    expert_ffn: int = 0
    expert_shared_ffn: int = 0
    moe_renorm: bool = True  # renormalise the top-k router weights (Mixtral, Qwen3-MoE; not Qwen2-MoE)
    qk_norm: bool = False  # per-head RMSNorm of q and k before RoPE (Qwen3, Gemma 3)
    # Gemma family (llama.cpp src/llama-model.cpp build_gemma*/ LLM_ARCH_GEMMA2/3 hparams)
    ffn_act: str = "silu"  # gate activation: silu (SwiGLU) | gelu (GeGLU, tanh approximation)
    post_norms: bool = False  # RMSNorm of the attention / FFN output before the residual add (Gemma 2/3)
    attn_softcap: float = 0.0  # scores -> c * tanh(scores / c) (Gemma 2)
    final_softcap: float = 0.0  # logits -> c * tanh(logits / c) (Gemma 2)
    sliding_window: int = 0  # local-attention window of the windowed layers (0 = none)
    swa_pattern: int = 0  # layer i is global iff (i + 1) % swa_pattern == 0 (Gemma 2: 2, Gemma 3: 6); 0/1 = all windowed
    rope_base_local: float = 0.0  # RoPE base of the windowed layers (Gemma 3: 10000; 0 = rope_base)
    attn_scale: float = 0.0  # softmax scale (0 = 1/sqrt(head_dim))
    name: str = "llama"
    extra: dict = field(default_factory=dict)

    @property
    def neox(self) -> bool:
        return self.arch in NEOX_ARCHS

    @property
    def q_dim(self) -> int:
        return self.n_heads * self.head_dim

    @property
    def kv_dim(self) -> int:
        return self.n_kv_heads * self.head_dim

    def layer_window(self, i: int) -> int:
        """Sliding-window size of layer i (0 = full causal attention)."""
        if self.sliding_window <= 0:
            return 0
        if self.swa_pattern > 1 and (i + 1) % self.swa_pattern == 0:
            return 0
        return self.sliding_window

    def n_params(self) -> int:
        h, f, L = self.hidden, self.ffn, self.n_layers
        if self.n_expert:
            ffn_p = self.n_expert * (3 * h * self.expert_ffn + h) + 3 * h * self.expert_shared_ffn
        else:
            ffn_p = 3 * h * f
        per = h * (self.q_dim + 2 * self.kv_dim) + self.q_dim * h + ffn_p + 2 * h
        emb = self.vocab * h * (1 if self.tie_embeddings else 2)
        return L * per + emb + h

    @classmethod
    def from_gguf_metadata(cls, md: dict) -> "LlamaConfig":
        arch = str(md.get("general.architecture", "llama"))

        def g(k, d=None):
            return md.get(f"{arch}.{k}", d)

        hidden = int(g("embedding_length"))
        n_heads = int(g("attention.head_count"))
        kv = g("attention.head_count_kv", n_heads)
        if hasattr(kv, "__len__"):
            kv = int(kv[0])
        head_dim = int(g("attention.key_length", hidden // n_heads))
        vocab = g("vocab_size")
        if vocab is None:
            toks = md.get("tokenizer.ggml.tokens")
            vocab = len(toks) if toks is not None else 32000
        ffn = g("feed_forward_length")
        if hasattr(ffn, "__len__"):
            ffn = int(ffn[0])
        rs_type = str(g("rope.scaling.type", "none") or "none")
        rs_factor = float(g("rope.scaling.factor", 0.0) or 0.0)
        cfg = cls(
            arch=arch,
            n_layers=int(g("block_count")),
            hidden=hidden,
            ffn=int(ffn),
            n_heads=n_heads,
            n_kv_heads=int(kv),
            head_dim=head_dim,
            vocab=int(vocab),
            ctx_train=int(g("context_length", 4096)),
            rope_base=float(g("rope.freq_base", 10000.0)),
            rope_dim=int(g("rope.dimension_count", head_dim)),
            rope_scaling=rs_type,
            rope_scale=(1.0 / rs_factor) if rs_factor else 1.0,
            rope_orig_ctx=int(g("rope.scaling.original_context_length", 0) or 0),
            rms_eps=float(g("attention.layer_norm_rms_epsilon", 1e-5)),
            qkv_bias=arch in BIAS_QKV_ARCHS,
            name=str(md.get("general.name", arch)),
        )
        if arch in ("gemma", "gemma2", "gemma3"):
            # llama.cpp build_gemma*: embeddings * sqrt(n_embd), GeGLU FFN, norms stored as (1 + w)
            cfg.embed_scale = hidden ** 0.5
            cfg.ffn_act = "gelu"
            cfg.tie_embeddings = True
        if arch == "gemma2":
            cfg.post_norms = True
            cfg.attn_softcap = float(g("attn_logit_softcapping", 50.0) or 0.0)
            cfg.final_softcap = float(g("final_logit_softcapping", 30.0) or 0.0)
            cfg.sliding_window = int(g("attention.sliding_window", 4096) or 0)
            cfg.swa_pattern = 2
            if cfg.n_layers == 46:  # Gemma-2-27B: query_pre_attn_scalar = n_embd / n_head
                cfg.attn_scale = (hidden / n_heads) ** -0.5
        if arch == "gemma3":
            cfg.post_norms = True
            cfg.sliding_window = int(g("attention.sliding_window", 1024) or 0)
            cfg.swa_pattern = int(g("attention.sliding_window_pattern", 6) or 6)
            cfg.rope_base_local = 10000.0
            cfg.final_softcap = float(g("final_logit_softcapping", 0.0) or 0.0)
            if cfg.n_layers == 62:  # Gemma-3-27B: query_pre_attn_scalar = n_embd / n_head
                cfg.attn_scale = (hidden / n_heads) ** -0.5
        ne = int(g("expert_count", 0) or 0)
        if ne:
            cfg.n_expert = ne
            cfg.n_expert_used = int(g("expert_used_count", 2))
            cfg.expert_ffn = int(g("expert_feed_forward_length", 0) or 0) or cfg.ffn
            cfg.expert_shared_ffn = int(g("expert_shared_feed_forward_length", 0) or 0)
            cfg.moe_renorm = bool(g("expert_weights_norm", arch != "qwen2moe"))
        cfg.qk_norm = arch in ("qwen3", "qwen3moe", "gemma3")
        return cfg


LLAMA3_8B = LlamaConfig(name="Llama-3-8B-Instruct")
LLAMA3_70B = LlamaConfig(name="Llama-3-70B-Instruct", n_layers=80, hidden=8192, ffn=28672, n_heads=64,
                         n_kv_heads=8)
LLAMA32_1B = LlamaConfig(name="Llama-3.2-1B", n_layers=16, hidden=2048, ffn=8192, n_heads=32, n_kv_heads=8,
                         head_dim=64, rope_dim=64, tie_embeddings=True)


QWEN3_30B_A3B = LlamaConfig(arch="qwen3moe", name="Qwen3-30B-A3B", n_layers=48, hidden=2048, ffn=6144,
                            n_heads=32, n_kv_heads=4, head_dim=128, rope_dim=128, vocab=151936, ctx_train=40960,
                            rope_base=1000000.0, rms_eps=1e-6, n_expert=128, n_expert_used=8, expert_ffn=768,
                            qk_norm=True)
MIXTRAL_8X7B = LlamaConfig(name="Mixtral-8x7B-Instruct", n_layers=32, hidden=4096, ffn=14336, n_heads=32,
                           n_kv_heads=8, vocab=32000, ctx_train=32768, rope_base=1000000.0, n_expert=8,
                           n_expert_used=2, expert_ffn=14336)
QWEN3_8B = LlamaConfig(arch="qwen3", name="Qwen3-8B", n_layers=36, hidden=4096, ffn=12288, n_heads=32,
                       n_kv_heads=8, vocab=151936, ctx_train=40960, rope_base=1000000.0, rms_eps=1e-6, qk_norm=True)
GEMMA2_9B = LlamaConfig(arch="gemma2", name="gemma-2-9b-it", n_layers=42, hidden=3584, ffn=14336, n_heads=16,
                        n_kv_heads=8, head_dim=256, rope_dim=256, vocab=256000, ctx_train=8192, rope_base=10000.0,
                        rms_eps=1e-6, tie_embeddings=True, embed_scale=3584 ** 0.5, ffn_act="gelu", post_norms=True,
                        attn_softcap=50.0, final_softcap=30.0, sliding_window=4096, swa_pattern=2)
GEMMA3_12B = LlamaConfig(arch="gemma3", name="gemma-3-12b-it", n_layers=48, hidden=3840, ffn=15360, n_heads=16,
                         n_kv_heads=8, head_dim=256, rope_dim=256, vocab=262208, ctx_train=131072,
                         rope_base=1000000.0, rope_scaling="linear", rope_scale=0.125, rms_eps=1e-6,
                         tie_embeddings=True, embed_scale=3840 ** 0.5, ffn_act="gelu", post_norms=True, qk_norm=True,
                         sliding_window=1024, swa_pattern=6, rope_base_local=10000.0)


def tiny_config(**kw) -> LlamaConfig:
    """A small Llama-architecture config for CPU tests."""
    base = dict(name="tiny-llama", n_layers=2, hidden=256, ffn=512, n_heads=4, n_kv_heads=2, head_dim=64,
                vocab=512, ctx_train=2048, rope_base=10000.0, rope_dim=64)
    base.update(kw)
    return LlamaConfig(**base)
