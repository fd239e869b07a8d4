"""Architecture hyper-parameters read from GGUF metadata (or built for synthetic checkpoints)."""
from __future__ import annotations

from dataclasses import dataclass, field

# llama.cpp rope type per architecture: NORM (adjacent pairs) vs NEOX (half split)
NEOX_ARCHS = {"qwen2", "qwen2moe", "qwen3", "phi2", "phi3", "gemma", "gemma2", "gemma3", "starcoder2",
              "falcon", "gptneox", "stablelm", "olmo2", "bert", "nomic-bert", "jina-bert-v2"}
BIAS_QKV_ARCHS = {"qwen2", "qwen2moe"}


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

    def n_params(self) -> int:
        h, f, L = self.hidden, self.ffn, self.n_layers
        per = h * (self.q_dim + 2 * self.kv_dim) + self.q_dim * h + 3 * h * f + 2 * h
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
            cfg.embed_scale = hidden ** 0.5
        return cfg


LLAMA3_8B = LlamaConfig(name="Llama-3-8B-Instruct")
LLAMA3_70B = LlamaConfig(name="Llama-3-70B-Instruct", n_layers=80, hidden=8192, ffn=28672, n_heads=64,
                         n_kv_heads=8)
LLAMA32_1B = LlamaConfig(name="Llama-3.2-1B", n_layers=16, hidden=2048, ffn=8192, n_heads=32, n_kv_heads=8,
                         head_dim=64, rope_dim=64, tie_embeddings=True)


def tiny_config(**kw) -> LlamaConfig:
    """A small Llama-architecture config for CPU tests."""
    base = dict(name="tiny-llama", n_layers=2, hidden=256, ffn=512, n_heads=4, n_kv_heads=2, head_dim=64,
                vocab=512, ctx_train=2048, rope_base=10000.0, rope_dim=64)
    base.update(kw)
    return LlamaConfig(**base)
