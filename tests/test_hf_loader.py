"""HF safetensors LLM directories (vllm / transformers backends, models/hf.py): logits of our Llama-family
graph loaded from a `save_pretrained` directory against transformers' own forward of the same weights
(fp32, CPU). Reference: backend/python/vllm/backend.py:81-141, backend/python/transformers/backend.py:68-284.
The checkpoints are random-init tiny models written by transformers here (no network)."""
import json

import numpy as np
import pytest
import torch

from localai_tfp_amd.models.loader import load_llm

transformers = pytest.importorskip("transformers")

COMMON = dict(vocab_size=320, hidden_size=128, intermediate_size=256, num_hidden_layers=2, num_attention_heads=4,
              num_key_value_heads=2, max_position_embeddings=512)


def _make(arch, tmp_path):
    torch.manual_seed(0)
    T = transformers
    if arch == "llama":
        hc = T.LlamaConfig(**COMMON, rope_theta=10000.0)
        m = T.LlamaForCausalLM(hc)
    elif arch == "llama31":
        hc = T.LlamaConfig(**COMMON, rope_theta=500000.0,
                           rope_scaling={"rope_type": "llama3", "factor": 8.0, "low_freq_factor": 1.0,
                                         "high_freq_factor": 4.0, "original_max_position_embeddings": 64})
        m = T.LlamaForCausalLM(hc)
    elif arch == "qwen2":
        hc = T.Qwen2Config(**COMMON, rope_theta=1e6, tie_word_embeddings=True)
        m = T.Qwen2ForCausalLM(hc)
    elif arch == "qwen3":
        hc = T.Qwen3Config(**COMMON, head_dim=32, rope_theta=1e6)
        m = T.Qwen3ForCausalLM(hc)
    elif arch == "phi3":
        hc = T.Phi3Config(**COMMON, rope_theta=10000.0, pad_token_id=0)
        m = T.Phi3ForCausalLM(hc)
    elif arch == "mixtral":
        hc = T.MixtralConfig(**COMMON, num_local_experts=4, num_experts_per_tok=2, rope_theta=1e6)
        m = T.MixtralForCausalLM(hc)
    elif arch == "qwen2moe":
        hc = T.Qwen2MoeConfig(**COMMON, num_experts=4, num_experts_per_tok=2, moe_intermediate_size=64,
                              shared_expert_intermediate_size=128, rope_theta=1e6)
        m = T.Qwen2MoeForCausalLM(hc)
    elif arch == "gemma2":
        hc = T.Gemma2Config(**COMMON, head_dim=32, query_pre_attn_scalar=32, sliding_window=8,
                            attn_logit_softcapping=30.0, final_logit_softcapping=20.0,
                            hidden_activation="gelu_pytorch_tanh")
        m = T.Gemma2ForCausalLM(hc)
    else:
        raise KeyError(arch)
    hc._attn_implementation = "eager"
    with torch.no_grad():  # norms away from 1 so the (1 + w) Gemma convention and per-norm mapping matter
        for n, p in m.named_parameters():
            if "norm" in n:
                p.add_(torch.randn_like(p) * 0.2)
            if n.endswith(".bias"):
                p.add_(torch.randn_like(p) * 0.1)
            if n.endswith("mlp.gate.weight"):  # decisive routing: no top-k ties flipped by rounding
                p.mul_(30.0)
    m = m.eval()
    d = tmp_path / arch
    m.save_pretrained(str(d))
    return m, str(d)


def _ours(model, prompt):
    from test_model_gpu import _run
    return _run(model, "cpu", prompt, [])[0][0]


@pytest.mark.parametrize("arch", ["llama", "llama31", "qwen2", "qwen3", "phi3", "mixtral", "qwen2moe", "gemma2"])
def test_hf_dir_matches_transformers(arch, tmp_path):
    hm, d = _make(arch, tmp_path)
    rng = np.random.default_rng(3)
    prompt = [int(x) for x in rng.integers(3, COMMON["vocab_size"], 19)]
    with torch.no_grad():
        ref = hm(torch.tensor([prompt])).logits[0, -1].float()
    model, tok, cfg, _ = load_llm(d, "cpu", overrides={"hf_quant": "f32"})
    got = _ours(model, prompt)
    rel = float((got - ref).norm() / ref.norm())
    assert rel < 5e-3, (arch, rel)
    # default: bf16 (the reference's vLLM / transformers precision); `quant: q8_0` -> Q8_0 blocks (qmm / qmv layout)
    modelb, *_ = load_llm(d, "cpu")
    assert modelb.layers[0].wo.qtype == "dense"
    relb = float((_ours(modelb, prompt) - ref).norm() / ref.norm())
    assert relb < 2e-2, (arch, relb)
    model8, *_ = load_llm(d, "cpu", overrides={"hf_quant": "q8_0"})
    assert model8.layers[0].wo.qtype == 8
    got8 = _ours(model8, prompt)
    rel8 = float((got8 - ref).norm() / ref.norm())
    assert rel8 < 3e-2, (arch, rel8)


def test_hf_config_mapping(tmp_path):
    from localai_tfp_amd.models.hf import config_from_hf
    c = config_from_hf({"architectures": ["LlamaForCausalLM"], "hidden_size": 4096, "num_attention_heads": 32,
                        "num_key_value_heads": 8, "num_hidden_layers": 32, "intermediate_size": 14336,
                        "vocab_size": 128256, "rope_theta": 500000.0,
                        "rope_scaling": {"rope_type": "llama3", "factor": 8.0, "low_freq_factor": 1.0,
                                         "high_freq_factor": 4.0, "original_max_position_embeddings": 8192}})
    assert (c.arch, c.n_kv_heads, c.head_dim, c.rope_base) == ("llama", 8, 128, 500000.0)
    assert c.rope_llama3["factor"] == 8.0
    y = config_from_hf({"architectures": ["Qwen2ForCausalLM"], "hidden_size": 1024, "num_attention_heads": 16,
                        "num_hidden_layers": 4, "vocab_size": 1000,
                        "rope_scaling": {"type": "yarn", "factor": 4.0, "original_max_position_embeddings": 32768}})
    assert y.qkv_bias and y.rope_scaling == "yarn" and y.rope_scale == 0.25 and y.rope_orig_ctx == 32768


def test_hf_tokenizer_dir(tmp_path):
    """tokenizer.json (byte-level BPE, as Llama-3 / Qwen ship) + tokenizer_config.json chat template."""
    from tokenizers import Tokenizer, decoders, models, pre_tokenizers, trainers
    tk = Tokenizer(models.BPE())
    tk.pre_tokenizer = pre_tokenizers.ByteLevel(add_prefix_space=False)
    tk.decoder = decoders.ByteLevel()
    tr = trainers.BpeTrainer(vocab_size=300, special_tokens=["<|begin_of_text|>", "<|eot_id|>"],
                             initial_alphabet=pre_tokenizers.ByteLevel.alphabet())
    tk.train_from_iterator(["hello world, hello there " * 20, "the quick brown fox"], tr)
    tk.save(str(tmp_path / "tokenizer.json"))
    (tmp_path / "tokenizer_config.json").write_text(json.dumps({
        "bos_token": "<|begin_of_text|>", "eos_token": "<|eot_id|>", "add_bos_token": True,
        "chat_template": "{% for m in messages %}{{ m['content'] }}<|eot_id|>{% endfor %}"}))
    from localai_tfp_amd.tokenizer import from_hf_dir
    t = from_hf_dir(str(tmp_path))
    ids = t.encode("hello world")
    assert ids[0] == t.bos_token_id == 0 and t.decode(ids) == "hello world"
    assert t.eos_token_id == 1 and 1 in t.eos_token_ids
    assert "messages" in t.chat_template
    tb = t.token_bytes()
    assert b"".join(tb[i] for i in ids[1:]) == b"hello world" and tb[0] == b""
    assert t.encode("<|eot_id|>", add_special=False) == [1]


@pytest.mark.gpu
def test_hf_dir_gpu_q8_0(tmp_path):
    """The HF checkpoint on the GPU: Q8_0 blocks re-laid out for qmm / qmv (no dense copy), logits vs
    the transformers fp32 forward."""
    torch.manual_seed(0)
    hc = transformers.LlamaConfig(vocab_size=512, hidden_size=512, intermediate_size=1024, num_hidden_layers=2,
                                  num_attention_heads=8, num_key_value_heads=2, max_position_embeddings=512)
    hm = transformers.LlamaForCausalLM(hc).eval()
    hm.save_pretrained(str(tmp_path))
    prompt = [int(x) for x in np.random.default_rng(5).integers(3, 512, 23)]
    with torch.no_grad():
        ref = hm(torch.tensor([prompt])).logits[0, -1].float()
    model, *_ = load_llm(str(tmp_path), "cuda:0", overrides={"hf_quant": "q8_0"})
    w = model.layers[0].wo
    assert w.is_quant and w.layout == "t32" and w.bf16_cache is None
    from test_model_gpu import _run
    got = _run(model, "cuda", prompt, [])[0][0].float().cpu()
    rel = float((got - ref).norm() / ref.norm())
    assert rel < 5e-2, rel
    # default: bf16 weights (the reference's vLLM / transformers precision), small batches on the 16-bit path
    model, *_ = load_llm(str(tmp_path), "cuda:0")
    assert not model.layers[0].wo.is_quant and not model._gemv_ok
    got = _run(model, "cuda", prompt, [])[0][0].float().cpu()
    rel = float((got - ref).norm() / ref.norm())
    assert rel < 3e-2, rel
