"""Gemma 2 / Gemma 3 on the Llama-family graph: GeGLU, post-attention / post-FFN norms, sliding-window
layers, attention + final-logit soft-capping, Gemma 3 QK-norm and local RoPE base.

Oracles: transformers' Gemma2ForCausalLM / Gemma3ForCausalLM (eager attention) loaded with the
dequantised weights of the same synthetic GGUF tensors — GGUF stores Gemma norms as (1 + w), the
HF modules add the 1 themselves — and our own fp32 CPU path for the HIP kernels (attention window /
softcap, D=256 prefill, GeGLU epilogues, mxk_rmsnorm_add). Reference parity: llama.cpp
build_gemma2 / build_gemma3 as run by the reference's llama-cpp backend
(backend/cpp/llama/grpc-server.cpp)."""
import math

import numpy as np
import pytest
import torch

from localai_tfp_amd.models.config import LlamaConfig, tiny_config
from localai_tfp_amd.models.llama import LlamaModel
from localai_tfp_amd.models.synthetic import gguf_metadata, synthetic_source
from localai_tfp_amd.ops import core as K
from localai_tfp_amd.ops.quant import dequantize

transformers = pytest.importorskip("transformers")


def _deq(src, name, minus_one=False):
    raw, qt, shape = src(name)
    t = torch.from_numpy(np.ascontiguousarray(dequantize(raw, qt, shape)).reshape(tuple(reversed(shape))).copy())
    return t.float() - (1.0 if minus_one else 0.0)


def _gemma_cfg(arch, **kw):
    H = kw.pop("hidden", 256)
    base = dict(arch=arch, hidden=H, ffn=512, n_heads=4, n_kv_heads=2, head_dim=64, rope_dim=64, vocab=512,
                n_layers=4, rms_eps=1e-6, tie_embeddings=True, embed_scale=H ** 0.5, ffn_act="gelu",
                post_norms=True, sliding_window=8)
    if arch == "gemma2":
        base.update(rope_base=10000.0, attn_softcap=2.0, final_softcap=3.0, swa_pattern=2)
    else:
        base.update(rope_base=1e6, rope_base_local=1e4, qk_norm=True, swa_pattern=3)
    base.update(kw)
    return tiny_config(**base)


def _hf_state(cfg, src):
    sd = {"model.embed_tokens.weight": _deq(src, "token_embd.weight"),
          "model.norm.weight": _deq(src, "output_norm.weight", True)}
    for i in range(cfg.n_layers):
        p, q = f"blk.{i}.", f"model.layers.{i}."
        sd[q + "input_layernorm.weight"] = _deq(src, p + "attn_norm.weight", True)
        sd[q + "post_attention_layernorm.weight"] = _deq(src, p + "post_attention_norm.weight", True)
        sd[q + "pre_feedforward_layernorm.weight"] = _deq(src, p + "ffn_norm.weight", True)
        sd[q + "post_feedforward_layernorm.weight"] = _deq(src, p + "post_ffw_norm.weight", True)
        for a, b in (("q", "attn_q"), ("k", "attn_k"), ("v", "attn_v"), ("o", "attn_output")):
            sd[q + f"self_attn.{a}_proj.weight"] = _deq(src, p + b + ".weight")
        if cfg.qk_norm:
            sd[q + "self_attn.q_norm.weight"] = _deq(src, p + "attn_q_norm.weight", True)
            sd[q + "self_attn.k_norm.weight"] = _deq(src, p + "attn_k_norm.weight", True)
        for a, b in (("gate", "ffn_gate"), ("up", "ffn_up"), ("down", "ffn_down")):
            sd[q + f"mlp.{a}_proj.weight"] = _deq(src, p + b + ".weight")
    return sd


def _hf_model(cfg):
    common = dict(vocab_size=cfg.vocab, hidden_size=cfg.hidden, intermediate_size=cfg.ffn,
                  num_hidden_layers=cfg.n_layers, num_attention_heads=cfg.n_heads,
                  num_key_value_heads=cfg.n_kv_heads, head_dim=cfg.head_dim, rms_norm_eps=cfg.rms_eps,
                  hidden_activation="gelu_pytorch_tanh", query_pre_attn_scalar=cfg.head_dim,
                  sliding_window=cfg.sliding_window, tie_word_embeddings=True)
    if cfg.arch == "gemma2":
        from transformers import Gemma2Config as HC, Gemma2ForCausalLM as HM
        hc = HC(attn_logit_softcapping=cfg.attn_softcap, final_logit_softcapping=cfg.final_softcap, **common)
        hc.rope_parameters = {"rope_type": "default", "rope_theta": cfg.rope_base}
    else:
        from transformers import Gemma3ForCausalLM as HM, Gemma3TextConfig as HC
        hc = HC(sliding_window_pattern=cfg.swa_pattern,
                rope_parameters={"full_attention": {"rope_type": "default", "rope_theta": cfg.rope_base},
                                 "sliding_attention": {"rope_type": "default", "rope_theta": cfg.rope_base_local}},
                **common)
    hc._attn_implementation = "eager"
    layer_types = [("full_attention" if cfg.layer_window(i) == 0 else "sliding_attention") for i in range(cfg.n_layers)]
    assert list(hc.layer_types) == layer_types, (hc.layer_types, layer_types)
    return HM(hc).eval()


def _our_logits(model, prompt, forced=()):
    from test_model_gpu import _run
    return _run(model, model.device.type, prompt, list(forced))


@pytest.mark.parametrize("arch", ["gemma2", "gemma3"])
def test_gemma_matches_transformers(arch):
    cfg = _gemma_cfg(arch)
    src = synthetic_source(cfg, "Q8_0", seed=11)
    hm = _hf_model(cfg)
    missing, unexpected = hm.load_state_dict(_hf_state(cfg, src), strict=False)
    assert not unexpected and not [k for k in missing if "rotary" not in k and "lm_head" not in k], \
        (missing, unexpected)
    ours = LlamaModel.load(cfg, src, "cpu")
    rng = np.random.default_rng(4)
    prompt = [int(x) for x in rng.integers(0, cfg.vocab, 21)]  # > 2x the window
    forced = [int(x) for x in rng.integers(0, cfg.vocab, 3)]
    with torch.no_grad():
        ref = hm(torch.tensor([prompt + forced])).logits[0].float()
    got = _our_logits(ours, prompt, forced)
    for i, g in enumerate(got):  # prefill logits of the last prompt token, then each decode step
        r = ref[len(prompt) - 1 + i]
        rel = float((g[0] - r).norm() / r.norm())
        assert rel < 2e-2, (i, rel)
        assert int(g[0].argmax()) == int(r.argmax())
    if cfg.final_softcap:
        assert float(got[0].abs().max()) <= cfg.final_softcap


def test_gemma_window_and_softcap_matter():
    """The features under test change the result (guards against a silently ignored option)."""
    cfg = _gemma_cfg("gemma2", attn_softcap=0.5, final_softcap=0.0)
    src = synthetic_source(cfg, "Q8_0", seed=11)
    prompt = [int(x) for x in np.random.default_rng(4).integers(0, cfg.vocab, 21)]
    base = _our_logits(LlamaModel.load(cfg, src, "cpu"), prompt)[0]
    for kw in (dict(sliding_window=0), dict(attn_softcap=0.0), dict(post_norms=False)):
        c2 = _gemma_cfg("gemma2", **{"attn_softcap": 0.5, "final_softcap": 0.0, **kw})
        other = _our_logits(LlamaModel.load(c2, src, "cpu"), prompt)[0]
        assert float((other - base).norm() / base.norm()) > 1e-3, kw


@pytest.mark.parametrize("arch", ["gemma2", "gemma3"])
def test_gemma_gguf_metadata_roundtrip(arch):
    from localai_tfp_amd.models.config import GEMMA2_9B, GEMMA3_12B
    full = GEMMA2_9B if arch == "gemma2" else GEMMA3_12B
    cfg = LlamaConfig.from_gguf_metadata(gguf_metadata(full))
    for f in ("arch", "head_dim", "ffn_act", "post_norms", "attn_softcap", "final_softcap", "sliding_window",
              "swa_pattern", "rope_base_local", "qk_norm", "tie_embeddings", "rope_scale"):
        assert getattr(cfg, f) == getattr(full, f), f
    assert math.isclose(cfg.embed_scale, full.embed_scale)
    wins = [cfg.layer_window(i) for i in range(12)]
    if arch == "gemma2":
        assert wins == [4096, 0] * 6  # even layers local (HF: sliding iff (i + 1) % 2)
    else:
        assert wins == [1024] * 5 + [0] + [1024] * 5 + [0]


def test_attention_window_softcap_reference():
    """_attn_ref_one semantics: key kp visible to query qp iff qp - window < kp <= qp; scores capped."""
    D, Hkv, bs = 8, 1, 4
    g = torch.Generator().manual_seed(0)
    kc = torch.randn(4, Hkv, bs, D, generator=g)
    vc = torch.randn(4, Hkv, bs, D, generator=g)
    table = torch.tensor([0, 1, 2, 3])
    q = torch.randn(1, 1, D, generator=g)
    ctx = 13
    out = K._attn_ref_one(q, kc, vc, table, ctx, ctx - 1, 0.5, bs, window=5, softcap=1.5)
    k = kc.permute(1, 0, 2, 3).reshape(Hkv, -1, D)[:, :ctx]
    v = vc.permute(1, 0, 2, 3).reshape(Hkv, -1, D)[:, :ctx]
    s = (k[0] @ q[0, 0]) * 0.5
    s = 1.5 * torch.tanh(s / 1.5)
    s[: ctx - 5] = float("-inf")
    ref = torch.softmax(s, 0) @ v[0]
    assert torch.allclose(out[0, 0], ref, atol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("D,Hq,Hkv", [(256, 8, 4), (256, 16, 8), (128, 32, 8)])
@pytest.mark.parametrize("window,softcap", [(0, 0.0), (37, 0.0), (0, 5.0), (100, 50.0)])
def test_attention_window_softcap_gpu(D, Hq, Hkv, window, softcap):
    bs, nb = 16, 512
    g = torch.Generator().manual_seed(D + window)
    kc = torch.randn(nb, Hkv, bs, D, generator=g).bfloat16()
    vc = torch.randn(nb, Hkv, bs, D, generator=g).bfloat16()
    scale = 1 / math.sqrt(D)

    def rel(a, b):
        return float((a.float().cpu() - b.float()).norm() / b.float().norm())

    # decode (partitioned: the window start falls inside a partition and whole partitions are empty)
    lens = [1, 40, 700, 1300]
    B = len(lens)
    maxb = max((l + bs - 1) // bs for l in lens)
    perm = torch.randperm(nb - 1, generator=g)[: B * maxb] + 1
    bt = perm.view(B, maxb).int()
    seq = torch.tensor(lens, dtype=torch.int32)
    q = torch.randn(B, Hq, D, generator=g).bfloat16()
    ref = torch.empty(B, Hq, D)
    K.attn_decode(q, kc, vc, bt, seq, scale, ref, window=window, softcap=softcap)
    for part in (256, 128):
        for impl in ("mfma", "valu"):
            out = torch.empty(B, Hq, D, dtype=torch.bfloat16, device="cuda")
            K.attn_decode(q.cuda(), kc.cuda(), vc.cuda(), bt.cuda(), seq.cuda(), scale, out, part_size=part,
                          window=window, softcap=softcap, impl=impl)
            assert rel(out, ref) < 1.5e-2, ("decode", part, impl)
    # prefill with cached prefixes (query 0 of a chunk sits mid-context)
    q_lens, ctx = [37, 1, 130, 64], [37, 20, 300, 200]
    S = len(q_lens)
    maxb = max((c + bs - 1) // bs for c in ctx)
    bt = (torch.randperm(nb - 1, generator=g)[: S * maxb] + 1).view(S, maxb).int()
    cu = torch.tensor([0] + list(np.cumsum(q_lens)), dtype=torch.int32)
    T = int(cu[-1])
    q = torch.randn(T, Hq, D, generator=g).bfloat16()
    ctx_t = torch.tensor(ctx, dtype=torch.int32)
    ref = torch.empty(T, Hq, D)
    K.attn_prefill(q, kc, vc, bt, cu, ctx_t, scale, ref, q_lens, ctx, window=window, softcap=softcap)
    for vmode in (0, 1):
        out = torch.empty(T, Hq, D, dtype=torch.bfloat16, device="cuda")
        K.attn_prefill(q.cuda(), kc.cuda(), vc.cuda(), bt.cuda(), cu.cuda(), ctx_t.cuda(), scale, out, q_lens, ctx,
                       vmode=vmode, window=window, softcap=softcap)
        assert rel(out, ref) < 1.5e-2, ("prefill", vmode)


@pytest.mark.gpu
@pytest.mark.parametrize("arch", ["gemma2", "gemma3"])
def test_gemma_gpu_matches_cpu_and_engine(arch):
    """head_dim 256 (Gemma's), GeGLU through the GEMV / MFMA epilogues, post-norm residual kernel,
    window + softcap in decode and prefill, and the whole step inside a hipGraph."""
    from localai_tfp_amd.engine.engine import EngineConfig, LLMEngine
    from localai_tfp_amd.ops.sampling import SamplingParams
    from localai_tfp_amd.tokenizer import ByteTokenizer
    from test_model_gpu import _run
    cfg = _gemma_cfg(arch, hidden=512, ffn=1024, n_heads=4, n_kv_heads=2, head_dim=256, rope_dim=256,
                     sliding_window=16)
    src = synthetic_source(cfg, "Q4_K_M", seed=9)
    mc = LlamaModel.load(cfg, src, "cpu")
    mg = LlamaModel.load(cfg, src, "cuda")
    prompt = [int(x) for x in np.random.default_rng(0).integers(0, cfg.vocab, 40)]
    a = _run(mc, "cpu", prompt, [5, 99, 300])
    b = _run(mg, "cuda", prompt, [5, 99, 300])
    for x, y in zip(a, b):
        assert float((x - y).norm() / x.norm()) < 6e-2
    tok = ByteTokenizer(cfg.vocab)
    streams = []
    for graphs in (False, True):
        eng = LLMEngine(mg, tok, EngineConfig(num_blocks=256, max_num_seqs=8, max_batched_tokens=256,
                                              max_model_len=512, use_graphs=graphs))
        outs = [eng.generate(tok.encode(f"gemma prompt number {i} " * 3), SamplingParams(temperature=0.0, ignore_eos=True),
                             max_tokens=24) for i in range(2)]
        assert all(len(o.token_ids) == 24 for o in outs)
        streams.append([o.token_ids for o in outs])
    assert streams[0] == streams[1]
