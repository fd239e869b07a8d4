"""Model families beyond dense Llama: Qwen3 (per-head q/k RMSNorm), Qwen3-MoE / Mixtral / Qwen2-MoE
(routed experts, shared expert) and Phi-3 (fused QKV / gate|up tensors).

Oracles: transformers' Qwen3MoeForCausalLM / Qwen3ForCausalLM loaded with the dequantised weights of
the same synthetic GGUF tensors (CPU), and the fp32 CPU path of our own model for the HIP kernels
(moe.hip route/sort/combine, qgemm16 grouped mode, rope_kv QK-norm) on the GPU. Reference parity:
llama.cpp build_moe_ffn / build_qwen3moe as run by the reference's llama-cpp backend."""
import numpy as np
import pytest
import torch

from localai_tfp_amd.models.config import tiny_config
from localai_tfp_amd.models.llama import LlamaModel
from localai_tfp_amd.models.synthetic import synthetic_source
from localai_tfp_amd.ops import moe as MO
from localai_tfp_amd.ops.linear import QWeight
from localai_tfp_amd.ops.quant import dequantize, random_quantized
from localai_tfp_amd.formats.gguf import QType

transformers = pytest.importorskip("transformers")


def _deq(src, name):
    raw, qt, shape = src(name)
    return torch.from_numpy(np.ascontiguousarray(dequantize(raw, qt, shape)).reshape(tuple(reversed(shape))).copy()).float()


def _moe_cfg(**kw):
    base = dict(arch="qwen3moe", hidden=256, n_heads=4, n_kv_heads=2, head_dim=64, rope_dim=64, vocab=512,
                n_layers=2, n_expert=8, n_expert_used=2, expert_ffn=256, qk_norm=True, rope_base=1e6,
                rms_eps=1e-6)
    base.update(kw)
    return tiny_config(**base)


def _hf_state(cfg, src):
    sd = {"model.embed_tokens.weight": _deq(src, "token_embd.weight"),
          "model.norm.weight": _deq(src, "output_norm.weight"), "lm_head.weight": _deq(src, "output.weight")}
    for i in range(cfg.n_layers):
        p, q = f"blk.{i}.", f"model.layers.{i}."
        sd[q + "input_layernorm.weight"] = _deq(src, p + "attn_norm.weight")
        sd[q + "post_attention_layernorm.weight"] = _deq(src, p + "ffn_norm.weight")
        for a, b in (("q", "attn_q"), ("k", "attn_k"), ("v", "attn_v"), ("o", "attn_output")):
            sd[q + f"self_attn.{a}_proj.weight"] = _deq(src, p + b + ".weight")
        if cfg.qk_norm:
            sd[q + "self_attn.q_norm.weight"] = _deq(src, p + "attn_q_norm.weight")
            sd[q + "self_attn.k_norm.weight"] = _deq(src, p + "attn_k_norm.weight")
        if cfg.n_expert:
            sd[q + "mlp.gate.weight"] = _deq(src, p + "ffn_gate_inp.weight")
            g, u = _deq(src, p + "ffn_gate_exps.weight"), _deq(src, p + "ffn_up_exps.weight")
            sd[q + "mlp.experts.gate_up_proj"] = torch.cat([g, u], 1)
            sd[q + "mlp.experts.down_proj"] = _deq(src, p + "ffn_down_exps.weight")
        else:
            for a, b in (("gate", "ffn_gate"), ("up", "ffn_up"), ("down", "ffn_down")):
                sd[q + f"mlp.{a}_proj.weight"] = _deq(src, p + b + ".weight")
    return sd


def _our_logits(model, prompt):
    from test_model_gpu import _run
    return _run(model, model.device.type, prompt, [])[0]


@pytest.mark.parametrize("moe", [True, False])
def test_qwen3_family_matches_transformers(moe):
    if moe:
        from transformers import Qwen3MoeConfig as HC, Qwen3MoeForCausalLM as HM
        cfg = _moe_cfg()
        hc = HC(vocab_size=cfg.vocab, hidden_size=cfg.hidden, intermediate_size=cfg.ffn,
                moe_intermediate_size=cfg.expert_ffn, num_hidden_layers=cfg.n_layers,
                num_attention_heads=cfg.n_heads, num_key_value_heads=cfg.n_kv_heads, head_dim=cfg.head_dim,
                num_experts=cfg.n_expert, num_experts_per_tok=cfg.n_expert_used, norm_topk_prob=True,
                decoder_sparse_step=1, mlp_only_layers=[], rope_theta=cfg.rope_base, rms_norm_eps=cfg.rms_eps,
                tie_word_embeddings=False)
    else:
        from transformers import Qwen3Config as HC, Qwen3ForCausalLM as HM
        cfg = _moe_cfg(arch="qwen3", n_expert=0, n_expert_used=0, expert_ffn=0, ffn=512)
        hc = HC(vocab_size=cfg.vocab, hidden_size=cfg.hidden, intermediate_size=cfg.ffn,
                num_hidden_layers=cfg.n_layers, num_attention_heads=cfg.n_heads,
                num_key_value_heads=cfg.n_kv_heads, head_dim=cfg.head_dim, rope_theta=cfg.rope_base,
                rms_norm_eps=cfg.rms_eps, tie_word_embeddings=False)
    hc.rope_parameters = {"rope_type": "default", "rope_theta": cfg.rope_base}
    src = synthetic_source(cfg, "Q8_0", seed=3)
    hm = HM(hc).eval()
    missing, unexpected = hm.load_state_dict(_hf_state(cfg, src), strict=False)
    assert not unexpected and not [k for k in missing if "rotary" not in k], (missing, unexpected)
    ours = LlamaModel.load(cfg, src, "cpu")
    prompt = [int(x) for x in np.random.default_rng(1).integers(0, cfg.vocab, 24)]
    with torch.no_grad():
        ref = hm(torch.tensor([prompt])).logits[0, -1].float()
    got = _our_logits(ours, prompt)[0]
    rel = float((got - ref).norm() / ref.norm())
    assert rel < 2e-2, rel
    assert int(got.argmax()) == int(ref.argmax())


def test_route_ref_semantics():
    logits = torch.tensor([[0.1, 2.0, 2.0, -1.0], [3.0, 0.0, 1.0, 0.5]])
    ids, w = MO.route_ref(logits, 2, True)
    assert ids[1].tolist() == [0, 2] and set(ids[0].tolist()) == {1, 2}
    assert torch.allclose(w.sum(-1), torch.ones(2))
    _, w2 = MO.route_ref(logits, 2, False)
    assert float(w2[1].sum()) < 1.0


def test_phi3_fused_tensors_split():
    """attn_qkv / fused ffn_up (gate rows first, as ggml_swiglu splits) load into the same model as the
    separate tensors."""
    cfg = tiny_config(arch="phi3", n_layers=1)
    src = synthetic_source(cfg, "Q8_0", seed=2)

    def fused(name):
        p = name.rsplit(".", 2)[0] + "."
        if name.endswith("attn_qkv.weight"):
            parts = [src(p + f"attn_{x}.weight") for x in "qkv"]
        elif name.endswith("ffn_up.weight"):
            parts = [src(p + "ffn_gate.weight"), src(p + "ffn_up.weight")]
        elif name.endswith(("attn_q.weight", "attn_k.weight", "attn_v.weight", "ffn_gate.weight")):
            return None
        else:
            return src(name)
        raw = np.concatenate([np.asarray(r).view(np.uint8).reshape(int(np.prod(s[1:])), -1) for r, _, s in parts])
        K = parts[0][2][0]
        return raw.reshape(-1), parts[0][1], (K, sum(int(np.prod(s[1:])) for _, _, s in parts))

    a = LlamaModel.load(cfg, src, "cpu")
    b = LlamaModel.load(cfg, fused, "cpu")
    prompt = [3, 50, 7, 99, 12]
    assert torch.allclose(_our_logits(a, prompt), _our_logits(b, prompt), atol=1e-5)


def _rand_qweight(rng, qt, N, K, dev):
    raw = random_quantized(rng, qt, N, K, std=0.05).reshape(N, -1)
    return QWeight.from_ggml(raw, int(qt), N, K, dev)


@pytest.mark.gpu
@pytest.mark.parametrize("t32", [True, False])
@pytest.mark.parametrize("E,k,H,F,qt,renorm", [(8, 2, 512, 512, QType.Q4_K, True),
                                               (128, 8, 256, 768, QType.Q4_K, True),
                                               (16, 4, 256, 256, QType.Q6_K, False),
                                               (8, 2, 256, 256, QType.Q8_0, True),
                                               (16, 4, 512, 256, QType.Q5_K, True)])
def test_moe_ffn_gpu_matches_fp32(E, k, H, F, qt, renorm, t32):
    """The GPU MoE layer (fused router + route, then either the t32 kernels — grouped decode GEMV for <= 64 pairs,
    sorted grouped qmm2 above — or the row-layout qgemm16 grouped kernel) against the fp32 CPU path."""
    from localai_tfp_amd.ops.linear import ACT_DTYPE, interleave_gate_up
    rng = np.random.default_rng(E + k)
    raws = {n: random_quantized(rng, qt, r, c, std=0.05).reshape(r, -1)
            for n, r, c in (("g", E * F, H), ("u", E * F, H), ("d", E * H, F))}
    router = torch.randn(E, H) * 0.5

    def build(dev):
        g = QWeight.from_ggml(raws["g"], int(qt), E * F, H, dev)
        u = QWeight.from_ggml(raws["u"], int(qt), E * F, H, dev)
        d = QWeight.from_ggml(raws["d"], int(qt), E * H, F, dev)
        gpu = dev == "cuda"
        return MO.MoEWeights(router=router.to(dev), gate=None if gpu else g, up=None if gpu else u,
                             gate_up=interleave_gate_up(g, u) if gpu else None, down=d, n_expert=E, n_used=k,
                             ffn=F, renorm=renorm)
    wc, wg = build("cpu"), build("cuda")
    if t32:
        assert wg.to_t32()
    elif qt == QType.Q5_K:
        pytest.skip("Q5_K expert stacks run only on the t32 kernels")
    for T in (1, 3, 16, 37, 300):
        x = torch.randn(T, H).to(ACT_DTYPE)
        h0 = torch.randn(T, H)
        ref = MO.moe_ffn(wc, x.float(), h0.clone())
        got = MO.moe_ffn(wg, x.cuda(), h0.cuda().clone()).cpu()
        torch.cuda.synchronize()
        rel = float((got - ref).norm() / (ref - h0).norm())
        # the grouped decode GEMV (t32, <= 64 pairs) runs on q8 activations per 32 (llama.cpp's MMVQ numerics): the
        # activations are quantised twice (x, then the SwiGLU output), ~1 % more error than the 16-bit GEMM paths
        tol = 2.5e-2 if (t32 and T * k <= MO.GEMV_MAX_PAIRS) else 1e-2
        assert rel < tol, (T, rel)


@pytest.mark.gpu
@pytest.mark.parametrize("T", [1, 5, 37, 300])
def test_moe_router_fused_norm_gpu(T):
    """moe_ffn(norm=(h, gamma, eps)): the router kernel computes the FFN RMSNorm (and writes the normed rows the expert
    GEMMs read) — same result as the norm kernel followed by the unfused layer, and the written rows match it."""
    from localai_tfp_amd.ops import core as K
    from localai_tfp_amd.ops.linear import ACT_DTYPE, interleave_gate_up
    E, k, H, F, qt = 128, 8, 256, 768, QType.Q4_K
    rng = np.random.default_rng(3)
    raws = {n: random_quantized(rng, qt, r, c, std=0.05).reshape(r, -1)
            for n, r, c in (("g", E * F, H), ("u", E * F, H), ("d", E * H, F))}
    g = QWeight.from_ggml(raws["g"], int(qt), E * F, H, "cuda")
    u = QWeight.from_ggml(raws["u"], int(qt), E * F, H, "cuda")
    d = QWeight.from_ggml(raws["d"], int(qt), E * H, F, "cuda")
    w = MO.MoEWeights(router=(torch.randn(E, H) * 0.5).cuda(), gate=None, up=None, gate_up=interleave_gate_up(g, u),
                      down=d, n_expert=E, n_used=k, ffn=F, renorm=True)
    assert w.to_t32()
    h = torch.randn(T, H, device="cuda") * 3
    gamma = (1 + 0.2 * torch.randn(H)).cuda()
    xa = torch.empty(T, H, dtype=ACT_DTYPE, device="cuda")
    K.rmsnorm(h, gamma, 1e-6, out_bf16=xa)
    ref = MO.moe_ffn(w, xa, h.clone())
    xb = torch.empty_like(xa)
    got = MO.moe_ffn(w, xb, h.clone(), norm=(h, gamma, 1e-6))
    torch.cuda.synchronize()
    assert float((xb.float() - xa.float()).abs().max()) <= 2e-3 * float(xa.float().abs().max())
    rel = float((got - ref).norm() / (ref - h).norm())
    assert rel < 1e-2, rel


@pytest.mark.gpu
def test_moe_router_route_fused_gpu(monkeypatch):
    """MX_MOE_ROUTE_FUSE: the top-k routing inside the router launch (last workgroup of each token block, fence-free
    hand-off of the logits) selects the same experts and weights as the separate routing launch."""
    from localai_tfp_amd.ops.linear import ACT_DTYPE
    E, k, H = 128, 8, 512
    router = (torch.randn(E, H) * 0.5).cuda()
    for T in (1, 9, 64, 300):
        x = torch.randn(T, H).to(ACT_DTYPE).cuda()
        res = []
        for fuse in (False, True):
            monkeypatch.setattr(MO, "ROUTE_FUSE", fuse)
            ids = torch.empty(T, k, dtype=torch.int32, device="cuda")
            wts = torch.empty(T, k, dtype=torch.float32, device="cuda")
            logits = torch.empty(T, E, dtype=torch.float32, device="cuda")
            tk = MO._router_tickets(x.device, (T + 7) // 8) if fuse else None
            from localai_tfp_amd import _native as N
            N.ensure_act(x.dtype)
            N.kcall("mxk_moe_router", x.data_ptr(), x.stride(0), router.data_ptr(), T, H, E, k, 1, ids.data_ptr(),
                    wts.data_ptr(), logits.data_ptr(), N.ptr(tk), None, 0, None, 0.0, N.stream_ptr())
            torch.cuda.synchronize()
            res.append((ids.cpu(), wts.cpu()))
        assert torch.equal(res[0][0], res[1][0]), T
        assert torch.allclose(res[0][1], res[1][1], atol=1e-6), T


@pytest.mark.gpu
def test_moe_model_gpu_matches_cpu_and_engine():
    from localai_tfp_amd.engine.engine import EngineConfig, LLMEngine
    from localai_tfp_amd.ops.sampling import SamplingParams
    from localai_tfp_amd.tokenizer import ByteTokenizer
    from test_model_gpu import _run
    cfg = _moe_cfg(hidden=512, expert_ffn=512, n_expert=16, n_expert_used=4)
    src = synthetic_source(cfg, "Q4_K_M", seed=7)
    mc = LlamaModel.load(cfg, src, "cpu")
    mg = LlamaModel.load(cfg, src, "cuda")
    prompt = [int(x) for x in np.random.default_rng(0).integers(0, cfg.vocab, 40)]
    a = _run(mc, "cpu", prompt, [5, 99, 300])
    b = _run(mg, "cuda", prompt, [5, 99, 300])
    for x, y in zip(a, b):
        assert float((x - y).norm() / x.norm()) < 6e-2
    tok = ByteTokenizer(cfg.vocab)
    streams = []
    for graphs in (False, True):  # the MoE layer (route/sort/grouped GEMMs) inside a captured hipGraph
        eng = LLMEngine(mg, tok, EngineConfig(num_blocks=256, max_num_seqs=8, max_batched_tokens=256,
                                              max_model_len=512, use_graphs=graphs))
        outs = [eng.generate(tok.encode(f"moe prompt {i}"), SamplingParams(temperature=0.0, ignore_eos=True),
                             max_tokens=12) for i in range(2)]
        assert all(len(o.token_ids) == 12 for o in outs)
        streams.append([o.token_ids for o in outs])
    assert streams[0] == streams[1]


@pytest.mark.gpu
@pytest.mark.parametrize("t32", [True, False])
@pytest.mark.parametrize("tp", [2, 4])
def test_moe_expert_parallel_gpu(tp, t32):
    """Expert parallelism (tensor-parallel MoE layers): every rank's share computed by the GPU kernels
    with the off-rank pairs in the null bucket; the shares sum to the unsharded MoE output."""
    from localai_tfp_amd.ops.linear import ACT_DTYPE, interleave_gate_up
    E, k, H, F, qt = 8, 2, 256, 256, QType.Q4_K
    rng = np.random.default_rng(11)
    raws = {n: random_quantized(rng, qt, r, c, std=0.05).reshape(r, -1)
            for n, r, c in (("g", E * F, H), ("u", E * F, H), ("d", E * H, F))}
    router = torch.randn(E, H) * 0.5

    def build(e0, el):
        g = QWeight.from_ggml(np.ascontiguousarray(raws["g"][e0 * F:(e0 + el) * F]), int(qt), el * F, H, "cuda")
        u = QWeight.from_ggml(np.ascontiguousarray(raws["u"][e0 * F:(e0 + el) * F]), int(qt), el * F, H, "cuda")
        d = QWeight.from_ggml(np.ascontiguousarray(raws["d"][e0 * H:(e0 + el) * H]), int(qt), el * H, F, "cuda")
        w = MO.MoEWeights(router=router.cuda(), gate=None, up=None, gate_up=interleave_gate_up(g, u), down=d,
                          n_expert=E, n_used=k, ffn=F, renorm=True, e0=e0, n_local=0 if el == E else el)
        if t32:
            assert w.to_t32()
        return w
    full = build(0, E)
    shards = [build(r * E // tp, E // tp) for r in range(tp)]
    for T in (1, 5, 64):
        x = torch.randn(T, H).to(ACT_DTYPE).cuda()
        ref = MO.moe_ffn(full, x, torch.zeros(T, H, device="cuda"))
        acc = torch.zeros(T, H, device="cuda")
        for w in shards:
            y = torch.zeros(T, H, device="cuda")
            MO.moe_ffn(w, x, y)
            acc += y
        torch.cuda.synchronize()
        rel = float((acc - ref).norm() / ref.norm())
        assert rel < 1e-4, (T, rel)
