"""fp8 (OCP e4m3) paged KV cache — the reference's `cache_type_k` / `cache_type_v` 8-bit cache types
(llama.cpp `--cache-type-k q8_0`), stored as gfx950-native fp8: rope_kv.hip writes saturated e4m3
bytes, attention.hip widens them in registers (decode) or while staging K/V tiles to LDS (prefill).

Oracles: the fp32 CPU path over the SAME fp8 cache contents (kernels vs reference read identical
bytes), torch's float8_e4m3fn cast for the stores, and the bf16-cache model for end-to-end drift."""
import math

import numpy as np
import pytest
import torch

from localai_tfp_amd.engine.engine import EngineConfig, LLMEngine, kv_torch_dtype
from localai_tfp_amd.engine.kv_cache import KVCache
from localai_tfp_amd.models.config import tiny_config
from localai_tfp_amd.models.llama import ForwardBatch, LlamaModel, Workspace
from localai_tfp_amd.models.synthetic import synthetic_source
from localai_tfp_amd.ops import core as K
from localai_tfp_amd.ops.sampling import SamplingParams
from localai_tfp_amd.tokenizer import ByteTokenizer

F8 = torch.float8_e4m3fn


def test_cache_type_names():
    # llama.cpp's block formats are stored as real blocks (uint8 rows, tests/test_kv_quant.py); fp8 stays e4m3
    assert kv_torch_dtype("q8_0") == torch.uint8 and kv_torch_dtype("q4_0") == torch.uint8 and kv_torch_dtype("fp8") == F8
    assert kv_torch_dtype("f16") == torch.bfloat16 and kv_torch_dtype("") == torch.bfloat16
    with pytest.raises(ValueError):
        kv_torch_dtype("int3")


def test_fp8_store_saturates():
    x = torch.tensor([1000.0, -1000.0, 3.3, 0.01])
    y = K._to_cache(x, F8).float()
    assert y[0] == 448 and y[1] == -448 and abs(float(y[2]) - 3.25) < 1e-6


def _prefill_logits(model, dev, prompt, kv_dtype):
    cfg = model.cfg
    bs = 16
    kv = KVCache(cfg.n_layers, 64, model.n_kv, bs, cfg.head_dim, dev, kv_dtype)
    ws = Workspace(cfg, 256, 8, dev)
    P = len(prompt)
    blocks = list(range(1, 2 + P // bs))
    bt = torch.tensor([blocks], dtype=torch.int32, device=dev)
    slots = torch.tensor([blocks[p // bs] * bs + p % bs for p in range(P)], dtype=torch.int32, device=dev)
    fb = ForwardBatch(torch.tensor(prompt, dtype=torch.int32, device=dev), torch.arange(P, dtype=torch.int32, device=dev),
                      slots, torch.tensor([P - 1], dtype=torch.int32, device=dev), n_decode=0, pf_block_tables=bt,
                      pf_cu_q=torch.tensor([0, P], dtype=torch.int32, device=dev),
                      pf_ctx_lens=torch.tensor([P], dtype=torch.int32, device=dev), pf_q_lens_host=[P],
                      pf_ctx_lens_host=[P])
    out = [model.forward(fb, kv, ws).float().cpu().clone()]
    # one decode step on top (reads the fp8 prefix through the decode kernel)
    p = P
    fb = ForwardBatch(torch.tensor([7], dtype=torch.int32, device=dev), torch.tensor([p], dtype=torch.int32, device=dev),
                      torch.tensor([blocks[p // bs] * bs + p % bs], dtype=torch.int32, device=dev),
                      torch.tensor([0], dtype=torch.int32, device=dev), n_decode=1, dec_block_tables=bt,
                      dec_seq_lens=torch.tensor([p + 1], dtype=torch.int32, device=dev), dec_max_len=p + 1)
    out.append(model.forward(fb, kv, ws).float().cpu().clone())
    return out


def test_fp8_cache_model_drift_cpu():
    cfg = tiny_config(n_layers=2)
    m = LlamaModel.load(cfg, synthetic_source(cfg, "Q8_0", seed=3), "cpu")
    prompt = [int(x) for x in np.random.default_rng(0).integers(0, cfg.vocab, 30)]
    a = _prefill_logits(m, "cpu", prompt, torch.bfloat16)
    b = _prefill_logits(m, "cpu", prompt, F8)
    for x, y in zip(a, b):
        assert float((x - y).norm() / x.norm()) < 5e-2


def test_engine_fp8_kv_cpu():
    cfg = tiny_config(n_layers=2)
    m = LlamaModel.load(cfg, synthetic_source(cfg, "Q4_K_M", seed=11), "cpu")
    tok = ByteTokenizer(cfg.vocab)
    e = LLMEngine(m, tok, EngineConfig(num_blocks=128, max_num_seqs=4, max_batched_tokens=64, max_model_len=256,
                                       kv_dtype="fp8"))
    assert e.kv.k.dtype == F8
    o = e.generate(tok.encode("fp8 cache"), SamplingParams(temperature=0.0, ignore_eos=True), max_tokens=8)
    assert len(o.token_ids) == 8


@pytest.mark.gpu
def test_rope_kv_fp8_gpu():
    T, Hq, Hkv, D, bs, nb = 37, 8, 2, 128, 16, 8
    g = torch.Generator().manual_seed(0)
    qkv = torch.randn(T, (Hq + 2 * Hkv) * D, generator=g) * 4
    pos = torch.arange(T, dtype=torch.int32) + 5
    slots = torch.randperm(nb * bs, generator=g)[:T].int()
    inv, af = K.rope_inv_freq(D, 500000.0)
    outs = []
    for dev in ("cpu", "cuda"):
        q = torch.empty(T, Hq, D, dtype=torch.bfloat16, device=dev)
        kc = torch.zeros(nb, Hkv, bs, D, dtype=F8, device=dev)
        vc = torch.zeros_like(kc)
        K.rope_kv(qkv.to(dev), None, pos.to(dev), slots.to(dev), inv.to(dev), af, Hq, Hkv, D, D, False, q, kc, vc, bs)
        outs.append((kc.cpu().float(), vc.cpu().float()))
    for a, b in zip(*outs):
        assert float((a - b).norm() / a.norm()) < 2e-2
        assert float((a == b).float().mean()) > 0.97  # same bytes up to rounding of near-ties


@pytest.mark.gpu
@pytest.mark.parametrize("D,Hq,Hkv", [(128, 32, 8), (64, 16, 4), (256, 8, 4)])
def test_attention_fp8_cache_gpu(D, Hq, Hkv):
    bs, nb = 16, 512
    g = torch.Generator().manual_seed(D)
    kc = (torch.randn(nb, Hkv, bs, D, generator=g) * 2).to(F8)
    vc = torch.randn(nb, Hkv, bs, D, generator=g).to(F8)
    scale = 1 / math.sqrt(D)

    def rel(a, b):
        return float((a.float().cpu() - b.float()).norm() / b.float().norm())

    lens = [1, 40, 700, 1300]
    B = len(lens)
    maxb = max((l + bs - 1) // bs for l in lens)
    bt = (torch.randperm(nb - 1, generator=g)[: B * maxb] + 1).view(B, maxb).int()
    seq = torch.tensor(lens, dtype=torch.int32)
    q = torch.randn(B, Hq, D, generator=g).bfloat16()
    ref = torch.empty(B, Hq, D)
    K.attn_decode(q, kc, vc, bt, seq, scale, ref)
    for impl in ("mfma", "valu"):
        out = torch.empty(B, Hq, D, dtype=torch.bfloat16, device="cuda")
        K.attn_decode(q.cuda(), kc.cuda(), vc.cuda(), bt.cuda(), seq.cuda(), scale, out, impl=impl)
        assert rel(out, ref) < 1.5e-2, impl
    q_lens, ctx = [37, 1, 130, 64], [37, 20, 300, 200]
    S = len(q_lens)
    maxb = max((c + bs - 1) // bs for c in ctx)
    bt = (torch.randperm(nb - 1, generator=g)[: S * maxb] + 1).view(S, maxb).int()
    cu = torch.tensor([0] + list(np.cumsum(q_lens)), dtype=torch.int32)
    T = int(cu[-1])
    q = torch.randn(T, Hq, D, generator=g).bfloat16()
    ctx_t = torch.tensor(ctx, dtype=torch.int32)
    ref = torch.empty(T, Hq, D)
    K.attn_prefill(q, kc, vc, bt, cu, ctx_t, scale, ref, q_lens, ctx)
    for vmode in (0, 1):
        out = torch.empty(T, Hq, D, dtype=torch.bfloat16, device="cuda")
        K.attn_prefill(q.cuda(), kc.cuda(), vc.cuda(), bt.cuda(), cu.cuda(), ctx_t.cuda(), scale, out, q_lens, ctx,
                       vmode=vmode)
        assert rel(out, ref) < 1.5e-2, vmode


@pytest.mark.gpu
def test_model_and_engine_fp8_kv_gpu():
    cfg = tiny_config(n_layers=2, hidden=512, n_heads=4, n_kv_heads=2, head_dim=128, rope_dim=128)
    src = synthetic_source(cfg, "Q4_K_M", seed=4)
    mc, mg = LlamaModel.load(cfg, src, "cpu"), LlamaModel.load(cfg, src, "cuda")
    prompt = [int(x) for x in np.random.default_rng(1).integers(0, cfg.vocab, 45)]
    a = _prefill_logits(mc, "cpu", prompt, F8)
    b = _prefill_logits(mg, "cuda", prompt, F8)
    for x, y in zip(a, b):
        assert float((x - y).norm() / x.norm()) < 6e-2
    tok = ByteTokenizer(cfg.vocab)
    e = LLMEngine(mg, tok, EngineConfig(num_blocks=256, max_num_seqs=8, max_batched_tokens=256, max_model_len=512,
                                        kv_dtype="fp8"))
    outs = [e.generate(tok.encode(f"fp8 kv {i}"), SamplingParams(temperature=0.0, ignore_eos=True), max_tokens=16)
            for i in range(3)]
    assert all(len(o.token_ids) == 16 for o in outs) and e.stats["graph_steps"] > 0
