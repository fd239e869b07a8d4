"""LLM LoRA adapters (reference: backend/cpp/llama/grpc-server.cpp:2402-2410 — LoraAdapter relative to
the model directory, LoraScale default 1.0, handed to llama.cpp which scales by scale*alpha/rank).

Runtime mode (the default, as llama.cpp): adapters stay beside the untouched quantised base weights and
`B (A x)` is added to every adapted projection's output (models/lora_runtime.py); the merge modes fold them into
the GGUF weights at load (Q8_0, the base block format, or exact fp32). Checked:
runtime logits == exact-fp32-merge logits, every projection adapted, prefill + decode, CPU and GPU;
merged tensor == quantise(dequantise(W) + scale*alpha/r * B@A) byte for byte (Q4_K, Q6_K, Q8_0, F32);
llama.cpp adapter GGUF and HF PEFT safetensors name mapping (incl. the q/k rotary-row permutation);
through the gRPC worker an adapter changes the greedy output, deterministically."""
import json

import numpy as np
import pytest

from localai_tfp_amd.formats.gguf import GGUFWriter, QType
from localai_tfp_amd.models import config as C
from localai_tfp_amd.models import lora as L
from localai_tfp_amd.ops import quant as Q


def _src(tensors):
    return lambda n: tensors.get(n)


@pytest.mark.parametrize("requant", ["same", "q8_0"])
@pytest.mark.parametrize("qt", [QType.Q4_K, QType.Q6_K, QType.Q8_0, QType.F32])
def test_merge_bytes_exact(qt, requant):
    rng = np.random.default_rng(0)
    N, K, r = 64, 256, 4
    w = rng.standard_normal((N, K)).astype(np.float32) * 0.02
    raw = {QType.Q4_K: Q.quantize_q4_k, QType.Q6_K: Q.quantize_q6_k, QType.Q8_0: Q.quantize_q8_0,
           QType.F32: lambda x: x.view(np.uint8)}[qt](w).reshape(N, -1)
    a = rng.standard_normal((r, K)).astype(np.float32) * 0.1
    b = rng.standard_normal((N, r)).astype(np.float32) * 0.1
    ad = L.Adapter({"blk.0.attn_q.weight": (a, b)}, alpha=8.0, scale=0.5, path="x")
    get = L.with_adapters(_src({"blk.0.attn_q.weight": (raw, int(qt), (K, N))}), [ad], requant)
    mraw, mqt, mshape = get("blk.0.attn_q.weight")
    want = Q.dequantize(raw, qt, (K, N)) + 0.5 * 8.0 / r * (b @ a)
    if requant == "q8_0" and qt != QType.F32:
        qt = QType.Q8_0
    assert mqt == int(qt) and tuple(mshape) == (K, N)
    if qt == QType.F32:
        np.testing.assert_allclose(Q.dequantize(mraw, mqt, mshape), want, rtol=1e-6, atol=1e-7)
    else:
        ref = {QType.Q4_K: Q.quantize_q4_k, QType.Q6_K: Q.quantize_q6_k, QType.Q8_0: Q.quantize_q8_0}[qt](want)
        assert np.array_equal(np.asarray(mraw).reshape(-1), ref.reshape(-1))
    with pytest.raises(ValueError, match="not in the base model"):
        L.with_adapters(_src({}), [ad])


def _write_adapter(path, pairs, alpha):
    wr = GGUFWriter(str(path))
    wr.add("general.type", "adapter")
    wr.add("adapter.type", "lora")
    wr.add("adapter.lora.alpha", float(alpha))
    for name, (a, b) in pairs.items():
        wr.add_tensor(name + ".lora_a", a.astype(np.float32))
        wr.add_tensor(name + ".lora_b", b.astype(np.float32))
    wr.write()


def test_gguf_and_peft_loading(tmp_path):
    rng = np.random.default_rng(1)
    cfg = C.tiny_config()
    a = rng.standard_normal((8, cfg.hidden)).astype(np.float32)
    b = rng.standard_normal((cfg.q_dim, 8)).astype(np.float32)
    _write_adapter(tmp_path / "ad.gguf", {"blk.1.attn_q.weight": (a, b)}, 16)
    ad = L.load_adapter(str(tmp_path / "ad.gguf"), 0.5)
    np.testing.assert_array_equal(ad.pairs["blk.1.attn_q.weight"][0], a)
    np.testing.assert_array_equal(ad.pairs["blk.1.attn_q.weight"][1], b)
    assert ad.mult(8) == pytest.approx(0.5 * 16 / 8)

    from safetensors.numpy import save_file
    pd = tmp_path / "peft"
    pd.mkdir()
    bk = rng.standard_normal((cfg.kv_dim, 8)).astype(np.float32)
    save_file({"base_model.model.model.layers.0.self_attn.k_proj.lora_A.weight": a,
               "base_model.model.model.layers.0.self_attn.k_proj.lora_B.weight": bk,
               "base_model.model.model.layers.1.mlp.down_proj.lora_A.weight": a[:, :1].repeat(cfg.ffn, 1),
               "base_model.model.model.layers.1.mlp.down_proj.lora_B.weight": bk[:, :1].repeat(1, 1)[:1].repeat(cfg.hidden, 0)},
              str(pd / "adapter_model.safetensors"))
    (pd / "adapter_config.json").write_text(json.dumps({"lora_alpha": 32, "r": 8}))
    ad = L.load_adapter(str(pd), 1.0, cfg)
    assert set(ad.pairs) == {"blk.0.attn_k.weight", "blk.1.ffn_down.weight"} and ad.alpha == 32
    hd = cfg.head_dim
    want = bk.reshape(cfg.n_kv_heads, 2, hd // 2, 8).swapaxes(1, 2).reshape(cfg.kv_dim, 8)
    np.testing.assert_array_equal(ad.pairs["blk.0.attn_k.weight"][1], want)  # GGUF rotary row order


def _predict(adapter=None, scale=0.0, tmp=None, device="cpu"):
    from localai_tfp_amd.grpc import pb
    from localai_tfp_amd.grpc.client import BackendClient
    from localai_tfp_amd.grpc.server import AioServer
    from localai_tfp_amd.workers.llm import LLMServicer
    svc = LLMServicer(device=device)
    server = AioServer(svc, "127.0.0.1:0", max_workers=4)
    c = BackendClient(f"127.0.0.1:{server.port}")
    try:
        kw = dict(LoraAdapter=adapter, LoraScale=scale, ModelPath=str(tmp)) if adapter else {}
        r = c.load_model(pb.ModelOptions(Model="synthetic:tiny", ContextSize=256, **kw))
        assert r.success, r.message
        return c.predict(pb.PredictOptions(Prompt="Hello world", Tokens=12, Temperature=0.0, IgnoreEOS=True)).message
    finally:
        c.close()
        svc.engine.shutdown()
        server.stop()


def test_worker_lora_changes_output(tmp_path):
    rng = np.random.default_rng(2)
    cfg = C.tiny_config()
    pairs = {f"blk.{i}.{n}.weight": (rng.standard_normal((4, k)).astype(np.float32),
                                     rng.standard_normal((nout, 4)).astype(np.float32))
             for i in range(cfg.n_layers)
             for n, k, nout in (("attn_v", cfg.hidden, cfg.kv_dim), ("ffn_down", cfg.ffn, cfg.hidden))}
    _write_adapter(tmp_path / "style.gguf", pairs, 4)
    base = _predict()
    assert _predict("style.gguf", 1.0, tmp_path) != base
    assert _predict("style.gguf", 1.0, tmp_path) == _predict("style.gguf", 1.0, tmp_path)


@pytest.mark.gpu
def test_worker_lora_gpu(tmp_path):
    """Merged Q8_0 tensors run on the native quantised GEMM/GEMV kernels inside the hipGraph decode."""
    rng = np.random.default_rng(3)
    cfg = C.tiny_config()
    pairs = {f"blk.{i}.attn_q.weight": (rng.standard_normal((8, cfg.hidden)).astype(np.float32),
                                        rng.standard_normal((cfg.q_dim, 8)).astype(np.float32))
             for i in range(cfg.n_layers)}
    _write_adapter(tmp_path / "q.gguf", pairs, 8)
    base = _predict(device="cuda:0")
    a = _predict("q.gguf", 1.0, tmp_path, device="cuda:0")
    assert a != base and a == _predict("q.gguf", 1.0, tmp_path, device="cuda:0")


def _all_proj_adapter(path, cfg, rng, r=4, layers=None):
    dims = {"attn_q": (cfg.hidden, cfg.q_dim), "attn_k": (cfg.hidden, cfg.kv_dim), "attn_v": (cfg.hidden, cfg.kv_dim),
            "attn_output": (cfg.q_dim, cfg.hidden), "ffn_gate": (cfg.hidden, cfg.ffn), "ffn_up": (cfg.hidden, cfg.ffn),
            "ffn_down": (cfg.ffn, cfg.hidden)}
    pairs = {f"blk.{i}.{n}.weight": (rng.standard_normal((r, k)).astype(np.float32) * 0.05,
                                     rng.standard_normal((nout, r)).astype(np.float32) * 0.05)
             for i in (layers if layers is not None else range(cfg.n_layers)) for n, (k, nout) in dims.items()}
    _write_adapter(path, pairs, 2 * r)


def _runtime_vs_merged(tmp_path, device, model="synthetic:tiny"):
    import torch
    from localai_tfp_amd.models.loader import SYNTHETIC, load_llm
    from test_model_gpu import _run
    cfg = SYNTHETIC[model.split(":")[1]]
    _all_proj_adapter(tmp_path / "a.gguf", cfg, np.random.default_rng(7))
    _all_proj_adapter(tmp_path / "b.gguf", cfg, np.random.default_rng(8), r=2, layers=[0])
    ads = [(str(tmp_path / "a.gguf"), 0.7), (str(tmp_path / "b.gguf"), 1.3)]
    rng = np.random.default_rng(0)
    prompt, forced = rng.integers(0, cfg.vocab, 19).tolist(), rng.integers(0, cfg.vocab, 3).tolist()
    outs = {}
    for mode in ("runtime", "f32", None):
        ov = {"lora": ads, "lora_requant": mode} if mode else {}
        m, _, _, _ = load_llm(model, device, overrides=ov)
        if mode == "runtime":
            assert all(L.lora is not None and L.lora.any for L in m.layers)
        outs[mode] = _run(m, torch.device(device), prompt, forced)
        del m
    for got, want, base in zip(outs["runtime"], outs["f32"], outs[None]):
        rel = float((got - want).norm() / want.norm())
        assert rel < (1e-3 if device == "cpu" else 2e-2), rel  # q-kernel vs dense fp32 rounding
        assert float((base - want).norm() / want.norm()) > 10 * rel  # the adapters do change the logits


def test_runtime_lora_matches_exact_merge(tmp_path):
    _runtime_vs_merged(tmp_path, "cpu")


@pytest.mark.gpu
def test_runtime_lora_matches_exact_merge_gpu(tmp_path):
    """GPU: the LoRA GEMMs run beside the quantised qmm/qmv kernels (batch-1 GEMV path, fused prologues off where
    the update needs the normed rows; prefill path with the gated activation after the update)."""
    _runtime_vs_merged(tmp_path, "cuda:0")


def test_runtime_lora_pipeline_stage(tmp_path):
    """A pipeline stage holding blocks l0..l1 attaches only its own blocks' adapters, at local indices."""
    from localai_tfp_amd.models import lora_runtime as LRT
    from localai_tfp_amd.models.llama import LlamaModel
    from localai_tfp_amd.models.loader import SYNTHETIC
    from localai_tfp_amd.models.synthetic import synthetic_source
    cfg = SYNTHETIC["tiny-4l"]
    _all_proj_adapter(tmp_path / "a.gguf", cfg, np.random.default_rng(3), layers=[2])
    m = LlamaModel.load(cfg, synthetic_source(cfg, "Q4_K_M", seed=1), "cpu", layer_range=(1, 3))
    n = LRT.build(m, [L.load_adapter(str(tmp_path / "a.gguf"), 1.0, cfg)], l0=1)
    assert n == 7 and m.layers[0].lora is None and m.layers[1].lora.any
