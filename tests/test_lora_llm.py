"""LLM LoRA adapters (reference: backend/cpp/llama/grpc-server.cpp:2402-2410 — LoraAdapter relative to
the model directory, LoraScale default 1.0, handed to llama.cpp which scales by scale*alpha/rank).

Adapters are merged into the GGUF weights at load and re-quantised (Q8_0 by default, or the base block
format). Checked:
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
