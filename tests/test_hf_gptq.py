"""GPTQ / AWQ / EXL2 HF checkpoints (vLLM `quantization: gptq / awq`, backend/python/vllm/backend.py:106-107; the
exllama2 backend's EXL2 and GPTQ, backend/python/exllama2/backend.py:49-56): models/hf.py dequantises `qweight /
qzeros / scales [/ g_idx]` and EXL2's `q_weight / q_scale / q_scale_max / q_groups / q_invperm` at load. The packed tensors
here come from an independent packer written in this test (AutoGPTQ v1 zero-point storage, act-order g_idx,
AWQ's GEMM nibble order); the loaded model's logits match transformers' forward of the same dequantised
weights. AutoGPTQ / AutoAWQ are not installed: parity with their kernels is unpinned."""
import json

import numpy as np
import pytest
import torch

from localai_tfp_amd.models.hf import AWQ_ORDER, dequant_awq, dequant_gptq
from localai_tfp_amd.models.loader import load_llm

transformers = pytest.importorskip("transformers")
from safetensors.torch import load_file, save_file  # noqa: E402

LINEARS = ("q_proj", "k_proj", "v_proj", "o_proj", "gate_proj", "up_proj", "down_proj")


def quantize(w: np.ndarray, group: int, rng, act_order: bool):
    """w [N, K] -> (q [K, N] 0..15, z [G, N] 1..15, s16 [G, N], g_idx [K]); asymmetric min/max per group."""
    N, K = w.shape
    G = K // group
    g_idx = (rng.permutation(K) // group) if act_order else np.arange(K) // group
    wt = w.T  # [K, N]
    q = np.zeros((K, N), np.int64)
    z = np.zeros((G, N), np.int64)
    s16 = np.zeros((G, N), np.float16)
    for g in range(G):
        rows = np.nonzero(g_idx == g)[0]
        blk = wt[rows]
        lo, hi = blk.min(0), blk.max(0)
        s = np.maximum((hi - lo) / 15.0, 1e-6)
        zz = np.clip(np.round(-lo / s), 1, 15)  # v1 storage keeps z >= 1 representable
        s16[g] = s.astype(np.float16)
        sf = s16[g].astype(np.float32)
        q[rows] = np.clip(np.round(blk / sf + zz), 0, 15)
        z[g] = zz
    return q, z, s16, g_idx


def pack_rows(q):  # [K, N] -> int32 [K/8, N], 8 consecutive k per word, low nibble first
    K, N = q.shape
    out = np.zeros((K // 8, N), np.uint32)
    for j in range(8):
        out |= (q[j::8].astype(np.uint32) & 0xF) << np.uint32(4 * j)
    return out.view(np.int32)


def pack_cols(v, order=None):  # [R, C] -> int32 [R, C/8]
    R, C = v.shape
    out = np.zeros((R, C // 8), np.uint32)
    for i in range(8):
        col = order[i] if order else i
        out |= (v[:, col::8].astype(np.uint32) & 0xF) << np.uint32(4 * i)
    return out.view(np.int32)


def test_gptq_and_awq_dequant_formulas():
    rng = np.random.default_rng(0)
    w = rng.standard_normal((64, 256)).astype(np.float32)
    for act in (False, True):
        q, z, s16, g_idx = quantize(w, 64, rng, act)
        ref = (s16.astype(np.float32)[g_idx] * (q - z[g_idx])).T
        got = dequant_gptq(pack_rows(q), pack_cols(z - 1), s16, g_idx if act else None, 4, 64)
        np.testing.assert_array_equal(got, ref.astype(np.float32))
        got2 = dequant_gptq(pack_rows(q), pack_cols(z), s16, g_idx if act else None, 4, 64, v2=True)
        np.testing.assert_array_equal(got2, ref.astype(np.float32))
    q, z, s16, g_idx = quantize(w, 64, rng, False)
    ref = (s16.astype(np.float32)[g_idx] * (q - z[g_idx])).T
    got = dequant_awq(pack_cols(q, AWQ_ORDER), pack_cols(z, AWQ_ORDER), s16, 4, 64)
    np.testing.assert_array_equal(got, ref.astype(np.float32))


@pytest.mark.parametrize("method", ["gptq", "gptq_actorder", "awq", "gptq_bf16"])
def test_quantized_hf_dir_matches_transformers(method, tmp_path):
    torch.manual_seed(0)
    T = transformers
    hc = T.LlamaConfig(vocab_size=320, hidden_size=128, intermediate_size=256, num_hidden_layers=2,
                       num_attention_heads=4, num_key_value_heads=2, max_position_embeddings=512)
    hc._attn_implementation = "eager"
    m = T.LlamaForCausalLM(hc).eval()
    d = tmp_path / method
    m.save_pretrained(str(d))
    sd = load_file(str(d / "model.safetensors"))
    rng = np.random.default_rng(1)
    group, act = 32, method == "gptq_actorder"
    deq = {}
    for k in list(sd):
        if not any(f".{n}.weight" in k for n in LINEARS):
            continue
        w = sd.pop(k).float().numpy()
        q, z, s16, g_idx = quantize(w, group, rng, act)
        base = k[: -len("weight")]
        if method.startswith("gptq"):
            sd[base + "qweight"] = torch.from_numpy(pack_rows(q))
            sd[base + "qzeros"] = torch.from_numpy(pack_cols(z - 1))
            sd[base + "g_idx"] = torch.from_numpy(g_idx.astype(np.int32))
        else:
            sd[base + "qweight"] = torch.from_numpy(pack_cols(q, AWQ_ORDER))
            sd[base + "qzeros"] = torch.from_numpy(pack_cols(z, AWQ_ORDER))
        if method == "gptq_bf16":  # scales stored in bf16 (numpy cannot hold them: widened at load)
            sb = torch.from_numpy(s16).to(torch.bfloat16)
            sd[base + "scales"] = sb
            s16 = sb.float().numpy()
        else:
            sd[base + "scales"] = torch.from_numpy(s16)
        deq[k] = torch.from_numpy((s16.astype(np.float32)[g_idx] * (q - z[g_idx])).T.astype(np.float32).copy())
    (d / "model.safetensors").unlink()
    save_file(sd, str(d / "model.safetensors"), metadata={"format": "pt"})
    cj = json.loads((d / "config.json").read_text())
    cj["quantization_config"] = ({"quant_method": "gptq", "bits": 4, "group_size": group, "desc_act": act, "sym": False}
                                 if method.startswith("gptq") else
                                 {"quant_method": "awq", "bits": 4, "group_size": group, "version": "gemm", "zero_point": True})
    (d / "config.json").write_text(json.dumps(cj))
    with torch.no_grad():  # the oracle: transformers on the dequantised weights
        sdm = m.state_dict()
        for k, v in deq.items():
            sdm[k].copy_(v)
        prompt = [int(x) for x in np.random.default_rng(3).integers(3, 320, 17)]
        ref = m(torch.tensor([prompt])).logits[0, -1].float()
    model, tok, cfg, _ = load_llm(str(d), "cpu", overrides={"hf_quant": "f32"})
    from test_model_gpu import _run
    got = _run(model, "cpu", prompt, [])[0][0]
    rel = float((got - ref).norm() / ref.norm())
    assert rel < 5e-3, (method, rel)


# ----------------------------------------------------------------------------------------------- EXL2 (exllamav2)
def exl2_pack(w: np.ndarray, group_bits, gs: int, rng):
    """Independent EXL2 packer: w [N, K] -> (tensors, dequantised reference [N, K]). Random row permutation, group g
    of the permuted rows quantised symmetrically at group_bits[g] bits with per-(group, column) 4-bit scale codes
    against the group's fp16 maximum scale; codes written one Python-int bitstream per column."""
    N, K = w.shape
    G = len(group_bits)
    perm = rng.permutation(K)  # packed row i holds input feature perm[i]
    wp = w[:, perm]
    words, groups, qs = [], [], np.zeros((G, N // 8), np.uint32)
    smax16 = np.zeros(G, np.float16)
    deq_p = np.zeros((N, K), np.float32)
    start = 0
    for g, b in enumerate(group_bits):
        blk = wp[:, g * gs:(g + 1) * gs]  # [N, rows]
        need = np.maximum(np.abs(blk).max(1) / (2 ** (b - 1) - 1), 1e-8)
        smax16[g] = np.float16(need.max())
        smax = float(smax16[g])
        s = np.clip(np.ceil(16 * np.sqrt(need / smax)) - 1, 0, 15).astype(np.int64)
        scale = ((s + 1) / 16.0) ** 2 * smax
        q = np.clip(np.round(blk / scale[:, None]) + 2 ** (b - 1), 0, 2 ** b - 1).astype(np.int64)
        deq_p[:, g * gs:(g + 1) * gs] = ((q - 2 ** (b - 1)) * scale[:, None]).astype(np.float32)
        for n in range(N):
            qs[g, n // 8] |= np.uint32(s[n] << (4 * (n % 8)))
        nw = blk.shape[1] * b // 32
        colw = np.zeros((nw, N), np.uint32)
        for n in range(N):
            acc = 0
            for i, c in enumerate(q[n]):
                acc |= int(c) << (i * b)
            for j in range(nw):
                colw[j, n] = (acc >> (32 * j)) & 0xFFFFFFFF
        words.append(colw)
        groups += [b, start]
        start += nw
    t = {"q_weight": np.concatenate(words).view(np.int32), "q_scale": qs.view(np.int32), "q_scale_max": smax16,
         "q_groups": np.array(groups, np.int16), "q_invperm": np.argsort(perm).astype(np.int16)}
    ref = np.empty_like(deq_p)
    ref[:, perm] = deq_p
    return t, ref


def test_exl2_dequant_formula():
    from localai_tfp_amd.models.hf import dequant_exl2
    rng = np.random.default_rng(0)
    w = rng.standard_normal((16, 384)).astype(np.float32)
    bits = [8, 8, 6, 5, 5, 4, 4, 4, 3, 3, 2, 2]  # sorted by width, as exllamav2's permutation leaves them
    t, ref = exl2_pack(w, bits, 32, rng)
    got = dequant_exl2(t["q_weight"], t["q_scale"], t["q_scale_max"], t["q_groups"], t["q_invperm"])
    np.testing.assert_allclose(got, ref, rtol=0, atol=1e-6)
    assert float(np.abs(got - w).mean()) < 0.3  # a quantisation of w (2-bit groups coarse, 8-bit ones close)


def test_exl2_hf_dir_matches_transformers(tmp_path):
    """A Llama directory with every linear in EXL2 tensors (mixed 8..2-bit groups, quant_method exl2) loads through the
    vllm / exllama2 path and matches transformers' forward of the same dequantised weights."""
    torch.manual_seed(0)
    T = transformers
    hc = T.LlamaConfig(vocab_size=320, hidden_size=128, intermediate_size=256, num_hidden_layers=2,
                       num_attention_heads=4, num_key_value_heads=2, max_position_embeddings=512)
    hc._attn_implementation = "eager"
    m = T.LlamaForCausalLM(hc).eval()
    d = tmp_path / "exl2"
    m.save_pretrained(str(d))
    sd = load_file(str(d / "model.safetensors"))
    rng = np.random.default_rng(1)
    deq = {}
    for k in list(sd):
        if not any(f".{n}.weight" in k for n in LINEARS):
            continue
        w = sd.pop(k).float().numpy()
        G = w.shape[1] // 32
        bits = sorted((8, 6, 5, 4)[i % 4] for i in range(G))[::-1]
        t, ref = exl2_pack(w, bits, 32, rng)
        base = k[: -len("weight")]
        for n, a in t.items():
            sd[base + n] = torch.from_numpy(np.ascontiguousarray(a))
        deq[k] = torch.from_numpy(ref.copy())
    (d / "model.safetensors").unlink()
    save_file(sd, str(d / "model.safetensors"), metadata={"format": "pt"})
    cj = json.loads((d / "config.json").read_text())
    cj["quantization_config"] = {"quant_method": "exl2", "version": "0.2.8", "bits": 5.75, "head_bits": 0}
    (d / "config.json").write_text(json.dumps(cj))
    with torch.no_grad():
        sdm = m.state_dict()
        for k, v in deq.items():
            sdm[k].copy_(v)
        prompt = [int(x) for x in np.random.default_rng(3).integers(3, 320, 17)]
        ref = m(torch.tensor([prompt])).logits[0, -1].float()
    model, tok, cfg, _ = load_llm(str(d), "cpu", overrides={"hf_quant": "f32"})
    from test_model_gpu import _run
    got = _run(model, "cpu", prompt, [])[0][0]
    rel = float((got - ref).norm() / ref.norm())
    assert rel < 5e-3, rel


def test_unknown_quant_method_refused(tmp_path):
    from localai_tfp_amd.models.hf import hf_source
    d = tmp_path / "q"
    d.mkdir()
    cfg = {"architectures": ["LlamaForCausalLM"], "model_type": "llama", "hidden_size": 64, "intermediate_size": 128,
           "num_hidden_layers": 1, "num_attention_heads": 4, "num_key_value_heads": 4, "vocab_size": 32,
           "rms_norm_eps": 1e-5, "max_position_embeddings": 64,
           "quantization_config": {"quant_method": "hqq"}}
    (d / "config.json").write_text(json.dumps(cfg))
    save_file({"model.embed_tokens.weight": torch.zeros(32, 64)}, str(d / "model.safetensors"), metadata={"format": "pt"})
    with pytest.raises(ValueError, match="hqq"):
        hf_source(str(d), "bf16")
