"""Lumina-Image 2.0 (diffusers Lumina2Text2ImgPipeline, backend/python/diffusers/backend.py:35,213-216).

* the Gemma-2 text encoder (a bare `Gemma2Model` in `text_encoder/`) read at hidden_states[-2] through the
  repo's LLM engine matches transformers' own forward of the same weights;
* the Next-DiT transformer matches a float64 re-statement of diffusers' Lumina2Transformer2DModel written
  here independently (complex-number RoPE, repeat-based grouped-query attention, sandwich norms);
* a synthetic directory in diffusers' layout (model_index.json, transformer/, text_encoder/, tokenizer/,
  vae/, scheduler/) loads and generates through the diffusion worker.
diffusers itself is not installed: parity with its images stays unpinned."""
import json
import math

import numpy as np
import pytest
import torch

from localai_tfp_amd.models.diffusion import lumina2 as LU

transformers = pytest.importorskip("transformers")


def _ref_forward(tr: LU.Lumina2Transformer, x, t, cap):
    c = tr.cfg
    sd = {k: v.double() for k, v in tr.state_dict().items()}
    D, Hq, Hk, hd, p = c.hidden, c.heads, c.kv_heads, c.head_dim, c.patch

    def rmsn(v, w, eps=c.eps):
        return v * torch.rsqrt(v.pow(2).mean(-1, keepdim=True) + eps) * w

    def linear(v, name, bias=True):
        y = v @ sd[name + ".weight"].T
        return y + sd[name + ".bias"] if bias and name + ".bias" in sd else y

    silu = torch.nn.functional.silu
    half = 128
    freqs = torch.exp(-math.log(10000.0) * torch.arange(half, dtype=torch.float64) / half)
    a = float(t) * freqs
    tproj = torch.cat([torch.cos(a), torch.sin(a)])[None]
    temb = linear(silu(linear(tproj, "time_caption_embed.timestep_embedder.linear_1")),
                  "time_caption_embed.timestep_embedder.linear_2")
    ctx = linear(rmsn(cap.double(), sd["time_caption_embed.caption_embedder.0.weight"]),
                 "time_caption_embed.caption_embedder.1")
    C, H, W = x.shape
    hp, wp = H // p, W // p
    tc = cap.shape[0]
    tables = []
    for d, n in zip(c.axes, c.axes_lens):
        f = 1.0 / c.theta ** (torch.arange(0, d, 2, dtype=torch.float64)[: d // 2] / d)
        tables.append(torch.polar(torch.ones(n, d // 2, dtype=torch.float64), torch.outer(torch.arange(n).double(), f)))
    ids = []
    for i in range(tc):
        ids.append((i, 0, 0))
    for r in range(hp):
        for q in range(wp):
            ids.append((tc, r, q))
    fc = torch.stack([torch.cat([tables[a][ii[a]] for a in range(3)]) for ii in ids])  # [L, hd/2] complex

    def rope(v, f):
        vc = torch.view_as_complex(v.reshape(*v.shape[:-1], -1, 2).contiguous())
        return torch.view_as_real(vc * f[:, None, :]).flatten(2)

    def attn(pre, xn, f):
        L = xn.shape[0]
        q = linear(xn, pre + "attn.to_q", False).view(L, Hq, hd)
        k = linear(xn, pre + "attn.to_k", False).view(L, Hk, hd)
        v = linear(xn, pre + "attn.to_v", False).view(L, Hk, hd)
        q, k = rmsn(q, sd[pre + "attn.norm_q.weight"]), rmsn(k, sd[pre + "attn.norm_k.weight"])
        q, k = rope(q, f), rope(k, f)
        n_rep = Hq // Hk
        k = k.unsqueeze(2).repeat(1, 1, n_rep, 1).flatten(1, 2)
        v = v.unsqueeze(2).repeat(1, 1, n_rep, 1).flatten(1, 2)
        s = torch.einsum("qhd,khd->hqk", q, k) / math.sqrt(hd)
        o = torch.einsum("hqk,khd->qhd", torch.softmax(s, -1), v).reshape(L, Hq * hd)
        return linear(o, pre + "attn.to_out.0", False)

    def block(pre, h, f, modulated):
        if modulated:
            e = linear(silu(temb), pre + "norm1.linear")
            s_msa, g_msa, s_mlp, g_mlp = e.chunk(4, dim=1)
            xn = rmsn(h, sd[pre + "norm1.norm.weight"]) * (1 + s_msa)
        else:
            xn = rmsn(h, sd[pre + "norm1.weight"])
        a = rmsn(attn(pre, xn, f), sd[pre + "norm2.weight"])
        h = h + (torch.tanh(g_msa) * a if modulated else a)
        y = rmsn(h, sd[pre + "ffn_norm1.weight"])
        if modulated:
            y = y * (1 + s_mlp)
        ff = linear(silu(linear(y, pre + "feed_forward.linear_1", False)) * linear(y, pre + "feed_forward.linear_3", False),
                    pre + "feed_forward.linear_2", False)
        ff = rmsn(ff, sd[pre + "ffn_norm2.weight"])
        return h + (torch.tanh(g_mlp) * ff if modulated else ff)

    img = x.double().view(C, hp, p, wp, p).permute(1, 3, 2, 4, 0).reshape(hp * wp, -1)
    h = linear(img, "x_embedder")
    for i in range(c.refiner_layers):
        ctx = block(f"context_refiner.{i}.", ctx, fc[:tc], False)
    for i in range(c.refiner_layers):
        h = block(f"noise_refiner.{i}.", h, fc[tc:], True)
    j = torch.cat([ctx, h])
    for i in range(c.layers):
        j = block(f"layers.{i}.", j, fc, True)
    scale = linear(silu(temb), "norm_out.linear_1")
    y = torch.nn.functional.layer_norm(j[tc:], (D,), eps=1e-6) * (1 + scale)
    out = linear(y, "norm_out.linear_2")
    return out.view(hp, wp, p, p, C).permute(4, 0, 2, 1, 3).reshape(C, H, W)


def _synthetic_tr(device="cpu", dtype=torch.float32, seed=1):
    from localai_tfp_amd.models.diffusion.nn import cast_module, init_synthetic
    with torch.device(device):
        tr = LU.Lumina2Transformer(LU.LUMINA2_TEST)
    init_synthetic(tr, seed, std=0.05)
    with torch.no_grad():
        for n, prm in tr.named_parameters():
            if n.endswith("norm.weight") or ".norm" in n or n.endswith("0.weight") and "caption" in n:
                prm.copy_(1 + 0.2 * torch.randn_like(prm))
    return cast_module(tr, device, dtype).eval()


def test_lumina2_transformer_matches_reference():
    tr = _synthetic_tr()
    g = torch.Generator().manual_seed(0)
    x = torch.randn(16, 12, 16, generator=g)
    cap = torch.randn(7, LU.LUMINA2_TEST.cap_dim, generator=g)
    t = torch.tensor(0.37)
    got = tr(x, t, cap)
    ref = _ref_forward(tr, x, t, cap).float()
    rel = float((got - ref).norm() / ref.norm())
    assert rel < 1e-4, rel


def _gemma_dir(tmp_path):
    T = transformers
    hc = T.Gemma2Config(vocab_size=300, hidden_size=64, intermediate_size=128, num_hidden_layers=3,
                        num_attention_heads=2, num_key_value_heads=1, head_dim=32, query_pre_attn_scalar=32,
                        sliding_window=16, attn_logit_softcapping=50.0, final_logit_softcapping=30.0,
                        hidden_activation="gelu_pytorch_tanh", max_position_embeddings=512)
    hc._attn_implementation = "eager"
    torch.manual_seed(0)
    m = T.Gemma2Model(hc).eval()
    with torch.no_grad():
        for n, prm in m.named_parameters():
            if "norm" in n:
                prm.add_(torch.randn_like(prm) * 0.2)
    d = tmp_path / "text_encoder"
    m.save_pretrained(str(d))
    return m, d


def test_gemma2_text_encoder_penultimate_hidden(tmp_path):
    """Bare Gemma2Model directory (no `model.` prefix, no lm_head) -> hidden_states[-2] equals transformers'."""
    from localai_tfp_amd.models.hf import hf_source
    from localai_tfp_amd.models.llama import LlamaModel
    hm, d = _gemma_dir(tmp_path)
    ids = [2, 17, 99, 45, 3, 250, 8, 61, 7, 7, 140, 33, 21, 90, 5, 11, 12, 200, 1]  # > sliding window
    with torch.no_grad():
        ref = hm(torch.tensor([ids]), output_hidden_states=True).hidden_states
    cfg, src = hf_source(str(d), "f32")
    m = LlamaModel.load(cfg, src, "cpu")
    got = m.prompt_hidden(ids, cfg.n_layers - 1)
    r = ref[-2][0].float()
    # the engine's 16-bit GEMM operands (CPU path mirrors the GPU numerics): same bound as test_hf_loader
    assert float((got - r).norm() / r.norm()) < 5e-3
    fin = m.prompt_hidden(ids)  # last_hidden_state (final norm)
    assert float((fin - ref[-1][0]).norm() / ref[-1][0].norm()) < 5e-3


def _tokenizer_dir(d):
    from tokenizers import Tokenizer, decoders, models, pre_tokenizers, trainers
    d.mkdir(parents=True)
    tk = Tokenizer(models.BPE())
    tk.pre_tokenizer = pre_tokenizers.ByteLevel(add_prefix_space=False)
    tk.decoder = decoders.ByteLevel()
    tr = trainers.BpeTrainer(vocab_size=290, special_tokens=["<pad>", "<eos>", "<bos>"],
                             initial_alphabet=pre_tokenizers.ByteLevel.alphabet())
    tk.train_from_iterator(["a photo of a red fox in the snow " * 10], tr)
    tk.save(str(d / "tokenizer.json"))
    (d / "tokenizer_config.json").write_text(json.dumps({"bos_token": "<bos>", "eos_token": "<eos>",
                                                         "add_bos_token": True}))


def _write_dir(tmp_path):
    from safetensors.torch import save_file
    from localai_tfp_amd.models.diffusion.nn import init_synthetic
    from localai_tfp_amd.models.diffusion.vae import VAE_TEST, AutoencoderKL, VAEConfig
    root = tmp_path / "lumina2"
    root.mkdir()
    (root / "model_index.json").write_text(json.dumps({"_class_name": "Lumina2Pipeline"}))
    c = LU.Lumina2Config(hidden=192, layers=2, refiner_layers=1, heads=2, kv_heads=1, multiple_of=64, cap_dim=64)
    tr = LU.Lumina2Transformer(c)
    init_synthetic(tr, 3)
    (root / "transformer").mkdir()
    save_file({k: v.contiguous() for k, v in tr.state_dict().items()}, str(root / "transformer" / "model.safetensors"))
    (root / "transformer" / "config.json").write_text(json.dumps({
        "_class_name": "Lumina2Transformer2DModel", "patch_size": 2, "in_channels": 16, "hidden_size": 192,
        "num_layers": 2, "num_refiner_layers": 1, "num_attention_heads": 2, "num_kv_heads": 1, "multiple_of": 64,
        "ffn_dim_multiplier": None, "norm_eps": 1e-5, "axes_dim_rope": [32, 32, 32], "axes_lens": [300, 512, 512],
        "cap_feat_dim": 64}))
    _, _ = _gemma_dir(root)
    _tokenizer_dir(root / "tokenizer")
    vc = VAEConfig(latent=16, channels=VAE_TEST.channels, layers=1, groups=8, scaling=0.3611, shift=0.1159)
    vae = AutoencoderKL(vc)
    init_synthetic(vae, 5)
    (root / "vae").mkdir()
    save_file({k: v.contiguous() for k, v in vae.state_dict().items()}, str(root / "vae" / "model.safetensors"))
    (root / "vae" / "config.json").write_text(json.dumps({
        "latent_channels": 16, "block_out_channels": list(VAE_TEST.channels), "layers_per_block": 1,
        "norm_num_groups": 8, "scaling_factor": 0.3611, "shift_factor": 0.1159, "use_quant_conv": False}))
    (root / "scheduler").mkdir()
    (root / "scheduler" / "scheduler_config.json").write_text(json.dumps({"shift": 6.0, "use_dynamic_shifting": False}))
    return root, tr


def test_lumina2_diffusers_dir_through_worker(tmp_path):
    # the text encoder's width must equal cap_feat_dim: 64
    root, tr = _write_dir(tmp_path)
    from localai_tfp_amd.grpc import pb
    from localai_tfp_amd.workers.diffusion import DiffusionServicer
    s = DiffusionServicer(device="cpu")
    r = s.LoadModel(pb.ModelOptions(Model=str(root)), None)
    assert r.success, r.message
    assert isinstance(s.pipe, LU.Lumina2Pipeline) and s.defaults["cfg_scale"] == 4.0
    sd = s.pipe.tr.state_dict()
    assert all(torch.equal(sd[k], v) for k, v in tr.state_dict().items())
    dst = str(tmp_path / "o.png")
    r = s.GenerateImage(pb.GenerateImageRequest(positive_prompt="a red fox", negative_prompt="blurry", width=64,
                                                height=64, step=2, seed=3, dst=dst), None)
    assert r.success, r.message
    from PIL import Image
    with Image.open(dst) as im:
        assert im.size == (64, 64)


def test_lumina2_synthetic_pipeline_type():
    from localai_tfp_amd.grpc import pb
    from localai_tfp_amd.workers.diffusion import DiffusionServicer
    s = DiffusionServicer(device="cpu")
    r = s.LoadModel(pb.ModelOptions(Model="synthetic:lumina2-test", PipelineType="Lumina2Text2ImgPipeline"), None)
    assert r.success, r.message
    from localai_tfp_amd.models.diffusion.pipeline import GenParams
    a = s.pipe.generate("x", GenParams(width=32, height=32, steps=2, cfg_scale=4.0, seed=1))
    b = s.pipe.generate("x", GenParams(width=32, height=32, steps=2, cfg_scale=4.0, seed=1))
    assert torch.equal(a, b) and a.shape == (3, 32, 32)


@pytest.mark.gpu
def test_lumina2_transformer_gpu():
    """bf16 on the repo kernels (GQA q/k norm + RoPE at head dim 96, grouped-query flash attention) vs fp32 CPU."""
    import copy
    from localai_tfp_amd.models.diffusion.nn import cast_module
    tr = _synthetic_tr()  # weights drawn on the CPU (a CUDA generator would draw different ones)
    trg = cast_module(copy.deepcopy(tr), "cuda", torch.bfloat16)
    g = torch.Generator().manual_seed(0)
    x = torch.randn(16, 24, 32, generator=g)
    cap = torch.randn(19, LU.LUMINA2_TEST.cap_dim, generator=g)
    t = torch.tensor(0.61)
    ref = tr(x, t, cap)
    got = trg(x.cuda(), t.cuda(), cap.cuda().bfloat16()).cpu()
    rel = float((got - ref).norm() / ref.norm())
    assert rel < 3e-2, rel


@pytest.mark.gpu
def test_qk_norm_rope_gqa_kernel():
    torch.manual_seed(1)
    rows, Hq, Hk, hd = 37, 6, 2, 96
    x = torch.randn(rows, (Hq + 2 * Hk) * hd).bfloat16()
    wq, wk = 1 + 0.1 * torch.randn(hd), 1 + 0.1 * torch.randn(hd)
    cs = LU.rope_table(LU.position_ids(5, 4, 8), (32, 32, 32), 10000.0)
    ref = LU.norm_rope_(x.clone(), Hq, Hk, hd, wq, wk, cs, 1e-5)
    got = LU.norm_rope_(x.cuda(), Hq, Hk, hd, wq.cuda(), wk.cuda(), cs.cuda(), 1e-5).cpu()
    assert float((got.float() - ref.float()).abs().max()) < 3e-2
    assert torch.equal(got[:, (Hq + Hk) * hd:], x[:, (Hq + Hk) * hd:])  # v untouched
