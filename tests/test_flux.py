"""Flux transformer + pipeline: the fused forward (one modulation GEMM, fused QKV / QKV|MLP GEMMs,
in-place QK-norm + RoPE) vs a plain re-statement of diffusers' FluxTransformer2DModel math, the
qk_norm_rope HIP kernel vs fp32, pack/unpack, schedules, and synthetic txt2img on CPU / GPU.

Parity note: diffusers is not importable here, so the oracle is the diffusers formulation written
out below (AdaLayerNormZero / Single / Continuous, FluxPosEmbed + apply_rotary_emb, joint
[text; image] attention); "parity unpinned" against diffusers outputs themselves."""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from localai_tfp_amd.models.diffusion import flux as FX
from localai_tfp_amd.models.diffusion.nn import init_synthetic, timestep_embedding


def _ref_forward(m: FX.FluxTransformer, x, img_ids, t, ctx, pooled, guidance):
    c = m.cfg
    D, H, hd = c.dim, c.heads, c.head_dim
    B, S, _ = x.shape
    T = ctx.shape[1]
    lin = lambda mod, v: F.linear(v, mod.weight.float(), mod.bias.float())  # noqa: E731
    te = m.time_text_embed
    emb = lambda e, v: lin(e.linear_2, F.silu(lin(e.linear_1, v)))  # noqa: E731
    temb = emb(te.timestep_embedder, timestep_embedding(t * 1000, 256))
    if c.guidance:
        temb = temb + emb(te.guidance_embedder, timestep_embedding(guidance * 1000, 256))
    temb = temb + emb(te.text_embedder, pooled)
    ids = torch.cat([torch.zeros(T, 3), img_ids], 0)
    cos, sin = [], []
    for i, d in enumerate(c.axes):
        fr = 1.0 / c.theta ** (torch.arange(0, d, 2, dtype=torch.float64) / d)
        a = ids[:, i].double()[:, None] * fr[None]
        cos.append(a.cos().repeat_interleave(2, 1))
        sin.append(a.sin().repeat_interleave(2, 1))
    cos, sin = torch.cat(cos, 1).float(), torch.cat(sin, 1).float()

    def rope(v):  # [B, H, L, hd]
        xr, xi = v.reshape(*v.shape[:-1], -1, 2).unbind(-1)
        rot = torch.stack([-xi, xr], -1).flatten(3)
        return v * cos + rot * sin

    def rms(v, w):
        return v * torch.rsqrt(v.pow(2).mean(-1, keepdim=True) + 1e-6) * w.float()

    def ln(v):
        return F.layer_norm(v, (D,), eps=1e-6)

    def attn(q, k, v):
        sh = lambda z: z.view(B, -1, H, hd).transpose(1, 2)  # noqa: E731
        return F.scaled_dot_product_attention(q, k, v).transpose(1, 2).reshape(B, -1, D)

    h = lin(m.x_embedder, x)
    cx = lin(m.context_embedder, ctx)
    st = F.silu(temb)
    heads = lambda z: z.view(B, -1, H, hd).transpose(1, 2)  # noqa: E731
    for blk in m.transformer_blocks:
        sh, sc, g, sh2, sc2, g2 = lin(blk.norm1.linear, st)[:, None].chunk(6, -1)
        csh, csc, cg, csh2, csc2, cg2 = lin(blk.norm1_context.linear, st)[:, None].chunk(6, -1)
        n = ln(h) * (1 + sc) + sh
        cn = ln(cx) * (1 + csc) + csh
        a = blk.attn
        q = torch.cat([rms(heads(lin(a.add_q_proj, cn)), a.norm_added_q.weight), rms(heads(lin(a.to_q, n)), a.norm_q.weight)], 2)
        k = torch.cat([rms(heads(lin(a.add_k_proj, cn)), a.norm_added_k.weight), rms(heads(lin(a.to_k, n)), a.norm_k.weight)], 2)
        v = torch.cat([heads(lin(a.add_v_proj, cn)), heads(lin(a.to_v, n))], 2)
        o = F.scaled_dot_product_attention(rope(q), rope(k), v).transpose(1, 2).reshape(B, -1, D)
        h = h + g * lin(a.to_out[0], o[:, T:])
        cx = cx + cg * lin(a.to_add_out, o[:, :T])
        n = ln(h) * (1 + sc2) + sh2
        h = h + g2 * lin(blk.ff.net[2], F.gelu(lin(blk.ff.net[0].proj, n), approximate="tanh"))
        cn = ln(cx) * (1 + csc2) + csh2
        cx = cx + cg2 * lin(blk.ff_context.net[2], F.gelu(lin(blk.ff_context.net[0].proj, cn), approximate="tanh"))
    xs = torch.cat([cx, h], 1)
    for blk in m.single_transformer_blocks:
        sh, sc, g = lin(blk.norm.linear, st)[:, None].chunk(3, -1)
        n = ln(xs) * (1 + sc) + sh
        a = blk.attn
        q, k, v = rms(heads(lin(a.to_q, n)), a.norm_q.weight), rms(heads(lin(a.to_k, n)), a.norm_k.weight), heads(lin(a.to_v, n))
        o = F.scaled_dot_product_attention(rope(q), rope(k), v).transpose(1, 2).reshape(B, -1, D)
        mlp = F.gelu(lin(blk.proj_mlp, n), approximate="tanh")
        xs = xs + g * lin(blk.proj_out, torch.cat([o, mlp], -1))
    sc, sh = lin(m.norm_out.linear, st)[:, None].chunk(2, -1)
    return lin(m.proj_out, ln(xs[:, T:]) * (1 + sc) + sh)


def _inputs(cfg, B=2, h2=4, w2=6, T=5, seed=0):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(B, h2 * w2, cfg.in_channels, generator=g)
    ctx = torch.randn(B, T, cfg.joint_dim, generator=g)
    pooled = torch.randn(B, cfg.pooled_dim, generator=g)
    return x, FX.image_ids(h2, w2, "cpu"), torch.tensor([0.7, 0.3][:B]), ctx, pooled, torch.tensor([3.5, 2.0][:B])


def _model(cfg, seed=1):
    m = FX.FluxTransformer(cfg)
    init_synthetic(m, seed)
    with torch.no_grad():  # non-trivial norm weights / biases so every term is exercised
        for n, p in m.named_parameters():
            if p.dim() == 1:
                p.add_(torch.randn_like(p) * 0.1)
    return m.eval()


@pytest.mark.parametrize("guidance", [True, False])
def test_flux_forward_matches_reference_cpu(guidance):
    cfg = FX.FluxConfig(layers=2, single_layers=2, heads=2, joint_dim=64, pooled_dim=32, guidance=guidance)
    m = _model(cfg)
    args = _inputs(cfg)
    got = m(*args)
    ref = _ref_forward(m, *args)
    torch.testing.assert_close(got, ref, rtol=2e-4, atol=2e-4)


def test_pack_unpack_and_sigmas():
    z = torch.randn(2, 16, 8, 12)
    p = FX.pack_latents(z)
    assert p.shape == (2, 24, 64)
    torch.testing.assert_close(FX.unpack_latents(p, 8, 12), z)
    s = FX.flux_sigmas(4, 4096)
    assert len(s) == 5 and s[0] == pytest.approx(1.0) and s[-1] == 0.0
    mu = 1.15  # at 4096 tokens
    t = 0.25
    assert s[3] == pytest.approx(math.exp(mu) * t / (1 + (math.exp(mu) - 1) * t))
    assert FX.flux_sigmas(4, 1024, dynamic=False) == pytest.approx([1.0, 0.75, 0.5, 0.25, 0.0])


def test_flux_pipeline_synthetic_cpu():
    from localai_tfp_amd.models.diffusion.pipeline import GenParams
    pipe = FX.FluxPipeline.synthetic("flux-test", "cpu")
    img = pipe.generate("a red fox", GenParams(width=64, height=64, steps=2, seed=3, cfg_scale=3.5))
    assert img.shape == (3, 64, 64) and torch.isfinite(img).all()


# ------------------------------------------------------------------------------------------------ GPU
@pytest.mark.gpu
def test_qk_norm_rope_kernel():
    dev = torch.device("cuda", 0)
    H, D, L, rows = 3, 384, 7, 21
    qkv = (torch.randn(rows, 3 * D + 8) * 2).to(torch.bfloat16)[:, :3 * D]  # strided rows
    wq, wk = torch.rand(128) + 0.5, torch.rand(128) + 0.5
    ids = torch.stack([torch.zeros(L), torch.arange(L).float(), torch.arange(L).float() * 2], 1)
    cs = FX.rope_table(ids, (16, 56, 56), 10000.0)
    ref = FX.qk_norm_rope(qkv.clone(), D, H, wq, wk, cs, L)
    g = qkv.clone().to(dev)
    FX.qk_norm_rope(g, D, H, wq.to(dev), wk.to(dev), cs.to(dev), L)
    torch.testing.assert_close(g.float().cpu(), ref.float(), rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(g[:, 2 * D:].cpu(), qkv[:, 2 * D:])  # v untouched


@pytest.mark.gpu
def test_flux_forward_gpu_vs_cpu_fp32():
    from localai_tfp_amd.models.diffusion.nn import cast_module
    cfg = FX.FluxConfig(layers=2, single_layers=2, heads=2, joint_dim=64, pooled_dim=32)
    m = _model(cfg)
    args = _inputs(cfg)
    ref = m(*args)
    import copy
    mg = cast_module(copy.deepcopy(m), torch.device("cuda", 0), torch.bfloat16)
    mg._prep = None
    got = mg(*[a.to("cuda:0") for a in args]).float().cpu()
    err = (got - ref).norm() / ref.norm()
    assert err < 3e-2, float(err)


@pytest.mark.gpu
def test_flux_pipeline_synthetic_gpu():
    from localai_tfp_amd.models.diffusion.pipeline import GenParams
    pipe = FX.FluxPipeline.synthetic("flux-test", "cuda:0")
    img = pipe.generate("a red fox", GenParams(width=128, height=96, steps=3, seed=3))
    assert img.shape == (3, 96, 128) and torch.isfinite(img).all()


def test_flux_worker_generate(tmp_path):
    from localai_tfp_amd.grpc import pb
    from localai_tfp_amd.workers.diffusion import DiffusionServicer
    sv = DiffusionServicer(device="cpu")
    r = sv.LoadModel(pb.ModelOptions(Model="synthetic:flux-test"), None)
    assert r.success, r.message
    assert sv.defaults["cfg_scale"] == 3.5
    dst = str(tmp_path / "out.png")
    r = sv.GenerateImage(pb.GenerateImageRequest(positive_prompt="a fox", width=64, height=64, step=2, seed=1, dst=dst),
                         None)
    assert r.success, r.message
    from PIL import Image
    assert Image.open(dst).size == (64, 64)
    r = sv.GenerateImage(pb.GenerateImageRequest(positive_prompt="a fox", width=64, height=64, step=4, seed=1,
                                                 src=dst, dst=str(tmp_path / "i2i.png")), None)
    assert r.success, r.message
