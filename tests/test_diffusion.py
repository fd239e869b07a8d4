"""Diffusion stack: MMDiT vs a plain fp32 PyTorch SD3 transformer, samplers, VAE, pipeline, worker and
/v1/images/generations (reference coverage: core/http/app_test.go stablediffusion case,
backend/python/diffusers/test.py)."""
import base64
import io
import math

import pytest
import torch
import torch.nn.functional as F
import yaml

from localai_tfp_amd.models.diffusion import samplers as S
from localai_tfp_amd.models.diffusion.mmdit import MMDIT_TEST, MMDITX_TEST, MMDiT
from localai_tfp_amd.models.diffusion.nn import cast_module, init_synthetic, timestep_embedding
from localai_tfp_amd.models.diffusion.pipeline import GenParams, SD3Pipeline
from localai_tfp_amd.models.diffusion.vae import VAE_TEST, AutoencoderKL


def ref_mmdit(m: MMDiT, latent, t, ctx, pooled):
    """Straightforward SD3 transformer forward (diffusers semantics), fp32."""
    c = m.cfg
    B, C, Hh, Ww = latent.shape
    p, D, H = c.patch, c.dim, c.heads
    x = F.conv2d(latent, m.pos_embed.proj.weight, m.pos_embed.proj.bias, stride=p).flatten(2).transpose(1, 2)
    x = x + m._pos(Hh // p, Ww // p)[None]
    te = m.time_text_embed
    temb = te.timestep_embedder.linear_2(F.silu(te.timestep_embedder.linear_1(timestep_embedding(t, 256))))
    temb = temb + te.text_embedder.linear_2(F.silu(te.text_embedder.linear_1(pooled)))
    cx = m.context_embedder(ctx)

    def ln(z):
        return F.layer_norm(z, (D,), eps=1e-6)

    def attn(q, k, v):
        q, k, v = (z.view(B, -1, H, D // H).transpose(1, 2) for z in (q, k, v))
        return F.scaled_dot_product_attention(q, k, v).transpose(1, 2).reshape(B, -1, D)

    def rms(z, mod, name):  # per-head RMS QK-norm (diffusers qk_norm="rms_norm", eps 1e-6)
        if not c.qk_norm:
            return z
        zh = z.view(*z.shape[:-1], H, D // H)
        return (zh * torch.rsqrt(zh.pow(2).mean(-1, keepdim=True) + 1e-6) * getattr(mod, name).weight).flatten(-2)
    S_ = x.shape[1]
    for blk in m.transformer_blocks:
        e = blk.norm1.linear(F.silu(temb))
        sh, sc, g, sh2, sc2, g2, *dual = e.chunk(9 if blk.dual else 6, 1)
        xn = ln(x) * (1 + sc[:, None]) + sh[:, None]
        if blk.dual:  # SD35AdaLayerNormZeroX: second modulation of the same normalised input
            xn2 = ln(x) * (1 + dual[1][:, None]) + dual[0][:, None]
        ec = blk.norm1_context.linear(F.silu(temb))
        if blk.pre_only:
            csc, csh = ec.chunk(2, 1)
        else:
            csh, csc, cg, csh2, csc2, cg2 = ec.chunk(6, 1)
        cn = ln(cx) * (1 + csc[:, None]) + csh[:, None]
        a = blk.attn
        q = torch.cat([rms(a.to_q(xn), a, "norm_q"), rms(a.add_q_proj(cn), a, "norm_added_q")], 1)
        k = torch.cat([rms(a.to_k(xn), a, "norm_k"), rms(a.add_k_proj(cn), a, "norm_added_k")], 1)
        v = torch.cat([a.to_v(xn), a.add_v_proj(cn)], 1)
        o = attn(q, k, v)
        x = x + g[:, None] * a.to_out[0](o[:, :S_])
        if blk.dual:
            a2 = blk.attn2
            o2 = attn(rms(a2.to_q(xn2), a2, "norm_q"), rms(a2.to_k(xn2), a2, "norm_k"), a2.to_v(xn2))
            x = x + dual[2][:, None] * a2.to_out[0](o2)
        xn = ln(x) * (1 + sc2[:, None]) + sh2[:, None]
        x = x + g2[:, None] * blk.ff.net[2](F.gelu(blk.ff.net[0].proj(xn), approximate="tanh"))
        if not blk.pre_only:
            cx = cx + cg[:, None] * a.to_add_out(o[:, S_:])
            cn = ln(cx) * (1 + csc2[:, None]) + csh2[:, None]
            cx = cx + cg2[:, None] * blk.ff_context.net[2](F.gelu(blk.ff_context.net[0].proj(cn), approximate="tanh"))
    sc, sh = m.norm_out.linear(F.silu(temb)).chunk(2, 1)
    x = ln(x) * (1 + sc[:, None]) + sh[:, None]
    out = m.proj_out(x)
    h, w = Hh // p, Ww // p
    out = out.view(B, h, w, p, p, c.out_channels)
    return torch.einsum("nhwpqc->nchpwq", out).reshape(B, c.out_channels, Hh, Ww)


def _mmdit(dev="cpu"):
    m = init_synthetic(MMDiT(MMDIT_TEST), 3)
    return m


def test_mmdit_matches_reference():
    m = _mmdit()
    g = torch.Generator().manual_seed(0)
    lat = torch.randn(2, 16, 16, 16, generator=g)
    t = torch.tensor([500.0, 20.0])
    ctx = torch.randn(2, 9, MMDIT_TEST.joint_dim, generator=g)
    pooled = torch.randn(2, MMDIT_TEST.pooled_dim, generator=g)
    with torch.no_grad():
        ref = ref_mmdit(m, lat, t, ctx, pooled)
        got = m(lat, t, ctx, pooled)
    assert (got - ref).abs().max() < 1e-3 * max(1.0, ref.abs().max().item())


def test_mmditx_dual_attention_matches_reference():
    """SD3.5-medium MMDiT-X blocks (attn2 + 9-vector adaLN) and RMS QK-norm against the fp32 reference."""
    m = init_synthetic(MMDiT(MMDITX_TEST), 4)
    assert m.transformer_blocks[0].dual and not m.transformer_blocks[2].dual
    g = torch.Generator().manual_seed(1)
    lat = torch.randn(2, 16, 16, 16, generator=g)
    t = torch.tensor([700.0, 3.0])
    ctx = torch.randn(2, 7, MMDITX_TEST.joint_dim, generator=g)
    pooled = torch.randn(2, MMDITX_TEST.pooled_dim, generator=g)
    with torch.no_grad():
        ref = ref_mmdit(m, lat, t, ctx, pooled)
        got = m(lat, t, ctx, pooled)
    assert (got - ref).abs().max() < 1e-3 * max(1.0, ref.abs().max().item())


def test_flow_euler_reaches_target():
    target = torch.randn(1, 4, 8, 8)
    sched = S.FlowSchedule(3.0)
    sig = S.get_sigmas(sched, 10)
    assert sig[0] == pytest.approx(1.0) and sig[-1] == 0.0 and all(a > b for a, b in zip(sig, sig[1:]))
    x = torch.randn(1, 4, 8, 8)
    for name in ("euler", "heun", "dpm++2m", "ipndm", "ddim_trailing"):
        out = S.sample(lambda xt, s: target, x.clone(), sig, name, flow=True)
        assert torch.allclose(out, target, atol=1e-4), name


def test_eps_schedules():
    sched = S.EpsSchedule()
    for kind in ("default", "karras", "exponential"):
        sig = S.get_sigmas(sched, 8, kind)
        assert len(sig) == 9 and sig[-1] == 0 and sig[0] > 10
    assert sched.t_of(sched.sigma_of(421.0)) == pytest.approx(421.0, abs=1e-3)


def test_vae_roundtrip_shapes():
    vae = init_synthetic(AutoencoderKL(VAE_TEST), 1).eval()
    z = torch.randn(1, 16, 8, 8)
    img = vae.decode(z)
    assert img.shape == (1, 3, 64, 64) and torch.isfinite(img).all()
    z2 = vae.encode(img)
    assert z2.shape == z.shape


def test_pipeline_txt2img_img2img():
    p = SD3Pipeline.synthetic("sd3-test", "cpu")
    a = p.generate("a red fox", GenParams(width=64, height=48, steps=3, seed=5))
    b = p.generate("a red fox", GenParams(width=64, height=48, steps=3, seed=5))
    c = p.generate("a red fox", GenParams(width=64, height=48, steps=3, seed=6))
    assert a.shape == (3, 48, 64) and torch.equal(a, b) and not torch.equal(a, c)
    d = p.generate("a red fox", GenParams(width=64, height=48, steps=4, seed=5, strength=0.5), init_image=a)
    assert d.shape == a.shape


@pytest.fixture(scope="module")
def client(tmp_path_factory):
    from fastapi.testclient import TestClient
    from localai_tfp_amd.config.app_config import ApplicationConfig
    from localai_tfp_amd.gateway.app import create_app
    d = tmp_path_factory.mktemp("sd")
    models = d / "models"
    models.mkdir()
    (models / "sd3.yaml").write_text(yaml.safe_dump({
        "name": "sd3", "backend": "diffusers", "parameters": {"model": "synthetic:sd3-test"},
        "options": ["sampler:euler", "cfg_scale:4.5"]}))
    cfg = ApplicationConfig(models_path=str(models), generated_content_dir=str(d / "gen"),
                            upload_dir=str(d / "up"), config_dir=str(d / "cfg"), api_keys=[])
    app = create_app(cfg, inproc=True)
    with TestClient(app) as c:
        yield c
    app.state.localai.shutdown()


def test_http_images(client):
    from PIL import Image
    r = client.post("/v1/images/generations", json={"model": "sd3", "prompt": "a cat|blurry", "size": "64x64",
                                                    "n": 2, "step": 2, "response_format": "b64_json"})
    assert r.status_code == 200, r.text
    data = r.json()["data"]
    assert len(data) == 2
    im = Image.open(io.BytesIO(base64.b64decode(data[0]["b64_json"])))
    assert im.size == (64, 64)
    r = client.post("/v1/images/generations", json={"model": "sd3", "prompt": "a dog", "size": "32x32", "step": 1})
    url = r.json()["data"][0]["url"]
    assert client.get(url.split("://", 1)[1].split("/", 1)[1].join(["/", ""])).status_code == 200


# ------------------------------------------------------------------------------------------------ GPU

@pytest.mark.gpu
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
def test_diffusion_kernels_gpu(dt):
    from localai_tfp_amd.ops import core as K
    g = torch.Generator().manual_seed(1)
    # layernorm_mod
    B, Sq, H = 2, 37, 1536
    x = torch.randn(B * Sq, H, generator=g) * 3 + 1
    mod = torch.randn(B, 4 * H, generator=g)
    ref = torch.empty(B * Sq, H)
    K.layernorm_mod(x, mod[:, H:2 * H], mod[:, :H], Sq, ref)
    out = torch.empty(B * Sq, H, dtype=dt, device="cuda")
    md = mod.cuda()
    K.layernorm_mod(x.cuda(), md[:, H:2 * H], md[:, :H], Sq, out)
    assert (out.float().cpu() - ref).abs().max() < 3e-2 * ref.abs().max()
    # gate_add
    y = torch.randn(B * Sq, H, generator=g).to(dt)
    xr = x.clone()
    K.gate_add(xr, y, mod[:, 2 * H:3 * H], Sq)
    xg = x.cuda()
    K.gate_add(xg, y.cuda(), md[:, 2 * H:3 * H], Sq)
    assert (xg.cpu() - xr).abs().max() < 1e-4 * xr.abs().max()
    # groupnorm (+silu) NHWC for VAE / UNet channel counts
    # 2560 / 2880: SDXL up-block concatenations (more than 256 8-channel chunks per pixel)
    for C, G, HW in ((128, 32, (64, 48)), (512, 32, (17, 9)), (320, 32, (8, 8)), (2560, 32, (16, 16)), (2880, 32, (5, 7))):
        t = (torch.randn(2, C, *HW, generator=g) * 2 + 0.5).to(dt)
        w = torch.rand(C, generator=g) + 0.5
        b = torch.randn(C, generator=g)
        ref = F.silu(F.group_norm(t.float(), G, w, b, 1e-6))
        got = K.groupnorm16(t.cuda().contiguous(memory_format=torch.channels_last), w.cuda(), b.cuda(), G, 1e-6, True)
        assert (got.float().cpu() - ref).abs().max() < 3e-2 * max(1.0, ref.abs().max().item()), C


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", [MMDIT_TEST, MMDITX_TEST], ids=["mmdit", "mmditx"])
def test_mmdit_gpu_matches_fp32(cfg):
    m = init_synthetic(MMDiT(cfg), 3)
    gm = cast_module(MMDiT(cfg), "cuda", torch.bfloat16)
    gm.load_state_dict({k: v.to(torch.bfloat16) if v.dim() > 1 else v for k, v in m.state_dict().items()})
    cast_module(gm, "cuda", torch.bfloat16)
    # reference sees the same bf16-rounded weights
    m.load_state_dict({k: v.to(torch.bfloat16).float() for k, v in m.state_dict().items()})
    g = torch.Generator().manual_seed(0)
    lat = torch.randn(2, 16, 32, 32, generator=g)
    t = torch.tensor([500.0, 20.0])
    ctx = torch.randn(2, 77, cfg.joint_dim, generator=g)
    pooled = torch.randn(2, cfg.pooled_dim, generator=g)
    with torch.no_grad():
        ref = ref_mmdit(m, lat, t, ctx, pooled)
        got = gm(lat.cuda(), t.cuda(), ctx.cuda(), pooled.cuda()).cpu()
    err = (got - ref).abs().max() / ref.abs().max()
    assert err < 5e-2, err


@pytest.mark.gpu
def test_pipeline_gpu_generates():
    p = SD3Pipeline.synthetic("sd3-test", "cuda:0")
    img = p.generate("hello", GenParams(width=128, height=128, steps=3, seed=1))
    assert img.shape == (3, 128, 128) and torch.isfinite(img).all()
    vae_c = init_synthetic(AutoencoderKL(VAE_TEST), 1).eval()
    vae_g = cast_module(init_synthetic(AutoencoderKL(VAE_TEST), 1), "cuda", torch.bfloat16).eval()
    z = torch.randn(1, 16, 16, 16)
    a, b = vae_c.decode(z), vae_g.decode(z.cuda()).cpu()
    assert (a - b).abs().max() < 0.1
    assert math.isfinite(float(b.mean()))


def test_diffusers_scheduler_type_names():
    from localai_tfp_amd.models.diffusion.samplers import SAMPLERS
    from localai_tfp_amd.workers.diffusion import DIFFUSERS_SCHEDULERS, diffusers_scheduler
    assert diffusers_scheduler("k_dpmpp_2m") == ("dpm++2m", "karras")
    assert diffusers_scheduler("euler_a") == ("euler_a", "default")
    for n in DIFFUSERS_SCHEDULERS:
        assert diffusers_scheduler(n)[0] in SAMPLERS
    import pytest
    with pytest.raises(ValueError):
        diffusers_scheduler("nope")
