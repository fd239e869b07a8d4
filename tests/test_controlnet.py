"""ControlNet for the UNet pipelines (reference: backend/python/diffusers/backend.py:239-242, 309-312 —
ControlNetModel on the pipeline; with it, the request's src image is the control image).

Checks: residual shapes/count match the UNet skips (diffusers layout: one per ResNet/downsampler plus
conv_in); zero-initialised zero-convs (as a freshly created diffusers ControlNet) leave the image
bit-identical to the plain pipeline; a trained-like (random) ControlNet changes the image
deterministically; the worker routes src to the control image; GPU fp16 vs CPU fp32."""
import torch

from localai_tfp_amd.models.diffusion.pipeline import GenParams


def _pipe(dev="cpu"):
    from localai_tfp_amd.models.diffusion.sd_pipeline import UNetPipeline
    return UNetPipeline.synthetic("sd15-test", dev).set_controlnet("synthetic")


def test_controlnet_residuals_and_zero_init():
    p = _pipe()
    cn, un = p.controlnet, p.unet
    x = torch.randn(2, 4, 8, 8)
    t = torch.tensor([500.0, 500.0])
    ctx = torch.randn(2, 77, un.cfg.cross_dim)
    cond = torch.rand(2, 3, 64, 64)
    down, mid = cn(x, t, ctx, cond, 0.8)
    skips, h = un._encode(torch.nn.functional.conv2d(x, un.conv_in.weight, un.conv_in.bias, padding=1),
                          *un._prologue(x, t, ctx, None, None)[:3])
    assert len(down) == len(skips) and all(a.shape == b.shape for a, b in zip(down, skips))
    assert mid.shape == h.shape
    gp = GenParams(width=64, height=64, steps=2, seed=1, cfg_scale=3.0)
    base = p.generate("a house", gp)
    for m in list(cn.controlnet_down_blocks) + [cn.controlnet_mid_block]:
        torch.nn.init.zeros_(m.weight)
        torch.nn.init.zeros_(m.bias)
    gp.extra["control_image"] = torch.rand(3, 64, 64)
    assert torch.equal(p.generate("a house", gp), base)


def test_controlnet_changes_image_and_worker(tmp_path):
    p = _pipe()
    gp = GenParams(width=64, height=64, steps=2, seed=1, cfg_scale=3.0)
    base = p.generate("a house", gp)
    gp.extra["control_image"] = torch.rand(3, 64, 64, generator=torch.Generator().manual_seed(0))
    a = p.generate("a house", gp)
    assert not torch.equal(a, base) and torch.equal(a, p.generate("a house", gp))
    from localai_tfp_amd.grpc import pb
    from localai_tfp_amd.models.diffusion.pipeline import save_png
    from localai_tfp_amd.workers.diffusion import DiffusionServicer
    save_png(gp.extra["control_image"], str(tmp_path / "edges.png"))
    svc = DiffusionServicer("cpu")
    assert svc.LoadModel(pb.ModelOptions(Model="synthetic:sd15-test", ControlNet="synthetic",
                                         Options=["control_scale:0.5"]), None).success
    r = svc.GenerateImage(pb.GenerateImageRequest(positive_prompt="a house", width=64, height=64, step=2, seed=1,
                                                  src=str(tmp_path / "edges.png"), dst=str(tmp_path / "o.png")), None)
    assert r.success, r.message
    assert (tmp_path / "o.png").stat().st_size > 0


import pytest  # noqa: E402


@pytest.mark.gpu
def test_controlnet_gpu_matches_cpu():
    import copy

    from localai_tfp_amd.models.diffusion.nn import cast_module
    pc = _pipe("cpu")  # same weights on both sides: cast the CPU modules to the GPU (fp16)
    dev = torch.device("cuda:0")
    pg = type("P", (), {})()
    pg.controlnet = cast_module(copy.deepcopy(pc.controlnet), dev, torch.float16)
    pg.unet = cast_module(copy.deepcopy(pc.unet), dev, torch.float16)
    x = torch.randn(2, 4, 8, 8)
    t = torch.tensor([300.0, 300.0])
    ctx = torch.randn(2, 77, pc.unet.cfg.cross_dim)
    cond = torch.rand(2, 3, 64, 64)
    dc, mc = pc.controlnet(x, t, ctx, cond, 1.0)
    dg, mg = pg.controlnet(x.cuda(), t.cuda(), ctx.cuda(), cond.cuda(), 1.0)
    for a, b in zip(dc + [mc], dg + [mg]):
        torch.testing.assert_close(b.float().cpu(), a.float(), rtol=3e-2, atol=3e-2)
    ec = pc.unet(x, t, ctx, control=(dc, mc))
    eg = pg.unet(x.cuda(), t.cuda(), ctx.cuda(), control=(dg, mg))
    torch.testing.assert_close(eg.float().cpu(), ec, rtol=5e-2, atol=5e-2)
