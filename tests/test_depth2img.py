"""Depth-to-image (the reference diffusers backend's StableDiffusionDepth2ImgPipeline, backend.py:172-173):
a 5-channel UNet conditioned on the source image's DPT depth map. Random-init components (no checkpoint
offline), so what is checked is the pipeline's wiring: the depth map's range / grid, the depth channel
reaching the UNet, the source image being required, and the GenerateImage RPC path. Parity with diffusers'
images is unpinned (diffusers is not installed)."""
import numpy as np
import pytest
import torch

from localai_tfp_amd.models.diffusion.pipeline import GenParams
from localai_tfp_amd.models.diffusion.sd_pipeline import UNetPipeline


@pytest.fixture(scope="module")
def pipe():
    return UNetPipeline.synthetic("sd2-depth-test", "cpu")


def test_depth_map_range_and_grid(pipe):
    assert pipe.depth_cond and pipe.depth is not None
    img = torch.rand(3, 64, 64)
    d = pipe.depth_map(img, 8, 8)
    assert d.shape == (1, 1, 8, 8)
    assert -1.0 - 1e-5 <= float(d.min()) and float(d.max()) <= 1.0 + 1e-5
    # the normalisation itself: a known depth ramp maps onto [-1, 1]
    m, sz, mean, std = pipe.depth

    class Ramp(torch.nn.Module):
        def forward(self, pixel_values):
            b, _, h, w = pixel_values.shape
            return type("O", (), {"predicted_depth": torch.arange(h * w, dtype=torch.float32).view(1, h, w)})()
    pipe.depth = (Ramp(), sz, mean, std)
    try:
        d = pipe.depth_map(img, 8, 8)
    finally:
        pipe.depth = (m, sz, mean, std)
    assert float(d.min()) == pytest.approx(-1.0, abs=1e-5) and float(d.max()) == pytest.approx(1.0, abs=1e-5)


def test_depth2img_generates_and_uses_depth(pipe, monkeypatch):
    gp = GenParams(width=64, height=64, steps=2, seed=3)
    gp.strength = 0.8
    img = torch.rand(3, 64, 64)
    seen = []
    orig = pipe.unet.forward

    def spy(x, *a, **k):
        seen.append(x.shape[1])
        return orig(x, *a, **k)
    monkeypatch.setattr(pipe.unet, "forward", spy)
    out = pipe.generate("a house", gp, img)
    assert out.shape == (3, 64, 64) and torch.isfinite(out).all()
    assert seen and all(c == 5 for c in seen)  # latent (4) + depth (1)
    with pytest.raises(ValueError, match="source image"):
        pipe.generate("a house", gp, None)


def test_depth2img_rpc(tmp_path):
    from PIL import Image

    from localai_tfp_amd.grpc import pb
    from localai_tfp_amd.workers.diffusion import DiffusionServicer
    s = DiffusionServicer(device="cpu")
    r = s.LoadModel(pb.ModelOptions(Model="synthetic:sd2-depth-test", PipelineType="StableDiffusionDepth2ImgPipeline"), None)
    assert r.success, r.message
    src = tmp_path / "src.png"
    Image.fromarray((np.random.default_rng(0).random((64, 64, 3)) * 255).astype(np.uint8)).save(src)
    dst = tmp_path / "out.png"
    r = s.GenerateImage(pb.GenerateImageRequest(positive_prompt="a room", width=64, height=64, step=2, seed=1,
                                                src=str(src), dst=str(dst)), None)
    assert r.success, r.message
    assert Image.open(dst).size == (64, 64)
