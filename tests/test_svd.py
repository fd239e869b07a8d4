"""Stable Video Diffusion (models/diffusion/svd.py) — reference: backend/python/diffusers/backend.py:175-179,
338-341 (StableVideoDiffusionPipeline + export_to_video) and backend.proto GenerateVideo.

diffusers is not importable here, so parity with StableVideoDiffusionPipeline is unpinned. Instead:
* the spatial path with every temporal mixer closed equals the (separately tested) SD UNet with the same
  spatial weights;
* the temporal ResNet and temporal transformer blocks equal plain fp32 5-D re-statements of the diffusers
  modules (Conv3d, 5-D GroupNorm, per-pixel attention over frames);
* the pipeline, worker RPCs (GenerateImage with src, GenerateVideo) and the MP4 writer run end to end.
"""
import math
import struct

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from localai_tfp_amd.models.diffusion import svd as SV
from localai_tfp_amd.models.diffusion import unet as U
from localai_tfp_amd.models.diffusion.nn import init_synthetic


def _unet(seed=0):
    torch.manual_seed(seed)
    m = init_synthetic(SV.UNetSpatioTemporalConditionModel(SV.SVD_TEST), seed).eval()
    with torch.no_grad():  # non-trivial norms / biases
        for n, p in m.named_parameters():
            if n.endswith("bias") or (p.dim() == 1 and "mix_factor" not in n):
                p.add_(0.05 * torch.randn_like(p))
    return m


def test_spatial_path_equals_sd_unet():
    m = _unet(1)
    with torch.no_grad():
        for mod in m.modules():
            if isinstance(mod, SV.AlphaBlender):  # all weight on the spatial branch
                mod.mix_factor.fill_(-1e4 if mod.switch else 1e4)
    c = SV.SVD_TEST
    uc = U.UNetConfig(in_channels=c.in_channels, out_channels=c.out_channels, channels=c.channels,
                      down_types=("CrossAttnDownBlock2D", "DownBlock2D"), up_types=("UpBlock2D", "CrossAttnUpBlock2D"),
                      layers=c.layers, heads=c.heads, transformer_layers=c.transformer_layers, cross_dim=c.cross_dim,
                      linear_proj=True, groups=c.groups, addition_embed="text_time",
                      addition_time_dim=c.addition_time_dim, projection_class_dim=c.projection_dim,
                      mid_transformer_layers=1)
    ref = U.UNet2DConditionModel(uc).eval()
    sd = {}
    for k, v in m.state_dict().items():
        if "temporal" in k or "time_mixer" in k or "time_pos_embed" in k:
            continue
        sd[k.replace(".spatial_res_block.", ".")] = v
    missing, unexpected = ref.load_state_dict(sd, strict=False)
    assert not missing and not unexpected, (missing, unexpected)
    B, Fr = 1, 3
    torch.manual_seed(2)
    x = torch.randn(B, Fr, c.in_channels, 16, 16)
    t = torch.tensor([0.7])
    ctx = torch.randn(B, 1, c.cross_dim)
    tid = torch.tensor([[6.0, 127.0, 0.02]])
    got = m(x, t, ctx, tid)
    want = ref(x.reshape(B * Fr, *x.shape[2:]), t.repeat_interleave(Fr), ctx.repeat_interleave(Fr, 0),
               {"text_embeds": torch.zeros(B * Fr, 0), "time_ids": tid.repeat_interleave(Fr, 0)})
    assert got.shape == (B, Fr, c.out_channels, 16, 16)
    torch.testing.assert_close(got.reshape_as(want), want, rtol=1e-4, atol=1e-4)


def _gn5(x, mod):
    return F.group_norm(x, mod.num_groups, mod.weight, mod.bias, mod.eps)


def test_temporal_resnet_matches_5d_reference():
    torch.manual_seed(3)
    blk = init_synthetic(SV.TemporalResnetBlock(16, 12, 8, 1e-5), 3).eval()
    with torch.no_grad():
        for n, p in blk.named_parameters():
            if p.dim() == 1:
                p.add_(0.1 * torch.randn_like(p))
    B, Fr, C, H, W = 2, 5, 16, 3, 4
    x = torch.randn(B * Fr, C, H, W)
    temb = torch.randn(B * Fr, 12)
    t = F.linear(F.silu(temb), blk.time_emb_proj.weight, blk.time_emb_proj.bias)
    got = SV.untview(blk.run(SV.tview(x, B), t), H, W)
    # diffusers TemporalResnetBlock on [B, C, F, H, W]
    x5 = x.reshape(B, Fr, C, H, W).permute(0, 2, 1, 3, 4)
    h = F.conv3d(F.silu(_gn5(x5, blk.norm1)), blk.conv1.weight, blk.conv1.bias, padding=(1, 0, 0))
    h = h + t.reshape(B, Fr, C)[:, :, :, None, None].permute(0, 2, 1, 3, 4)
    h = F.conv3d(F.silu(_gn5(h, blk.norm2)), blk.conv2.weight, blk.conv2.bias, padding=(1, 0, 0))
    want = (x5 + h).permute(0, 2, 1, 3, 4).reshape(B * Fr, C, H, W)
    torch.testing.assert_close(got, want, rtol=1e-4, atol=1e-4)


def _mha(q, k, v, heads):
    B, Sq, C = q.shape
    D = C // heads
    qh, kh, vh = (t.reshape(B, -1, heads, D).transpose(1, 2) for t in (q, k, v))
    a = torch.softmax(qh @ kh.transpose(-1, -2) / math.sqrt(D), -1)
    return (a @ vh).transpose(1, 2).reshape(B, Sq, C)


def _attn_ref(attn, x, ctx, heads):
    ctx = x if ctx is None else ctx
    o = _mha(F.linear(x, attn.to_q.weight), F.linear(ctx, attn.to_k.weight), F.linear(ctx, attn.to_v.weight), heads)
    return F.linear(o, attn.to_out[0].weight, attn.to_out[0].bias)


def _ff_ref(ff, x):
    g = F.linear(x, ff.net[0].proj.weight, ff.net[0].proj.bias)
    a, gate = g.chunk(2, -1)
    return F.linear(a * F.gelu(gate), ff.net[2].weight, ff.net[2].bias)


@pytest.mark.parametrize("sc", [1, 3])
def test_temporal_transformer_block_matches_reference(sc):
    torch.manual_seed(4)
    C, heads, D = 16, 2, 24
    blk = init_synthetic(SV.TemporalBasicTransformerBlock(C, heads, D), 4).eval()
    with torch.no_grad():
        for n, p in blk.named_parameters():
            if p.dim() == 1:
                p.add_(0.1 * torch.randn_like(p))
    B, Fr, S = 2, 4, 6
    h = torch.randn(B * Fr * S, C)
    tctx = torch.randn(B, sc, D)
    got = blk.run(h.clone(), B, Fr, S, tctx)
    # diffusers TemporalBasicTransformerBlock: tokens [B*S, F, C]
    x = h.reshape(B, Fr, S, C).permute(0, 2, 1, 3).reshape(B * S, Fr, C)
    ln = lambda m, t: F.layer_norm(t, (C,), m.weight, m.bias, 1e-5)  # noqa: E731
    x = _ff_ref(blk.ff_in, ln(blk.norm_in, x)) + x
    x = _attn_ref(blk.attn1, ln(blk.norm1, x), None, heads) + x
    ctx = tctx[:, None].expand(B, S, sc, D).reshape(B * S, sc, D)
    x = _attn_ref(blk.attn2, ln(blk.norm2, x), ctx, heads) + x
    x = _ff_ref(blk.ff, ln(blk.norm3, x)) + x
    want = x.reshape(B, S, Fr, C).permute(0, 2, 1, 3).reshape(B * Fr * S, C)
    torch.testing.assert_close(got, want, rtol=1e-4, atol=1e-4)


def test_alpha_blender_modes():
    s, t = torch.full((2, 3), 2.0), torch.zeros(2, 3)
    a = SV.AlphaBlender(0.0, switch=False)  # sigmoid(0) = 0.5
    assert torch.allclose(a.blend(s, t), torch.full((2, 3), 1.0))
    b = SV.AlphaBlender(2.0, switch=True)  # a = 1 - sigmoid(2)
    w = 1 - 1 / (1 + math.exp(-2.0))
    assert torch.allclose(b.blend(s, t), torch.full((2, 3), 2.0 * w))


def test_karras_sigmas_and_param_count():
    s = SV.karras_sigmas(25)
    assert len(s) == 26 and abs(s[0] - 700.0) < 1e-3 and abs(s[-2] - 0.002) < 1e-6 and s[-1] == 0.0
    n = sum(p.numel() for p in SV.UNetSpatioTemporalConditionModel(SV.SVD_XT).parameters())
    assert 1.50e9 < n < 1.54e9, n  # SVD UNet: 1.52B parameters


def test_pipeline_and_video_file(tmp_path):
    from PIL import Image

    from localai_tfp_amd.utils.video import read_mp4_boxes, write_video
    p = SV.SVDPipeline.synthetic("svd-test", "cpu")
    im = Image.fromarray((np.random.RandomState(0).rand(48, 80, 3) * 255).astype("uint8"))
    vp = SV.VideoParams(width=64, height=64, steps=2, seed=5)
    a = p.generate(im, vp)
    b = p.generate(im, vp)
    assert len(a) == SV.SVD_TEST.num_frames and a[0].size == (64, 64)
    assert all(np.array_equal(np.asarray(x), np.asarray(y)) for x, y in zip(a, b))
    path = write_video(a, str(tmp_path / "v.mp4"), fps=7)
    data = open(path, "rb").read()
    top = [k for k, _, _ in read_mp4_boxes(data)]
    assert top == [b"ftyp", b"moov", b"mdat"]
    # the chunk offset points at the first JPEG (SOI marker) and the sample sizes cover mdat exactly
    stco = data.find(b"stco")
    off = struct.unpack(">I", data[stco + 12:stco + 16])[0]
    assert data[off:off + 2] == b"\xff\xd8"
    _, mo, ml = read_mp4_boxes(data)[2]
    stsz = data.find(b"stsz")
    n = struct.unpack(">I", data[stsz + 12:stsz + 16])[0]
    sizes = struct.unpack(f">{n}I", data[stsz + 16:stsz + 16 + 4 * n])
    assert n == len(a) and sum(sizes) == ml and mo == off
    gif = write_video(a, str(tmp_path / "v.gif"), fps=7)
    with Image.open(gif) as g:
        assert g.n_frames == len(a)


def test_worker_generate_video_and_image(tmp_path):
    from PIL import Image

    from localai_tfp_amd.grpc import pb
    from localai_tfp_amd.workers.diffusion import DiffusionServicer
    src = tmp_path / "start.png"
    Image.fromarray((np.random.RandomState(1).rand(64, 64, 3) * 255).astype("uint8")).save(src)
    w = DiffusionServicer(device="cpu")
    r = w.LoadModel(pb.ModelOptions(Model="synthetic:svd-test", Options=["steps:2", "fps:6"]), None)
    assert r.success, r.message
    dst = tmp_path / "out.mp4"
    r = w.GenerateVideo(pb.GenerateVideoRequest(start_image=str(src), width=64, height=64, num_frames=3, seed=2,
                                                dst=str(dst)), None)
    assert r.success, r.message
    assert dst.read_bytes()[4:8] == b"ftyp"
    r = w.GenerateImage(pb.GenerateImageRequest(src=str(src), width=64, height=64, dst=str(tmp_path / "o.gif")), None)
    assert r.success, r.message
    with Image.open(tmp_path / "o.gif") as g:
        assert g.n_frames == SV.SVD_TEST.num_frames
    r = w.GenerateVideo(pb.GenerateVideoRequest(width=64, height=64, dst=str(dst)), None)
    assert not r.success and "start image" in r.message
    # a text-to-image model answers GenerateVideo with a clear error
    w2 = DiffusionServicer(device="cpu")
    assert w2.LoadModel(pb.ModelOptions(Model="synthetic:sd15-test"), None).success
    r = w2.GenerateVideo(pb.GenerateVideoRequest(start_image=str(src), dst=str(dst)), None)
    assert not r.success and "video" in r.message


@pytest.mark.gpu
def test_svd_unet_gpu_matches_cpu():
    from localai_tfp_amd.models.diffusion.nn import cast_module
    m = _unet(5)
    with torch.no_grad():
        for mod in m.modules():
            if isinstance(mod, SV.AlphaBlender):
                mod.mix_factor.normal_()
    torch.manual_seed(6)
    x = torch.randn(1, 4, SV.SVD_TEST.in_channels, 16, 24)
    t = torch.tensor([0.3])
    ctx = torch.randn(1, 1, SV.SVD_TEST.cross_dim)
    tid = torch.tensor([[6.0, 127.0, 0.02]])
    ref = m(x, t, ctx, tid)
    g = cast_module(m, "cuda:0", torch.float16)
    got = g(x.cuda(), t.cuda(), ctx.cuda(), tid.cuda()).cpu()
    assert float((got - ref).norm() / ref.norm()) < 2e-2


@pytest.mark.gpu
def test_svd_pipeline_gpu(tmp_path):
    from PIL import Image
    p = SV.SVDPipeline.synthetic("svd-test", "cuda:0")
    im = Image.fromarray((np.random.RandomState(0).rand(64, 64, 3) * 255).astype("uint8"))
    fr = p.generate(im, SV.VideoParams(width=128, height=64, steps=3, seed=1))
    assert len(fr) == SV.SVD_TEST.num_frames and fr[0].size == (128, 64)
