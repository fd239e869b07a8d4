"""Implicit-GEMM MFMA conv2d (csrc/kernels/conv.hip, ops/conv.py) vs a plain fp32 PyTorch conv.

CPU tests pin the packed-weight k order (an im2col GEMM over the packed layout reproduces F.conv2d) and
the fused-epilogue reference; GPU tests run the HIP kernel on every tile config over UNet / VAE /
ControlNet / Whisper-shaped convolutions (odd channel counts, stride 2, asymmetric padding, fused 2x
upsampling, time-embedding / residual / SiLU epilogues) against fp32 F.conv2d.
"""
import pytest
import torch
import torch.nn.functional as F

from localai_tfp_amd.ops import conv as CV


def _im2col_packed(x, wp, cp, kh, kw, stride, pad, up):
    """CPU emulation of the kernel's k order: A[p, (i*KW + j)*Cp + c] over the (padded) NHWC input."""
    n, c, h, w = x.shape
    if up:
        x = F.interpolate(x, scale_factor=2.0, mode="nearest")
    t, l, b, r = pad
    xp = F.pad(x, (l, r, t, b))
    xp = F.pad(xp.permute(0, 2, 3, 1), (0, cp - c))  # [N, H', W', Cp]
    hl, wl = xp.shape[1], xp.shape[2]
    ho, wo = (hl - kh) // stride + 1, (wl - kw) // stride + 1
    cols = []
    for i in range(kh):
        for j in range(kw):
            cols.append(xp[:, i:i + stride * (ho - 1) + 1:stride, j:j + stride * (wo - 1) + 1:stride, :])
    a = torch.cat(cols, -1).reshape(n * ho * wo, kh * kw * cp)
    a = F.pad(a, (0, wp.shape[1] - a.shape[1]))
    return (a @ wp.float().t()).reshape(n, ho, wo, -1).permute(0, 3, 1, 2)


@pytest.mark.parametrize("cin,cout,k,stride,pad,up", [
    (4, 320, 3, 1, (1, 1, 1, 1), False),
    (3, 16, 3, 1, (1, 1, 1, 1), False),
    (64, 96, 3, 2, (0, 0, 1, 1), False),
    (40, 24, 3, 1, (1, 1, 1, 1), True),
    (80, 32, 1, 1, (0, 0, 0, 0), False),
])
def test_packed_weight_k_order(cin, cout, k, stride, pad, up):
    torch.manual_seed(0)
    x = torch.randn(2, cin, 9, 7)
    w = torch.randn(cout, cin, k, k)
    wp, cp = CV.pack_weight(w, torch.float32)
    assert cp % 8 == 0 and wp.shape[1] % 64 == 0
    got = _im2col_packed(x, wp, cp, k, k, stride, pad, up)
    ref = CV._reference(x, w, None, stride, pad, up, None, None, None)
    torch.testing.assert_close(got, ref, rtol=1e-4, atol=1e-4)


def test_reference_fused_epilogue():
    torch.manual_seed(1)
    m = torch.nn.Conv2d(8, 16, 3, 1, 1)
    x = torch.randn(2, 8, 5, 5)
    t = torch.randn(2, 16)
    res = torch.randn(2, 16, 5, 5)
    y = CV.conv2d(x, m, tadd=t, residual=res, act="silu")
    ref = F.silu(F.conv2d(x, m.weight, m.bias, 1, 1) + t[:, :, None, None] + res)
    torch.testing.assert_close(y, ref.detach(), rtol=1e-5, atol=1e-5)


# ------------------------------------------------------------------------------------------------ GPU
GPU_CASES = [
    # n, cin, cout, h, w, k, stride, pad, up, tadd, res, act
    (2, 320, 320, 32, 32, 3, 1, (1, 1, 1, 1), False, True, False, None),      # UNet resnet conv1 (+temb)
    (2, 640, 640, 16, 16, 3, 1, (1, 1, 1, 1), False, False, True, None),      # conv2 (+skip)
    (2, 320, 640, 16, 16, 1, 1, (0, 0, 0, 0), False, False, False, None),     # 1x1 shortcut
    (2, 4, 320, 32, 32, 3, 1, (1, 1, 1, 1), False, False, False, None),       # conv_in (Cin 4 -> padded 8)
    (2, 320, 4, 32, 32, 3, 1, (1, 1, 1, 1), False, False, False, None),       # conv_out (Cout 4)
    (1, 128, 3, 64, 64, 3, 1, (1, 1, 1, 1), False, False, False, None),       # VAE conv_out (Cout 3)
    (1, 3, 128, 64, 64, 3, 1, (1, 1, 1, 1), False, False, False, None),       # VAE encoder conv_in (Cin 3)
    (1, 128, 128, 33, 31, 3, 2, (0, 0, 1, 1), False, False, False, None),     # VAE downsample (asym pad)
    (2, 640, 640, 8, 8, 3, 1, (1, 1, 1, 1), True, False, False, None),        # UNet upsampler (fused 2x)
    (1, 256, 256, 17, 23, 3, 1, (1, 1, 1, 1), True, False, True, None),       # VAE upsampler + residual
    (1, 16, 32, 40, 40, 3, 2, (1, 1, 1, 1), False, False, False, "silu"),     # ControlNet cond embedding
    (3, 1280, 1280, 8, 8, 3, 1, (1, 1, 1, 1), False, True, True, None),       # low-res level, all epilogues
    (2, 80, 384, 1, 300, 3, 1, (0, 1, 0, 1), False, False, False, "gelu"),    # Whisper conv1 (H = 1)
    (2, 384, 384, 1, 300, 3, 2, (0, 1, 0, 1), False, False, False, "gelu"),   # Whisper conv2 (stride 2)
]


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("case", GPU_CASES)
def test_conv2d_gpu_vs_fp32(case, dtype):
    n, cin, cout, h, w, k, stride, pad, up, use_t, use_res, act = case
    dev = "cuda"
    g = torch.Generator().manual_seed(cin * 7 + cout)
    x = torch.randn(n, cin, h, w, generator=g)
    kh = 1 if h == 1 else k  # H = 1 cases are 1-D convs (Whisper stem)
    m = torch.nn.Conv2d(cin, cout, (kh, k), stride, 0)
    with torch.no_grad():
        m.weight.copy_(torch.randn(m.weight.shape, generator=g) / (cin * kh * k) ** 0.5)
        m.bias.copy_(torch.randn(cout, generator=g) * 0.1)
    t = torch.randn(n, cout, generator=g) if use_t else None
    hl, wl = (2 * h, 2 * w) if up else (h, w)
    ho, wo = (hl + pad[0] + pad[2] - kh) // stride + 1, (wl + pad[1] + pad[3] - k) // stride + 1
    res = torch.randn(n, cout, ho, wo, generator=g) if use_res else None
    ref = CV._reference(x, m.weight.detach(), m.bias.detach(), stride, pad, up, t, res, act).float()

    md = torch.nn.Conv2d(cin, cout, (kh, k), stride, 0).to(dev)
    md.load_state_dict(m.state_dict())
    md = md.to(dtype)
    xd = x.to(dev, dtype).contiguous(memory_format=torch.channels_last)
    rd = res.to(dev, dtype).contiguous(memory_format=torch.channels_last) if res is not None else None
    td = t.to(dev) if t is not None else None
    cfgs = [-1, 0x22, 0x14, 0x12, 0x11, 0x21]
    for cfg in cfgs:
        y = CV.conv2d(xd, md, stride=stride, pad=pad, upsample=up, tadd=td, residual=rd, act=act, cfg=cfg)
        torch.cuda.synchronize()
        assert y.shape == ref.shape and y.is_contiguous(memory_format=torch.channels_last)
        # the 16-bit input / weight rounding is the only difference from the fp32 oracle
        xr = x.to(dtype).float()
        ref16 = CV._reference(xr, m.weight.detach().to(dtype).float(), m.bias.detach(), stride, pad, up, t,
                              None if res is None else res.to(dtype).float(), act).float()
        err = (y.float().cpu() - ref16).abs().max().item()
        tol = (2e-2 if dtype == torch.float16 else 8e-2) * max(1.0, ref16.abs().max().item())
        assert err < tol, (cfg, err, tol)
        err32 = (y.float().cpu() - ref).norm() / ref.norm()
        assert err32 < (5e-3 if dtype == torch.float16 else 2e-2), (cfg, float(err32))


@pytest.mark.gpu
def test_conv_tadd_broadcast_and_module_cache():
    dev = "cuda"
    torch.manual_seed(3)
    m = torch.nn.Conv2d(64, 128, 3, 1, 1).to(dev).half()
    x = torch.randn(2, 64, 12, 12, device=dev).half().contiguous(memory_format=torch.channels_last)
    t = torch.randn(1, 128, device=dev)
    y = CV.conv2d(x, m, tadd=t)
    ref = F.conv2d(x.float(), m.weight.float(), m.bias.float(), 1, 1) + t[:, :, None, None]
    assert (y.float() - ref).abs().max().item() < 3e-2
    key0 = m._mx_conv_pack[0]
    with torch.no_grad():
        m.weight.mul_(2.0)  # an in-place merge (LoRA) bumps the version -> repack
    y2 = CV.conv2d(x, m)
    assert m._mx_conv_pack[0] != key0
    ref2 = F.conv2d(x.float(), m.weight.float(), m.bias.float(), 1, 1)
    assert (y2.float() - ref2).abs().max().item() < 6e-2


@pytest.mark.gpu
@pytest.mark.parametrize("dil,act", [(2, "elu"), (3, None), (1, "elu")])
def test_conv1d_rows_dilation_elu_gpu(dil, act):
    """EnCodec-style H = 1 convs: dilation and the ELU epilogue, vs fp32 F.conv1d."""
    dev = "cuda"
    g = torch.Generator().manual_seed(dil)
    x = torch.randn(2, 64, 1, 50, generator=g)
    m = torch.nn.Conv2d(64, 48, (1, 3), 1, 0, dilation=(1, dil))
    with torch.no_grad():
        m.weight.copy_(torch.randn(m.weight.shape, generator=g) / (64 * 3) ** 0.5)
    ref = F.conv1d(x[:, :, 0].half().float(), m.weight.detach()[:, :, 0].half().float(), m.bias.detach(),
                   padding=dil, dilation=dil)
    ref = F.elu(ref) if act == "elu" else ref
    md = torch.nn.Conv2d(64, 48, (1, 3), 1, 0, dilation=(1, dil)).to(dev)
    md.load_state_dict(m.state_dict())
    md = md.half()
    xd = x.to(dev).half().contiguous(memory_format=torch.channels_last)
    y = CV.conv2d(xd, md, pad=(0, dil, 0, dil), act=act)
    assert y.shape == (2, 48, 1, 50)
    assert (y[:, :, 0].float().cpu() - ref).abs().max().item() < 2e-2
