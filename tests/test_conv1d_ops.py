"""ops/conv.py conv1d / conv_transpose1d (the H = 1 conv.hip path used by Kokoro and the VITS vocoders) against
torch.nn.functional fp32 references: CPU runs the kernel's reference formulation, GPU runs conv.hip."""
import pytest
import torch
import torch.nn.functional as F

from localai_tfp_amd.ops import conv as CV


def _devs():
    return ["cpu"] + (["cuda"] if torch.cuda.is_available() else [])


@pytest.mark.parametrize("dev", ["cpu"])
@pytest.mark.parametrize("ci,co,k,stride,pad,dil", [(8, 16, 3, 1, 1, 1), (1, 8, 3, 2, 1, 1), (16, 8, 5, 1, 6, 3),
                                                    (24, 22, 7, 1, 3, 1), (12, 12, 1, 1, 0, 1), (4, 8, 12, 6, 3, 1)])
def test_conv1d_matches_torch(dev, ci, co, k, stride, pad, dil):
    g = torch.Generator().manual_seed(ci * 100 + k)
    x = torch.randn(2, ci, 37, generator=g)
    w = torch.randn(co, ci, k, generator=g) / (ci * k) ** 0.5
    b = torch.randn(co, generator=g)
    want = F.conv1d(x, w, b, stride=stride, padding=pad, dilation=dil)
    cw = CV.conv1d_weights(w.to(dev), b.to(dev), torch.float32 if dev == "cpu" else torch.float16)
    got = CV.conv1d(x.to(dev), cw, stride=stride, padding=pad, dilation=dil).cpu()
    assert got.shape == want.shape
    assert torch.allclose(got, want, atol=1e-4 if dev == "cpu" else 2e-2, rtol=1e-3 if dev == "cpu" else 2e-2)


@pytest.mark.parametrize("dev", ["cpu"])
@pytest.mark.parametrize("ci,co,r,pad", [(16, 8, 10, 5), (8, 8, 6, 3), (4, 6, 2, 1), (6, 4, 4, 0)])
def test_conv_transpose1d_matches_torch(dev, ci, co, r, pad):
    g = torch.Generator().manual_seed(r)
    x = torch.randn(2, ci, 19, generator=g)
    w = torch.randn(ci, co, 2 * r, generator=g) / ci ** 0.5
    b = torch.randn(co, generator=g)
    want = F.conv_transpose1d(x, w, b, stride=r, padding=pad)
    cwt = CV.conv_transpose1d_weights(w.to(dev), b.to(dev), r, torch.float32 if dev == "cpu" else torch.float16)
    got = CV.conv_transpose1d(x.to(dev), cwt, pad).cpu()
    assert got.shape == want.shape
    assert torch.allclose(got, want, atol=1e-4 if dev == "cpu" else 2e-2, rtol=1e-3 if dev == "cpu" else 2e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("ci,co,k,stride,pad,dil", [(8, 16, 3, 1, 1, 1), (1, 8, 3, 2, 1, 1), (16, 8, 5, 1, 6, 3),
                                                    (128, 22, 7, 1, 3, 1), (64, 64, 1, 1, 0, 1)])
def test_conv1d_gpu(ci, co, k, stride, pad, dil):
    test_conv1d_matches_torch("cuda", ci, co, k, stride, pad, dil)


@pytest.mark.gpu
@pytest.mark.parametrize("ci,co,r,pad", [(256, 128, 10, 5), (128, 64, 6, 3)])
def test_conv_transpose1d_gpu(ci, co, r, pad):
    test_conv_transpose1d_matches_torch("cuda", ci, co, r, pad)


@pytest.mark.parametrize("ci,co,k,stride,pad,dil", [(8, 16, 3, 1, 1, 1), (1, 8, 3, 2, 1, 1), (16, 8, 5, 1, 6, 3),
                                                    (12, 12, 1, 1, 0, 1)])
def test_conv1d_gemm_matches_torch(ci, co, k, stride, pad, dil):
    g = torch.Generator().manual_seed(k)
    x = torch.randn(2, ci, 23, generator=g)
    w = torch.randn(co, ci, k, generator=g)
    b = torch.randn(co, generator=g)
    want = F.conv1d(x, w, b, stride=stride, padding=pad, dilation=dil)
    got = CV.conv1d_gemm(x, w, b, stride=stride, padding=pad, dilation=dil)
    assert got.shape == want.shape and torch.allclose(got, want, atol=1e-4, rtol=1e-4)


@pytest.mark.parametrize("k,pad,dil", [(3, 1, 1), (3, 3, 3), (5, 2, 1)])
def test_depthwise_conv1d_matches_torch(k, pad, dil):
    g = torch.Generator().manual_seed(k + dil)
    x = torch.randn(2, 6, 29, generator=g)
    w = torch.randn(6, 1, k, generator=g)
    b = torch.randn(6, generator=g)
    want = F.conv1d(x, w, b, padding=pad, dilation=dil, groups=6)
    got = CV.depthwise_conv1d(x, w, b, padding=pad, dilation=dil)
    assert got.shape == want.shape and torch.allclose(got, want, atol=1e-5)
