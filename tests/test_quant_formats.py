"""The GGUF block formats without a dedicated kernel layout (Q4_0, Q5_0, IQ4_NL, IQ4_XS, Q3_K exactly;
Q4_1, Q5_1, Q2_K, Q5_K re-quantised to 8 bits) are carried on the Q8_0 qmm / qmv kernels instead of a
dense 16-bit copy (ops/quant.py to_q8_0). Reference: llama.cpp loads all of them
(backend/cpp/llama/grpc-server.cpp:509-556); the gallery ships 39 Q4_0, 30 Q5_K_M, 6 Q2_K and IQ models."""
import numpy as np
import pytest
import torch

from localai_tfp_amd.formats.gguf import BLOCK, QType
from localai_tfp_amd.ops import quant as Q

EXACT = [QType.Q4_0, QType.Q5_0, QType.IQ4_NL, QType.IQ4_XS]
REQUANT = [QType.Q4_1, QType.Q5_1, QType.Q2_K, QType.Q5_K, QType.Q3_K]
SCALE_FIELDS = {QType.Q4_0: [0], QType.Q5_0: [0], QType.IQ4_NL: [0], QType.IQ4_XS: [0], QType.Q3_K: [108],
                QType.Q4_1: [0, 2], QType.Q5_1: [0, 2], QType.Q2_K: [80, 82], QType.Q5_K: [0, 2]}


def rand_blocks(qt, n, k, seed=0):
    rng = np.random.default_rng(seed)
    be, bb = BLOCK[qt]
    b = rng.integers(0, 256, (n * k // be, bb), dtype=np.uint8)
    for o in SCALE_FIELDS[qt]:  # finite, small f16 scales
        b[:, o:o + 2] = np.float16(rng.uniform(0.001, 0.01, b.shape[0])).view(np.uint8).reshape(-1, 2)
    return b.reshape(n, -1)


def test_iq4_nl_known_values():
    blk = np.zeros(18, np.uint8)
    blk[0:2] = np.array([1.0], np.float16).view(np.uint8)
    qs = np.arange(16, dtype=np.uint8)
    blk[2:18] = qs | ((15 - qs) << 4)
    y = Q.dequantize(blk, QType.IQ4_NL, (32,))
    assert np.array_equal(y[:16], Q.IQ4_KVALUES.astype(np.float32))
    assert np.array_equal(y[16:], Q.IQ4_KVALUES[::-1].astype(np.float32))


def test_iq4_xs_scales():
    blk = np.zeros(136, np.uint8)
    blk[0:2] = np.array([0.5], np.float16).view(np.uint8)
    # sub-block ib: ls = low nibble (scales_l) | 2 high bits (scales_h); choose ls = 32 + ib
    ls = 32 + np.arange(8)
    sl = np.zeros(4, np.uint8)
    for ib in range(8):
        sl[ib // 2] |= (ls[ib] & 0xF) << (4 * (ib % 2))
    sh = sum(int((ls[ib] >> 4) & 3) << (2 * ib) for ib in range(8))
    blk[2:4] = np.array([sh], np.uint16).view(np.uint8)
    blk[4:8] = sl
    blk[8:136] = 0x88  # index 8 -> codebook value 1
    y = Q.dequantize(blk, QType.IQ4_XS, (256,)).reshape(8, 32)
    assert np.allclose(y, (0.5 * np.arange(8))[:, None] * 1.0)


@pytest.mark.parametrize("qt", EXACT + REQUANT)
def test_to_q8_0(qt):
    n, k = 16, 512
    raw = rand_blocks(qt, n, k)
    w = Q.dequantize(raw, qt, (k, n))
    q8 = Q.to_q8_0(raw, qt, n, k)
    assert q8.shape == (n, k // 32 * 34)
    w8 = Q.dequantize(q8, QType.Q8_0, (k, n))
    err = float(np.abs(w8 - w).max() / np.abs(w).max())
    if qt in EXACT[:3]:
        assert err == 0.0, err
    else:
        assert err < 5e-3, err


def test_iq_codebook_types_parse_but_refuse_clearly():
    raw = np.zeros(66, np.uint8)
    with pytest.raises(NotImplementedError, match="codebook"):
        Q.dequantize(raw, QType.IQ2_XXS, (256,))


@pytest.mark.gpu
@pytest.mark.parametrize("qt", EXACT + REQUANT)
def test_carried_formats_gpu(qt):
    """On the GPU these weights are Q8_0 t32 tiles (never a dense copy) and both kernels (qmv at
    M <= 4, qmm above) match the fp32 product with the checkpoint's own dequantisation."""
    from localai_tfp_amd.ops.linear import EPI_F32, QWeight, qmatmul
    from localai_tfp_amd.ops import core as K
    n, k = 256, 1024
    raw = rand_blocks(qt, n, k, seed=int(qt))
    dense = torch.from_numpy(Q.dequantize(raw, qt, (k, n)).copy())
    W = QWeight.from_ggml(raw, int(qt), n, k, "cuda")
    assert W.is_quant and int(W.qtype) == int(QType.Q8_0) and W.src_qtype == int(qt)
    assert W.to_t32()
    for M in (1, 3, 40, 200):
        x = torch.randn(M, k).half()
        ref = x.float() @ dense.t()
        out = torch.zeros(M, n, device="cuda")
        if M <= 4:
            xq = torch.empty(M, k, dtype=torch.int8, device="cuda")
            xds = torch.empty(M, k // 32, 2, device="cuda")
            K.quant_q8(x.cuda(), xq, xds)
            qmatmul(W, None, EPI_F32, out, xq=xq, xds=xds, out_zeroed=True)
            tol = 2e-2
        else:
            qmatmul(W, x.cuda(), EPI_F32, out, out_zeroed=True)
            tol = 1e-2
        rel = float((out.cpu() - ref).norm() / ref.norm())
        assert rel < tol, (qt.name, M, rel)


# ---- MX4F / MX5F: Q4_0 / Q4_1 / Q5_0 / Q5_1 at their own bit width in the t32 kernels --------------------
Q32 = [QType.Q4_0, QType.Q4_1, QType.Q5_0, QType.Q5_1]


@pytest.mark.parametrize("qt", Q32)
def test_to_mxf_exact(qt):
    """The re-layout is exact (w = s * code + m with the checkpoint's own f16 s / m; Q4_0 / Q5_0 offsets
    -8 d / -16 d are exact f16 products), 5 / 6 bits per weight instead of Q8_0's 8.5, and the t32 tiling is a
    byte permutation."""
    n, k = 64, 768
    raw = rand_blocks(qt, n, k, seed=3)
    ref = Q.dequantize(raw, qt, (k, n))
    mx, mt = Q.to_mxf(raw, qt, n, k)
    assert mt == (QType.MX5F if qt in (QType.Q5_0, QType.Q5_1) else QType.MX4F)
    assert mx.shape == (n, k // 256 * BLOCK[mt][1])
    assert np.array_equal(Q.dequantize(mx, mt, (k, n)), ref)
    t = Q.tile32(mx, None, mt, n, k)
    assert t.numel() == mx.size and np.array_equal(np.sort(t.numpy().reshape(-1)), np.sort(mx.reshape(-1)))
    q8 = Q.to_q8_0(mx, mt, n, k)  # the fallback for weights that cannot be tiled: exact for Q4_0 / Q5_0
    err = np.abs(Q.dequantize(q8, QType.Q8_0, (k, n)) - ref).max()
    assert err == 0.0 if qt in (QType.Q4_0, QType.Q5_0) else err < 5e-3 * np.abs(ref).max()


@pytest.mark.gpu
@pytest.mark.parametrize("qt", Q32)
def test_mxf_kernels_gpu(qt, monkeypatch):
    """MX4F / MX5F through every t32 kernel: decode GEMV (q8 rows and the fused quantise / RMSNorm prologue,
    every epilogue, split-K), the LDS-DMA MFMA GEMM (several tile shapes, ragged M / N, split-K, SwiGLU) and the
    row dequantisation, against the fp32 product with the checkpoint's own dequantisation."""
    from localai_tfp_amd.ops import core as K
    from localai_tfp_amd.ops import linear as L
    from localai_tfp_amd.ops.linear import EPI_ADD_F32, EPI_BF16, EPI_F32, EPI_SWIGLU, QWeight, qmatmul
    n, k = 416, 2304
    raw = rand_blocks(qt, n, k, seed=int(qt) + 5)
    dense = torch.from_numpy(Q.dequantize(raw, qt, (k, n)).copy())
    W = QWeight.from_ggml(raw, int(qt), n, k, "cuda", t32=True)
    assert int(W.qtype) in (int(QType.MX4F), int(QType.MX5F)) and W.src_qtype == int(qt)
    assert W.to_t32() and W.layout == "t32"
    rows = torch.tensor([0, 7, n - 1, 100], dtype=torch.int32, device="cuda")
    assert torch.equal(W.dequant_gpu(torch.float32, rows).cpu(), dense[rows.long().cpu()])

    def rel(a, b):
        return float((a.float().cpu() - b).norm() / b.norm())
    g = torch.Generator().manual_seed(1)
    for M in (1, 3, 4):
        x = torch.randn(M, k, generator=g).half().cuda()
        xq = torch.empty(M, k, dtype=torch.int8, device="cuda")
        xds = torch.empty(M, k // 32, 2, device="cuda")
        K.quant_q8(x, xq, xds)
        xr = (xq.float().reshape(M, k // 32, 32) * xds[:, :, :1]).reshape(M, k).cpu()
        ref = xr @ dense.t()
        out = torch.empty(M, n, device="cuda")
        qmatmul(W, None, EPI_F32, out, xq=xq, xds=xds)
        assert rel(out, ref) < 2e-3, M
        acc = torch.randn(M, n, device="cuda")
        acc0 = acc.clone()
        qmatmul(W, None, EPI_ADD_F32, acc, xq=xq, xds=xds)
        assert rel(acc - acc0, ref) < 2e-3
        sw = torch.empty(M, n // 2, dtype=torch.float16, device="cuda")
        qmatmul(W, None, EPI_SWIGLU, sw, xq=xq, xds=xds)
        gg = ref.reshape(M, n // 32, 2, 16)
        assert rel(sw, torch.nn.functional.silu(gg[:, :, 0].reshape(M, -1)) * gg[:, :, 1].reshape(M, -1)) < 1e-2
        # fused prologue: 16-bit rows quantised in the GEMV / fp32 residual rows RMS-normalised first
        o2 = torch.zeros(M, n, device="cuda")
        assert L.qmv_fused(W, x, EPI_F32, o2, out_zeroed=True)
        assert rel(o2, x.float().cpu() @ dense.t()) < 2e-2
        r32 = torch.randn(M, k, generator=g).cuda()
        nw = (torch.rand(k, generator=g) + 0.5).cuda()
        o3 = torch.empty(M, n, device="cuda")
        assert L.qmv_fused(W, r32, EPI_F32, o3, norm=nw, eps=1e-5)
        y = (r32 * torch.rsqrt(r32.pow(2).mean(-1, keepdim=True) + 1e-5) * nw).cpu()
        assert rel(o3, y @ dense.t()) < 2e-2
    for M, cfg in ((40, None), (200, None), (77, (4, 2, 1, 2)), (130, (2, 10, 1, 2)), (96, (2, 1, 2, 1)),
                   (256, (4, 1, 2, 1)), (300, (8, 1, 1, 3))):
        monkeypatch.setattr(L, "QMM2", cfg is not None)
        monkeypatch.setattr(L, "QMM2_FORCE", cfg)
        x = torch.randn(M, k, generator=g).half()
        ref = x.float() @ dense.t()
        out = torch.zeros(M, n, device="cuda")
        qmatmul(W, x.cuda(), EPI_F32, out, out_zeroed=True)
        assert rel(out, ref) < 5e-3, (M, cfg)
        ob = torch.empty(M, n, dtype=torch.float16, device="cuda")
        qmatmul(W, x.cuda(), EPI_BF16, ob)
        assert rel(ob, ref) < 5e-3, (M, cfg)
        sw = torch.empty(M, n // 2, dtype=torch.float16, device="cuda")
        qmatmul(W, x.cuda(), EPI_SWIGLU, sw)
        gg = ref.reshape(M, n // 32, 2, 16)
        assert rel(sw, torch.nn.functional.silu(gg[:, :, 0].reshape(M, -1)) * gg[:, :, 1].reshape(M, -1)) < 1e-2
