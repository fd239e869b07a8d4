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
