"""Q5_K weights on their native t32 kernels (decode GEMV, qmm2 / qmm3 GEMM, row dequantisation) against the fp32
product of the dequantised weight."""
import numpy as np
import pytest
import torch

from localai_tfp_amd.formats.gguf import QType
from localai_tfp_amd.ops import core as K
from localai_tfp_amd.ops import linear as L
from localai_tfp_amd.ops import quant as Q
from localai_tfp_amd.ops.linear import EPI_ADD_F32, EPI_BF16, EPI_F32, EPI_SWIGLU, QWeight

pytestmark = pytest.mark.gpu
DEV = "cuda"


def rel(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


def make_w(qt, n, k, seed):
    raw = Q.random_quantized(np.random.default_rng(seed), int(qt), n, k)
    dense = torch.from_numpy(Q.dequantize(raw, int(qt), (k, n)).copy()).float()
    return raw, dense


def test_q5k_native_paths():
    """Q5_K stays Q5_K on the GPU (t32 layout, no re-quantisation): the decode GEMV (q8 activations and the
    fused RMSNorm prologue), the f16-activation qmm2 / qmm3 GEMM (M > 4) and
    the row dequantisation all match the fp32 dequantised reference."""
    n, k = 384, 1024
    raw, dense = make_w(QType.Q5_K, n, k, seed=5)
    W = QWeight.from_ggml(raw, QType.Q5_K, n, k, DEV, t32=True)
    assert int(W.qtype) == int(QType.Q5_K) and W.to_t32()
    rows = torch.tensor([0, 5, 383, 77], dtype=torch.int32, device=DEV)
    got = W.dequant_gpu(torch.float32, rows)
    assert rel(got, dense[rows.long().cpu()]) < 1e-6
    torch.manual_seed(0)
    for M in (1, 3, 40):
        x = torch.randn(M, k, device=DEV)
        ref = x.cpu() @ dense.t()
        out = torch.zeros(M, n, device=DEV)
        L.qmatmul(W, x.half(), EPI_F32, out, out_zeroed=True)
        assert rel(out, ref) < 2e-2, M
        if M <= 4:
            xq = torch.empty(M, k, dtype=torch.int8, device=DEV)
            xds = torch.empty(M, k // 32, 2, device=DEV)
            K.quant_q8(x.half(), xq, xds)
            o2 = torch.zeros(M, n, device=DEV)
            L.qmatmul(W, None, EPI_F32, o2, xq=xq, xds=xds)
            assert rel(o2, ref) < 2e-2, M
