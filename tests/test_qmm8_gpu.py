"""int8-MFMA GEMM on Q8_K activations (csrc/kernels/qmm8.hip) and the Q8_K quantisers (norm.hip).

Numerics oracle: ggml's quantize_row_q8_K (ops.core.quant_q8k_ref, bit-exact) and, for the GEMM, the fp32
product of the DEQUANTISED operands (dequantised Q8_K rows x dequantised weight): the kernel computes
that product with exact integer sub-block sums, so the only difference is fp32 summation order. A second
check against the unquantised fp32 activations bounds the activation-quantisation error itself."""
import numpy as np
import pytest
import torch

from localai_tfp_amd.formats.gguf import QType
from localai_tfp_amd.ops import core as K
from localai_tfp_amd.ops import linear as L
from localai_tfp_amd.ops import quant as Q
from localai_tfp_amd.ops.core import Q8KAct
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


@pytest.mark.parametrize("src", ["f32", "f16"])
def test_quant_q8k_matches_ggml(src):
    torch.manual_seed(0)
    M, Kd = 37, 4096
    x = torch.randn(M, Kd) * 3
    x[3, 17] = -40.0  # a dominant negative element: iscale > 0 branch
    x[5, 256:512] = 0.0  # an all-zero block
    xs = x if src == "f32" else x.half().float()
    ref = Q8KAct.empty(M, Kd, "cpu")
    K.quant_q8k_ref(xs, ref)
    got = Q8KAct.empty(M, Kd, DEV)
    K.quant_q8k(xs.to(DEV) if src == "f32" else x.half().to(DEV), got)
    assert torch.equal(got.q.cpu(), ref.q)
    assert torch.equal(got.d.cpu(), ref.d)
    assert torch.equal(got.bs.cpu(), ref.bs)


def test_rmsnorm_q8k():
    torch.manual_seed(1)
    M, H = 9, 4096
    x = torch.randn(M, H, device=DEV)
    w = torch.rand(H, device=DEV) + 0.5
    a = Q8KAct.empty(M, H, DEV)
    xb = torch.empty(M, H, dtype=torch.float16, device=DEV)
    K.rmsnorm_q8k(x, w, 1e-5, a, xb)
    y = x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + 1e-5) * w
    assert rel(xb, y) < 1e-3
    ref = Q8KAct.empty(M, H, "cpu")
    K.quant_q8k_ref(y.cpu(), ref)
    # rsqrt on the GPU is not correctly rounded: allow off-by-one codes, but scales within 1e-5
    assert (a.q.cpu().int() - ref.q.int()).abs().max() <= 1
    assert rel(a.d, ref.d) < 1e-5
    assert rel(a.dequant(), y) < 1e-2


CFGS = [c for c in L.QMM8_CONFIGS]


@pytest.mark.parametrize("qt", [QType.Q4_K, QType.Q6_K, QType.Q5_K])
@pytest.mark.parametrize("cfg", CFGS, ids=lambda c: "x".join(map(str, c)))
def test_qmm8_configs(qt, cfg, monkeypatch):
    """Every compiled tile configuration, every epilogue, ragged M / N tails and split-K, against the
    dequantised-operand fp32 product (tight) and the unquantised product (loose)."""
    n, k = 416, 2304  # partial column tiles; 9 super-blocks (odd split counts)
    raw, dense = make_w(qt, n, k, seed=sum(cfg) + 3)
    W = QWeight.from_ggml(raw, qt, n, k, DEV, t32=True)
    monkeypatch.setattr(L, "QMM8", True)
    assert W.to_t32() and L.qmm8_ok(W)
    for M, splits in ((77, 1), (130, 3)):
        torch.manual_seed(M)
        x = torch.randn(M, k, device=DEV)
        a = Q8KAct.empty(M, k, DEV)
        K.quant_q8k(x, a)
        ref = a.dequant().cpu() @ dense.t()
        ref_x = x.cpu() @ dense.t()
        monkeypatch.setattr(L, "QMM8_FORCE", (*cfg, splits))
        z = torch.zeros(M, n, device=DEV)
        L.qmatmul8(W, a, EPI_F32, z, out_zeroed=True)
        assert rel(z, ref) < 2e-5, (M, splits)
        assert rel(z, ref_x) < 2e-2
        acc = torch.randn(M, n, device=DEV)
        acc0 = acc.clone()
        L.qmatmul8(W, a, EPI_ADD_F32, acc)
        assert rel(acc - acc0, ref) < 1e-4
        monkeypatch.setattr(L, "QMM8_FORCE", (*cfg, 1))
        out = torch.empty(M, n, device=DEV)
        L.qmatmul8(W, a, EPI_F32, out)
        assert rel(out, ref) < 2e-5
        ob = torch.empty(M, n, dtype=torch.float16, device=DEV)
        L.qmatmul8(W, a, EPI_BF16, ob)
        assert rel(ob, ref) < 1e-3
        sw = torch.empty(M, n // 2, dtype=torch.float16, device=DEV)
        L.qmatmul8(W, a, EPI_SWIGLU, sw)
        g = ref.reshape(M, n // 32, 2, 16)
        ref_sw = torch.nn.functional.silu(g[:, :, 0].reshape(M, -1)) * g[:, :, 1].reshape(M, -1)
        assert rel(sw, ref_sw) < 2e-3


@pytest.mark.parametrize("name,qt,n,k,epi", [
    ("qkv", QType.Q4_K, 6144, 4096, EPI_F32), ("gate_up", QType.Q4_K, 28672, 4096, EPI_SWIGLU),
    ("down", QType.Q4_K, 4096, 14336, EPI_ADD_F32), ("down_q6", QType.Q6_K, 4096, 14336, EPI_ADD_F32)])
@pytest.mark.parametrize("M", [5, 128, 320])
def test_qmm8_llama3_8b_shapes(name, qt, n, k, epi, M):
    """Llama-3-8B projection shapes through the default int8 dispatch against fp32 references."""
    raw, dense = make_w(qt, n, k, seed=n + k + M)
    W = QWeight.from_ggml(raw, qt, n, k, DEV, t32=True)
    assert W.to_t32()
    torch.manual_seed(M)
    x = torch.randn(M, k, device=DEV)
    a = Q8KAct.empty(M, k, DEV)
    K.quant_q8k(x, a)
    ref = a.dequant().cpu() @ dense.t()
    if epi == EPI_SWIGLU:
        out = torch.empty(M, n // 2, dtype=torch.float16, device=DEV)
        L.qmatmul8(W, a, epi, out)
        g = ref.reshape(M, n // 32, 2, 16)
        ref = torch.nn.functional.silu(g[:, :, 0].reshape(M, -1)) * g[:, :, 1].reshape(M, -1)
        assert rel(out, ref) < 2e-3
        return
    if epi == EPI_ADD_F32:
        out = torch.randn(M, n, device=DEV)
        base = out.clone()
        L.qmatmul8(W, a, epi, out)
        assert rel(out - base, ref) < 1e-4
        return
    out = torch.zeros(M, n, device=DEV)
    L.qmatmul8(W, a, epi, out, out_zeroed=True)
    assert rel(out, ref) < 2e-5


def test_q5k_native_paths():
    """Q5_K stays Q5_K on the GPU (t32 layout, no re-quantisation): the decode GEMV (q8 activations and the
    fused RMSNorm prologue), the int8-MFMA GEMM, the f16-activation entry (quantised to Q8_K on the fly) and
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
