"""Load-time GEMM autotuner (ops/autotune.py): plan lookup by M bucket on the CPU; on the GPU, every plan it can
pick computes the same product as the fp32 reference, and the tuned dispatch matches it too."""
import numpy as np
import pytest
import torch

from localai_tfp_amd.formats.gguf import QType
from localai_tfp_amd.ops import autotune as AT
from localai_tfp_amd.ops import linear as L


def test_lookup_buckets():
    key = AT._key(4096, 4096, int(QType.Q4_K), L.EPI_ADD_F32, True)
    AT.TUNED[key] = [(128, ("q2", 2, 2, 1, 2)), (256, ("q3", 1, 2)), (512, ("rows", 256))]
    try:
        assert AT.lookup(4096, 4096, int(QType.Q4_K), L.EPI_ADD_F32, True, 100) == ("q2", 2, 2, 1, 2)
        assert AT.lookup(4096, 4096, int(QType.Q4_K), L.EPI_ADD_F32, True, 129) == ("q3", 1, 2)
        assert AT.lookup(4096, 4096, int(QType.Q4_K), L.EPI_ADD_F32, True, 512) == ("rows", 256)
        assert AT.lookup(4096, 4096, int(QType.Q4_K), L.EPI_ADD_F32, True, 513) is None
        assert AT.lookup(4096, 4096, int(QType.Q4_K), L.EPI_F32, True, 100) is None  # other epilogue: untuned
    finally:
        AT.TUNED.pop(key)


def test_candidates_respect_split_and_rows():
    c = AT.candidates(384, 6144, 4096, int(QType.Q4_K), can_split=False)
    assert all(p[-1] == 1 for p in c if p[0] in ("q2", "q3"))
    assert ("rows", 256) in c and ("rows", 128) in c
    c2 = AT.candidates(256, 4096, 14336, int(QType.Q4_K), can_split=True)
    assert any(p[0] == "q3" and p[-1] == 8 for p in c2)
    assert not any(p[0] == "rows" and p[1] >= 256 for p in c2)


@pytest.mark.gpu
@pytest.mark.parametrize("epi", [L.EPI_F32, L.EPI_ADD_F32, L.EPI_SWIGLU, L.EPI_BF16])
def test_tuned_plans_match_reference(epi, tmp_path, monkeypatch):
    from localai_tfp_amd.ops.quant import random_quantized
    monkeypatch.setenv("MX_TUNE_CACHE", str(tmp_path / "tune.json"))
    dev = torch.device("cuda")
    N, K = (2048 if epi == L.EPI_SWIGLU else 1024), 1024
    raw = random_quantized(np.random.default_rng(2), int(QType.Q4_K), N, K)
    W = L.QWeight.from_ggml(raw, int(QType.Q4_K), N, K, dev)
    assert W.to_t32()
    dense = W.dequant_gpu(torch.float16).float()
    can_split = epi not in (L.EPI_SWIGLU, L.EPI_BF16)
    buckets = (64, 128, 192, 320)
    res = AT.tune_weight(W, epi, can_split, buckets, iters=2)
    assert [b for b, _ in res] == list(buckets)
    for M in (40, 128, 200, 300):
        x = (torch.randn(M, K, device=dev) * 0.5).half()
        y = x.float() @ dense.t()
        ref = y if epi != L.EPI_SWIGLU else (lambda v: torch.nn.functional.silu(v[:, :, 0]) * v[:, :, 1])(
            y.reshape(M, N // 32, 2, 16)).reshape(M, N // 2)
        out = torch.zeros(M, N // 2, device=dev, dtype=torch.float16) if epi == L.EPI_SWIGLU else \
            torch.zeros(M, N, device=dev, dtype=torch.float16) if epi == L.EPI_BF16 else \
            torch.zeros(M, N, device=dev, dtype=torch.float32)
        L.qmatmul(W, x, epi, out, out_zeroed=True)
        torch.cuda.synchronize()
        rel = float((out.float() - ref).norm() / ref.norm())
        assert rel < 3e-3, (M, AT.lookup(N, K, int(QType.Q4_K), epi, can_split, M), rel)
    AT.TUNED.clear()
