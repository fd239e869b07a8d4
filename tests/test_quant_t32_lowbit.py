"""Q3_K / Q2_K in their own t32 tiled layouts (ops/quant.py tile32; kernels: qmv.hip TUnit<Q3_K|Q2_K>,
qmm2.hip Q2B<Q3_K|Q2_K>, dequant_t32): a numpy decoder that indexes the tiled bytes exactly as the kernels do
(unit offsets, chunk / half / lane-half addressing, the kmask scale unpack, the 3-bit code sign handling) must
reproduce the ggml dequantisation (dq_q3_k / dq_q2_k) bit for bit; and QWeight keeps them native (no Q8_0
re-expression). Block-format parity with llama.cpp itself is unpinned (no GGUF fixture of these types here)."""
import numpy as np
import pytest
import torch

from localai_tfp_amd.formats.gguf import QType
from localai_tfp_amd.ops import quant as Q


def _decode_t32(t32: np.ndarray, qt, n: int, k: int) -> np.ndarray:
    """Tiled bytes -> fp32 [n, k], element by element through the kernels' addressing."""
    unit = Q.T32_UNIT[qt][0]
    nsb = k // 256
    out = np.zeros((n, k), np.float32)
    for col in range(n):
        g, r = col // 32, col % 32
        for sb in range(nsb):
            base = t32[g, sb * unit:(sb + 1) * unit]
            for e in range(256):
                nn, j, half, i = e >> 7, (e >> 5) & 3, (e >> 4) & 1, e & 15
                isx = 8 * nn + 2 * j + half
                if qt == QType.Q3_K:
                    qb = base[1536 + nn * 1024 + half * 512 + r * 16 + i]
                    hm = base[512 + half * 512 + r * 16 + i]
                    hd = base[r * 16:r * 16 + 16].copy()
                    w = hd[:12].view(np.uint32)
                    km1, km2 = np.uint32(0x03030303), np.uint32(0x0F0F0F0F)
                    sw = [(w[0] & km2) | ((w[2] & km1) << 4), (w[1] & km2) | (((w[2] >> 2) & km1) << 4),
                          ((w[0] >> 4) & km2) | (((w[2] >> 4) & km1) << 4), ((w[1] >> 4) & km2) | (((w[2] >> 6) & km1) << 4)]
                    sc = int((int(sw[isx >> 2]) >> (8 * (isx & 3))) & 0xFF) - 32
                    d = float(hd[12:14].view(np.float16)[0])
                    c = ((int(qb) >> (2 * j)) & 3) | (((int(hm) >> (4 * nn + j)) & 1) << 2)
                    out[col, sb * 256 + e] = np.float32(d) * np.float32(sc) * np.float32(c - 4)
                else:
                    qb = base[640 + nn * 1024 + half * 512 + r * 16 + i]
                    b = int(base[r * 16 + isx])
                    dd = base[512 + r * 4:512 + r * 4 + 4].copy().view(np.float16)
                    q = (int(qb) >> (2 * j)) & 3
                    out[col, sb * 256 + e] = (np.float32(dd[0]) * np.float32(b & 15) * np.float32(q)
                                              - np.float32(dd[1]) * np.float32(b >> 4))
    return out


@pytest.mark.parametrize("qt", [QType.Q3_K, QType.Q2_K])
def test_t32_layout_decodes_like_ggml(qt):
    n, k = 64, 512
    raw = Q.random_quantized(np.random.default_rng(int(qt)), int(qt), n, k)
    ref = Q.dequantize(raw, qt, (k, n)).reshape(n, k)
    assert np.isfinite(ref).all() and ref.std() > 0
    t = Q.tile32(np.asarray(raw).reshape(n, -1), None, int(qt), n, k).numpy()
    assert t.shape == (n // 32, (k // 256) * Q.T32_UNIT[qt][0])
    got = _decode_t32(t, qt, n, k)
    np.testing.assert_allclose(got, ref, rtol=1e-6, atol=1e-9)


def test_q3k_scale_pack_roundtrip():
    rng = np.random.default_rng(0)
    sc = rng.integers(0, 64, size=(50, 16)).astype(np.uint32)
    blk = np.zeros((50, 110), np.uint8)
    blk[:, 96:108] = Q._pack_q3k_scales(sc)
    blk[:, 108:110] = np.float16(1.0).tobytes()[0], np.float16(1.0).tobytes()[1]
    blk[:, 0:32] = 0xFF  # every high bit set: code = q, value = sc - 32 for q = 0 -> (sc-32)*(0+4-4)=0; use q = 1
    blk[:, 32:96] = 0x55  # every 2-bit field = 1 -> value = (sc - 32) * 1
    v = Q.dequantize(blk.reshape(-1), QType.Q3_K, (256, 50)).reshape(50, 16, 16)
    np.testing.assert_array_equal(v[:, :, 0], sc.astype(np.float32) - 32)


@pytest.mark.parametrize("qt", [QType.Q3_K, QType.Q2_K])
def test_qweight_keeps_lowbit_native_on_cpu(qt):
    from localai_tfp_amd.ops.linear import QWeight
    n, k = 32, 256
    raw = Q.random_quantized(np.random.default_rng(5), int(qt), n, k)
    w = QWeight.from_ggml(raw, int(qt), n, k, "cpu", t32=True)
    assert w.qtype == int(qt) and w.is_quant  # no Q8_0 / dense re-expression
    x = torch.randn(3, k)
    out = torch.empty(3, n)
    from localai_tfp_amd.ops.linear import EPI_F32, qmatmul
    qmatmul(w, x, EPI_F32, out)
    ref = x @ torch.from_numpy(Q.dequantize(raw, qt, (k, n)).reshape(n, k)).t()
    assert torch.allclose(out, ref, atol=1e-4)
