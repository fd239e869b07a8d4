"""t32 tiled weight layout (ops/quant.py tile32, consumed by csrc/kernels/qmm.hip / qmv.hip): a pure
byte permutation of the GPU-native block rows whose offsets are the ones the kernels compute."""
import numpy as np
import pytest
import torch

from localai_tfp_amd.formats.gguf import QType
from localai_tfp_amd.ops import quant as Q


def _native(qt, n, k, seed=0):
    raw = Q.random_quantized(np.random.default_rng(seed), int(qt), n, k)
    data, dpl = Q.repack_for_gpu(np.asarray(raw).view(np.uint8).reshape(n, -1), qt, n, k)
    return data.reshape(n, -1), (dpl.view(np.int16) if dpl is not None else None)


@pytest.mark.parametrize("qt", [QType.Q4_K, QType.Q6_K, QType.Q8_0])
def test_tile32_is_a_permutation(qt):
    n, k = 64, 512
    data, dpl = _native(qt, n, k)
    t = Q.tile32(data, dpl, int(qt), n, k).numpy()
    unit, elems = Q.T32_UNIT[qt]
    assert t.shape == (n // 32, (k // elems) * unit)
    src = np.concatenate([data.reshape(-1)] + ([dpl.view(np.uint8).reshape(-1)] if dpl is not None else []))
    # Q6_K pads each d to a dword (2 zero bytes per column per super-block)
    pad = (n * (k // 256) * 2) if qt == QType.Q6_K else 0
    assert t.size == src.size + pad
    assert np.array_equal(np.sort(t.reshape(-1)), np.sort(np.concatenate([src, np.zeros(pad, np.uint8)])))


def test_tile32_q4k_offsets():
    """byte (column n, super-block kb, quarter jq, chunk c, j) lands where qmm/qmv read it."""
    n, k = 64, 768
    data, _ = _native(QType.Q4_K, n, k, seed=3)
    t = Q.tile32(data, None, int(QType.Q4_K), n, k).numpy()
    nb = k // 256
    for col in (0, 17, 33, 63):
        g, r = divmod(col, 32)
        for kb in range(nb):
            blk = data[col, kb * 144:(kb + 1) * 144]
            base = kb * 4608
            assert np.array_equal(t[g, base + r * 16: base + r * 16 + 16], blk[:16])
            for jq in range(4):
                for c in range(2):
                    o = base + 512 + jq * 1024 + c * 512 + r * 16
                    assert np.array_equal(t[g, o:o + 16], blk[16 + 32 * jq + 16 * c: 16 + 32 * jq + 16 * c + 16])


def test_tile32_q6k_q8_offsets():
    n, k = 32, 512
    data, dpl = _native(QType.Q6_K, n, k, seed=4)
    t = Q.tile32(data, dpl, int(QType.Q6_K), n, k).numpy()
    for r in (0, 9, 31):
        for kb in range(2):
            blk = data[r, kb * 208:(kb + 1) * 208]
            base = kb * 6784
            assert np.array_equal(t[0, base + r * 16: base + r * 16 + 16], blk[192:208])
            assert t[0, base + 512 + r * 4: base + 512 + r * 4 + 2].view(np.int16)[0] == dpl[r, kb]
            for jq in range(4):
                p = base + 640 + jq * 1536
                assert np.array_equal(t[0, p + r * 16: p + r * 16 + 16], blk[32 * jq: 32 * jq + 16])
                assert np.array_equal(t[0, p + 512 + r * 16: p + 512 + r * 16 + 16], blk[32 * jq + 16: 32 * jq + 32])
                assert np.array_equal(t[0, p + 1024 + r * 16: p + 1024 + r * 16 + 16], blk[128 + 16 * jq: 128 + 16 * jq + 16])
    data, dpl = _native(QType.Q8_0, n, k, seed=5)
    t = Q.tile32(data, dpl, int(QType.Q8_0), n, k).numpy()
    for r in (0, 31):
        for kt in range(k // 64):
            base = kt * 2176
            assert np.array_equal(t[0, base + r * 4: base + r * 4 + 4].view(np.int16), dpl[r, 2 * kt: 2 * kt + 2])
            for s in range(4):
                o = base + 128 + s * 512 + r * 16
                assert np.array_equal(t[0, o:o + 16], data[r, kt * 64 + 16 * s: kt * 64 + 16 * s + 16])


def test_tile32_rejects_unaligned():
    data, _ = _native(QType.Q4_K, 48, 256)
    with pytest.raises(ValueError):
        Q.tile32(data, None, int(QType.Q4_K), 48, 256)
